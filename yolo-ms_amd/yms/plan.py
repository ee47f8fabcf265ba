"""Static execution plans for the YOLOv8 / YOLO-MS detector graph on MI355X.

A plan is built once per (module, input shape, compute dtype, train/eval) by walking
the module tree (each yolov8 module implements ``emit``).  It records

* NHWC activation buffers (channel stride ``ld`` = round8(C)) laid out in one arena;
  every channel concatenation of the reference (C2f ``torch.cat`` at
  components.py:119, SPPF :146, neck yolov8_neck.py:79-91, head yolov8_head.py:122)
  is a *placement*: producers write at a channel offset of the consumer's buffer,
  so no copy kernel exists;
* a list of ops (ConvOp, BiasConvOp, UpsampleOp, SppfPoolOp, InputOp) whose
  forward/backward are launches of the hand-written HIP kernels in libyms.so.

Training: forward stores the pre-BN conv output z, BN batch statistics are fused in
the conv epilogue (per-tile partial sums) and finalised by one tiny kernel which also
updates running_mean/var exactly like nn.BatchNorm2d(eps=1e-3, momentum=0.03).
Backward walks the ops in reverse: BN+SiLU backward (two-pass reduction), dgrad and
wgrad implicit GEMMs, fp32 parameter gradients written into one flat arena (ordered
in backward-completion order so that data-parallel all-reduce buckets complete
contiguously -- see yms.dist).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib as L

ALIGN = 256
# (the BN backward finalize inside the reduce launch -- last-arriving block -- was measured slower,
# 19.5-19.7 ms separate vs 20.4-21.3 ms fused, profiles/r02_ab_bn_fused_priority_graph.txt: it puts one
# block's serial sum of the partial table on the critical path; the fused launch serves the head's
# bias gradients only, yms_bias_bwd)
BN_MOMENTUM = 0.03   # components.py:73
BN_EPS = 1e-3


def r8(c):
    return (c + 7) // 8 * 8


def _al(x):
    return (x + ALIGN - 1) // ALIGN * ALIGN


class Buf:
    __slots__ = ("idx", "n", "h", "w", "ld", "name", "off", "zero", "needs_grad")

    def __init__(self, idx, n, h, w, ld, name, zero):
        self.idx, self.n, self.h, self.w, self.ld, self.name, self.zero = idx, n, h, w, ld, name, zero
        self.off = None
        self.needs_grad = True

    @property
    def npix(self):
        return self.n * self.h * self.w


class View:
    __slots__ = ("buf", "off", "c")

    def __init__(self, buf, off, c):
        self.buf, self.off, self.c = buf, off, c

    def slot(self, k, c):
        """Channel sub-view [off + k, off + k + c) (8-aligned: the kernels move 16-B chunks)."""
        if (self.off + k) % 8:
            raise RuntimeError(f"yms: channel slice at offset {self.off + k} is not a multiple of 8")
        return View(self.buf, self.off + k, c)

    @property
    def h(self):
        return self.buf.h

    @property
    def w(self):
        return self.buf.w


class Layout:
    """Arena allocator used while finalising a plan (byte offsets)."""

    def __init__(self):
        self.size = 0

    def alloc(self, nbytes):
        off = self.size
        self.size += _al(max(int(nbytes), 1))
        return off


def _overlap(a, b):
    return a.buf is b.buf and a.off < b.off + b.c and b.off < a.off + a.c


def _check_not_in_place(op, y):
    """GradTracker.release(y) clears y's gradient interval once its producer has taken it, so an
    earlier writer of that memory stores instead of accumulating.  That is only sound when no
    input of the same op lives in y's channels (an in-place op would lose its input's gradient):
    every op's inputs are checked here."""
    for name, v in vars(op).items() if hasattr(op, "__dict__") else ():
        vs = v if isinstance(v, (list, tuple)) else (v,)
        for u in vs:
            if isinstance(u, View) and u is not y and name != "y" and _overlap(u, y):
                raise RuntimeError(f"yms: {type(op).__name__}.{name} overlaps its output (in-place op)")


class GradTracker:
    """Backward-order simulation deciding, for every write into an activation-gradient slice,
    whether it is the first one (plain store) or must accumulate; buffers that are read
    before any write (or carry zero-padded channels) are zeroed once per backward."""

    def __init__(self):
        self.written = {}
        self.zero = set()
        self.writes = None       # buffers any op writes a gradient into (recorded after the seeds)

    def _iv(self, v):
        return v.off, v.off + v.c

    def _covered(self, v):
        lo, hi = self._iv(v)
        ivs = sorted(self.written.get(v.buf.idx, []))
        cur = lo
        for a, b in ivs:
            if a <= cur < b:
                cur = b
            if cur >= hi:
                return True
        return cur >= hi

    def _touch(self, v):
        lo, hi = self._iv(v)
        return any(a < hi and lo < b for a, b in self.written.get(v.buf.idx, []))

    def _zero_buf(self, v):
        self.zero.add(v.buf.idx)
        self.written[v.buf.idx] = [(0, v.buf.ld)]

    def read(self, v):
        if not self._covered(v):
            self._zero_buf(v)

    def release(self, v):
        """The producer of v has taken its gradient (backward order): the slice's gradient is dead,
        so a later (earlier-in-forward) writer of the same memory stores instead of accumulating.
        Only matters where one buffer slice holds two tensors in turn (MSBlock: Y_{i+1} written over
        X_{i+1}); buffers with zeroed padding always accumulate and are never reused that way."""
        if v.buf.zero:
            return
        lo, hi = self._iv(v)
        out = []
        for a, b in self.written.get(v.buf.idx, []):
            if b <= lo or a >= hi:
                out.append((a, b))
                continue
            if a < lo:
                out.append((a, lo))
            if b > hi:
                out.append((hi, b))
        self.written[v.buf.idx] = out

    def write(self, v):
        """-> accumulate flag (0 = first writer, plain store)."""
        if self.writes is not None:
            self.writes.add(v.buf.idx)
        if v.buf.zero:                       # padded channels must stay zero: zero whole buffer
            if v.buf.idx not in self.zero:
                self._zero_buf(v)
            return 1
        if not self._touch(v):
            self.written.setdefault(v.buf.idx, []).append(self._iv(v))
            return 0
        if not self._covered(v):
            self._zero_buf(v)
        return 1


class Rt:
    """Per-call runtime state."""

    def __init__(self, plan, base, stream, training):
        self.plan = plan
        self.base = base
        self.gbase = None
        self.st = stream
        self.training = training
        self.pg_base = None      # flat fp32 param-grad arena pointer
        self.eval_base = None    # eval cache base pointer (packed weights + folded BN)
        self.prepacked = False   # training: all weight packs already issued (Plan.prepack)
        self.stem_x = {}         # plan input index -> NCHW fp32 tensor read by a stem ConvOp
        self._ev = None          # wst(): main -> side ordering event
        self.main = None         # backward: torch stream objects (main, weight-gradient side stream)
        self.side = None
        self.gover = None        # backward: buffer idx -> incoming output-gradient tensor used in place
        # backward: enqueue each layer's weight gradient (side stream) BEFORE its input gradient, so
        # the side stream's wait on the main stream ends at the BN apply, not after the dgrad
        # (YMS_WGRAD_FIRST=1: every layer; default "tail": only the layers whose input is the stem's
        # output, the step's tail, where the main stream has nothing left but the stem's input-side
        # chain and the side stream's last weight gradient otherwise starts after it; 0: none)
        self.wgrad_first = os.environ.get("YMS_WGRAD_FIRST", "tail") == "1"

    def a(self, v):
        return self.base + v.buf.off

    def g(self, v):
        o = self.gover.get(v.buf.idx) if self.gover else None
        return o if o is not None else self.gbase + v.buf.off

    def cnt(self, i):
        """Arrival counter i of the in-launch BN-backward finalize (zeroed at backward start)."""
        return self.gbase + self.plan.gscratch["cnt"] + 16 * i

    def wst(self):
        """Stream for a weight-gradient GEMM (+ its split reduce): a side stream ordered after
        everything enqueued on the main stream so far.  wgrad is off the backward's critical
        path (only the optimizer consumes dw), so it overlaps the next layers' HBM-bound BN
        backward kernels and dgrads.  Only wgrads use the side stream, so the shared
        "wgrad" scratch stays in stream order."""
        if self.side is None:
            return self.st
        # one reusable event (a wait binds the record made before it), not a new one per layer
        if self._ev is None:
            self._ev = torch.cuda.Event()
        self._ev.record(self.main)
        self.side.wait_event(self._ev)
        return self.side.cuda_stream


class ConvOp:
    """Conv block = Conv2d(bias=False) -> BatchNorm2d -> SiLU/Identity (+ residual),
    components.py:69-77 (residual: Bottleneck :87-93)."""

    def __init__(self, b, mod, x, y, res, act):
        conv = mod.conv
        if conv.groups != 1 or conv.dilation != (1, 1) or conv.kernel_size[0] != conv.kernel_size[1]:
            raise RuntimeError("yms: only square, ungrouped, undilated convolutions are supported")
        if conv.stride[0] != conv.stride[1] or conv.padding[0] != conv.padding[1]:
            raise RuntimeError("yms: anisotropic stride/padding unsupported")
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        self.mod, self.x, self.y, self.res, self.act = mod, x, y, res, act
        self.shape = L.ConvShape(b.n, x.h, x.w, conv.in_channels, conv.out_channels, k, s, p,
                                 y.h, y.w, b.dt)
        self.sp = ctypes.pointer(self.shape)
        self.c = conv.out_channels
        self.npix = b.n * y.h * y.w
        self.pw = b.param(conv, "weight")
        self.pg = b.param(mod.bn, "weight")
        self.pb = b.param(mod.bn, "bias")
        self.flops = 2 * self.npix * self.c * conv.in_channels * k * k
        self.stem_input = None   # plan input index when this conv reads the NCHW input directly
        self.tail_wgrad_first = False   # enqueue the weight gradient before the input gradient (Plan)
        self.bnred_for = None    # producer whose BN-backward reduce this conv's input gradient computes
        self.bnred_by = None     # consumer whose input gradient computes this conv's BN-backward reduce
        self.bnred_key = None    # grad-scratch region of the partial rows of THIS conv's reduce
        self.bnred_wkey = None   # grad-scratch region this conv's input gradient writes (its producer's)

    def layout(self, plan, La, Le):
        es = plan.es
        self.wp_elems = L.lib().yms_conv_packed_elems(self.sp, 0)
        self.wpt_elems = L.lib().yms_conv_packed_elems(self.sp, 1)
        c = self.c
        # eval cache: packed fwd weights + folded scale/shift
        self.e_wp = Le.alloc(self.wp_elems * es)
        self.e_sc = Le.alloc(4 * c)
        self.e_sh = Le.alloc(4 * c)
        if plan.training:
            self.zld = r8(c)
            self.z = La.alloc(self.npix * self.zld * es)
            self.t_wp = La.alloc(self.wp_elems * es)
            self.t_wpt = La.alloc(self.wpt_elems * es)
            self.sc = La.alloc(4 * c)
            self.sh = La.alloc(4 * c)
            self.mi = La.alloc(8 * c)
            if self.stem_input is not None:
                self.stats_rows = L.lib().yms_conv_stem_stats_rows(self.sp)
            else:
                self.stats_rows = L.lib().yms_conv_stats_rows(self.sp)
            self.stats_ld = L.lib().yms_conv_stats_ld(self.sp)
            plan.need_scratch("stats", 4 * self.stats_rows * (2 * self.stats_ld + 1))
            self.bwd_rows = L.lib().yms_bn_bwd_rows(self.npix, c)
            plan.need_scratch("bwd", 4 * 2 * c * self.bwd_rows)
            plan.need_scratch("coef", 8 * c)
            self.wg_ws = L.lib().yms_conv_wgrad_ws_bytes(self.sp)
            plan.need_scratch("wgrad", self.wg_ws)
            if self.stem_input is not None:
                # its own scratch: the stem's wgrad runs on the MAIN stream while the side stream
                # may still be in the previous layers' wgrads, which share the "wgrad" scratch
                self.wg_ws = L.lib().yms_conv_stem_wgrad_ws_bytes(self.sp)
                plan.need_scratch("stemwg", self.wg_ws)

    def pack_specs(self):
        """(shape, fp32 weight, arena byte offset of the packed copy, for_dgrad) per training pack."""
        w = self.mod.conv.weight.data_ptr()
        return [(self.sp, w, self.t_wp, 0), (self.sp, w, self.t_wpt, 1)]

    def prepare_eval(self, rt):
        m = self.mod
        L.call("yms_conv_pack_weight", self.sp, m.conv.weight.data_ptr(), rt.eval_base + self.e_wp, 0, rt.st)
        bn = m.bn
        L.call("yms_bn_fold", self.c, bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
               bn.running_var.data_ptr(), ctypes.c_float(bn.eps), rt.eval_base + self.e_sc,
               rt.eval_base + self.e_sh, rt.st)

    def fwd(self, rt):
        x, y, r = self.x, self.y, self.res
        xl, yl = x.buf.ld, y.buf.ld
        rp = rt.a(r) if r is not None else None
        rl, ro = (r.buf.ld, r.off) if r is not None else (0, 0)
        stem = self.stem_input is not None
        if not rt.training:
            eb = rt.eval_base
            if stem:
                L.call("yms_conv_stem_fwd", self.sp, rt.stem_x[self.stem_input].data_ptr(),
                       self.mod.conv.weight.data_ptr(), rt.a(y), yl, y.off, eb + self.e_sc, eb + self.e_sh,
                       self.act, None, 0, rt.st)
                return
            L.call("yms_conv_fwd", self.sp, rt.a(x), xl, x.off, eb + self.e_wp, rt.a(y), yl, y.off,
                   eb + self.e_sc, eb + self.e_sh, self.act, rp, rl, ro, None, rt.st)
            return
        m = self.mod
        base = rt.base
        if not rt.prepacked:
            L.call("yms_conv_pack_weight", self.sp, m.conv.weight.data_ptr(), base + self.t_wp, 0, rt.st)
            L.call("yms_conv_pack_weight", self.sp, m.conv.weight.data_ptr(), base + self.t_wpt, 1, rt.st)
        stats = base + rt.plan.scratch["stats"]
        if stem:
            L.call("yms_conv_stem_fwd", self.sp, rt.stem_x[self.stem_input].data_ptr(), m.conv.weight.data_ptr(),
                   base + self.z, self.zld, 0, None, None, L.ACT_NONE, stats, self.stats_ld, rt.st)
        else:
            L.call("yms_conv_fwd", self.sp, rt.a(x), xl, x.off, base + self.t_wp, base + self.z, self.zld, 0,
                   None, None, L.ACT_NONE, None, 0, 0, stats, rt.st)
        bn = m.bn
        L.call("yms_bn_finalize", self.c, stats, self.stats_rows, self.stats_ld, self.npix, bn.weight.data_ptr(),
               bn.bias.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
               ctypes.c_float(bn.momentum if bn.momentum is not None else BN_MOMENTUM),
               ctypes.c_float(bn.eps), base + self.mi, base + self.sc, base + self.sh, rt.st)
        L.call("yms_affine_act", rt.plan.dt, self.npix, self.c, base + self.z, self.zld, 0, base + self.sc,
               base + self.sh, self.act, rp, rl, ro, rt.a(y), yl, y.off, rt.st)

    def plan_grads(self, T):
        T.read(self.y)
        self.acc_res = T.write(self.res) if self.res is not None else 0
        self.acc_x = T.write(self.x) if self.x.buf.needs_grad else 0

    def bwd(self, rt):
        x, y, r = self.x, self.y, self.res
        base, dt, c = rt.base, rt.plan.dt, self.c
        gy, gyl, gyo = rt.g(y), y.buf.ld, y.off
        ws = rt.gbase + rt.plan.gscratch["bwd"]
        coef = rt.gbase + rt.plan.gscratch["coef"]
        z = base + self.z
        if self.bnred_by is not None:
            # the consumer's input gradient (its last writer) already summed the partial rows
            L.call("yms_bn_act_bwd_finalize", c, rt.gbase + rt.plan.gscratch[self.bnred_key], self.bnred_rows,
                   self.npix, rt.pgrad(self.pg), rt.pgrad(self.pb), coef, rt.st)
        else:
            L.call("yms_bn_act_bwd_reduce", dt, self.npix, c, z, self.zld, 0, gy, gyl, gyo, base + self.sc,
                   base + self.sh, base + self.mi, self.act, ws, rt.st)
            L.call("yms_bn_act_bwd_finalize", c, ws, self.bwd_rows, self.npix,
                   rt.pgrad(self.pg), rt.pgrad(self.pb), coef, rt.st)
        if self.stem_input is not None:
            # the stem's input needs no gradient: the apply pass is fused into the weight
            # gradient, which reads gy, z and the NCHW input.
            # It runs on the MAIN stream: the stem is the backward's last layer, so the main stream
            # is idle from here on while the side stream still drains the previous layers'
            # weight gradients -- the two then overlap instead of queueing (step tail 0.53 ms).
            dw = rt.pgrad(self.pw)
            if dw is not None:
                st = rt.st
                xs = rt.stem_x[self.stem_input]
                L.call("yms_conv_stem_wgrad", self.sp, xs.data_ptr(), gy, gyl, gyo, z, self.zld, 0, base + self.sc,
                       base + self.sh, base + self.mi, coef, self.act,
                       rt.gbase + rt.plan.gscratch["stemwg"],
                       self.wg_ws, dw, 0, st)
            return
        gres = rt.g(r) if r is not None else None
        gro = (r.buf.ld, r.off) if r is not None else (0, 0)
        dz = z                   # dz overwrites z in place
        L.call("yms_bn_act_bwd_apply", dt, self.npix, c, z, self.zld, 0, gy, gyl, gyo, base + self.sc,
               base + self.sh, base + self.mi, coef, self.act, dz, self.zld, 0, gres, gro[0], gro[1], self.acc_res,
               rt.st)
        def dgrad():
            if not x.buf.needs_grad:
                return
            q = self.bnred_for
            if q is not None:
                # + the producer's BN-backward reduce in the epilogue (dx = the producer's final gy)
                L.call("yms_conv_dgrad_bnred", self.sp, dz, self.zld, 0, base + self.t_wpt, rt.g(x), x.buf.ld, x.off,
                       self.acc_x, base + q.z, q.zld, 0, base + q.sc, base + q.sh, base + q.mi, q.act,
                       rt.gbase + rt.plan.gscratch[self.bnred_wkey], rt.st)
            else:
                L.call("yms_conv_dgrad", self.sp, dz, self.zld, 0, base + self.t_wpt, rt.g(x), x.buf.ld, x.off,
                       self.acc_x, rt.st)

        dw = rt.pgrad(self.pw)
        first = rt.wgrad_first or self.tail_wgrad_first
        if not first:
            dgrad()
        if dw is not None:
            wsz = self.wg_ws
            L.call("yms_conv_wgrad", self.sp, rt.a(x), x.buf.ld, x.off, dz, self.zld, 0,
                   rt.gbase + rt.plan.gscratch["wgrad"], wsz, dw, 0, rt.wst())
        if first:
            dgrad()

    def grad_params(self):
        return [self.pb, self.pg, self.pw]


class SiblingConvOp:
    """Two Conv blocks (Conv2d -> BN -> act, components.py:69-77) that read the SAME input view --
    the head's box[i][0] and cls[i][0] (yolov8_head.py:84-85, 99-100: Conv(c_i, 4*ch) and
    Conv(c_i, nc), both 3x3 of x_i) -- with their outputs as the two channel slots of one buffer
    [.., c_a | c_b].  The forward runs each member's conv (its own tile shape) into its slot of one
    z buffer and its own BN finalize; everything after is one pass over the c_a + c_b channels:
    ONE affine pass; in the backward ONE BN reduce / finalize / apply, ONE input gradient (a single
    GEMM with K = k^2 (c_a + c_b): dx is stored once instead of stored, re-read and accumulated by a
    second dgrad) and ONE weight gradient (M = c_a + c_b).  The members' parameter gradients are
    adjacent in the flat gradient arena (grad_params order), so the fused backward writes them in
    place; the transposed dgrad weight is packed from both fp32 weights by one pack job (w2 / split)."""

    def __init__(self, b, mods, x, y, act):
        self.x, self.y, self.res, self.act = x, y, None, act
        self.members, self.offs = [], []
        off = 0
        for m in mods:
            self.offs.append(off)
            self.members.append(ConvOp(b, m, x, y.slot(off, m.conv.out_channels), None, act))
            off += m.conv.out_channels
        self.c = off
        m0 = self.members[0]
        sh0 = m0.shape
        self.shape = L.ConvShape(sh0.n, sh0.h, sh0.w, sh0.cin, self.c, sh0.k, sh0.stride, sh0.pad, sh0.ho, sh0.wo, sh0.dtype)
        self.sp = ctypes.pointer(self.shape)
        self.npix = m0.npix
        self.flops = sum(m.flops for m in self.members)
        self.stem_input = None

    def layout(self, plan, La, Le):
        es = plan.es
        for m in self.members:
            m.wp_elems = L.lib().yms_conv_packed_elems(m.sp, 0)
            m.e_wp = Le.alloc(m.wp_elems * es)
            m.e_sc = Le.alloc(4 * m.c)
            m.e_sh = Le.alloc(4 * m.c)
        if not plan.training:
            return
        c = self.c
        self.zld = r8(c)
        self.z = La.alloc(self.npix * self.zld * es)
        for m in self.members:
            m.t_wp = La.alloc(m.wp_elems * es)
            m.stats_rows = L.lib().yms_conv_stats_rows(m.sp)
            m.stats_ld = L.lib().yms_conv_stats_ld(m.sp)
            plan.need_scratch("stats", 4 * m.stats_rows * (2 * m.stats_ld + 1))
        self.wpt_elems = L.lib().yms_conv_packed_elems(self.sp, 1)
        self.t_wpt = La.alloc(self.wpt_elems * es)
        self.sc = La.alloc(4 * c)
        self.sh = La.alloc(4 * c)
        self.mi = La.alloc(8 * c)
        self.bwd_rows = L.lib().yms_bn_bwd_rows(self.npix, c)
        plan.need_scratch("bwd", 4 * 2 * c * self.bwd_rows)
        plan.need_scratch("coef", 8 * c)
        # the fallback when the members' parameter gradients are not adjacent (some frozen):
        # dgamma / dbeta into scratch, then per member
        plan.need_scratch("sib", 8 * c)
        self.wg_ws = L.lib().yms_conv_wgrad_ws_bytes(self.sp)
        plan.need_scratch("wgrad", self.wg_ws)
        for m in self.members:
            m.wg_ws = L.lib().yms_conv_wgrad_ws_bytes(m.sp)
            plan.need_scratch("wgrad", m.wg_ws)

    def pack_specs(self):
        """(shape, fp32 weight, arena offset, for_dgrad[, (second weight, split)]) per pack."""
        specs = [(m.sp, m.mod.conv.weight.data_ptr(), m.t_wp, 0) for m in self.members]
        a, bb = self.members
        specs.append((self.sp, a.mod.conv.weight.data_ptr(), self.t_wpt, 1,
                      (bb.mod.conv.weight.data_ptr(), a.c)))
        return specs

    def prepare_eval(self, rt):
        for m in self.members:
            m.prepare_eval(rt)

    def bn_modules(self):
        return [m.mod for m in self.members]

    def fwd(self, rt):
        if not rt.training:
            for m in self.members:      # eval: BN + act fused in each member's epilogue, into its slot
                m.fwd(rt)
            return
        if not rt.prepacked:
            raise RuntimeError("yms: sibling convs need the batched pack (Plan.prepack)")
        x, y = self.x, self.y
        base = rt.base
        stats = base + rt.plan.scratch["stats"]
        for m, off in zip(self.members, self.offs):
            L.call("yms_conv_fwd", m.sp, rt.a(x), x.buf.ld, x.off, base + m.t_wp, base + self.z, self.zld, off,
                   None, None, L.ACT_NONE, None, 0, 0, stats, rt.st)
            bn = m.mod.bn
            L.call("yms_bn_finalize_ld", m.c, stats, m.stats_rows, m.stats_ld, self.npix, bn.weight.data_ptr(),
                   bn.bias.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                   ctypes.c_float(bn.momentum if bn.momentum is not None else BN_MOMENTUM),
                   ctypes.c_float(bn.eps), base + self.mi + 4 * off, self.c, base + self.sc + 4 * off,
                   base + self.sh + 4 * off, rt.st)
        L.call("yms_affine_act", rt.plan.dt, self.npix, self.c, base + self.z, self.zld, 0, base + self.sc,
               base + self.sh, self.act, None, 0, 0, rt.a(y), y.buf.ld, y.off, rt.st)

    def plan_grads(self, T):
        T.read(self.y)
        self.acc_x = T.write(self.x) if self.x.buf.needs_grad else 0

    def _adjacent(self, rt, attr):
        ps = [rt.pgrad(getattr(m, attr)) for m in self.members]
        if any(p is None for p in ps):
            return None
        for m, p, q in zip(self.members, ps, ps[1:]):
            per = m.mod.conv.weight[0].numel() if attr == "pw" else 1
            if q != p + 4 * per * m.c:
                return None
        return ps[0]

    def bwd(self, rt):
        x, y = self.x, self.y
        base, dt, c = rt.base, rt.plan.dt, self.c
        gy, gyl, gyo = rt.g(y), y.buf.ld, y.off
        ws = rt.gbase + rt.plan.gscratch["bwd"]
        coef = rt.gbase + rt.plan.gscratch["coef"]
        z = base + self.z
        L.call("yms_bn_act_bwd_reduce", dt, self.npix, c, z, self.zld, 0, gy, gyl, gyo, base + self.sc,
               base + self.sh, base + self.mi, self.act, ws, rt.st)
        dg, db = self._adjacent(rt, "pg"), self._adjacent(rt, "pb")
        if dg is not None and db is not None:
            L.call("yms_bn_act_bwd_finalize", c, ws, self.bwd_rows, self.npix, dg, db, coef, rt.st)
        else:
            tmp = rt.gbase + rt.plan.gscratch["sib"]
            L.call("yms_bn_act_bwd_finalize", c, ws, self.bwd_rows, self.npix, tmp, tmp + 4 * c, coef, rt.st)
            for m, off in zip(self.members, self.offs):
                for src, pi in ((tmp, m.pg), (tmp + 4 * c, m.pb)):
                    d = rt.pgrad(pi)
                    if d is not None:
                        L.call("yms_copy", d, src + 4 * off, 4 * m.c, rt.st)
        dz = z                   # dz overwrites z in place
        L.call("yms_bn_act_bwd_apply", dt, self.npix, c, z, self.zld, 0, gy, gyl, gyo, base + self.sc,
               base + self.sh, base + self.mi, coef, self.act, dz, self.zld, 0, None, 0, 0, 0, rt.st)
        def dgrad():
            if x.buf.needs_grad:
                L.call("yms_conv_dgrad", self.sp, dz, self.zld, 0, base + self.t_wpt, rt.g(x), x.buf.ld, x.off,
                       self.acc_x, rt.st)

        if not rt.wgrad_first:
            dgrad()
        dw = self._adjacent(rt, "pw")
        if dw is not None:
            L.call("yms_conv_wgrad", self.sp, rt.a(x), x.buf.ld, x.off, dz, self.zld, 0,
                   rt.gbase + rt.plan.gscratch["wgrad"], self.wg_ws, dw, 0, rt.wst())
        else:
            for m, off in zip(self.members, self.offs):
                d = rt.pgrad(m.pw)
                if d is not None:
                    L.call("yms_conv_wgrad", m.sp, rt.a(x), x.buf.ld, x.off, dz, self.zld, off,
                           rt.gbase + rt.plan.gscratch["wgrad"], m.wg_ws, d, 0, rt.wst())
        if rt.wgrad_first:
            dgrad()

    def grad_params(self):
        # member-major within each kind: the flat arena then holds [dbeta_a | dbeta_b],
        # [dgamma_a | dgamma_b] and [dw_a | dw_b] contiguously (_adjacent)
        return [m.pb for m in self.members] + [m.pg for m in self.members] + [m.pw for m in self.members]


class BiasConvOp:
    """Plain nn.Conv2d with bias (the head's final 1x1 layers, yolov8_head.py:86-109)."""

    def __init__(self, b, conv, x, y):
        if conv.groups != 1 or conv.bias is None:
            raise RuntimeError("yms: biased ungrouped conv expected")
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        self.conv, self.x, self.y = conv, x, y
        self.shape = L.ConvShape(b.n, x.h, x.w, conv.in_channels, conv.out_channels, k, s, p, y.h, y.w, b.dt)
        self.sp = ctypes.pointer(self.shape)
        self.c = conv.out_channels
        self.npix = b.n * y.h * y.w
        self.pw = b.param(conv, "weight")
        self.pbias = b.param(conv, "bias")
        self.flops = 2 * self.npix * self.c * conv.in_channels * k * k
        self.stem_input = None   # plan input index when this conv reads the NCHW input directly
        self.tail_wgrad_first = False   # enqueue the weight gradient before the input gradient (Plan)

    def layout(self, plan, La, Le):
        es = plan.es
        self.wp_elems = L.lib().yms_conv_packed_elems(self.sp, 0)
        self.wpt_elems = L.lib().yms_conv_packed_elems(self.sp, 1)
        self.e_wp = Le.alloc(self.wp_elems * es)
        if plan.training:
            self.t_wp = La.alloc(self.wp_elems * es)
            self.t_wpt = La.alloc(self.wpt_elems * es)
            plan.need_scratch("bwd", 4 * 2 * self.c * L.lib().yms_bn_bwd_rows(self.npix, self.c))
            self.wg_ws = L.lib().yms_conv_wgrad_ws_bytes(self.sp)
            plan.need_scratch("wgrad", self.wg_ws)
            self.cnt = plan.counter()

    def prepare_eval(self, rt):
        L.call("yms_conv_pack_weight", self.sp, self.conv.weight.data_ptr(), rt.eval_base + self.e_wp, 0, rt.st)

    def pack_specs(self):
        w = self.conv.weight.data_ptr()
        return [(self.sp, w, self.t_wp, 0), (self.sp, w, self.t_wpt, 1)]

    def fwd(self, rt):
        x, y = self.x, self.y
        if rt.training:
            wp = rt.base + self.t_wp
            if not rt.prepacked:
                L.call("yms_conv_pack_weight", self.sp, self.conv.weight.data_ptr(), wp, 0, rt.st)
                L.call("yms_conv_pack_weight", self.sp, self.conv.weight.data_ptr(), rt.base + self.t_wpt, 1, rt.st)
        else:
            wp = rt.eval_base + self.e_wp
        L.call("yms_conv_fwd", self.sp, rt.a(x), x.buf.ld, x.off, wp, rt.a(y), y.buf.ld, y.off,
               None, self.conv.bias.data_ptr(), L.ACT_NONE, None, 0, 0, None, rt.st)

    def plan_grads(self, T):
        T.read(self.y)
        self.acc_x = T.write(self.x) if self.x.buf.needs_grad else 0

    def bwd(self, rt):
        x, y = self.x, self.y
        gy, gyl, gyo = rt.g(y), y.buf.ld, y.off
        db = rt.pgrad(self.pbias)
        if db is not None:
            L.call("yms_bias_bwd", rt.plan.dt, self.npix, self.c, gy, gyl, gyo,
                   rt.gbase + rt.plan.gscratch["bwd"], rt.cnt(self.cnt), db, rt.st)
        def dgrad():
            if x.buf.needs_grad:
                L.call("yms_conv_dgrad", self.sp, gy, gyl, gyo, rt.base + self.t_wpt, rt.g(x), x.buf.ld, x.off,
                       self.acc_x, rt.st)

        if not rt.wgrad_first:
            dgrad()
        dw = rt.pgrad(self.pw)
        if dw is not None:
            L.call("yms_conv_wgrad", self.sp, rt.a(x), x.buf.ld, x.off, gy, gyl, gyo,
                   rt.gbase + rt.plan.gscratch["wgrad"], self.wg_ws, dw, 0, rt.wst())
        if rt.wgrad_first:
            dgrad()

    def grad_params(self):
        return [self.pbias, self.pw]


class DWConvOp(ConvOp):
    """Depthwise Conv block (YOLO-MS IB_k mid conv, yolov8/model/yolo_ms.py): Conv2d(groups=C,
    bias=False, k x k, stride 1, pad k//2) -> BatchNorm2d -> SiLU, on the dwconv kernels.  BN
    forward/backward are the ConvOp path; weights are read unpacked (fp32 [C][k][k])."""

    def __init__(self, b, mod, x, y, act):
        conv = mod.conv
        k = conv.kernel_size[0]
        c = conv.out_channels
        if not (conv.groups == c == conv.in_channels and conv.kernel_size[0] == conv.kernel_size[1]
                and k in (3, 5, 7, 9) and conv.stride == (1, 1) and conv.padding == (k // 2, k // 2)
                and conv.dilation == (1, 1)):
            raise RuntimeError("yms: grouped convolutions are supported as depthwise k x k (k = 3/5/7/9), "
                               "stride 1, pad k//2")
        self.mod, self.x, self.y, self.res, self.act = mod, x, y, None, act
        self.dshape = L.DwShape(b.n, x.h, x.w, c, k, b.dt)
        self.sp = ctypes.pointer(self.dshape)
        self.c = c
        self.npix = b.n * y.h * y.w
        self.pw = b.param(conv, "weight")
        self.pg = b.param(mod.bn, "weight")
        self.pb = b.param(mod.bn, "bias")
        self.flops = 0          # not an MFMA contraction: excluded from the conv roofline
        self.dw_flops = 2 * self.npix * c * k * k
        self.stem_input = None
        self.bnred_for = self.bnred_by = self.bnred_key = self.bnred_wkey = None   # (ConvOp's fused-reduce links: unused)

    def layout(self, plan, La, Le):
        es, c = plan.es, self.c
        self.e_sc = Le.alloc(4 * c)
        self.e_sh = Le.alloc(4 * c)
        if plan.training:
            self.zld = r8(c)
            self.z = La.alloc(self.npix * self.zld * es)
            self.sc = La.alloc(4 * c)
            self.sh = La.alloc(4 * c)
            self.mi = La.alloc(8 * c)
            self.stats_rows = L.lib().yms_dwconv_stats_rows(self.sp)
            self.stats_ld = r8(c)
            plan.need_scratch("stats", 4 * self.stats_rows * (2 * self.stats_ld + 1))
            plan.need_scratch("bwd", 4 * 2 * c * L.lib().yms_bn_bwd_rows(self.npix, c))
            plan.need_scratch("coef", 8 * c)
            # sized once here and passed as-is at backward time: the C side reads its tiling knobs
            # on every call, so a recomputed size could outgrow the region reserved here
            self.wg_ws = L.lib().yms_dwconv_wgrad_ws_bytes(self.sp)
            plan.need_scratch("wgrad", self.wg_ws)

    def pack_specs(self):
        return []

    def prepare_eval(self, rt):
        bn = self.mod.bn
        L.call("yms_bn_fold", self.c, bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
               bn.running_var.data_ptr(), ctypes.c_float(bn.eps), rt.eval_base + self.e_sc,
               rt.eval_base + self.e_sh, rt.st)

    def fwd(self, rt):
        x, y = self.x, self.y
        w = self.mod.conv.weight.data_ptr()
        if not rt.training:
            eb = rt.eval_base
            L.call("yms_dwconv_fwd", self.sp, rt.a(x), x.buf.ld, x.off, w, rt.a(y), y.buf.ld, y.off, eb + self.e_sc,
                   eb + self.e_sh, self.act, None, 0, rt.st)
            return
        base = rt.base
        stats = base + rt.plan.scratch["stats"]
        L.call("yms_dwconv_fwd", self.sp, rt.a(x), x.buf.ld, x.off, w, base + self.z, self.zld, 0, None, None,
               L.ACT_NONE, stats, self.stats_ld, rt.st)
        bn = self.mod.bn
        L.call("yms_bn_finalize", self.c, stats, self.stats_rows, self.stats_ld, self.npix, bn.weight.data_ptr(),
               bn.bias.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
               ctypes.c_float(bn.momentum if bn.momentum is not None else BN_MOMENTUM),
               ctypes.c_float(bn.eps), base + self.mi, base + self.sc, base + self.sh, rt.st)
        L.call("yms_affine_act", rt.plan.dt, self.npix, self.c, base + self.z, self.zld, 0, base + self.sc,
               base + self.sh, self.act, None, 0, 0, rt.a(y), y.buf.ld, y.off, rt.st)

    def bwd(self, rt):
        x, y = self.x, self.y
        base, dt, c = rt.base, rt.plan.dt, self.c
        z = base + self.z
        ws = rt.gbase + rt.plan.gscratch["bwd"]
        coef = rt.gbase + rt.plan.gscratch["coef"]
        L.call("yms_bn_act_bwd_reduce", dt, self.npix, c, z, self.zld, 0, rt.g(y), y.buf.ld, y.off, base + self.sc,
               base + self.sh, base + self.mi, self.act, ws, rt.st)
        L.call("yms_bn_act_bwd_finalize", c, ws, L.lib().yms_bn_bwd_rows(self.npix, c), self.npix,
               rt.pgrad(self.pg), rt.pgrad(self.pb), coef, rt.st)
        L.call("yms_bn_act_bwd_apply", dt, self.npix, c, z, self.zld, 0, rt.g(y), y.buf.ld, y.off, base + self.sc,
               base + self.sh, base + self.mi, coef, self.act, z, self.zld, 0, None, 0, 0, 0, rt.st)
        w = self.mod.conv.weight.data_ptr()
        if x.buf.needs_grad and not rt.wgrad_first:
            L.call("yms_dwconv_dgrad", self.sp, z, self.zld, 0, w, rt.g(x), x.buf.ld, x.off, self.acc_x, rt.st)
        dw = rt.pgrad(self.pw)
        if dw is not None:
            wsz = self.wg_ws
            L.call("yms_dwconv_wgrad", self.sp, rt.a(x), x.buf.ld, x.off, z, self.zld, 0,
                   rt.gbase + rt.plan.gscratch["wgrad"], wsz, dw, 0, rt.wst())
        if x.buf.needs_grad and rt.wgrad_first:
            L.call("yms_dwconv_dgrad", self.sp, z, self.zld, 0, w, rt.g(x), x.buf.ld, x.off, self.acc_x, rt.st)


class AddOp:
    """y = a + b (b None: y = a) over channel views: the MS-Block branch sums X_i + Y_{i-1} and
    the Y_1 = X_1 placement.  Backward routes dy into both addends (store or accumulate)."""

    def __init__(self, b, a, bb, y):
        self.a, self.b, self.y = a, bb, y
        self.npix = b.n * y.h * y.w
        self.c = y.c
        self.flops = 0

    def layout(self, plan, La, Le):
        pass

    def fwd(self, rt):
        a, b, y = self.a, self.b, self.y
        bp = rt.a(b) if b is not None else None
        bl, bo = (b.buf.ld, b.off) if b is not None else (0, 0)
        L.call("yms_add_views", rt.plan.dt, self.npix, self.c, rt.a(a), a.buf.ld, a.off, bp, bl, bo, rt.a(y),
               y.buf.ld, y.off, 0, rt.st)

    def plan_grads(self, T):
        T.read(self.y)
        self.acc = [T.write(v) if (v is not None and v.buf.needs_grad) else None for v in (self.a, self.b)]

    def bwd(self, rt):
        y = self.y
        if all(v is not None and acc is not None for v, acc in zip((self.a, self.b), self.acc)):
            a, b = self.a, self.b
            L.call("yms_add_grad2", rt.plan.dt, self.npix, self.c, rt.g(y), y.buf.ld, y.off, rt.g(a), a.buf.ld,
                   a.off, self.acc[0], rt.g(b), b.buf.ld, b.off, self.acc[1], rt.st)
            return
        for v, acc in zip((self.a, self.b), self.acc):
            if v is None or acc is None:
                continue
            L.call("yms_add_views", rt.plan.dt, self.npix, self.c, rt.g(y), y.buf.ld, y.off, None, 0, 0, rt.g(v),
                   v.buf.ld, v.off, acc, rt.st)

    def grad_params(self):
        return []


class UpsampleOp:
    """nearest x2, components.py:153-160."""

    def __init__(self, b, x, y):
        self.x, self.y, self.n = x, y, b.n
        self.flops = 0

    def layout(self, plan, La, Le):
        pass

    def fwd(self, rt):
        x, y = self.x, self.y
        L.call("yms_upsample2x_fwd", rt.plan.dt, self.n, x.h, x.w, x.c, rt.a(x), x.buf.ld, x.off,
               rt.a(y), y.buf.ld, y.off, rt.st)

    def plan_grads(self, T):
        T.read(self.y)
        self.acc_x = T.write(self.x) if self.x.buf.needs_grad else 0

    def bwd(self, rt):
        x, y = self.x, self.y
        if not x.buf.needs_grad:
            return
        L.call("yms_upsample2x_bwd", rt.plan.dt, self.n, x.h, x.w, x.c, rt.g(y), y.buf.ld, y.off,
               rt.g(x), x.buf.ld, x.off, self.acc_x, rt.st)

    def grad_params(self):
        return []


class SppfPoolOp:
    """The three chained MaxPool2d(5,1,2) of SPPF (components.py:136-146) over a 4-slot buffer."""

    def __init__(self, b, v4, c):
        self.v, self.c, self.n = v4, c, b.n
        self.flops = 0

    def layout(self, plan, La, Le):
        if plan.training:
            plan.need_scratch("sppf", L.lib().yms_sppf_ws_bytes(self.n, self.v.h, self.v.w, self.c))

    def fwd(self, rt):
        v = self.v
        L.call("yms_sppf_pool_fwd", rt.plan.dt, self.n, v.h, v.w, self.c, rt.a(v), v.buf.ld, v.off, rt.st)

    def plan_grads(self, T):
        T.read(self.v)        # slot grads come from conv2's dgrad; the pool chain accumulates in place

    def bwd(self, rt):
        v = self.v
        L.call("yms_sppf_pool_bwd", rt.plan.dt, self.n, v.h, v.w, self.c, rt.a(v), v.buf.ld, v.off,
               rt.g(v), v.buf.ld, v.off, rt.gbase + rt.plan.gscratch["sppf"], rt.st)

    def grad_params(self):
        return []


class Builder:
    """Collects buffers, ops and parameter references while modules ``emit``."""

    def __init__(self, n, dt, training):
        self.n, self.dt, self.training = n, dt, training
        self.es = 4 if dt == L.F32 else 2
        self.bufs = []
        self.ops = []
        self.param_refs = []      # (module, attr)
        self._pidx = {}

    def new(self, h, w, c, name="act", ld=None):
        b = Buf(len(self.bufs), self.n, h, w, ld if ld is not None else r8(c), name, zero=(c % 8 != 0))
        self.bufs.append(b)
        return View(b, 0, c)

    def param(self, mod, attr):
        key = (id(mod), attr)
        if key not in self._pidx:
            self._pidx[key] = len(self.param_refs)
            self.param_refs.append((mod, attr))
        return self._pidx[key]

    # --- emitters used by the yolov8 modules -------------------------------------------
    def conv(self, mod, x, out=None, res=None, act=None):
        conv = mod.conv
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        ho, wo = (x.h + 2 * p - k) // s + 1, (x.w + 2 * p - k) // s + 1
        if out is None:
            out = self.new(ho, wo, conv.out_channels)
        assert out.c == conv.out_channels and out.h == ho and out.w == wo, "yms: output view mismatch"
        if act is None:
            act = L.ACT_SILU if isinstance(mod.activation, torch.nn.SiLU) else L.ACT_NONE
        if conv.groups != 1:
            if res is not None:
                raise RuntimeError("yms: residual epilogue is not supported on depthwise convolutions")
            self.ops.append(DWConvOp(self, mod, x, out, act))
        else:
            self.ops.append(ConvOp(self, mod, x, out, res, act))
        return out

    def sibling_convs(self, mods, x):
        """Two Conv blocks reading the same input x -> their output views, the channel slots of one
        buffer (SiblingConvOp), or two separate ConvOps when they cannot share one (different
        geometry or activation, a first member whose width is not a multiple of 8, or
        YMS_HEAD_FUSE=0)."""
        ks = {(m.conv.kernel_size, m.conv.stride, m.conv.padding, m.conv.groups, m.conv.dilation,
               isinstance(m.activation, torch.nn.SiLU)) for m in mods}
        fuse = (len(mods) == 2 and len(ks) == 1 and mods[0].conv.groups == 1 and mods[0].conv.out_channels % 8 == 0
                and os.environ.get("YMS_HEAD_FUSE", "1") != "0")
        if not fuse:
            return [m.emit(self, x) for m in mods]
        conv = mods[0].conv
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        ho, wo = (x.h + 2 * p - k) // s + 1, (x.w + 2 * p - k) // s + 1
        y = self.new(ho, wo, sum(m.conv.out_channels for m in mods))
        act = L.ACT_SILU if isinstance(mods[0].activation, torch.nn.SiLU) else L.ACT_NONE
        op = SiblingConvOp(self, mods, x, y, act)
        self.ops.append(op)
        return [m.y for m in op.members]

    def add(self, a, b, out=None):
        """y = a + b (b may be None: a placement copy) -> view."""
        if b is not None and (a.h, a.w, a.c) != (b.h, b.w, b.c):
            raise RuntimeError("yms: add of mismatched views")
        if out is None:
            out = self.new(a.h, a.w, a.c)
        self.ops.append(AddOp(self, a, b, out))
        return out

    def conv2d_bias(self, conv, x, out=None):
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        ho, wo = (x.h + 2 * p - k) // s + 1, (x.w + 2 * p - k) // s + 1
        if out is None:
            out = self.new(ho, wo, conv.out_channels)
        self.ops.append(BiasConvOp(self, conv, x, out))
        return out

    def upsample(self, x, out=None):
        if out is None:
            out = self.new(2 * x.h, 2 * x.w, x.c)
        self.ops.append(UpsampleOp(self, x, out))
        return out

    def sppf_pool(self, v4, c):
        self.ops.append(SppfPoolOp(self, v4, c))


class Plan:
    def __init__(self, b: Builder, inputs, outputs, kind):
        self.n, self.dt, self.training, self.es = b.n, b.dt, b.training, b.es
        self.bufs, self.ops, self.param_refs = b.bufs, b.ops, b.param_refs
        self.inputs, self.outputs, self.kind = inputs, outputs, kind
        self.scratch_req = {}
        self.n_counters = 0
        self.stem_inputs = self._find_stems()
        if self.training and os.environ.get("YMS_WGRAD_FIRST", "tail") == "tail":
            stem_out = {op.y.buf.idx for op in self.stem_inputs.values()}
            for op in self.ops:
                if type(op) is ConvOp and op.x.buf.idx in stem_out:
                    op.tail_wgrad_first = True
        self._find_bnred()
        La, Le = Layout(), Layout()
        # an input the stem conv reads as NCHW fp32 has no NHWC buffer: no arena bytes, and no
        # per-step zeroing of its padding channels (3 -> 8: 419 MB, 51 us per configs[2] step)
        stem_bufs = {self.inputs[i].buf.idx for i in self.stem_inputs}
        for buf in self.bufs:
            if buf.idx in stem_bufs:
                buf.off, buf.zero = 0, False
                continue
            buf.off = La.alloc(buf.npix * buf.ld * self.es)
        self.act_bytes = La.size
        for op in self.ops:
            op.layout(self, La, Le)
        self.scratch = {}
        if self.training:
            self.scratch["stats"] = La.alloc(self.scratch_req.get("stats", 0))
        self.arena_bytes = La.size
        # grad arena: activation grads share the activation layout, then backward scratch
        Lg = Layout()
        Lg.size = self.act_bytes
        self.gscratch = {k: Lg.alloc(self.scratch_req.get(k, 0)) for k in ("bwd", "coef", "wgrad", "sppf", "stemwg", "sib")}
        for k in sorted(k for k in self.scratch_req if k.startswith("bnr")):
            self.gscratch[k] = Lg.alloc(self.scratch_req[k])
        self.gscratch["cnt"] = Lg.alloc(16 * max(self.n_counters, 1))
        self.garena_bytes = Lg.size
        self.eval_bytes = Le.size
        self.zero_ranges = [(bf.off, bf.npix * bf.ld * self.es) for bf in self.bufs if bf.zero]
        # training z buffers with padding channels (c % 8 != 0, e.g. a head with nc = 3): the convs and
        # the BN apply (dz written over z) touch only the c real channels, while the input gradient
        # reads the whole 16-B groups -- padding left as arena garbage (NaN / Inf bit patterns) times
        # the zero weight rows is NaN, so those z buffers start zeroed and their padding stays zero
        if self.training:
            for op in self.ops:
                zld, z = getattr(op, "zld", None), getattr(op, "z", None)
                if zld is not None and z is not None and zld != op.c:
                    self.zero_ranges.append((z, op.npix * zld * self.es))
        if self.training:
            T = GradTracker()
            self.seed_acc = [T.write(v) for v in self.outputs]
            T.writes = set()
            for op in reversed(self.ops):
                op.plan_grads(T)
                y = getattr(op, "y", None)
                if isinstance(y, View) and not any(y is o for o in self.outputs):
                    _check_not_in_place(op, y)
                    T.release(y)
            # output buffers whose gradient no op writes (only reads): the incoming gradient tensor
            # can serve as that buffer's gradient in place (runner._seed_grad), no copy
            self.grad_read_only = {v.buf.idx for v in self.outputs if v.buf.idx not in T.writes}
            self.gzero_ranges = [(bf.off, bf.npix * bf.ld * self.es) for bf in self.bufs if bf.idx in T.zero]
            self.gzero_ranges.append((self.gscratch["cnt"], 16 * max(self.n_counters, 1)))
        self.flops = sum(op.flops for op in self.ops)
        # parameter-gradient arena in backward-completion order (reverse op order)
        order = []
        seen = set()
        for op in reversed(self.ops):
            for pi in op.grad_params():
                if pi not in seen:
                    seen.add(pi)
                    order.append(pi)
        self.pgrad_order = order
        self._eval_sig = None
        self._eval_arena = None

    def _find_stems(self):
        """Inputs whose only reader is a stem-shaped Conv (3x3 stride 2 over <= 3 channels, no
        residual, 16-bit compute, input without gradient): that conv reads the NCHW fp32 input
        itself (yms_conv_stem_fwd, and yms_conv_stem_wgrad with the BN backward apply fused in),
        so the NHWC input pack goes.  YMS_STEM=0 keeps the generic pack + implicit-GEMM path."""
        out = {}
        if self.dt == L.F32 or os.environ.get("YMS_STEM", "1") == "0":
            return out
        for i, v in enumerate(self.inputs):
            readers = [op for op in self.ops
                       if any(isinstance(a, View) and a.buf is v.buf for a in vars(op).values())]
            if len(readers) != 1 or type(readers[0]) is not ConvOp:
                continue
            op = readers[0]
            if (op.x.buf is v.buf and op.x.off == 0 and op.x.c == v.c and op.res is None and v.buf.ld == r8(v.c)
                    and not v.buf.needs_grad
                    and L.lib().yms_conv_stem_supported(op.sp)):
                op.stem_input = i
                out[i] = op
        return out

    def _find_bnred(self):
        """Training, 16-bit: a Conv whose input gradient runs on the direct 3x3 kernel
        (yms_conv_dgrad_bnred_rows > 0) and whose input view is exactly the output of an earlier
        Conv op P, with no op in between touching that view (so this dgrad is the LAST writer of
        P's output gradient, backward order), computes P's BN + act backward reduce in its epilogue
        (yms_conv_dgrad_bnred): P's separate reduce pass (z and gy read once more) goes, and P's
        finalize reads the partial rows from a grad-scratch region of their own.  YMS_BNRED=0 keeps
        the separate reduce (A/B)."""
        if not self.training or self.dt == L.F32 or os.environ.get("YMS_BNRED", "1") == "0":
            return

        def views(op):
            for v in vars(op).values():
                for u in (v if isinstance(v, (list, tuple)) else (v,)):
                    if isinstance(u, View):
                        yield u

        n = 0
        for i, c in enumerate(self.ops):
            if type(c) is not ConvOp or c.stem_input is not None or not c.x.buf.needs_grad:
                continue
            rows = L.lib().yms_conv_dgrad_bnred_rows(c.sp)
            if rows <= 0:
                continue
            x = c.x
            j = next((j for j in range(i - 1, -1, -1)
                      if isinstance(getattr(self.ops[j], "y", None), View) and _overlap(self.ops[j].y, x)), None)
            if j is None:
                continue
            q = self.ops[j]
            if (type(q) is not ConvOp or q.y.off != x.off or q.y.c != x.c or q.c != x.c or q.bnred_by is not None
                    or q.act not in (L.ACT_NONE, L.ACT_SILU)):
                continue
            if any(_overlap(v, x) for op in self.ops[j + 1:i] for v in views(op)):
                continue
            if any(_overlap(v, x) for k, v in vars(c).items() if isinstance(v, View) and k != "x"):
                continue
            key = f"bnr{n}"
            n += 1
            # a conv can be both: the consumer of one pair (wkey) and the producer of the next (key)
            c.bnred_for, c.bnred_wkey = q, key
            q.bnred_by, q.bnred_key, q.bnred_rows = c, key, rows
            self.need_scratch(key, 4 * rows * 2 * r8(x.c))

    def counter(self):
        """Reserve one 16-B arrival counter in the grad scratch (-> its index)."""
        self.n_counters += 1
        return self.n_counters - 1

    def need_scratch(self, key, nbytes):
        self.scratch_req[key] = max(self.scratch_req.get(key, 0), int(nbytes))

    def params(self):
        return [getattr(m, a) for (m, a) in self.param_refs]

    # ------------------------------------------------------------------------------------
    def ensure_eval_cache(self, device, stream):
        """(Re)pack weights and fold BN when any parameter / buffer changed."""
        sig = []
        for op in self.ops:
            if isinstance(op, (ConvOp, SiblingConvOp)):
                for m in (op.bn_modules() if isinstance(op, SiblingConvOp) else (op.mod,)):
                    for t in (m.conv.weight, m.bn.weight, m.bn.bias, m.bn.running_mean, m.bn.running_var):
                        sig.append((t.data_ptr(), t._version))
            elif isinstance(op, BiasConvOp):
                sig.append((op.conv.weight.data_ptr(), op.conv.weight._version))
        sig = tuple(sig)
        if self._eval_arena is None or self._eval_arena.device != device:
            self._eval_arena = torch.empty(max(self.eval_bytes, 1), dtype=torch.uint8, device=device)
            self._eval_sig = None
        if sig != self._eval_sig:
            rt = Rt(self, None, stream, False)
            rt.eval_base = self._eval_arena.data_ptr()
            for op in self.ops:
                if hasattr(op, "prepare_eval"):
                    op.prepare_eval(rt)
            self._eval_sig = sig
        return self._eval_arena.data_ptr()

    def pack_table(self):
        """The batched pack's device job table (built and uploaded on the CURRENT stream on a
        cache miss: call it before handing prepack to another stream)."""
        specs = [sp for op in self.ops if hasattr(op, "pack_specs") for sp in op.pack_specs()]
        key = tuple((sp[1], sp[2], sp[4] if len(sp) > 4 else None) for sp in specs)
        cache = self.__dict__.setdefault("_pack_tables", {})
        ent = cache.get(key)
        if ent is None:
            jobs, singles = [], []
            for spec in specs:
                sp, w, dst, fd = spec[:4]
                j = L.PackJob()
                st = L.lib().yms_pack_job_init(sp, w, dst, fd, ctypes.byref(j))
                if len(spec) > 4:                 # two sources (SiblingConvOp): batched only
                    if st != 0:
                        raise RuntimeError("yms: a two-source weight pack must be batchable")
                    j.w2, j.split = spec[4]
                if st == 0:
                    jobs.append(j)
                else:
                    singles.append((sp, w, dst, fd))
            arr = (L.PackJob * max(len(jobs), 1))(*jobs)
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            table = host.to(torch.device("cuda", torch.cuda.current_device()))
            if len(cache) >= 4:
                cache.clear()
            ent = cache[key] = (table, len(jobs), singles)
        return ent

    def prepack(self, rt, ent=None):
        """Training: issue every conv weight pack of the step on rt.st -- one batched launch for
        the plain packs (device job table of arena OFFSETS, cached per parameter set, so it is
        valid for any arena and is built before any graph capture) plus the stride-2 dgrad
        parity packs individually."""
        table, nj, singles = ent if ent is not None else self.pack_table()
        L.call("yms_conv_pack_weights_batched", nj, table.data_ptr(), rt.base, rt.st)
        for sp, w, dst, fd in singles:
            L.call("yms_conv_pack_weight", sp, w, rt.base + dst, fd, rt.st)
        rt.prepacked = True

    def new_arena(self, device, stream):
        arena = torch.empty(max(self.arena_bytes, 1), dtype=torch.uint8, device=device)
        base = arena.data_ptr()
        for off, nb in self.zero_ranges:
            L.call("yms_zero", base + off, nb, stream)
        return arena

    def act_tensor(self, arena, view, dtype):
        """torch view (NCHW-shaped, channels-last strided) of an activation buffer slice."""
        b = view.buf
        nb = b.npix * b.ld * self.es
        t = arena[b.off:b.off + nb].view(dtype).view(b.n, b.h, b.w, b.ld)
        return t[..., view.off:view.off + view.c].permute(0, 3, 1, 2)
