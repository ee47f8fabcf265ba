"""Module execution: plan cache, autograd bridge and dtype policy.

``run(module, inputs)`` is what every yolov8 module's ``forward`` calls.  The whole
module tree below it executes as ONE torch.autograd.Function whose forward/backward
launch the plan's HIP kernels on the current stream; parameter gradients come back
to autograd as views of a flat fp32 arena (so ``loss.backward(); opt.step()`` of the
reference training loop, train.py:356-372, works unchanged).  There is no CPU or
ATen-conv fallback: CPU tensors or a missing libyms.so raise RuntimeError.
"""
from __future__ import annotations

import os

import threading

import torch

from . import _lib as L
from .plan import Builder, Plan, Rt

_CACHE_ATTR = "_yms_plans"


def compute_dtype(module):
    """bf16/fp16 under torch.autocast('cuda'), else module.yms_dtype, else fp32."""
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return getattr(module, "yms_dtype", torch.float32)


def set_compute_dtype(module, dtype):
    """Run `module` (and its children when called through it) with bf16/fp16/fp32 kernels;
    parameters stay fp32 masters."""
    L.dtype_code(dtype)
    for m in module.modules():
        m.yms_dtype = dtype
    return module


class _State:
    pass


def _check_inputs(inputs):
    for x in inputs:
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
            raise RuntimeError("yms: the MI355X-native model runs on ROCm GPU tensors only "
                               "(move the model and inputs to 'cuda'); there is no CPU fallback")


def get_plan(module, inputs, dt, training):
    key = (tuple(tuple(x.shape) for x in inputs), tuple(bool(x.requires_grad) for x in inputs), dt, training)
    cache = module.__dict__.setdefault(_CACHE_ATTR, {})
    plan = cache.get(key)
    if plan is None:
        for x in inputs:
            if x.dim() != 4:
                raise RuntimeError(f"yms: expected NCHW 4-D input, got shape {tuple(x.shape)}")
        b = Builder(inputs[0].shape[0], L.dtype_code(dt), training)
        in_views, outs, kind = module._yms_plan(b, inputs)
        for v, x in zip(in_views, inputs):
            v.buf.name = "input"
            v.buf.needs_grad = bool(x.requires_grad)
        plan = Plan(b, in_views, outs, kind)
        cache[key] = plan
    return plan


def _load_inputs(plan, rt, inputs):
    for i, (x, v) in enumerate(zip(inputs, plan.inputs)):
        xc = x.contiguous()
        st = rt.st
        if i in plan.stem_inputs:
            # the stem conv reads the NCHW input itself, forward and weight gradient: no pack
            rt.stem_x[i] = xc if xc.dtype == torch.float32 else xc.float()
            continue
        if v.off == 0 and xc.dtype == torch.float32:
            L.call("yms_pack_input", plan.dt, xc.shape[0], xc.shape[1], xc.shape[2], xc.shape[3], xc.data_ptr(),
                   rt.a(v), v.buf.ld, st)
        else:
            L.call("yms_nchw_to_nhwc", L.dtype_code(xc.dtype), plan.dt, xc.shape[0], xc.shape[2], xc.shape[3],
                   xc.shape[1], xc.data_ptr(), rt.a(v), v.buf.ld, v.off, 0, rt.st)


def _outputs(plan, arena, dtype):
    return [plan.act_tensor(arena, v, dtype) for v in plan.outputs]


def _decode(plan, rt, arena):
    info = plan.kind[1].yms_decode_info()
    n = plan.n
    views = plan.outputs
    nc = info["nc"]
    A = sum(v.h * v.w for v in views)
    out = torch.empty((n, A, 4 + nc), dtype=torch.float32, device=arena.device)
    import ctypes
    lv = (ctypes.c_void_p * 4)(*[rt.a(v) for v in views] + [None] * (4 - len(views)))
    hs = (ctypes.c_int * 4)(*[v.h for v in views] + [0] * (4 - len(views)))
    ws = (ctypes.c_int * 4)(*[v.w for v in views] + [0] * (4 - len(views)))
    st = (ctypes.c_float * 4)(*(list(info["strides"]) + [0.0] * (4 - len(views))))
    ld = views[0].buf.ld
    for v in views:
        if v.buf.ld != ld or v.off != 0:
            raise RuntimeError("yms: head outputs must share one channel stride")
    L.call("yms_head_decode", plan.dt, n, nc, len(views), lv, hs, ws, ld, st, out.data_ptr(),
           ctypes.c_float(0.0), None, None, None, rt.st)
    return out


def _seed_grad(plan, rt, v, g, acc):
    """Incoming output gradient -> NHWC grad slice.  Channels-last grads (what elementwise
    losses on our channels-last outputs produce, and the fused loss's d/d maps) are already NHWC:
    when no op of the plan writes into that buffer's gradient (the head maps: the backward only
    reads them) the incoming tensor itself serves as the buffer's gradient -- no copy (the copies
    of the three head-map gradients were ~0.15 ms per configs[2] step); else one 2-D copy."""
    n, c, h, w = g.shape
    if (g.dtype == L_DTYPES[plan.dt] and g.stride(1) == 1 and g.stride(3) == c and g.stride(2) == w * c
            and g.stride(0) == h * w * c and not acc and c == v.buf.ld and v.off == 0):
        if os.environ.get("YMS_GRAD_INPLACE", "1") != "0" and v.buf.idx in plan.grad_read_only and not any(v2.buf is v.buf for v2 in plan.outputs if v2 is not v):
            if rt.gover is None:
                rt.gover = {}
            rt.gover[v.buf.idx] = g.data_ptr()
            return
        L.call("yms_copy", rt.g(v), g.data_ptr(), n * h * w * c * plan.es, rt.st)
        return
    gc = g.contiguous()
    L.call("yms_nchw_to_nhwc", L.dtype_code(gc.dtype), plan.dt, n, h, w, c, gc.data_ptr(), rt.g(v), v.buf.ld,
           v.off, acc, rt.st)


# weight-gradient GEMMs on a per-device side stream (YMS_WGRAD_STREAM=0: all on one stream)
WGRAD_SIDE_STREAM = os.environ.get("YMS_WGRAD_STREAM", "1") != "0"
_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


L_DTYPES = {L.F32: torch.float32, L.BF16: torch.bfloat16, L.F16: torch.float16}


class _PlanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, state, *args):
        plan = state.plan
        inputs = args[:len(plan.inputs)]
        dev = inputs[0].device
        stream = L.stream_ptr(dev)
        arena = plan.new_arena(dev, stream)
        rt = Rt(plan, arena.data_ptr(), stream, True)
        _load_inputs(plan, rt, inputs)
        ops = plan.ops
        if WGRAD_SIDE_STREAM and plan.ops and plan.ops[0] in plan.stem_inputs.values():
            # the stem conv reads the fp32 weight itself: the step's weight packs go to the side
            # stream and overlap it; every later conv is ordered after them
            main, side = torch.cuda.current_stream(dev), _side_stream(dev)
            ent = plan.pack_table()          # a first-call table upload goes on main, before the wait
            side.wait_stream(main)
            rt.st = side.cuda_stream
            plan.prepack(rt, ent)
            rt.st = stream
            ops[0].fwd(rt)
            # main joins the side stream right here, so any later reuse of the arena's or the
            # table's memory (main-stream ordered) comes after the packs: no record_stream (which
            # would defer the arena's reuse and, with the host steps ahead, make the caching
            # allocator map a second ~100 GB arena for YOLO-MS-L)
            main.wait_stream(side)
            ops = ops[1:]
        else:
            plan.prepack(rt)
        for op in ops:
            op.fwd(rt)
        state.arena = arena
        state.rt = rt
        state.in_meta = [(x.shape, x.dtype, x.requires_grad) for x in inputs]
        state.used = False
        ctx.state = state
        outs = _outputs(plan, arena, state.dtype)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        state = ctx.state
        if state.used:
            raise RuntimeError("yms: backward through the same forward twice (retain_graph) is unsupported")
        state.used = True
        plan, rt = state.plan, state.rt
        dev = state.arena.device
        rt.st = L.stream_ptr(dev)
        rt.main = torch.cuda.current_stream(dev)
        rt.side = _side_stream(dev) if WGRAD_SIDE_STREAM else None
        garena = torch.empty(max(plan.garena_bytes, 1), dtype=torch.uint8, device=dev)
        rt.gbase = garena.data_ptr()
        rt.gover = None
        for off, nb in plan.gzero_ranges:
            L.call("yms_zero", rt.gbase + off, nb, rt.st)
        for v, g, acc in zip(plan.outputs, gouts, plan.seed_acc):
            if g is None:
                if not acc:
                    L.call("yms_zero", rt.g(v), v.buf.npix * v.buf.ld * plan.es, rt.st)
                continue
            _seed_grad(plan, rt, v, g, acc)
        params = state.params
        # flat fp32 grad arena in backward-completion order; its layout is cached per plan and
        # requires_grad pattern, and the per-parameter torch views are built only after the
        # backward's kernels are enqueued (that host loop used to leave the GPU idle ~0.5 ms)
        need = tuple(p.requires_grad for p in params)
        lays = plan.__dict__.setdefault("_pg_layouts", {})
        lay = lays.get(need)
        if lay is None:
            offs, off = [], 0
            for i in plan.pgrad_order:
                if need[i]:
                    offs.append((i, off, params[i].numel(), tuple(params[i].shape)))
                    off += params[i].numel()
            lay = lays[need] = (off, offs)
        total, offs = lay
        pg = torch.empty(max(total, 1), dtype=torch.float32, device=dev)
        base = pg.data_ptr()
        ptrs = [None] * len(params)
        for i, off, _, _ in offs:
            ptrs[i] = base + 4 * off

        def param_views():
            v = [None] * len(params)
            chunks = torch.split(pg[:total], [n for _, _, n, _ in offs]) if offs else []
            for (i, _, _, shp), t in zip(offs, chunks):
                v[i] = t.view(shp)
            return v

        rt.pgrad = lambda i: ptrs[i]
        hook = state.grad_hook
        views = None
        if hook is not None:
            views = param_views()
            hook.begin(plan, pg, ptrs, views)
        for op in reversed(plan.ops):
            op.bwd(rt)
            if hook is not None and hook.pending(op):
                if rt.side is not None:
                    # the bucket's dw come from side-stream wgrads and its BN/bias grads from the main
                    # stream: order the side stream after main and issue the collective from the side
                    # stream, so the main stream never stalls on the wgrads (the collective's stream
                    # waits on the side stream; finish() joins main to the collectives)
                    rt.side.wait_stream(rt.main)
                    with torch.cuda.stream(rt.side):
                        hook.op_done(op)
                else:
                    hook.op_done(op)
        if rt.side is not None:
            rt.main.wait_stream(rt.side)
            rt.side = None
        if hook is not None:
            hook.finish()
        in_grads = []
        for (shape, dtype, rg), v in zip(state.in_meta, plan.inputs):
            if rg:
                gi = torch.empty(shape, dtype=dtype, device=dev)
                L.call("yms_nhwc_to_nchw", plan.dt, L.dtype_code(dtype), shape[0], shape[2], shape[3], shape[1],
                       rt.g(v), v.buf.ld, v.off, gi.data_ptr(), rt.st)
                in_grads.append(gi)
            else:
                in_grads.append(None)
        state.arena = None
        if views is None:
            views = param_views()
        return (None, *in_grads, *views)


_INFER_ARENAS_MAX = 4


def run(module, inputs, grad_hook=None):
    """Execute `module` on `inputs` (list of NCHW cuda tensors) through its plan."""
    _check_inputs(inputs)
    L.lib()
    if grad_hook is None:
        grad_hook = getattr(module, "_yms_grad_hook", None)
    dtype = compute_dtype(module)
    training = module.training
    plan = get_plan(module, inputs, dtype, training)
    params = plan.params()
    dev = inputs[0].device
    if training:
        state = _State()
        state.plan, state.dtype, state.params, state.grad_hook = plan, dtype, params, grad_hook
        outs = _PlanFn.apply(state, *inputs, *params)
        _bump_bn_counters(plan)
        return plan, list(outs)
    # eval / inference: no autograd graph, eval-cached packed weights + folded BN
    stream = L.stream_ptr(dev)
    decode = isinstance(plan.kind, tuple) and plan.kind[0] == "decode"
    with torch.no_grad():
        # a decode plan returns a fresh tensor, so its arena is internal: keep it per (stream, host
        # thread) -- the next call from that thread on that stream is ordered after this one, while
        # two threads sharing a stream would interleave their launches -- and skip
        # re-zeroing the pad ranges
        # (bounded -- the oldest entry goes once a plan holds _INFER_ARENAS_MAX, so a
        # thread pool churning through threads does not keep one full arena per dead thread)
        arena = None
        if decode:
            cache = plan.__dict__.setdefault("_infer_arenas", {})
            key = (stream, threading.get_ident())
            arena = cache.pop(key, None)
            if arena is not None and arena.device != dev:
                arena = None
        if arena is None:
            arena = plan.new_arena(dev, stream)
        if decode:
            while len(cache) >= _INFER_ARENAS_MAX:
                cache.pop(next(iter(cache)))
            cache[key] = arena           # re-inserted last: the dict's order is least-recently used first
        rt = Rt(plan, arena.data_ptr(), stream, False)
        rt.eval_base = plan.ensure_eval_cache(dev, stream)
        _load_inputs(plan, rt, inputs)
        for op in plan.ops:
            op.fwd(rt)
        if decode:
            return plan, [_decode(plan, rt, arena)]
        return plan, _outputs(plan, arena, dtype)


def _bump_bn_counters(plan):
    """nn.BatchNorm2d increments num_batches_tracked in training forward."""
    ts = getattr(plan, "_nbt", None)
    if ts is None:
        from .plan import ConvOp, SiblingConvOp
        ts = [m.bn.num_batches_tracked for op in plan.ops
              for m in (op.bn_modules() if isinstance(op, SiblingConvOp) else (op.mod,) if isinstance(op, ConvOp) else ())]
        plan._nbt = ts
    if ts:
        with torch.no_grad():
            torch._foreach_add_(ts, 1)
