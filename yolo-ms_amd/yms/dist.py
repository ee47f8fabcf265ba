"""Data-parallel training over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

One process per GPU.  The reference is single-device (train.py:177-181); this is the
new DP layer of SURVEY 5/8(e):

* parameters are broadcast from rank 0 once; BN running buffers are broadcast from
  rank 0 before every forward (DDP's default ``broadcast_buffers`` semantics; the
  reference has no SyncBN, so per-replica batch statistics are used);
* the plan's backward writes every fp32 parameter gradient into ONE flat arena,
  ordered by backward completion (yms.plan.Plan.pgrad_order).  The arena is cut into
  ~``bucket_cap_mb`` contiguous buckets; as soon as the last op contributing to a bucket
  has been enqueued, an async all-reduce(AVG) of that bucket is issued.  RCCL's stream
  waits on the compute stream at that point, so the collective overlaps the rest of the
  backward; ``finish`` joins the compute stream to every outstanding collective.
* gradients reach autograd as views of the reduced arena -- no copies.

xGMI is point-to-point (7 links per GPU); ~10 MB buckets give 4-5 ring collectives per step
for YOLOv8-s (10.5 M params = 42 MB fp32), the first one starting after about a fifth of the
backward, each issued from the wgrad side stream so the compute stream never waits for it.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn


class GradBucketer:
    """Issues bucketed all-reduces from inside the plan backward (see runner._PlanFn)."""

    def __init__(self, group=None, bucket_cap_mb=10.0):
        self.group = group
        self.cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        self._plans = {}
        self.works = []
        self.launched_buckets = 0

    def _buckets(self, plan, views):
        key = (id(plan), tuple(v is not None for v in views))
        bk = self._plans.get(key)
        if bk is not None:
            return bk
        # element ranges of each param in the flat arena (pgrad_order), only params with grads
        ranges = []
        off = 0
        for i in plan.pgrad_order:
            if views[i] is not None:
                n = views[i].numel()
                ranges.append((i, off, off + n))
                off += n
        # owner op position (in backward order) of every param: the LAST op that writes its grad
        # (a shared parameter is complete only after its final contribution)
        owner = {}
        for pos, op in enumerate(reversed(plan.ops)):
            for pi in op.grad_params():
                owner[pi] = max(owner.get(pi, -1), pos)
        buckets = []   # (start, end, ready_after_backward_pos)
        s, last = 0, -1
        for i, a, b in ranges:
            last = max(last, owner[i])
            if b - s >= self.cap:
                buckets.append((s, b, last))
                s, last = b, -1
        if s < off:
            buckets.append((s, off, last))
        ready = {}
        for bi, (a, b, pos) in enumerate(buckets):
            ready.setdefault(pos, []).append(bi)
        bk = (buckets, ready, {id(op): pos for pos, op in enumerate(reversed(plan.ops))})
        self._plans[key] = bk
        return bk

    def begin(self, plan, pg, ptrs, views):
        self.pg = pg
        self.buckets, self.ready, self.pos = self._buckets(plan, views)
        self.works = []
        self.launched_buckets = 0

    def _reduce(self, t):
        if dist.get_backend(self.group) == "nccl":
            return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def pending(self, op):
        """True when op_done(op) will launch a bucket all-reduce."""
        return bool(self.ready.get(self.pos[id(op)]))

    def op_done(self, op):
        for bi in self.ready.get(self.pos[id(op)], ()):
            a, b, _ = self.buckets[bi]
            self.works.append((self._reduce(self.pg[a:b]), a, b))
            self.launched_buckets += 1

    def finish(self):
        ws = dist.get_world_size(self.group)
        avg_native = dist.get_backend(self.group) == "nccl"
        for w, a, b in self.works:
            w.wait()
            if not avg_native:
                self.pg[a:b].div_(ws)
        self.works = []


class DataParallel(nn.Module):
    """``yms.dist.DataParallel(YOLOv8(...).cuda())`` -- drop-in for the single-device model
    inside the reference training loop; state_dict keys are prefixed ``module.`` exactly
    like torch DDP (the reference strips that prefix when loading, train.py:270-276)."""

    def __init__(self, module, group=None, bucket_cap_mb=10.0, broadcast_buffers=True):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("yms.dist.DataParallel: call torch.distributed.init_process_group first")
        self.module = module
        self.group = group
        self.broadcast_buffers = broadcast_buffers
        self.bucketer = GradBucketer(group, bucket_cap_mb)
        with torch.no_grad():
            for p in module.parameters():
                dist.broadcast(p.data, 0, group=group)
            self._flat_buffers()
            self._sync_buffers()
        module._yms_grad_hook = self.bucketer

    def _flat_buffers(self):
        """Re-home every floating-point buffer (BN running stats) as a view of ONE flat tensor, so
        the per-step broadcast is a single in-place collective with no flatten/unflatten copies."""
        mods = [(m, n, b) for m in self.module.modules() for n, b in m._buffers.items()
                if b is not None and b.is_floating_point()]
        self._flat = None
        if not mods:
            return
        groups = {}
        for m, n, b in mods:
            groups.setdefault((b.dtype, b.device), []).append((m, n, b))
        if len(groups) != 1:
            self._bufs = [b for _, _, b in mods]
            return
        flat = torch._utils._flatten_dense_tensors([b for _, _, b in mods])
        off = 0
        self._views = []
        for m, n, b in mods:
            m._buffers[n] = flat[off:off + b.numel()].view_as(b)
            self._views.append((m, n, m._buffers[n].data_ptr()))
            off += b.numel()
        self._flat = flat

    def _flat_is_current(self):
        """True while every buffer is still the view of ``_flat`` it was made: ``.to()``, ``.half()``
        or ``load_state_dict(assign=True)`` on the wrapped module replace buffers, and a broadcast of
        the stale flat tensor would then leave the ranks' BN statistics silently diverged."""
        return all(m._buffers.get(n) is not None and m._buffers[n].data_ptr() == p for m, n, p in self._views)

    def _sync_buffers(self):
        if self._flat is None or not self._flat_is_current():
            # mixed dtypes / devices keep per-buffer references: re-collect them from the module on
            # every call, so a replaced buffer is never the one broadcast into
            self._flat_buffers()
        if self._flat is not None:
            dist.broadcast(self._flat, 0, group=self.group)
            return
        bufs = getattr(self, "_bufs", [])
        if not bufs:
            return
        flat = torch._utils._flatten_dense_tensors(bufs)
        dist.broadcast(flat, 0, group=self.group)
        for b, f in zip(bufs, torch._utils._unflatten_dense_tensors(flat, bufs)):
            b.copy_(f)

    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.module.training:
            with torch.no_grad():
                self._sync_buffers()
        return self.module(*args, **kwargs)
