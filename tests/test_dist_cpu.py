"""CPU tier: the data-parallel layer (yms.dist) over gloo with world_size 2.

The GPU path issues the same calls over RCCL ("nccl" backend, ReduceOp.AVG); here gloo
(SUM + divide) exercises bucketing, completion-order triggering, averaging, parameter
broadcast and BN-buffer broadcast without a GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Op:
    def __init__(self, params):
        self.params = params

    def grad_params(self):
        return self.params


class _Plan:
    """Mimics yms.plan.Plan: ops in forward order, params owned by ops."""

    def __init__(self, sizes):
        self.ops = [_Op([2 * i, 2 * i + 1]) for i in range(len(sizes) // 2)]
        order = []
        for op in reversed(self.ops):
            order += op.grad_params()
        self.pgrad_order = order
        self.sizes = sizes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from yms.dist import DataParallel, GradBucketer
        sizes = [1000, 10, 5000, 20, 300, 3, 70000, 64]
        plan = _Plan(sizes)
        views = [None] * len(sizes)
        total = sum(sizes)
        pg = torch.empty(total)
        off = 0
        for i in plan.pgrad_order:
            views[i] = pg[off:off + sizes[i]]
            off += sizes[i]
        bk = GradBucketer(bucket_cap_mb=0.02)      # ~5K floats per bucket -> several buckets
        launched = []
        for it in range(2):                          # twice: cached bucket layout
            for i in plan.pgrad_order:
                views[i].copy_(torch.arange(sizes[i], dtype=torch.float32) * (rank + 1) + i)
            bk.begin(plan, pg, None, views)
            for op in reversed(plan.ops):
                # a bucket must only be launched once all its params are written
                before = bk.launched_buckets
                will = bk.pending(op)
                bk.op_done(op)
                assert will == (bk.launched_buckets > before)
            launched.append(bk.launched_buckets)
            bk.finish()
        exp = []
        for i in plan.pgrad_order:
            base = torch.arange(sizes[i], dtype=torch.float32)
            exp.append(base * (1 + world) / 2 + i)   # mean over ranks of base*(r+1)+i
        ok_grad = torch.allclose(pg, torch.cat(exp))
        # parameter + BN buffer broadcast from rank 0
        torch.manual_seed(rank)
        m = torch.nn.BatchNorm2d(4)
        with torch.no_grad():
            m.weight.fill_(rank + 1.0)
            m.running_mean.fill_(10.0 * (rank + 1))
        dp = DataParallel(m, bucket_cap_mb=1.0)
        ok_bcast = bool(torch.all(m.weight == 1.0)) and bool(torch.all(m.running_mean == 10.0))
        with torch.no_grad():
            m.running_mean.fill_(5.0 * (rank + 1))
        dp.train()
        dp(torch.zeros(2, 4, 3, 3))                   # buffers re-synced before forward
        rm1 = m.running_mean[0].item()
        # a cast after wrapping replaces the buffers: the broadcast must follow the new tensors
        m.double()
        with torch.no_grad():
            m.running_mean.fill_(7.0 * (rank + 1))
        dp(torch.zeros(2, 4, 3, 3, dtype=torch.float64))
        # mixed buffer dtypes (no single flat tensor): a replaced buffer must still be the one synced
        mm = torch.nn.Sequential(torch.nn.BatchNorm2d(4), torch.nn.BatchNorm2d(4).double())
        dpm = DataParallel(mm, bucket_cap_mb=1.0)
        mm[0].running_mean = torch.full((4,), 3.0 * (rank + 1))      # replaced after wrapping
        with torch.no_grad():
            mm[1].running_mean.fill_(2.0 * (rank + 1))
        dpm.eval()
        with torch.no_grad():
            dpm._sync_buffers()
        mixed = (mm[0].running_mean[0].item(), mm[1].running_mean[0].item())
        q.put((rank, ok_grad, launched, ok_bcast, (rm1, m.running_mean[0].item()), mixed))
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_gloo_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_grad, launched, ok_bcast, rm, mixed in res:
        assert ok_grad, rank
        assert launched[0] == launched[1] >= 3, launched
        assert ok_bcast, rank
        # rank 0's buffer (5.0) broadcast before forward, then BN2d(momentum 0.1) on zeros
        assert abs(rm[0] - 0.9 * 5.0) < 1e-5, rm
        assert abs(rm[1] - 0.9 * 7.0) < 1e-5, rm     # rank 0's value after .double()
        assert mixed == (3.0, 2.0), mixed              # rank 0's values, incl. the replaced buffer


def test_bucket_layout_on_the_real_plan():
    """Bucket readiness on the real YOLO-MS-S training plan (meta tensors, no GPU): the buckets tile
    the flat fp32 grad arena in backward-completion order, and each is triggered only after the
    last op owning any of its parameters (so no all-reduce starts before its grads are written)."""
    from yms import runner
    from yms.dist import GradBucketer
    from yolov8.yolov8 import YOLOv8
    m = YOLOv8("s", 80).train()
    plan = runner.get_plan(m, [torch.empty(64, 3, 640, 640, device="meta")], torch.bfloat16, True)
    params = plan.params()
    views = [torch.empty(p.shape, device="meta") if p.requires_grad else None for p in params]
    bk = GradBucketer(bucket_cap_mb=4.0)
    buckets, ready, pos = bk._buckets(plan, views)
    total = sum(v.numel() for v in views if v is not None)
    assert abs(total - 10_497_808) < 100            # YOLOv8-s grads (DFL conv frozen)
    assert buckets[0][0] == 0 and buckets[-1][1] == total
    assert all(buckets[i][1] == buckets[i + 1][0] for i in range(len(buckets) - 1))
    assert len(buckets) >= 8
    owner = {}
    for p_, op in enumerate(reversed(plan.ops)):
        for pi in op.grad_params():
            owner[pi] = max(owner.get(pi, -1), p_)
    off = 0
    ranges = []
    for i in plan.pgrad_order:
        if views[i] is not None:
            ranges.append((i, off, off + views[i].numel()))
            off += views[i].numel()
    for a, b, trig in buckets:
        for i, lo, hi in ranges:
            if lo < b and a < hi:
                assert owner[i] <= trig
    # every bucket is launched exactly once over a backward walk
    fired = [bi for p_ in range(len(plan.ops)) for bi in ready.get(p_, [])]
    assert sorted(fired) == list(range(len(buckets)))
