"""GPU tier: the real HIP model through yms.dist.DataParallel.

Two ranks share cuda:0 over gloo (gloo reduces CUDA tensors through host staging; on an 8-GPU node
the same calls go over RCCL).  Each rank trains on its own shard; the averaged gradients must equal
the mean of the single-process per-shard HIP gradients, buckets must be issued from inside the
plan backward (side-stream wgrad joined before each bucket), and BN running buffers must follow
rank 0 (DDP broadcast_buffers semantics).  The reference has no DP (train.py:177-181)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank):
    return torch.randn(2, 3, 64, 96, generator=torch.Generator().manual_seed(100 + rank))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import model_ref as M
        from yms.dist import DataParallel
        from yolov8.yolov8 import YOLOv8
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        sd = M.init_params("n", 80)
        model = YOLOv8("n", 80).to(dev)
        model.load_state_dict(sd)
        with torch.no_grad():            # rank-dependent buffers: the broadcast must undo this
            model.backbone.conv0.bn.running_mean.add_(float(rank))
        dp = DataParallel(model, bucket_cap_mb=0.25)          # ~65K floats/bucket -> many buckets
        ok_bcast = bool(torch.equal(model.backbone.conv0.bn.running_mean.cpu(),
                                    sd["backbone.conv0.bn.running_mean"]))
        dp.train()
        outs = dp(_shard(rank).to(dev))
        sum((o.double() ** 2).mean() for o in outs).backward()
        torch.cuda.synchronize()
        # numpy arrays pickle by value (torch CPU tensors would pass file descriptors that die with this process)
        grads = {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}
        launched = dp.bucketer.launched_buckets
        # a second step: buffers re-broadcast from rank 0 before the forward
        with torch.no_grad():
            model.neck.c2f_1.conv1.bn.running_var.mul_(1.0 + rank)
        dp.zero_grad(set_to_none=True)
        seen = []
        h = model.register_forward_pre_hook(
            lambda mod, inp: seen.append(mod.neck.c2f_1.conv1.bn.running_var.detach().cpu().clone()))
        outs = dp(_shard(rank).to(dev))
        h.remove()
        rv = seen[0].numpy()      # the buffer the forward started from (after DataParallel's broadcast)
        sum((o.double() ** 2).mean() for o in outs).backward()
        torch.cuda.synchronize()
        q.put((rank, grads, launched, ok_bcast, rv))
    except Exception as e:   # surface the error in the parent
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_dataparallel_real_model_two_ranks_gloo_on_gpu():
    from oracle import model_ref as M
    from yolov8.yolov8 import YOLOv8
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    # single-process HIP gradients of each shard, averaged
    sd = M.init_params("n", 80)
    per = []
    for rank in range(world):
        m = YOLOv8("n", 80).cuda()
        m.load_state_dict(sd)
        m.train()
        sum((o.double() ** 2).mean() for o in m(_shard(rank).cuda())).backward()
        per.append({k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None})
    (_, g0, l0, b0, rv0), (_, g1, l1, b1, rv1) = res
    assert b0 and b1
    assert l0 == l1 >= 3, (l0, l1)
    assert set(g0) == set(per[0])
    for k in per[0]:
        mean = (per[0][k].double() + per[1][k].double()) / 2
        for g in (g0, g1):
            err = ((torch.from_numpy(g[k]).double() - mean).norm() / (mean.norm() + 1e-30)).item()
            assert err < 1e-5, (k, err)
    assert (rv0 == rv1).all()   # rank 1's scaled running_var was replaced by rank 0's
