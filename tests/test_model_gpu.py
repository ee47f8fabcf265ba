"""GPU parity of the module API (yolov8.*) against golden vectors produced by the
reference model (tests/golden) and against the CPU oracle (oracle/model_ref.py)."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import model_ref as M
from yolov8.model import components as C
from yolov8.yolov8 import YOLOv8

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def _load(name):
    return dict(np.load(os.path.join(GOLD, name)))


def _closed_form_local(module):
    """Same closed-form init make_golden.py used (keys local to the block)."""
    sd = {}
    for k, v in module.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = torch.zeros_like(v)
        elif v.dim() == 4:
            fan = v.shape[1] * v.shape[2] * v.shape[3]
            sd[k] = M._closed_form(k, tuple(v.shape), (3.0 / fan) ** 0.5 * 1.2)
        elif k.endswith("bn.weight"):
            sd[k] = M._closed_form(k, tuple(v.shape), 0.25, base=1.0)
        elif k.endswith("bn.bias"):
            sd[k] = M._closed_form(k, tuple(v.shape), 0.2)
        elif k.endswith("running_mean"):
            sd[k] = M._closed_form(k, tuple(v.shape), 0.1)
        elif k.endswith("running_var"):
            sd[k] = M._closed_form(k, tuple(v.shape), 0.3, base=1.2)
        else:
            sd[k] = M._closed_form(k, tuple(v.shape), 0.5)
    module.load_state_dict(sd)
    return module


def _rel(got, ref):
    got = torch.as_tensor(got).double().cpu()
    ref = torch.as_tensor(ref).double()
    return ((got - ref).norm() / (ref.norm() + 1e-12)).item()


def _maxerr(got, ref):
    got = torch.as_tensor(got).float().cpu()
    ref = torch.as_tensor(ref).float()
    return ((got - ref).abs().max() / (ref.abs().max() + 1e-12)).item()


BLOCKS = {
    "conv1x1": lambda: C.Conv(16, 24, 1, 1, 0),
    "conv3x3s1": lambda: C.Conv(8, 16, 3, 1, 1),
    "conv3x3s2": lambda: C.Conv(3, 16, 3, 2, 1),
    "conv3x3s2_c24": lambda: C.Conv(24, 32, 3, 2, 1),
    "bottleneck": lambda: C.Bottleneck(16, 16),
    "c2f_n1": lambda: C.C2f(32, 32, 1),
    "c2f_n2": lambda: C.C2f(24, 48, 2),
    "sppf": lambda: C.SPPF(32, 32),
}


@pytest.mark.parametrize("name", sorted(BLOCKS))
def test_block_fp32_vs_reference_golden(name):
    g = _load(f"block_{name}.npz")
    m = _closed_form_local(BLOCKS[name]()).to(DEV)
    x = torch.from_numpy(g["x"]).to(DEV)
    m.eval()
    y = m(x)
    assert _maxerr(y, g["eval_y"]) < 1e-4
    m.train()
    xg = x.clone().requires_grad_(True)
    y = m(xg)
    assert _maxerr(y.detach(), g["train_y0"]) < 1e-4
    (y.float() * torch.from_numpy(g["cot0"]).to(DEV)).sum().backward()
    assert _rel(xg.grad, g["dx"]) < 1e-4
    pd = dict(m.named_parameters())
    for k in g:
        if k.startswith("grad:"):
            assert _rel(pd[k[5:]].grad, g[k]) < 1e-4, k
        if k.startswith("buf:") and "running" in k:
            assert _maxerr(dict(m.named_buffers())[k[4:]], g[k]) < 1e-5, k
        if k.startswith("buf:") and "num_batches" in k:
            assert int(dict(m.named_buffers())[k[4:]]) == int(g[k])


def test_upsample_and_dfl_golden():
    g = _load("block_upsample.npz")
    up = C.Upsample().to(DEV)
    y = up(torch.from_numpy(g["x"]).to(DEV))
    assert torch.equal(y.float().cpu(), torch.from_numpy(g["y"]))
    g = _load("block_dfl.npz")
    y = C.DFL().to(DEV)(torch.from_numpy(g["x"]).to(DEV))
    assert _maxerr(y, g["y"]) < 1e-5


@pytest.mark.parametrize("fname,v,nc", [("model_n80_2x64x64.npz", "n", 80),
                                        ("model_n80_1x128x96.npz", "n", 80),
                                        ("model_n1_2x64x64.npz", "n", 1)])
def test_full_model_fp32_vs_reference_golden(fname, v, nc):
    g = _load(fname)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(M.init_params(v, nc))
    x = torch.from_numpy(g["x"]).to(DEV)
    m.eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    y = m(x)
    assert y.shape == g["eval_y"].shape
    ref = torch.from_numpy(g["eval_y"])
    assert _maxerr(y[..., :4], ref[..., :4]) < 1e-4
    assert (y[..., 4:].cpu() - ref[..., 4:]).abs().max().item() < 1e-5
    m.train()
    ys = m(x)
    loss = 0
    for i, t in enumerate(ys):
        # batch-statistics BN over tiny maps amplifies fp32 summation-order noise: 1e-3 (north-star bar)
        assert _maxerr(t.detach(), g[f"train_y{i}"]) < 1e-3
        loss = loss + (t * torch.from_numpy(g[f"cot{i}"]).to(DEV)).sum()
    loss.backward()
    pd = dict(m.named_parameters())
    for k in g:
        if k.startswith("gsum:"):
            gr = pd[k[5:]].grad.double().cpu()
            s, a = g[k]
            assert abs(gr.abs().sum().item() - a) <= 2e-3 * abs(a) + 1e-6, k
        elif k.startswith("grad:"):
            # GPU-fp32 vs CPU-fp32: both carry fp32 noise (fp64-gated at 1e-3 in the next test)
            assert _rel(pd[k[5:]].grad, g[k]) < 2e-3, k
        elif k.startswith("buf:"):
            assert _maxerr(dict(m.named_buffers())[k[4:]], g[k]) < 1e-5, k


def test_s640_bf16_eval_against_oracle():
    """YOLO-MS-S (= YOLOv8-s graph) 640x640 bf16 inference vs the fp32 CPU oracle."""
    v, nc = "s", 80
    sd = M.init_params(v, nc)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    x = torch.randn(2, 3, 640, 640, generator=torch.Generator().manual_seed(0))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(DEV)).cpu()
    with torch.no_grad():
        ref = M.forward(dict(sd), v, nc, x, False)
    assert y.shape == (2, 8400, 84) and y.dtype == torch.float32
    cls_err = (y[..., 4:] - ref[..., 4:]).abs().max().item()
    box_rel = _rel(y[..., :4], ref[..., :4])
    # bf16 end-to-end drift (CPU bf16 autocast itself drifts 4.5e-2 box / 1.9e-3 cls)
    assert cls_err < 3e-2, cls_err
    assert box_rel < 2e-2, box_rel


def _oracle_grads(v, nc, sd, x, dtype, autocast=False):
    p = {k: (t.clone().to(dtype).requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else (t.clone().to(dtype) if t.is_floating_point() else t.clone()))
         for k, t in sd.items()}
    if autocast:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            r = M.forward(p, v, nc, x.to(dtype), True)
    else:
        r = M.forward(p, v, nc, x.to(dtype), True)
    sum((o.double() ** 2).mean() for o in r).backward()
    return {k: t.grad.double() for k, t in p.items() if t.grad is not None}


def test_full_model_fp32_grads_vs_fp64_oracle():
    """fp32 training gradients of every parameter within 1e-3 (relative L2) of an fp64 CPU run."""
    v, nc = "n", 80
    sd = M.init_params(v, nc)
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    g64 = _oracle_grads(v, nc, sd, x, torch.float64)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.train()
    sum((o.double() ** 2).mean() for o in m(x.to(DEV))).backward()
    pd = dict(m.named_parameters())
    worst = max(_rel(pd[k].grad, g64[k]) for k in g64 if k in pd)
    assert worst < 1e-3, worst


def test_s_bf16_train_grads_no_worse_than_cpu_bf16():
    """bf16 training drift (YOLO-MS-S graph): the HIP path's gradients, measured against an fp64
    oracle, must be no worse than the reference's own CPU path under bf16 autocast.  (Through ~60
    batch-stat BN layers at batch 2 both drift by tens of percent on the deepest layers; per-kernel
    bf16 parity is gated tightly in test_conv_gpu.py.)"""
    v, nc = "s", 80
    sd = M.init_params(v, nc)
    x = torch.randn(2, 3, 128, 128, generator=torch.Generator().manual_seed(1))
    g64 = _oracle_grads(v, nc, sd, x, torch.float64)
    gbf = _oracle_grads(v, nc, sd, x, torch.float32, autocast=True)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        outs = m(x.to(DEV))
    sum((o.double() ** 2).mean() for o in outs).backward()
    pd = dict(m.named_parameters())
    ours = sorted(_rel(pd[k].grad, g64[k]) for k in g64 if k in pd)
    cpu = sorted(_rel(gbf[k], g64[k]) for k in g64 if k in pd)
    # median and 90th percentile within 1.2x of the CPU bf16 drift; the single worst tensor (a
    # chaotic deep-layer extreme that moves with any rounding change) within 1.5x
    med, p90 = len(ours) // 2, (9 * len(ours)) // 10
    assert ours[med] <= 1.2 * cpu[med], (ours[med], cpu[med])
    assert ours[p90] <= 1.2 * cpu[p90], (ours[p90], cpu[p90])
    assert ours[-1] <= 1.5 * cpu[-1], (ours[-1], cpu[-1])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_c2f_lowp_train_grads(dt):
    """Shallow block in bf16/fp16 training: forward, input and parameter grads within 3e-2 of fp32."""
    torch.manual_seed(0)
    m = _closed_form_local(C.C2f(64, 64, 2)).to(DEV).train()
    x = torch.randn(4, 64, 20, 20, generator=torch.Generator().manual_seed(2))
    cot = torch.randn(4, 64, 20, 20, generator=torch.Generator().manual_seed(3))
    p = {"blk." + k: t.detach().cpu().clone() for k, t in m.state_dict().items()}
    pr = {k: (t.requires_grad_(True) if t.is_floating_point() and "running" not in k else t) for k, t in p.items()}
    xr = x.clone().requires_grad_(True)
    yr = M.c2f(pr, "blk", xr, 2, True)
    (yr * cot).sum().backward()
    xg = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        y = m(xg)
    assert y.dtype == dt
    (y.float() * cot.to(DEV)).sum().backward()
    assert _rel(y.detach().float(), yr.detach()) < 3e-2
    assert _rel(xg.grad, xr.grad) < 3e-2
    pd = dict(m.named_parameters())
    for k, t in pr.items():
        if t.grad is not None:
            assert _rel(pd[k[4:]].grad, t.grad) < 3e-2, k


def test_cpu_tensor_fails_loudly():
    m = C.Conv(3, 8).to(DEV)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 3, 8, 8))


# ---- configs[3] / configs[4] parity cases (BASELINE.json) ----------------------------------

def _eval_vs_oracle(v, size, batch, dt, seed):
    nc = 80
    sd = M.init_params(v, nc)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    x = torch.randn(batch, 3, size, size, generator=torch.Generator().manual_seed(seed))
    with torch.autocast("cuda", dtype=dt):
        y = m(x.to(DEV)).cpu()
    with torch.no_grad():
        ref = M.forward(dict(sd), v, nc, x, False)
    A = 21 * (size // 32) ** 2
    assert y.shape == (batch, A, 84) and y.dtype == torch.float32
    assert torch.isfinite(y).all()
    return (y[..., 4:] - ref[..., 4:]).abs().max().item(), _rel(y[..., :4], ref[..., :4])


def test_s1280_fp16_eval_against_oracle():
    """configs[4]: YOLO-MS-S 1280x1280 fp16 inference (A = 33600) vs the fp32 CPU oracle."""
    cls_err, box_rel = _eval_vs_oracle("s", 1280, 1, torch.float16, 4)
    # fp16 carries 3 more mantissa bits than bf16: tighter than the bf16 bound of the 640 test
    assert cls_err < 1e-2, cls_err
    assert box_rel < 5e-3, box_rel


def test_l640_eval_fp32_and_bf16_against_oracle():
    """configs[3] graph: YOLO-MS-L (deep 'l' backbone, 512-wide C2f stacks) 640x640 forward.
    fp32 within the north-star 1e-3 of the fp32 oracle (the oracle itself is 6e-4 from fp64 on the
    class probabilities).  bf16: the 'l' graph with this init is chaotic under bf16 -- the
    reference's own CPU bf16 autocast moves single class probabilities by up to 0.98 -- so bf16 is
    gated on the error distribution against the CPU bf16 path's (median / p90 / p99)."""
    v, nc = "l", 80
    sd = M.init_params(v, nc)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    x = torch.randn(1, 3, 640, 640, generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        ref = M.forward(dict(sd), v, nc, x, False)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            cpu_bf = M.forward(dict(sd), v, nc, x, False).float()
        y32 = m(x.to(DEV)).cpu()
        m2 = YOLOv8(v, nc).to(DEV)
        m2.load_state_dict(sd)
        m2.eval()
        m2.head.stride = torch.tensor([8.0, 16.0, 32.0])
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ybf = m2(x.to(DEV)).cpu()
    assert y32.shape == (1, 8400, 84) and ybf.dtype == torch.float32
    assert (y32[..., 4:] - ref[..., 4:]).abs().max().item() < 1e-3
    assert _rel(y32[..., :4], ref[..., :4]) < 1e-4
    ours = (ybf[..., 4:] - ref[..., 4:]).abs().flatten()
    cpu = (cpu_bf[..., 4:] - ref[..., 4:]).abs().flatten()
    for q in (0.5, 0.9, 0.99):
        a, b = torch.quantile(ours, q).item(), torch.quantile(cpu, q).item()
        assert a <= 1.3 * b + 1e-4, (q, a, b)
    assert _rel(ybf[..., :4], ref[..., :4]) <= 1.3 * _rel(cpu_bf[..., :4], ref[..., :4]) + 1e-4


def test_l_bf16_train_grads_no_worse_than_cpu_bf16():
    """configs[3]: YOLO-MS-L bf16 training gradients, drift vs fp64 no worse than the CPU bf16 path
    (same criterion as the 's' test above; batch 2 at 96x96 keeps the fp64 oracle within seconds)."""
    v, nc = "l", 80
    sd = M.init_params(v, nc)
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(6))
    g64 = _oracle_grads(v, nc, sd, x, torch.float64)
    gbf = _oracle_grads(v, nc, sd, x, torch.float32, autocast=True)
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        outs = m(x.to(DEV))
    sum((o.double() ** 2).mean() for o in outs).backward()
    pd = dict(m.named_parameters())
    keys = [k for k in g64 if k in pd]
    assert len(keys) == len([p for p in pd.values() if p.requires_grad])
    ours = sorted(_rel(pd[k].grad, g64[k]) for k in keys)
    cpu = sorted(_rel(gbf[k], g64[k]) for k in keys)
    med, p90 = len(ours) // 2, (9 * len(ours)) // 10
    assert ours[med] <= 1.2 * cpu[med], (ours[med], cpu[med])
    assert ours[p90] <= 1.2 * cpu[p90], (ours[p90], cpu[p90])
    assert ours[-1] <= 1.5 * cpu[-1], (ours[-1], cpu[-1])
