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


def _quantiles_no_worse(ours, cpu, qs=(0.5, 0.9, 0.99), factor=1.3):
    for q in qs:
        a, b = torch.quantile(ours, q).item(), torch.quantile(cpu, q).item()
        assert a <= factor * b + 1e-5, (q, a, b)


def test_s640_bf16_eval_against_oracle():
    """configs[1] graph: YOLO-MS-S (= YOLOv8-s graph) 640x640 bf16 inference vs the fp32 CPU oracle.
    Gate: the error distribution (median / p90 / p99 of |ours - fp32 oracle| over class
    probabilities, and the box L2 drift) within 1.3x of the reference's own CPU bf16 autocast path
    on the same input (SURVEY 7.3 measured that path's class drift at 1.9e-3)."""
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
        with torch.autocast("cpu", dtype=torch.bfloat16):
            cpu_bf = M.forward(dict(sd), v, nc, x, False).float()
    assert y.shape == (2, 8400, 84) and y.dtype == torch.float32
    ours = (y[..., 4:] - ref[..., 4:]).abs().flatten()
    cpu = (cpu_bf[..., 4:] - ref[..., 4:]).abs().flatten()
    _quantiles_no_worse(ours, cpu)
    assert ours.max().item() <= 1.5 * cpu.max().item() + 1e-4, (ours.max().item(), cpu.max().item())
    assert _rel(y[..., :4], ref[..., :4]) <= 1.3 * _rel(cpu_bf[..., :4], ref[..., :4]) + 1e-4


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


# ---- BASELINE.json configs at their own sizes (VERDICT r1 "untested configs") ---------------

def _train_grads_vs(v, nc, sd, x, dtype):
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.train()
    if dtype == torch.float32:
        outs = m(x.to(DEV))
    else:
        with torch.autocast("cuda", dtype=dtype):
            outs = m(x.to(DEV))
    sum((o.double() ** 2).mean() for o in outs).backward()
    return m, [o.detach().float().cpu() for o in outs], dict(m.named_parameters())


def test_configs0_n320_fp32_eval_train_grads():
    """configs[0]: YOLO-MS-XS -> reference 'n' graph, 320x320, B=2, fp32: eval output, train-mode
    head maps, every parameter gradient and the BN running buffers against the oracle within the
    north-star 1e-3 (grads against fp64, as the oracle's own fp32 noise is ~1e-4 there)."""
    v, nc = "n", 80
    sd = M.init_params(v, nc)
    x = torch.randn(2, 3, 320, 320, generator=torch.Generator().manual_seed(10))
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    y = m(x.to(DEV)).cpu()
    with torch.no_grad():
        ref = M.forward(dict(sd), v, nc, x, False)
    assert y.shape == (2, 2100, 84)
    assert (y[..., 4:] - ref[..., 4:]).abs().max().item() < 1e-3
    assert _rel(y[..., :4], ref[..., :4]) < 1e-4
    # train mode: head maps vs the fp32 oracle, grads vs fp64, running buffers
    p = {k: (t.clone().requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else t.clone()) for k, t in sd.items()}
    r = M.forward(p, v, nc, x, True)
    g64 = _oracle_grads(v, nc, sd, x, torch.float64)
    m2, outs, pd = _train_grads_vs(v, nc, sd, x, torch.float32)
    for o, rr in zip(outs, r):
        assert _maxerr(o, rr.detach()) < 1e-3
    worst = max(_rel(pd[k].grad, g64[k]) for k in g64 if k in pd)
    assert worst < 1e-3, worst
    bufs = dict(m2.named_buffers())
    for k, t in p.items():
        if "running" in k:
            assert _maxerr(bufs[k], t) < 1e-4, k


def test_configs3_l640_fp32_train_grads_vs_fp64():
    """configs[3] at its own resolution: YOLO-MS-L 640x640 training (B=2) on the closed-form
    weights: every parameter gradient within the north-star 1e-3 of an fp64 oracle (the CPU fp32
    oracle's own drift is printed beside it).  The bf16 gates run on the well-conditioned fixture
    (tests/test_train_conditioned_gpu.py), where the CPU bf16 yardstick is not chaotic."""
    v, nc = "l", 80
    sd = M.init_params(v, nc)
    x = torch.randn(2, 3, 640, 640, generator=torch.Generator().manual_seed(22))
    g64 = _oracle_grads(v, nc, sd, x, torch.float64)
    g32 = _oracle_grads(v, nc, sd, x, torch.float32)
    _, _, pd = _train_grads_vs(v, nc, sd, x, torch.float32)
    keys = [k for k in g64 if k in pd]
    assert len(keys) == len([p for p in pd.values() if p.requires_grad])
    errs = sorted(_rel(pd[k].grad, g64[k]) for k in keys)
    cerr = sorted(_rel(g32[k], g64[k]) for k in keys)
    n = len(errs)
    print(f"L640 fp32 grad drift vs fp64: ours median {errs[n // 2]:.3g} p90 {errs[9 * n // 10]:.3g} max "
          f"{errs[-1]:.3g}; CPU fp32 median {cerr[n // 2]:.3g} p90 {cerr[9 * n // 10]:.3g} max {cerr[-1]:.3g}")
    assert errs[-1] < 1e-3, (errs[-1], cerr[-1])


def test_configs2_s640_b64_fp32_train_step_vs_oracle():
    """The bench's batch: YOLO-MS-S 640x640, B=64, fp32 training forward + backward against the fp32
    oracle at B=64.  Covers what only the full batch reaches: 256-row tiles with per-128-row BN
    statistics, multi-split wgrad slabs, the capped (<= 512-row) BN-backward partial sums and
    > 2^31-byte arenas.  Gate: head maps within 1e-3 (rel to max) and every parameter gradient
    within 2e-3 relative L2 (two fp32 summation orders over 26 M pixels per channel)."""
    v, nc = "s", 80
    sd = M.init_params(v, nc)
    x = torch.randn(64, 3, 640, 640, generator=torch.Generator().manual_seed(23))
    p = {k: (t.clone().requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else t.clone()) for k, t in sd.items()}
    r = M.forward(p, v, nc, x, True)
    sum((o.double() ** 2).mean() for o in r).backward()
    rd = [o.detach() for o in r]
    del r
    _, outs, pd = _train_grads_vs(v, nc, sd, x, torch.float32)
    for o, rr in zip(outs, rd):
        assert _maxerr(o, rr) < 1e-3
    errs = sorted((_rel(pd[k].grad, t.grad.double()), k) for k, t in p.items() if t.grad is not None)
    assert errs[-1][0] < 2e-3, errs[-3:]


def _gemm_conv(x, w, s):
    """fp32 conv as unfold + GEMM on the GPU (torch im2col + BLAS; no conv library involved)."""
    import torch.nn.functional as F
    n, cin, h, wd = x.shape
    cout, _, k, _ = w.shape
    ho, wo = (h + 2 * (k // 2) - k) // s + 1, (wd + 2 * (k // 2) - k) // s + 1
    cols = F.unfold(x, k, padding=k // 2, stride=s)                    # [n, cin*k*k, L]
    return (w.view(cout, -1) @ cols).view(n, cout, ho, wo)


def _gemm_conv_bwd(x, w, dz, s):
    import torch.nn.functional as F
    n, cin, h, wd = x.shape
    cout, _, k, _ = w.shape
    dzf = dz.reshape(n, cout, -1)                                        # [n, cout, L]
    dcols = w.view(cout, -1).t() @ dzf                                   # [n, cin*k*k, L]
    dx = F.fold(dcols, (h, wd), k, padding=k // 2, stride=s)
    del dcols
    cols = F.unfold(x, k, padding=k // 2, stride=s)
    dw = torch.einsum("nol,nkl->ok", dzf, cols).view(cout, cin, k, k)
    return dx, dw


def _dw_ref(x, w):
    """fp32 depthwise k x k conv (stride 1, pad k//2) as a sum of k^2 shifted products on the GPU
    (no conv library involved)."""
    import torch.nn.functional as F
    k = w.shape[-1]
    p = k // 2
    h, wd = x.shape[2], x.shape[3]
    xp = F.pad(x, (p, p, p, p))
    z = torch.zeros_like(x)
    for dy in range(k):
        for dx in range(k):
            z += xp[:, :, dy:dy + h, dx:dx + wd] * w[:, 0, dy, dx].view(1, -1, 1, 1)
    return z


# Bench-scale gates of the bf16 kernels against fp32 torch on the same bf16 operands.  The
# outputs are fp32 accumulations rounded once to bf16: per element at most half an ulp, 2^-9 of
# its magnitude (~1.95e-3 of max|ref|), so the max gate is 2x that; the relative L2 error of such
# rounding is ~2^-9 / sqrt(3) ~ 1.1e-3 and a dropped k-tile (one of K/64) would give ~sqrt(64 / K)
# >= 0.05 even at K = 2304.  The fp32 weight gradients carry no output rounding.
BF16_MAX_GATE = 4e-3
BF16_L2_GATE = 2.5e-3
FP32_OUT_L2_GATE = 2e-4


def _rel_dev(got, ref):
    """relative L2 error on the device (fp32 norms of fp32 differences)"""
    return ((got.float() - ref.float()).norm() / (ref.float().norm() + 1e-30)).item()


def _dw_wgrad_ref(x, dz, k):
    import torch.nn.functional as F
    p = k // 2
    h, wd = x.shape[2], x.shape[3]
    xp = F.pad(x, (p, p, p, p))
    dw = torch.empty(x.shape[1], 1, k, k, device=x.device)
    for dy in range(k):
        for dx in range(k):
            dw[:, 0, dy, dx] = (xp[:, :, dy:dy + h, dx:dx + wd] * dz).sum((0, 2, 3))
    return dw


def _dw_layer_vs_fp32(key, g, dt):
    """One depthwise layer at its bench shape through the C-ABI: forward with BN statistics, dgrad
    (rot-180 taps) and the split wgrad, against fp32 shifted-sum references on the same bf16 operands."""
    import ctypes

    from hiputil import check_moments, nchw, nhwc, r8, split_stats, stats_buffer
    from yms import _lib as L
    n, h, w, c, k = key
    x = torch.randn(n, c, h, w, device=DEV, generator=g).to(dt).float()
    wt = torch.randn(c, 1, k, k, device=DEV, generator=g) / k
    sh = L.DwShape(n, h, w, c, k, L.dtype_code(dt))
    sp = ctypes.pointer(sh)
    xb = nhwc(x, dt)
    rows = L.lib().yms_dwconv_stats_rows(sp)
    buf = stats_buffer(rows, r8(c))
    y = torch.zeros((n, h, w, r8(c)), dtype=dt, device=DEV)
    L.call("yms_dwconv_fwd", sp, xb.data_ptr(), xb.shape[-1], 0, wt.data_ptr(), y.data_ptr(), y.shape[-1], 0,
           None, None, 0, buf.data_ptr(), r8(c), L.stream_ptr())
    z = _dw_ref(x, wt)
    yz = nchw(y, c)
    err = (yz - z).abs().max().item()
    # bf16 output, fp32 accumulation: one rounding, half-ulp 2^-9 of the element (BF16_MAX_GATE)
    assert err <= BF16_MAX_GATE * z.abs().max().item(), (key, "dw fwd", err)
    assert _rel_dev(yz, z) <= BF16_L2_GATE, (key, "dw fwd L2", _rel_dev(yz, z))
    del yz
    check_moments(split_stats(buf, rows, r8(c)), z, 1e-3)
    del y, buf
    dz = torch.randn(n, c, h, w, device=DEV, generator=g).to(dt).float()
    ref_dx = _dw_ref(dz, wt.flip(2, 3))
    dzb = nhwc(dz, dt)
    dx = torch.zeros((n, h, w, r8(c)), dtype=dt, device=DEV)
    L.call("yms_dwconv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wt.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
           0, L.stream_ptr())
    dxz = nchw(dx, c)
    err = (dxz - ref_dx).abs().max().item()
    assert err <= BF16_MAX_GATE * ref_dx.abs().max().item(), (key, "dw dgrad", err)
    assert _rel_dev(dxz, ref_dx) <= BF16_L2_GATE, (key, "dw dgrad L2", _rel_dev(dxz, ref_dx))
    del dxz
    del dx, ref_dx
    wsb = L.lib().yms_dwconv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4 + 1, device=DEV)
    dw = torch.zeros(c, 1, k, k, device=DEV)
    L.call("yms_dwconv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0, ws.data_ptr(),
           wsb, dw.data_ptr(), 0, L.stream_ptr())
    ref_dw = _dw_wgrad_ref(x, dz, k)
    err = (dw - ref_dw).abs().max().item()
    assert err <= 2e-3 * ref_dw.abs().max().item(), (key, "dw wgrad", err)
    assert _rel_dev(dw, ref_dw) <= FP32_OUT_L2_GATE, (key, "dw wgrad L2", _rel_dev(dw, ref_dw))


@pytest.mark.parametrize("version", ["s", "l", "ms-s", "ms-l"])
def test_configs_b64_bf16_layers_vs_fp32(version):
    """Every distinct conv layer of YOLO-MS-S (configs[2]) / YOLO-MS-L (configs[3]) at 640x640,
    B=64 in bf16 -- forward with BN statistics, dgrad and wgrad -- through the C-ABI against fp32
    PyTorch on the GPU over the same bf16-rounded operands (the per-kernel reference of a
    floating-point kernel), for the reference's YOLOv8 s / l graphs and the MS-Block / HKS graphs
    (ms-s, ms-l: every depthwise k = 3/5/7/9 layer too).  These are the bench's exact shapes:
    256-row tiles, split-K wgrad slab counts, the depthwise strip walks and wide wgrad reductions,
    32-bit offsets."""
    import ctypes

    from hiputil import nhwc, pack, shape
    from yms import _lib as L
    from yms import runner
    from yms.plan import DWConvOp
    m = YOLOv8(version, 80)
    m.train()
    plan = runner.get_plan(m, [torch.empty(64, 3, 640, 640, device="meta")], torch.bfloat16, True)
    seen = set()
    g = torch.Generator(device=DEV).manual_seed(31)
    dt = torch.bfloat16
    n_dw = 0
    for op in plan.ops:
        if isinstance(op, DWConvOp):
            d = op.dshape
            key = (d.n, d.h, d.w, d.c, d.k)
            if key not in seen:
                seen.add(key)
                n_dw += 1
                _dw_layer_vs_fp32(key, g, dt)
                torch.cuda.empty_cache()
            continue
        sh = getattr(op, "shape", None)
        if sh is None:
            continue
        key = (sh.n, sh.h, sh.w, sh.cin, sh.cout, sh.k, sh.stride)
        if key in seen:
            continue
        seen.add(key)
        n, h, w, cin, cout, k, s = key
        x = torch.randn(n, cin, h, w, device=DEV, generator=g).to(dt)
        wt = (torch.randn(cout, cin, k, k, device=DEV, generator=g) / (cin * k * k) ** 0.5).to(dt)
        shp = shape(n, h, w, cin, cout, k, s, dt)
        sp = ctypes.pointer(shp)
        xb = nhwc(x.float(), dt)
        # forward (+ BN partial statistics)
        wp = pack(wt.float(), shp, dt, 0)
        y = torch.zeros((n, shp.ho, shp.wo, (cout + 7) // 8 * 8), dtype=dt, device=DEV)
        rows, ld = L.lib().yms_conv_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
        buf = torch.full((rows * (2 * ld + 1),), float("nan"), dtype=torch.float32, device=DEV)
        st, cnt = buf[:rows * 2 * ld].view(rows, 2, ld), buf[rows * 2 * ld:]
        L.call("yms_conv_fwd", sp, xb.data_ptr(), xb.shape[-1], 0, wp.data_ptr(), y.data_ptr(), y.shape[-1], 0,
               None, None, 0, None, 0, 0, buf.data_ptr(), L.stream_ptr())
        z = _gemm_conv(x.float(), wt.float(), s)
        zs = z.abs().max().item()
        yz = y[..., :cout].permute(0, 3, 1, 2).float()
        err = (yz - z).abs().max().item()
        assert err <= BF16_MAX_GATE * zs, (key, "fwd", err, zs)
        assert _rel_dev(yz, z) <= BF16_L2_GATE, (key, "fwd L2", _rel_dev(yz, z))
        del yz
        # rows of (sum z, sum (z - row mean)^2) over cnt[r] pixels, merged (Chan) in fp64
        npx = n * shp.ho * shp.wo
        nr = cnt.double().view(-1, 1)
        assert nr.sum().item() == npx and (nr > 0).all() and torch.isfinite(st[:, :, :cout]).all(), key
        r1, r2 = st[:, 0, :cout].double(), st[:, 1, :cout].double()
        s1 = r1.sum(0)
        s2 = (r2 + nr * (r1 / nr - s1 / npx) ** 2).sum(0)
        zd = z.double()
        assert _rel(s1.cpu(), zd.sum((0, 2, 3)).cpu()) < 1e-3, (key, "sum")
        assert _rel(s2.cpu(), ((zd - zd.mean((0, 2, 3), keepdim=True)) ** 2).sum((0, 2, 3)).cpu()) < 1e-3, (key, "M2")
        del z, zd
        # dgrad / wgrad
        dz = torch.randn(n, cout, shp.ho, shp.wo, device=DEV, generator=g).to(dt)
        ref_dx, ref_dw = _gemm_conv_bwd(x.float(), wt.float(), dz.float(), s)
        dzb = nhwc(dz.float(), dt)
        if cin > 3:
            wpt = pack(wt.float(), shp, dt, 1)
            dx = torch.zeros((n, h, w, (cin + 7) // 8 * 8), dtype=dt, device=DEV)
            L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(),
                   dx.shape[-1], 0, 0, L.stream_ptr())
            dxz = dx[..., :cin].permute(0, 3, 1, 2).float()
            err = (dxz - ref_dx).abs().max().item()
            assert err <= BF16_MAX_GATE * ref_dx.abs().max().item(), (key, "dgrad", err)
            assert _rel_dev(dxz, ref_dx) <= BF16_L2_GATE, (key, "dgrad L2", _rel_dev(dxz, ref_dx))
            del dxz
            del dx
        wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=DEV)
        dw = torch.zeros(cout, cin, k, k, device=DEV)
        L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0,
               ws.data_ptr(), wsb, dw.data_ptr(), 0, L.stream_ptr())
        err = (dw - ref_dw).abs().max().item()
        assert err <= 2e-3 * ref_dw.abs().max().item(), (key, "wgrad", err)
        assert _rel_dev(dw, ref_dw) <= FP32_OUT_L2_GATE, (key, "wgrad L2", _rel_dev(dw, ref_dw))
        del x, wt, xb, y, st, dz, dzb, ws, dw, ref_dx, ref_dw
        torch.cuda.empty_cache()
    assert len(seen) >= 20
    if version.startswith("ms-"):
        assert n_dw >= 4 and {op.dshape.k for op in plan.ops if isinstance(op, DWConvOp)} == {3, 5, 7, 9}
    else:
        assert n_dw == 0
