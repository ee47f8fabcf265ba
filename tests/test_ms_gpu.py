"""GPU parity of the YOLO-MS family (MS-Block with depthwise k x k IB_k, HKS backbone k = 3/5/7/9;
yolov8/model/yolo_ms.py) against the build's CPU restatement oracle/ms_ref.py.  NOT
reference-pinned: the reference holds no MS-Block code (annotations.md:66-133 is a diagram), so
the oracle is the SURVEY 7.4 structure written independently of the product modules."""
import pytest
import torch

from oracle import ms_ref as MS
from yolov8.model.yolo_ms import MSBlock
from yolov8.yolov8 import YOLOv8

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(got, ref):
    got = torch.as_tensor(got).double().cpu()
    ref = torch.as_tensor(ref).double()
    return ((got - ref).norm() / (ref.norm() + 1e-12)).item()


def _maxerr(got, ref):
    got = torch.as_tensor(got).float().cpu()
    ref = torch.as_tensor(ref).float()
    return ((got - ref).abs().max() / (ref.abs().max() + 1e-12)).item()


def _model(v, nc, sd):
    m = YOLOv8(v, nc).to(DEV)
    m.load_state_dict(sd)
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    return m


def _grads(v, nc, sd, x, dtype):
    p = {k: (t.clone().to(dtype).requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else (t.clone().to(dtype) if t.is_floating_point() else t.clone()))
         for k, t in sd.items()}
    r = MS.forward(p, v, nc, x.to(dtype), True)
    sum((o.double() ** 2).mean() for o in r).backward()
    return p, r


def _quantiles(errs, qs=(0.5, 0.9, 1.0)):
    t = torch.tensor(sorted(errs), dtype=torch.float64)
    return [torch.quantile(t, q).item() for q in qs]


def test_msblock_module_hks9_fp32_and_bf16():
    """One MS-Block with the largest HKS kernel (k = 9, two IB layers per branch) as a standalone
    module (well conditioned: 1920 pixels per BN): forward, input and parameter gradients in fp32
    against the fp32 oracle (1e-4, parameters 3e-4), and in bf16 within 2x (+1e-3) of the CPU
    bf16 autocast drift of the same block."""
    torch.manual_seed(0)
    blk = MSBlock(64, 64, kernel_size=9, layers=2)
    sd = {("blk." + k): t for k, t in blk.state_dict().items()}
    gen = MS.init_params("ms-xs", 80)           # reuse the closed-form initializer's per-key rule
    from oracle import model_ref as M
    for k, t in list(sd.items()):
        if k.endswith("num_batches_tracked"):
            continue
        if k.endswith("conv.weight"):
            sd[k] = M._closed_form(k, tuple(t.shape), (3.0 / (t.shape[1] * t.shape[2] * t.shape[3])) ** 0.5 * 1.2)
        elif k.endswith("bn.weight"):
            sd[k] = M._closed_form(k, tuple(t.shape), 0.25, base=1.0)
        elif k.endswith("running_var"):
            sd[k] = M._closed_form(k, tuple(t.shape), 0.3, base=1.2)
        else:
            sd[k] = M._closed_form(k, tuple(t.shape), 0.1)
    del gen
    blk.load_state_dict({k[4:]: v for k, v in sd.items()})
    blk = blk.to(DEV).train()
    x = torch.randn(2, 64, 24, 40, generator=torch.Generator().manual_seed(3))
    cot = torch.randn(2, 64, 24, 40, generator=torch.Generator().manual_seed(4))
    pr = {k: (t.clone().requires_grad_(True) if t.is_floating_point() and "running" not in k else t.clone())
          for k, t in sd.items()}
    xr = x.clone().requires_grad_(True)
    yr = MS.msblock(pr, "blk", xr, 9, 2, True)
    (yr * cot).sum().backward()
    # CPU bf16 autocast drift of the same block: the yardstick for the bf16 path
    pc = {k: (t.clone().requires_grad_(True) if t.is_floating_point() and "running" not in k else t.clone())
          for k, t in sd.items()}
    xc = x.clone().requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        yc = MS.msblock(pc, "blk", xc, 9, 2, True)
    (yc.float() * cot).sum().backward()
    pkeys = [k for k, t in pr.items() if t.grad is not None]
    cpu_bf = [_rel(yc.detach().float(), yr.detach()), _rel(xc.grad, xr.grad)]
    cpu_bf_p = _quantiles([_rel(pc[k].grad, pr[k].grad) for k in pkeys], (0.5, 1.0))
    for dt in (torch.float32, torch.bfloat16):
        blk.zero_grad(set_to_none=True)
        xg = x.to(DEV).requires_grad_(True)
        if dt == torch.float32:
            y = blk(xg)
        else:
            with torch.autocast("cuda", dtype=dt):
                y = blk(xg)
        (y.float() * cot.to(DEV)).sum().backward()
        pd = dict(blk.named_parameters())
        ey, ex = _rel(y.detach().float(), yr.detach()), _rel(xg.grad, xr.grad)
        ep = [_rel(pd[k[4:]].grad, pr[k].grad) for k in pkeys]
        if dt == torch.float32:
            assert ey < 1e-4 and ex < 1e-4, (ey, ex)
            assert max(ep) < 3e-4, max(ep)
        else:
            assert ey <= 2 * cpu_bf[0] + 1e-3 and ex <= 2 * cpu_bf[1] + 1e-3, (ey, ex, cpu_bf)
            for a, b in zip(_quantiles(ep, (0.5, 1.0)), cpu_bf_p):
                assert a <= 2 * b + 1e-3, (a, b)


def _calibrated(v, nc, size):
    return MS.calibrate(MS.init_params(v, nc), v, nc,
                        torch.randn(1, 3, size, size, generator=torch.Generator().manual_seed(5)))


def test_ms_s640_bf16_eval_vs_cpu_bf16_drift():
    """YOLO-MS-S (HKS) 640x640 bf16 inference (running statistics calibrated on another 640x640
    input): class-probability error quantiles and box drift within 1.3x of the same graph's CPU
    bf16 autocast path."""
    v, nc = "ms-s", 80
    sd = _calibrated(v, nc, 640)
    x = torch.randn(1, 3, 640, 640, generator=torch.Generator().manual_seed(8))
    m = _model(v, nc, sd).eval()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(DEV)).cpu()
    with torch.no_grad():
        ref = MS.forward(dict(sd), v, nc, x, False)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            cpu_bf = MS.forward(dict(sd), v, nc, x, False).float()
    assert torch.isfinite(y).all()
    ours = (y[..., 4:] - ref[..., 4:]).abs().flatten()
    cpu = (cpu_bf[..., 4:] - ref[..., 4:]).abs().flatten()
    for q in (0.5, 0.9, 0.99):
        a, b = torch.quantile(ours, q).item(), torch.quantile(cpu, q).item()
        assert a <= 1.3 * b + 1e-4, (q, a, b)
    assert _rel(y[..., :4], ref[..., :4]) <= 1.3 * _rel(cpu_bf[..., :4], ref[..., :4]) + 1e-4


@pytest.mark.parametrize("v", ["ms-l", "ms-s"])
def test_ms_640_fp32_eval_vs_oracle(v):
    """configs[3]'s large-kernel graph (YOLO-MS-L: HKS 3/5/7/9, 3 IB layers per branch) and MS-S at
    640x640 in fp32, running statistics calibrated on another 640x640 input.  Even so ms-l at
    random init is chaotic (CPU fp32 vs fp64: class error median ~2.5e-2), so: class error
    quantiles (median, p99) and box drift vs the fp64 oracle within 2x of the CPU fp32 oracle's."""
    nc = 80
    sd = _calibrated(v, nc, 640)
    x = torch.randn(1, 3, 640, 640, generator=torch.Generator().manual_seed(9))
    m = _model(v, nc, sd).eval()
    y = m(x.to(DEV)).cpu().double()
    with torch.no_grad():
        r32 = MS.forward(dict(sd), v, nc, x, False).double()
        r64 = MS.forward({k: (t.double() if t.is_floating_point() else t) for k, t in sd.items()}, v, nc,
                         x.double(), False)
    assert y.shape == r64.shape and torch.isfinite(y).all()
    ours = (y[..., 4:] - r64[..., 4:]).abs().flatten()
    cpu = (r32[..., 4:] - r64[..., 4:]).abs().flatten()
    for q in (0.5, 0.99):
        a, b = torch.quantile(ours, q).item(), torch.quantile(cpu, q).item()
        assert a <= 2 * b + 1e-5, (q, a, b)
    assert _rel(y[..., :4], r64[..., :4]) <= 2 * _rel(r32[..., :4], r64[..., :4]) + 1e-6
