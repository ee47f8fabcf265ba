"""Stem convolution (yms_conv_stem_fwd: NCHW fp32 input -> NHWC, 3x3 stride 2, cin <= 3) against
torch fp32 on the dtype-rounded operands, and the model with the stem path against the generic
pack + implicit-GEMM path (YMS_STEM=0).  Reference layer: yolov8/model/yolov8_backbone.py:30-40
(Conv(in_channels, int(64*w), 3, 2, 1) -> BN -> SiLU, components.py:69-77)."""
import ctypes
import os
import sys

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(__file__))
from hiputil import DT, r8, shape  # noqa: E402
from yms import _lib as L  # noqa: E402

pytestmark = pytest.mark.gpu


def _ref(x, w, dt):
    """conv of the dtype-rounded operands in fp32 (the kernel's products are exact)."""
    xr = x.to(DT[dt]).float()
    wr = w.to(DT[dt]).float()
    return F.conv2d(xr, wr, stride=2, padding=1)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 64, 64, 3, 32), (3, 37, 70, 3, 48), (1, 130, 66, 2, 16),
                                            (2, 40, 40, 1, 80), (1, 17, 9, 3, 96), (2, 48, 64, 3, 24)])
def test_stem_eval_affine_silu(dt, n, h, w, cin, cout):
    g = torch.Generator().manual_seed(n * 1000 + h + cout)
    x = torch.randn(n, cin, h, w, generator=g) * 2.0
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.3
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.2
    sh_ = shape(n, h, w, cin, cout, 3, 2, DT[dt])
    sp = ctypes.pointer(sh_)
    assert L.lib().yms_conv_stem_supported(sp) == 1
    ld = r8(cout) + 8                     # a wider buffer: the output is a channel slot (off 8)
    y = torch.full((n, sh_.ho, sh_.wo, ld), float("nan"), dtype=DT[dt], device="cuda")
    xd, wd = x.cuda(), wt.cuda()
    scd, shd = sc.cuda(), sh.cuda()
    L.call("yms_conv_stem_fwd", sp, xd.data_ptr(), wd.data_ptr(), y.data_ptr(), ld, 8, scd.data_ptr(),
           shd.data_ptr(), L.ACT_SILU, None, 0, L.stream_ptr())
    torch.cuda.synchronize()
    ref = F.silu(_ref(x, wt, dt) * sc[:, None, None] + sh[:, None, None])
    out = y[..., 8:8 + cout].permute(0, 3, 1, 2).float().cpu()
    assert torch.isnan(y[..., :8].float()).all()          # channels outside the slot untouched
    tol = 8e-3 if dt == "bf16" else 1e-3
    err = (out - ref).abs().max().item()
    assert err <= tol * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("n,h,w,cout", [(2, 64, 64, 32), (3, 45, 77, 48), (2, 48, 64, 24), (2, 40, 40, 56)])
def test_stem_training_z_and_statistics(n, h, w, cout):
    dt = "bf16"
    g = torch.Generator().manual_seed(h * w + cout)
    x = torch.randn(n, 3, h, w, generator=g) + 3.0      # |mean| >> std: centred moments matter
    wt = torch.randn(cout, 3, 3, 3, generator=g) * 0.3
    sh_ = shape(n, h, w, 3, cout, 3, 2, DT[dt])
    sp = ctypes.pointer(sh_)
    rows = L.lib().yms_conv_stem_stats_rows(sp)
    ld_s = L.lib().yms_conv_stats_ld(sp)
    assert rows == n * ((sh_.ho + 7) // 8) * ((sh_.wo + 31) // 32)
    stats = torch.full((rows * (2 * ld_s + 1),), float("nan"), device="cuda")
    z = torch.empty((n, sh_.ho, sh_.wo, r8(cout)), dtype=DT[dt], device="cuda")
    xd, wd = x.cuda(), wt.cuda()
    L.call("yms_conv_stem_fwd", sp, xd.data_ptr(), wd.data_ptr(), z.data_ptr(), r8(cout), 0, None, None,
           L.ACT_NONE, stats.data_ptr(), ld_s, L.stream_ptr())
    npix = n * sh_.ho * sh_.wo
    gam, bet = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
    rm, rv = torch.zeros(cout, device="cuda"), torch.ones(cout, device="cuda")
    mi = torch.empty(2 * cout, device="cuda")
    sc, sf = torch.empty(cout, device="cuda"), torch.empty(cout, device="cuda")
    L.call("yms_bn_finalize", cout, stats.data_ptr(), rows, ld_s, npix, gam.data_ptr(), bet.data_ptr(),
           rm.data_ptr(), rv.data_ptr(), ctypes.c_float(0.03), ctypes.c_float(1e-3), mi.data_ptr(),
           sc.data_ptr(), sf.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    ref = _ref(x, wt, dt).double()
    zz = z[..., :cout].permute(0, 3, 1, 2).double().cpu()
    assert (zz - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    # statistics are of the fp32 accumulators (as the implicit-GEMM epilogue's)
    mean = ref.mean((0, 2, 3))
    var = ref.var((0, 2, 3), unbiased=False)
    assert torch.allclose(mi[:cout].double().cpu(), mean, rtol=1e-5, atol=1e-4 * mean.abs().max().item())
    istd = 1.0 / (var + 1e-3).sqrt()
    assert torch.allclose(mi[cout:].double().cpu(), istd, rtol=2e-4)
    cnt = stats[rows * 2 * ld_s:].cpu()
    assert cnt.sum().item() == npix


def test_stem_rejects_unsupported():
    sp = ctypes.pointer(shape(2, 64, 64, 4, 32, 3, 2, torch.bfloat16))      # cin 4
    assert L.lib().yms_conv_stem_supported(sp) == 0
    sp = ctypes.pointer(shape(2, 64, 64, 3, 32, 3, 1, torch.bfloat16))      # stride 1
    assert L.lib().yms_conv_stem_supported(sp) == 0
    sp = ctypes.pointer(shape(2, 64, 64, 3, 32, 3, 2, torch.float32))       # fp32: generic path
    assert L.lib().yms_conv_stem_supported(sp) == 0
    x = torch.zeros(1, device="cuda")
    assert L.lib().yms_conv_stem_fwd(sp, x.data_ptr(), x.data_ptr(), x.data_ptr(), 32, 0, None, None, 0, None, 0,
                                     None) != 0


@pytest.mark.parametrize("v,training", [("n", False), ("s", True), ("ms-xs", True)])
def test_model_stem_path_matches_generic_path(v, training, monkeypatch):
    from yms import set_compute_dtype
    from yolov8.yolov8 import YOLOv8

    from oracle import model_ref as M
    from oracle import ms_ref

    # the well-conditioned fixture: at the default random init the graphs are chaotic enough
    # (ms-xs bf16 output drift ~0.4 on the CPU alone) that the stem's fp32 statistics summation
    # order (1e-7 relative in the batch mean) flips a few bf16 roundings and grows to 0.2 at the head
    sd = M.ordered_init((ms_ref if v.startswith("ms") else M).init_params(v, 80))
    torch.manual_seed(0)
    x = torch.randn(2, 3, 96, 128, device="cuda")
    outs = {}
    for stem in ("1", "0"):
        monkeypatch.setenv("YMS_STEM", stem)
        m = YOLOv8(v, 80)
        m.load_state_dict(sd)
        m = m.cuda()
        set_compute_dtype(m, torch.bfloat16)
        m.train(training)
        if not training:
            m.head.stride = torch.tensor([8.0, 16.0, 32.0])
            outs[stem] = (m(x).float(),)
        else:
            o = m(x)
            sum((t.float() ** 2).mean() for t in o).backward()
            outs[stem] = tuple(t.float() for t in o) + (m.backbone.conv0.conv.weight.grad.clone(),)
        plans = list(m.__dict__["_yms_plans"].values())
        assert sum(len(p.stem_inputs) for p in plans) == (1 if stem == "1" else 0)
    for a, b in zip(outs["1"], outs["0"]):
        err = ((a - b).norm() / b.norm()).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("n,h,w,cout", [(2, 64, 64, 32), (3, 45, 78, 48), (1, 33, 20, 16), (2, 48, 64, 24),
                                       (2, 40, 40, 56)])
def test_stem_wgrad_with_fused_bn_backward(dt, n, h, w, cout):
    """yms_conv_stem_wgrad = BN+SiLU backward apply (bn_bwd_apply_kernel's dz, rounded to the
    dtype) followed by the conv weight gradient against the NCHW input, vs fp64 torch."""
    g = torch.Generator().manual_seed(n * 7 + h + cout)
    x = torch.randn(n, 3, h, w, generator=g)
    sh_ = shape(n, h, w, 3, cout, 3, 2, DT[dt])
    sp = ctypes.pointer(sh_)
    ho, wo = sh_.ho, sh_.wo
    z = torch.randn(n, ho, wo, cout, generator=g).to(DT[dt])
    gy = (torch.randn(n, ho, wo, cout, generator=g) * 0.1).to(DT[dt])
    sc = torch.rand(cout, generator=g) + 0.5
    sf = torch.randn(cout, generator=g) * 0.2
    mu = torch.randn(cout, generator=g) * 0.1
    istd = torch.rand(cout, generator=g) + 0.5
    coef = torch.randn(2 * cout, generator=g) * 0.05
    # reference dz exactly as bn_bwd_apply_kernel forms it (fp32), rounded to the dtype
    zf, gf = z.float(), gy.float()
    a = zf * sc + sf
    s_ = torch.sigmoid(a)
    da = gf * (s_ * (1 + a * (1 - s_)))
    bz = -sc * coef[cout:] * istd
    a0 = -sc * coef[:cout] - bz * mu
    dz = (sc * da + a0 + bz * zf).to(DT[dt]).double()                   # [n, ho, wo, cout]
    xr = x.to(DT[dt]).double()
    ref = torch.nn.grad.conv2d_weight(xr, (cout, 3, 3, 3), dz.permute(0, 3, 1, 2), stride=2, padding=1)
    ws = torch.empty(L.lib().yms_conv_stem_wgrad_ws_bytes(sp) // 4 + 1, device="cuda")
    dw = torch.full((cout, 3, 3, 3), float("nan"), device="cuda")
    xd, zd, gd = x.cuda(), z.cuda(), gy.cuda()
    mi = torch.cat([mu, istd]).cuda()
    scd, sfd, cd = sc.cuda(), sf.cuda(), coef.cuda()
    L.call("yms_conv_stem_wgrad", sp, xd.data_ptr(), gd.data_ptr(), cout, 0, zd.data_ptr(), cout, 0, scd.data_ptr(),
           sfd.data_ptr(), mi.data_ptr(), cd.data_ptr(), L.ACT_SILU, ws.data_ptr(), ws.numel() * 4, dw.data_ptr(), 0,
           L.stream_ptr())
    torch.cuda.synchronize()
    out = dw.double().cpu()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 2e-3, rel


def test_stem_b64_640_fwd_stats_and_wgrad():
    """The bench's stem: 64 x 3 x 640 x 640 fp32 input -> 32 channels at 320^2 (configs[2]), in bf16.
    Forward z and its BN statistics (25,600 partial rows) vs an fp32 im2col GEMM on the GPU, and the
    weight gradient with the fused BN+SiLU backward apply vs an fp32 GEMM over the same dz."""
    import torch.nn.functional as F
    from hiputil import check_moments, split_stats, stats_buffer
    n, h, w, cout, dt = 64, 640, 640, 32, torch.bfloat16
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(64)
    x = torch.randn(n, 3, h, w, device=dev, generator=g)
    wt = torch.randn(cout, 3, 3, 3, device=dev, generator=g) * 0.3
    sh_ = shape(n, h, w, 3, cout, 3, 2, dt)
    sp = ctypes.pointer(sh_)
    ho, wo = sh_.ho, sh_.wo
    rows, ld_s = L.lib().yms_conv_stem_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
    buf = stats_buffer(rows, ld_s)
    z = torch.empty((n, ho, wo, r8(cout)), dtype=dt, device=dev)
    L.call("yms_conv_stem_fwd", sp, x.data_ptr(), wt.data_ptr(), z.data_ptr(), r8(cout), 0, None, None,
           L.ACT_NONE, buf.data_ptr(), ld_s, L.stream_ptr())
    xr, wr = x.to(dt).float(), wt.to(dt).float()
    cols = F.unfold(xr, 3, padding=1, stride=2)                              # [n, 27, ho*wo]
    ref = (wr.view(cout, -1) @ cols).view(n, cout, ho, wo)
    zz = z[..., :cout].permute(0, 3, 1, 2).float()
    assert (zz - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    check_moments(split_stats(buf, rows, ld_s), ref, 1e-4)
    del buf
    # backward: dz = BN+SiLU backward apply (fp32, rounded to bf16) of (gy, z), then dW = dz^T im2col(x)
    gy = (torch.randn(n, ho, wo, cout, device=dev, generator=g) * 0.1).to(dt)
    sc = torch.rand(cout, device=dev, generator=g) + 0.5
    sf = torch.randn(cout, device=dev, generator=g) * 0.2
    mu = torch.randn(cout, device=dev, generator=g) * 0.1
    istd = torch.rand(cout, device=dev, generator=g) + 0.5
    coef = torch.randn(2 * cout, device=dev, generator=g) * 0.05
    zf, gf = z[..., :cout].float(), gy.float()
    a = zf * sc + sf
    s_ = torch.sigmoid(a)
    da = gf * (s_ * (1 + a * (1 - s_)))
    bz = -sc * coef[cout:] * istd
    a0 = -sc * coef[:cout] - bz * mu
    dz = (sc * da + a0 + bz * zf).to(dt).float()                            # [n, ho, wo, cout]
    del a, s_, da
    ref_dw = torch.einsum("nlo,nkl->ok", dz.reshape(n, ho * wo, cout), cols).view(cout, 3, 3, 3)
    del cols, dz
    ws = torch.empty(L.lib().yms_conv_stem_wgrad_ws_bytes(sp) // 4 + 1, device=dev)
    dw = torch.full((cout, 3, 3, 3), float("nan"), device=dev)
    mi = torch.cat([mu, istd])
    zc = z.contiguous()
    L.call("yms_conv_stem_wgrad", sp, x.data_ptr(), gy.data_ptr(), cout, 0, zc.data_ptr(), r8(cout), 0, sc.data_ptr(),
           sf.data_ptr(), mi.data_ptr(), coef.data_ptr(), L.ACT_SILU, ws.data_ptr(), ws.numel() * 4, dw.data_ptr(), 0,
           L.stream_ptr())
    torch.cuda.synchronize()
    rel = ((dw.double() - ref_dw.double()).norm() / ref_dw.double().norm()).item()
    assert rel < 2e-3, rel
