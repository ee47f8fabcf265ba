"""GPU parity of the direct small-channel 3x3 convolution (csrc/conv_direct.hip) -- the path
yms_conv_fwd / yms_conv_dgrad take for 16-bit 3x3 stride-1 convs with 32 / 64 reduction channels
and <= 64 output channels (components.py:69-93 Bottleneck convs of the 160^2 / 80^2 C2f stages, the
80^2 head branches) -- against fp32 PyTorch on the same dtype-rounded operands, and against the
implicit-GEMM path of the same op (yms_conv_direct_set(0)).  Covers both tile widths (TW 32 / 16), both
reduction widths, one and two output fragments, ragged map heights, padded input channels, channel
slices of wider buffers, every epilogue (BN+SiLU+residual, statistics, store, accumulate)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from hiputil import DT, check_moments, conv_fwd, nchw, nhwc, pack, r8, ref_conv, shape
from yms import _lib as L

pytestmark = pytest.mark.gpu

# (n, cin, h, w, cout): tile width 32 (w % 32 == 0) / 16, ragged heights (h % tile rows != 0),
# cin padded to 32 (30), cout 40 (second fragment partly valid), 8 and 24 output channels
SHAPES = [
    (2, 32, 16, 32, 32),
    (1, 64, 20, 32, 64),
    (3, 64, 16, 16, 64),
    (2, 32, 23, 48, 64),
    (2, 64, 9, 32, 32),
    (2, 30, 11, 64, 40),
    (1, 64, 37, 16, 8),
    (2, 32, 8, 96, 24),
]
TOL = {"bf16": 1e-2, "f16": 2e-3}


def _close(got, ref, tol):
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"max err {err:.3g} vs scale {scale:.3g} (tol {tol})"


def _direct_rows(sh):
    """yms_conv_stats_rows of the direct kernel (one row per persistent block) vs the NT kernels'."""
    return L.lib().yms_conv_stats_rows(ctypes.pointer(sh))


@pytest.fixture
def direct_switch():
    """yms_conv_direct_set(on) for the test, the process' setting restored after it."""
    prev = L.lib().yms_conv_direct_set(-1)
    yield lambda on: L.lib().yms_conv_direct_set(int(on))
    L.lib().yms_conv_direct_set(prev)


def test_direct_route_taken(direct_switch):
    """The direct kernel's statistics rows are one per persistent block (<= ntiles); the route
    switched off (yms_conv_direct_set(0), YMS_DIRECT=0 at start-up) restores the NT kernels' row
    count (one per block and 128-row half of its tiles)."""
    sh = shape(64, 80, 80, 64, 64, 3, 1, torch.bfloat16)
    ntiles = 64 * (80 // 16) * (80 // 16)
    rows = _direct_rows(sh)
    assert 1 <= rows <= ntiles
    direct_switch(0)
    assert _direct_rows(sh) != rows
    direct_switch(1)
    assert _direct_rows(shape(64, 80, 80, 128, 64, 3, 1, torch.bfloat16)) != rows   # 128-ch reduction: NT


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("shp", SHAPES)
def test_direct_fwd_affine_silu_residual(shp, dt):
    n, cin, h, w, cout = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(sum(shp))
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sf = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, cout, h, w, generator=g)
    sh = shape(n, h, w, cin, cout, 3, 1, dtype)
    z = ref_conv(x, wt, 1, dtype)
    act = F.silu(z * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1))
    y, _ = conv_fwd(nhwc(x, dtype), wt, sh, dtype, sc.cuda(), sf.cuda(), L.ACT_SILU, nhwc(res, dtype))
    _close(nchw(y, cout).cpu(), act + res.to(dtype).float(), TOL[dt])
    if r8(cout) != cout or y.shape[-1] > cout:
        assert y[..., cout:].abs().max().item() == 0        # channels past cout untouched
    y2, _ = conv_fwd(nhwc(x, dtype), wt, sh, dtype, sc.cuda(), sf.cuda(), L.ACT_SILU)   # no residual
    _close(nchw(y2, cout).cpu(), act, TOL[dt])


@pytest.mark.parametrize("shp", SHAPES)
def test_direct_fwd_stats(shp):
    n, cin, h, w, cout = shp
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(7 + sum(shp))
    x = torch.randn(n, cin, h, w, generator=g) + 0.5      # non-zero mean: centred moments matter
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    sh = shape(n, h, w, cin, cout, 3, 1, dtype)
    y, st = conv_fwd(nhwc(x, dtype), wt, sh, dtype, stats=True)
    z = ref_conv(x, wt, 1, dtype)
    _close(nchw(y, cout).cpu(), z, TOL["bf16"])
    check_moments(st, z, 1e-3)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("shp", SHAPES)
def test_direct_dgrad_store_and_accumulate(shp, dt):
    """Input gradient: reduction over cout (the direct kernel takes cout in {32, 64} rounded to 8,
    cin <= 64): shapes are read as (n, cout_of_dgrad=cin, h, w, reduction=cout) swapped."""
    n, cred, h, w, cin = shp          # dgrad: reduction channels = conv cout = cred, outputs = cin
    dtype = DT[dt]
    g = torch.Generator().manual_seed(11 + sum(shp))
    wt = torch.randn(cred, cin, 3, 3, generator=g) / (cred * 9) ** 0.5
    dz = torch.randn(n, cred, h, w, generator=g)
    sh = shape(n, h, w, cin, cred, 3, 1, dtype)
    sp = ctypes.pointer(sh)
    xr = torch.zeros(n, cin, h, w, requires_grad=True)
    F.conv2d(xr, wt.to(dtype).float(), None, 1, 1).backward(dz.to(dtype).float())
    wpt = pack(wt, sh, dtype, 1)
    dzb = nhwc(dz, dtype)
    dx = nhwc(torch.zeros(n, cin, h, w), dtype)
    L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
           0, L.stream_ptr())
    _close(nchw(dx, cin).cpu(), xr.grad, TOL[dt])
    base = torch.randn(n, cin, h, w, generator=g)
    dx = nhwc(base, dtype)
    L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
           1, L.stream_ptr())
    _close(nchw(dx, cin).cpu(), xr.grad + base.to(dtype).float(), 2 * TOL[dt])


def test_direct_channel_slices():
    """Input read from / output written to / residual read from channel slices of wider buffers
    (the C2f / concat placement of plan.py)."""
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(3)
    n, cin, h, w, cout = 2, 64, 13, 32, 32
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / 24
    res = torch.randn(n, cout, h, w, generator=g)
    sh = shape(n, h, w, cin, cout, 3, 1, dtype)
    sp = ctypes.pointer(sh)
    xb = nhwc(x, dtype, ld=128, off=32)
    rb = nhwc(res, dtype, ld=96, off=64)
    y = torch.zeros(n, h, w, 80, dtype=dtype, device="cuda")
    wp = pack(wt, sh, dtype, 0)
    sc, sf = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
    L.call("yms_conv_fwd", sp, xb.data_ptr(), 128, 32, wp.data_ptr(), y.data_ptr(), 80, 40, sc.data_ptr(),
           sf.data_ptr(), 0, rb.data_ptr(), 96, 64, None, L.stream_ptr())
    ref = ref_conv(x, wt, 1, dtype).to(dtype).float() + res.to(dtype).float()
    _close(nchw(y, cout, off=40).cpu(), ref, 1e-2)
    assert y[..., :40].abs().max().item() == 0 and y[..., 72:].abs().max().item() == 0


@pytest.mark.parametrize("shp", [(64, 64, 80, 80, 64), (64, 32, 160, 160, 32), (8, 32, 320, 320, 32)])
def test_direct_matches_implicit_gemm_bench_shapes(shp, direct_switch):
    """Bench-scale layers (B=64 S@640 stages; the S@1280 320^2 stage): forward with statistics and
    input gradient of the direct kernel against the implicit-GEMM kernels (route off) on the same
    operands -- both fp32-accumulated MFMA sums of the same products, so they agree to the bf16
    rounding of the output."""
    n, cin, h, w, cout = shp
    dtype = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(5)
    xb = torch.randn(n, h, w, cin, device="cuda", generator=g).to(dtype)
    wt = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) / (cin * 9) ** 0.5
    dz = torch.randn(n, h, w, cout, device="cuda", generator=g).to(dtype)
    sh = shape(n, h, w, cin, cout, 3, 1, dtype)
    sp = ctypes.pointer(sh)
    wp, wpt = pack(wt, sh, dtype, 0), pack(wt, sh, dtype, 1)
    outs = {}
    for mode in ("1", "0"):
        direct_switch(int(mode))
        rows, ld = L.lib().yms_conv_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
        stt = torch.full((rows * (2 * ld + 1),), float("nan"), device="cuda")
        y = torch.empty(n, h, w, cout, dtype=dtype, device="cuda")
        L.call("yms_conv_fwd", sp, xb.data_ptr(), cin, 0, wp.data_ptr(), y.data_ptr(), cout, 0, None, None, 0,
               None, 0, 0, stt.data_ptr(), L.stream_ptr())
        dx = torch.empty(n, h, w, cin, dtype=dtype, device="cuda")
        L.call("yms_conv_dgrad", sp, dz.data_ptr(), cout, 0, wpt.data_ptr(), dx.data_ptr(), cin, 0, 0,
               L.stream_ptr())
        cnt = stt[rows * 2 * ld:]
        mom = stt[:rows * 2 * ld].view(rows, 2, ld)[:, :, :cout].double()
        nn = cnt.double().view(-1, 1)
        mean = mom[:, 0].sum(0) / nn.sum()
        m2 = (mom[:, 1] + nn * (mom[:, 0] / nn - mean) ** 2).sum(0)
        assert nn.sum().item() == n * h * w
        outs[mode] = (y.float(), dx.float(), mean, m2)
    (y1, d1, m1, v1), (y0, d0, m0, v0) = outs["1"], outs["0"]
    for a, b in ((y1, y0), (d1, d0)):
        err = (a - b).abs().max().item()
        assert err <= 8e-3 * b.abs().max().item(), err
    assert torch.allclose(m1, m0, rtol=1e-5, atol=1e-6 * m0.abs().max().item())
    assert torch.allclose(v1, v0, rtol=1e-4)


# stride-2 input gradient by parity class: (n, cin = dgrad outputs, h, w, cout = reduction); class
# grids ceil(w/2) of 32 / 16, odd h / w (the last class row / column masked), cin of 8..64
S2 = [
    (2, 32, 64, 64, 64),
    (1, 32, 40, 64, 64),
    (2, 16, 32, 32, 32),
    (2, 64, 30, 64, 64),
    (1, 24, 33, 63, 64),
    (3, 8, 18, 31, 32),
]


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("shp", S2)
def test_direct_dgrad_stride2(shp, dt):
    n, cin, h, w, cout = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(13 + sum(shp))
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (cout * 9) ** 0.5
    sh = shape(n, h, w, cin, cout, 3, 2, dtype)
    dz = torch.randn(n, cout, sh.ho, sh.wo, generator=g)
    sp = ctypes.pointer(sh)
    xr = torch.zeros(n, cin, h, w, requires_grad=True)
    F.conv2d(xr, wt.to(dtype).float(), None, 2, 1).backward(dz.to(dtype).float())
    wpt = pack(wt, sh, dtype, 1)
    dzb = nhwc(dz, dtype)
    for acc in (0, 1):
        base = torch.randn(n, cin, h, w, generator=g) if acc else torch.zeros(n, cin, h, w)
        dx = nhwc(base, dtype, ld=r8(cin) + 8)           # a wider buffer: channel slice of it
        L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(),
               dx.shape[-1], 0, acc, L.stream_ptr())
        exp = xr.grad + (base.to(dtype).float() if acc else 0)
        _close(nchw(dx, cin).cpu(), exp, TOL[dt] * (2 if acc else 1))
        assert dx[..., r8(cin):].abs().max().item() == 0


def test_direct_dgrad_stride2_bench_shape(direct_switch):
    """The 320^2 32->64 stride-2 layer of the S@640 backbone: direct kernel vs the implicit GEMM's
    parity-class path (route off) on the same operands."""
    n, cin, h, w, cout = 16, 32, 320, 320, 64
    dtype = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(6)
    wt = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) / (cout * 9) ** 0.5
    sh = shape(n, h, w, cin, cout, 3, 2, dtype)
    dz = torch.randn(n, sh.ho, sh.wo, cout, device="cuda", generator=g).to(dtype)
    sp = ctypes.pointer(sh)
    wpt = pack(wt, sh, dtype, 1)
    outs = []
    for mode in ("1", "0"):
        direct_switch(int(mode))
        dx = torch.empty(n, h, w, cin, dtype=dtype, device="cuda")
        L.call("yms_conv_dgrad", sp, dz.data_ptr(), cout, 0, wpt.data_ptr(), dx.data_ptr(), cin, 0, 0,
               L.stream_ptr())
        outs.append(dx.float())
    err = (outs[0] - outs[1]).abs().max().item()
    assert err <= 8e-3 * outs[1].abs().max().item(), err
