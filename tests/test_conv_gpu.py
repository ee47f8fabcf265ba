"""GPU parity of the implicit-GEMM convolution kernels (forward with every epilogue,
dgrad, wgrad) against fp32 PyTorch-CPU convolution on the same dtype-rounded operands."""
import ctypes
import os

import pytest
import torch
import torch.nn.functional as F

from hiputil import DT, check_moments, conv_fwd, nchw, nhwc, pack, r8, ref_conv, shape
from yms import _lib as L

pytestmark = pytest.mark.gpu

# (n, cin, h, w, cout, k, stride): stem, odd sizes, padded channels, wide outputs, 1x1
SHAPES = [
    (2, 3, 13, 10, 16, 3, 2),
    (2, 16, 9, 7, 24, 1, 1),
    (1, 64, 20, 20, 80, 3, 1),
    (2, 32, 40, 40, 64, 3, 2),
    (1, 256, 10, 10, 512, 1, 1),
    (3, 8, 17, 19, 130, 3, 1),
    (1, 1, 8, 8, 1, 3, 1),
    (2, 80, 11, 12, 80, 1, 1),
    (2, 16, 9, 7, 24, 1, 2),        # 1x1 stride 2 (odd parity classes have no taps)
    (1, 40, 15, 17, 48, 3, 2),      # odd sizes: unequal parity classes
]
# bf16/f16 outputs are rounded to 8/11 significant bits; fp32 uses the exact-f32 MFMA
TOL = {"f32": 2e-5, "bf16": 1e-2, "f16": 2e-3}


def _close(got, ref, tol):
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"max err {err:.3g} vs scale {scale:.3g} (tol {tol})"


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("shp", SHAPES)
def test_conv_fwd_affine_silu_residual(shp, dt):
    n, cin, h, w, cout, k, s = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(hash(shp) % 1000)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh_ = torch.randn(cout, generator=g) * 0.1
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    res = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    y, _ = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, sc.cuda(), sh_.cuda(), L.ACT_SILU, nhwc(res, dtype))
    z = ref_conv(x, wt, s, dtype)
    ref = F.silu(z * sc.view(1, -1, 1, 1) + sh_.view(1, -1, 1, 1)) + res.to(dtype).float()
    _close(nchw(y, cout).cpu(), ref, TOL[dt])
    # padded channels of the output buffer stay zero
    if r8(cout) != cout:
        assert y[..., cout:].abs().max().item() == 0


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("shp", SHAPES[:6])
def test_conv_fwd_stats(shp, dt):
    n, cin, h, w, cout, k, s = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    y, st = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, stats=True)
    z = ref_conv(x, wt, s, dtype)
    _close(nchw(y, cout).cpu(), z, TOL[dt])
    check_moments(st, z, 1e-4 if dt == "f32" else 1e-3)


def test_conv_fwd_channel_offsets():
    """Input read from / output written to channel slices of wider buffers (concat placement)."""
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 24, 9, 9, generator=g)
    wt = torch.randn(40, 24, 3, 3, generator=g) / 15
    xb = nhwc(x, dtype, ld=48, off=16)
    shp_ = shape(2, 9, 9, 24, 40, 3, 1, dtype)
    y, _ = conv_fwd(xb, wt, shp_, dtype, act=0, yld=64, yoff=8, xoff=16)
    ref = ref_conv(x, wt, 1, dtype)
    _close(nchw(y, 40, off=8).cpu(), ref, TOL["bf16"])
    assert y[..., :8].abs().max().item() == 0 and y[..., 48:].abs().max().item() == 0


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("shp", SHAPES)
def test_conv_dgrad_wgrad(shp, dt):
    n, cin, h, w, cout, k, s = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    xr = x.to(dtype).float().requires_grad_(True)
    wr = wt.to(dtype).float().requires_grad_(True)
    F.conv2d(xr, wr, None, s, k // 2).backward(dz.to(dtype).float())
    sp = ctypes.pointer(shp_)
    # dgrad, accumulate onto a pre-filled buffer
    base = torch.randn(n, cin, h, w, generator=g)
    dx = nhwc(base, dtype)
    wpt = pack(wt, shp_, dtype, 1)
    dzb = nhwc(dz, dtype)
    L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
           1, L.stream_ptr())
    _close(nchw(dx, cin).cpu(), xr.grad + base.to(dtype).float(), TOL[dt] * 2)
    # wgrad (fp32 result, split-K slabs)
    xb = nhwc(x, dtype)
    wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device="cuda")
    dw = torch.zeros(cout, cin, k, k, device="cuda")
    L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0, ws.data_ptr(),
           wsb, dw.data_ptr(), 0, L.stream_ptr())
    _close(dw.cpu(), wr.grad, 1e-4 if dt == "f32" else 2e-3)


def test_invalid_arguments_rejected():
    sh = shape(1, 8, 8, 8, 8, 3, 1, torch.float32)
    sh.ho = 5   # inconsistent
    st = L.lib().yms_conv_fwd(ctypes.pointer(sh), 1, 8, 0, 1, 1, 8, 0, None, None, 0, None, 0, 0, None,
                              L.stream_ptr())
    assert st == 1
    sh = shape(1, 8, 8, 8, 8, 3, 1, torch.float32)
    st = L.lib().yms_conv_fwd(ctypes.pointer(sh), 1, 12, 0, 1, 1, 8, 0, None, None, 0, None, 0, 0, None,
                              L.stream_ptr())
    assert st == 1   # ld not a multiple of 8


# full-size tiles: 256-row tiles with BN statistics per 128 rows (M not a multiple of 256),
# multi-split wgrad
BIG = [(3, 32, 40, 40, 32, 3, 1), (2, 64, 40, 40, 64, 3, 1), (2, 128, 20, 30, 128, 1, 1),
       (2, 64, 40, 40, 128, 3, 2)]


@pytest.mark.parametrize("shp", BIG)
def test_conv_bf16_large_tiles(shp):
    n, cin, h, w, cout, k, s = shp
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    y, st = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, stats=True)
    z = ref_conv(x, wt, s, dtype)
    _close(nchw(y, cout).cpu(), z, TOL["bf16"])
    check_moments(st, z, 1e-3)
    sc = torch.rand(cout, generator=g) + 0.5
    sh_ = torch.randn(cout, generator=g) * 0.1
    ya, _ = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, sc.cuda(), sh_.cuda(), L.ACT_SILU)
    _close(nchw(ya, cout).cpu(), F.silu(z * sc.view(1, -1, 1, 1) + sh_.view(1, -1, 1, 1)), TOL["bf16"])
    dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    xr = x.to(dtype).float().requires_grad_(True)
    wr = wt.to(dtype).float().requires_grad_(True)
    F.conv2d(xr, wr, None, s, k // 2).backward(dz.to(dtype).float())
    sp = ctypes.pointer(shp_)
    dx = nhwc(torch.zeros(n, cin, h, w), dtype)
    wpt = pack(wt, shp_, dtype, 1)
    dzb = nhwc(dz, dtype)
    L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
           0, L.stream_ptr())
    _close(nchw(dx, cin).cpu(), xr.grad, TOL["bf16"] * 2)
    xb = nhwc(x, dtype)
    wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device="cuda")
    dw = torch.zeros(cout, cin, k, k, device="cuda")
    L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0, ws.data_ptr(),
           wsb, dw.data_ptr(), 0, L.stream_ptr())
    _close(dw.cpu(), wr.grad, 2e-3)


# halo-tiled 3x3 stride-1 kernel (conv_halo.hip): reduction channels % 64 == 0.  Widths < 64 use
# full-width tiles (TW = W), widths >= 64 with W % 16 == 0 use 16x16 tiles; the batch is one tall
# virtual image with a zero separator row per image, so tiles straddle images.  Odd heights /
# widths, several images per tile, cout not a multiple of 8 / 64 / 128, one and two column tiles.
S1 = [
    (3, 64, 7, 7, 64, 3, 1),
    (2, 64, 20, 20, 80, 3, 1),
    (5, 128, 9, 13, 40, 3, 1),
    (2, 128, 40, 40, 128, 3, 1),
    (1, 64, 48, 17, 72, 3, 1),
    (2, 64, 64, 64, 64, 3, 1),
    (1, 192, 16, 80, 136, 3, 1),
    (2, 256, 20, 20, 256, 3, 1),
    (1, 64, 3, 96, 64, 3, 1),
]


@pytest.mark.parametrize("shp", S1)
def test_conv3x3_s1_default_paths(shp):
    """3x3 stride-1 layers through the default routing (the direct small-channel kernel where it
    applies, else the implicit GEMM): forward with statistics, eval forward with BN+SiLU+residual
    into a channel slice, stride-1 input gradient (store and accumulate)."""
    n, cin, h, w, cout, k, s = shp
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(hash(shp) % 997)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    z = ref_conv(x, wt, s, dtype)
    # forward + BN statistics
    y, st = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, stats=True)
    _close(nchw(y, cout).cpu(), z, TOL["bf16"])
    check_moments(st, z, 1e-3)
    if r8(cout) != cout:
        assert y[..., cout:].abs().max().item() == 0
    # forward with folded BN + SiLU + residual, output at a channel offset of a wider buffer
    sc = torch.rand(cout, generator=g) + 0.5
    sh_ = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, cout, h, w, generator=g)
    ya, _ = conv_fwd(nhwc(x, dtype), wt, shp_, dtype, sc.cuda(), sh_.cuda(), L.ACT_SILU, nhwc(res, dtype),
                     yld=r8(cout) + 16, yoff=8)
    ref = F.silu(z * sc.view(1, -1, 1, 1) + sh_.view(1, -1, 1, 1)) + res.to(dtype).float()
    _close(nchw(ya, cout, off=8).cpu(), ref, TOL["bf16"])
    assert ya[..., :8].abs().max().item() == 0
    # stride-1 dgrad (reduction over cout): store and accumulate
    if cout % 64 == 0:
        dz = torch.randn(n, cout, h, w, generator=g)
        xr = x.to(dtype).float().requires_grad_(True)
        F.conv2d(xr, wt.to(dtype).float(), None, 1, 1).backward(dz.to(dtype).float())
        sp = ctypes.pointer(shp_)
        wpt = pack(wt, shp_, dtype, 1)
        dzb = nhwc(dz, dtype)
        base = torch.randn(n, cin, h, w, generator=g)
        for acc in (0, 1):
            dx = nhwc(base, dtype)
            L.call("yms_conv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(),
                   dx.shape[-1], 0, acc, L.stream_ptr())
            exp = xr.grad + (base.to(dtype).float() if acc else 0)
            _close(nchw(dx, cin).cpu(), exp, TOL["bf16"] * 2)


# halo-tiled 3x3 weight gradient (wgrad_halo.hip): patch widths TW = W (W <= 40), divisors of W,
# W not a multiple of TW; stride 1 / 2 with odd sizes (halo clipping at every border); cout of one
# or two 32-blocks with padding (16, 48, 80, 130); cin not a multiple of 32 (8, 40, 96); many
# patches per split (n = 6); images spanning patch rows; the 64-input-channel block variant.
WGH = [
    (2, 32, 20, 20, 32, 1), (3, 40, 13, 27, 48, 1), (2, 64, 80, 80, 64, 1), (1, 96, 50, 70, 80, 1),
    (2, 8, 33, 41, 16, 2), (2, 64, 40, 40, 130, 2), (1, 32, 161, 97, 64, 2), (6, 64, 24, 24, 64, 1),
    (1, 16, 7, 300, 32, 1), (2, 48, 9, 5, 40, 2),
    # one block over all 64 input channels (4 x 16 patches): ragged patch rows, padded input channels
    (3, 64, 21, 32, 64, 1), (1, 60, 18, 48, 64, 1),
]


@pytest.mark.parametrize("mode", ["2", "1"])
@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("shp", WGH)
def test_wgrad_3x3_halo(shp, dt, mode, monkeypatch):
    """mode 2 forces the halo kernel on every shape; mode 1 is the default selection (halo for
    stride-1 layers with 32 / 64 output channels, the im2col kernel otherwise)."""
    monkeypatch.setenv("YMS_WG_HALO", mode)
    n, cin, h, w, cout, s = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(n * 7919 + cin * 31 + h + w + cout + s)
    x = torch.randn(n, cin, h, w, generator=g)
    shp_ = shape(n, h, w, cin, cout, 3, s, dtype)
    dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    xr, dzr = x.to(dtype).double(), dz.to(dtype).double()
    ref = torch.nn.grad.conv2d_weight(xr, (cout, cin, 3, 3), dzr, stride=s, padding=1)
    sp = ctypes.pointer(shp_)
    # channel slots of wider buffers (x at offset 8, dz at offset 16)
    xb = nhwc(x, dtype, ld=r8(cin) + 16, off=8)
    dzb = nhwc(dz, dtype, ld=r8(cout) + 16, off=16)
    wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
    ws = torch.full((wsb // 4 + 1,), float("nan"), dtype=torch.float32, device="cuda")
    for acc in (0, 1):
        dw = torch.full((cout, cin, 3, 3), 0.25, device="cuda")
        L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 8, dzb.data_ptr(), dzb.shape[-1], 16,
               ws.data_ptr(), wsb, dw.data_ptr(), acc, L.stream_ptr())
        got = dw.double().cpu() - (0.25 if acc else 0.0)
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel < 1e-5 and (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6, (acc, rel)


# LDS-DMA ring weight gradient (wgrad_ring.hip): 1x1 and 3x3, stride 1 / 2, 64- and 128-row tiles
# (cout 48, 64, 80, 128, 130, 256), 64-column GEMMs (1x1 with cin <= 64 on 128-row tiles), cin
# not a multiple of 64 (40, 96, 200), pixel counts not a multiple of the k-tile, many splits,
# channel slots of wider buffers
WGR = [
    (2, 64, 40, 40, 128, 3, 1), (3, 40, 13, 27, 48, 3, 1), (2, 96, 20, 20, 80, 1, 1), (1, 200, 17, 19, 130, 1, 1),
    (2, 32, 33, 41, 256, 3, 2), (2, 64, 24, 24, 64, 1, 1), (4, 128, 20, 20, 256, 3, 1), (2, 48, 9, 5, 96, 3, 2),
    (8, 128, 40, 40, 128, 1, 1), (1, 16, 7, 300, 72, 3, 1), (2, 256, 10, 10, 512, 3, 2),
]


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("shp", WGR)
def test_wgrad_ring(shp, dt, monkeypatch):
    monkeypatch.setenv("YMS_WG_HALO", "0")
    monkeypatch.setenv("YMS_WG_RING", "2")
    n, cin, h, w, cout, k, s = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(n * 7919 + cin * 31 + h + w + cout + s + k)
    x = torch.randn(n, cin, h, w, generator=g)
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    xr, dzr = x.to(dtype).double(), dz.to(dtype).double()
    ref = torch.nn.grad.conv2d_weight(xr, (cout, cin, k, k), dzr, stride=s, padding=k // 2)
    sp = ctypes.pointer(shp_)
    xb = nhwc(x, dtype, ld=r8(cin) + 16, off=8)
    dzb = nhwc(dz, dtype, ld=r8(cout) + 16, off=16)
    wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
    ws = torch.full((wsb // 4 + 1,), float("nan"), dtype=torch.float32, device="cuda")
    for acc in (0, 1):
        dw = torch.full((cout, cin, k, k), 0.25, device="cuda")
        L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 8, dzb.data_ptr(), dzb.shape[-1], 16,
               ws.data_ptr(), wsb, dw.data_ptr(), acc, L.stream_ptr())
        got = dw.double().cpu() - (0.25 if acc else 0.0)
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel < 1e-5 and (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6, (acc, rel)


@pytest.mark.parametrize("route", ["tt", "ring", "halo"])
@pytest.mark.parametrize("ratio", ["0.05", "1.0", "0"])
def test_wgrad_split_k_slab_cap(route, ratio, monkeypatch):
    """The split-K slab cap (YMS_WG_SLAB_RATIO: default 0.05 of the layer's x + dz bytes; 1.0 the
    round-3 default; 0 uncapped) changes only how many fp32 partial slabs the weight gradient sums
    in its fixed-order reduce: every setting on every wgrad kernel (register-staged TT, LDS-DMA ring,
    halo-staged 3x3) matches the fp32 torch gradient on bf16 operands, on layers deep enough in
    pixels (B*H*W up to 32k) that the split count differs between the settings."""
    monkeypatch.setenv("YMS_WG_SLAB_RATIO", ratio)
    monkeypatch.setenv("YMS_WG_RING", "1" if route == "ring" else "0")
    monkeypatch.setenv("YMS_WG_HALO", "1" if route == "halo" else "0")
    dtype = torch.bfloat16
    cases = [(8, 64, 40, 40, 64, 3, 1), (8, 128, 20, 20, 256, 1, 1), (4, 32, 80, 80, 32, 3, 1),
             (8, 96, 40, 40, 128, 3, 2)]
    for n, cin, h, w, cout, k, s in cases:
        g = torch.Generator().manual_seed(n + cin + cout + k)
        x = torch.randn(n, cin, h, w, generator=g)
        shp_ = shape(n, h, w, cin, cout, k, s, dtype)
        dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
        xr = x.to(dtype).float()
        wr = torch.zeros(cout, cin, k, k, requires_grad=True)
        F.conv2d(xr, wr, None, s, k // 2).backward(dz.to(dtype).float())
        sp = ctypes.pointer(shp_)
        xb, dzb = nhwc(x, dtype), nhwc(dz, dtype)
        wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device="cuda")
        dw = torch.zeros(cout, cin, k, k, device="cuda")
        L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0,
               ws.data_ptr(), wsb, dw.data_ptr(), 0, L.stream_ptr())
        _close(dw.cpu(), wr.grad, 2e-3)


@pytest.mark.parametrize("route", ["tt", "ring", "halo"])
def test_wgrad_workspace_smaller_than_planned(route, monkeypatch):
    """A workspace sized under other YMS_WG_* settings than the call's (here: fewer bytes than
    yms_conv_wgrad_ws_bytes asks for) runs fewer split-K partial slabs instead of failing: the
    gradient still matches; below one slab the call is refused."""
    monkeypatch.setenv("YMS_WG_SLAB_RATIO", "1.0")       # many splits, so the shrink has room
    monkeypatch.setenv("YMS_WG_RING", "1" if route == "ring" else "0")
    monkeypatch.setenv("YMS_WG_HALO", "1" if route == "halo" else "0")
    dtype = torch.bfloat16
    n, cin, h, w, cout, k, s = (8, 64, 40, 40, 64, 3, 1) if route != "ring" else (8, 128, 20, 20, 256, 1, 1)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, cin, h, w, generator=g)
    shp_ = shape(n, h, w, cin, cout, k, s, dtype)
    dz = torch.randn(n, cout, shp_.ho, shp_.wo, generator=g)
    wr = torch.zeros(cout, cin, k, k, requires_grad=True)
    F.conv2d(x.to(dtype).float(), wr, None, s, k // 2).backward(dz.to(dtype).float())
    sp = ctypes.pointer(shp_)
    xb, dzb = nhwc(x, dtype), nhwc(dz, dtype)
    full = L.lib().yms_conv_wgrad_ws_bytes(sp)
    slab = 4 * cout * k * k * cin                       # at least one slab (tiles round it up)
    assert full > 2 * slab
    for wsb in (full // 2 + 4, full // 3 + 4):
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device="cuda")
        dw = torch.zeros(cout, cin, k, k, device="cuda")
        L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0,
               ws.data_ptr(), wsb, dw.data_ptr(), 0, L.stream_ptr())
        _close(dw.cpu(), wr.grad, 2e-3)
    ws = torch.empty(16, dtype=torch.float32, device="cuda")
    st = L.lib().yms_conv_wgrad(sp, xb.data_ptr(), xb.shape[-1], 0, dzb.data_ptr(), dzb.shape[-1], 0, ws.data_ptr(),
                                64, dw.data_ptr(), 0, L.stream_ptr())
    assert st != 0
