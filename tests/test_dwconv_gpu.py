"""Depthwise k x k conv kernels (YOLO-MS MS-Block IB_k mid conv) through the C-ABI
against fp32 PyTorch-CPU grouped convolution (groups = C) on the same dtype-rounded operands:
forward (folded BN + SiLU, and BN statistics: per-tile sum and centred M2), dgrad (store / accumulate), wgrad; plus the
branch-sum kernel yms_add_views.  Parity here is against torch's definition of a depthwise conv,
not against the reference (which has no MS-Block code: annotations.md:66-133)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from hiputil import DT, check_moments, nchw, nhwc, r8, split_stats, stats_buffer
from yms import _lib as L

pytestmark = pytest.mark.gpu

# the tile width follows the map width (32 where it divides it, else 40 / 20 / 32: every width below
# is covered), and k = 3 with C % 64 == 0 takes 64-channel blocks: the list holds each kernel
# geometry -- TX 20 (w 20, 9), 40 (33, 40, 80, 23), 32 (70, 45, 64, 96), 64-channel k = 3 blocks
# (C 64 / 128 / 192), 56-channel k = 3 blocks (C 112 / 168), 32-channel blocks for every k; fp32 runs the tile weight-gradient kernel.
# 16-bit k = 5 / 7 / 9 at widths <= 64 (k = 5: 96) take the MFMA weight gradient: one (w 9, 20, 24,
# 28, 30), two (33, 40, 45, 50) and three (70, 96) column chunks (each k with one and two), partial
# channel groups (C 24, 40), partial last row blocks (h 13, 19, 21, 33), several units per block
# (n 40) and 32-row units for maps of 17-32 rows in one chunk (h 18, 20, 21, 25, 32).  16-bit k = 7 at widths
# <= 48 runs forward / dgrad on MFMA too: two (w 28) and three (40, 45) column blocks, a 2-row last
# row block (h 18), several units per block (n 16)
SHAPES = [(2, 20, 20, 64, 3), (1, 17, 33, 48, 5), (3, 40, 40, 32, 7), (2, 13, 9, 16, 9), (1, 80, 80, 64, 9),
          (2, 8, 70, 40, 5), (2, 24, 80, 32, 3), (2, 11, 45, 24, 7), (2, 40, 40, 128, 3), (1, 9, 23, 192, 3),
          (2, 16, 64, 64, 3), (1, 12, 96, 40, 7), (2, 20, 20, 128, 9),
          (2, 21, 30, 40, 9), (40, 20, 20, 256, 9), (2, 19, 70, 24, 5), (1, 33, 96, 40, 5),
          (2, 18, 28, 48, 7), (16, 40, 40, 256, 7), (2, 17, 50, 24, 9), (2, 12, 24, 32, 5),
          (2, 25, 16, 16, 5), (1, 32, 32, 24, 7), (2, 24, 40, 112, 3), (1, 20, 20, 168, 3)]
TOL = {"f32": 2e-5, "bf16": 1e-2, "f16": 2e-3}
# f16 through the 16-bit paths (the MFMA kernels' f16 builtins) on the k >= 5 shapes
F16_SHAPES = [sh for sh in SHAPES if sh[4] >= 5]


def _close(got, ref, tol):
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"max err {err:.3g} vs scale {scale:.3g} (tol {tol})"


@pytest.mark.parametrize("dt,shp", [(d, sh) for sh in SHAPES for d in ("f32", "bf16")] +
                         [("f16", sh) for sh in F16_SHAPES])
def test_dwconv_fwd_dgrad_wgrad(shp, dt):
    n, h, w, c, k = shp
    dtype = DT[dt]
    g = torch.Generator().manual_seed(sum(shp))
    x = torch.randn(n, c, h, w, generator=g)
    wt = torch.randn(c, 1, k, k, generator=g) / k
    xr = x.to(dtype).float()
    z = F.conv2d(xr, wt, None, 1, k // 2, 1, c)
    sh = L.DwShape(n, h, w, c, k, L.dtype_code(dtype))
    sp = ctypes.pointer(sh)
    st = L.stream_ptr()
    wd = wt.contiguous().cuda()
    xb = nhwc(x, dtype, ld=r8(c) + 8, off=8)
    # eval: folded BN + SiLU, written at a channel offset
    sc = torch.rand(c, generator=g) + 0.5
    sf = torch.randn(c, generator=g) * 0.1
    scd, sfd = sc.cuda(), sf.cuda()          # keep the device copies alive across the async launch
    y = torch.zeros((n, h, w, r8(c) + 16), dtype=dtype, device="cuda")
    L.call("yms_dwconv_fwd", sp, xb.data_ptr(), xb.shape[-1], 8, wd.data_ptr(), y.data_ptr(), y.shape[-1], 16,
           scd.data_ptr(), sfd.data_ptr(), L.ACT_SILU, None, 0, st)
    _close(nchw(y, c, off=16).cpu(), F.silu(z * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)), TOL[dt])
    assert y[..., :16].abs().max().item() == 0
    # train: z + BN partial statistics
    rows = L.lib().yms_dwconv_stats_rows(sp)
    buf = stats_buffer(rows, r8(c))
    y2 = torch.zeros((n, h, w, r8(c)), dtype=dtype, device="cuda")
    L.call("yms_dwconv_fwd", sp, xb.data_ptr(), xb.shape[-1], 8, wd.data_ptr(), y2.data_ptr(), y2.shape[-1], 0,
           None, None, 0, buf.data_ptr(), r8(c), st)
    _close(nchw(y2, c).cpu(), z, TOL[dt])
    check_moments(split_stats(buf, rows, r8(c)), z, 1e-4 if dt == "f32" else 1e-3)
    # backward
    dz = torch.randn(n, c, h, w, generator=g)
    xg = xr.clone().requires_grad_(True)
    wg = wt.clone().requires_grad_(True)
    F.conv2d(xg, wg, None, 1, k // 2, 1, c).backward(dz.to(dtype).float())
    dzb = nhwc(dz, dtype)
    base = torch.randn(n, c, h, w, generator=g)
    for acc in (0, 1):
        dx = nhwc(base, dtype)
        L.call("yms_dwconv_dgrad", sp, dzb.data_ptr(), dzb.shape[-1], 0, wd.data_ptr(), dx.data_ptr(), dx.shape[-1], 0,
               acc, st)
        _close(nchw(dx, c).cpu(), xg.grad + (base.to(dtype).float() if acc else 0), TOL[dt] * 2)
    wsb = L.lib().yms_dwconv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4, device="cuda")
    dw = torch.full((c, 1, k, k), 0.5, device="cuda")
    L.call("yms_dwconv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 8, dzb.data_ptr(), dzb.shape[-1], 0, ws.data_ptr(),
           wsb, dw.data_ptr(), 1, st)
    _close(dw.cpu() - 0.5, wg.grad, {"f32": 1e-4, "bf16": 2e-3, "f16": 5e-4}[dt])


def test_add_views():
    g = torch.Generator().manual_seed(3)
    a = torch.randn(2, 24, 5, 7, generator=g)
    b = torch.randn(2, 24, 5, 7, generator=g)
    ab = nhwc(a, torch.bfloat16, ld=40, off=8)
    bb = nhwc(b, torch.bfloat16, ld=32, off=0)
    y = nhwc(torch.ones(2, 24, 5, 7), torch.bfloat16, ld=24)
    L.call("yms_add_views", L.BF16, 70, 24, ab.data_ptr(), 40, 8, bb.data_ptr(), 32, 0, y.data_ptr(), 24, 0, 1,
           L.stream_ptr())
    ref = a.to(torch.bfloat16).float() + b.to(torch.bfloat16).float() + 1
    _close(nchw(y, 24).cpu(), ref, 1e-2)
    L.call("yms_add_views", L.BF16, 70, 24, ab.data_ptr(), 40, 8, None, 0, 0, y.data_ptr(), 24, 0, 0, L.stream_ptr())
    assert torch.equal(nchw(y, 24).cpu(), a.to(torch.bfloat16).float())


@pytest.mark.parametrize("acc1,acc2", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_add_grad2_routes_into_both_addends(acc1, acc2):
    """yms_add_grad2: the MS-Block branch-sum backward, ga (+)= g and gb (+)= g in one pass."""
    g = torch.Generator().manual_seed(acc1 * 2 + acc2)
    npix, c = 3001, 24
    gy = torch.randn(npix, 40, generator=g).to(torch.bfloat16).cuda()          # a 40-wide buffer, slot at 8
    ga = torch.randn(npix, 32, generator=g).to(torch.bfloat16).cuda()
    gb = torch.randn(npix, 48, generator=g).to(torch.bfloat16).cuda()
    ea = (ga[:, 0:24].float() * acc1 + gy[:, 8:32].float()).to(torch.bfloat16)
    eb = (gb[:, 16:40].float() * acc2 + gy[:, 8:32].float()).to(torch.bfloat16)
    rest_a, rest_b = ga[:, 24:].clone(), gb[:, :16].clone()
    L.call("yms_add_grad2", L.BF16, npix, c, gy.data_ptr(), 40, 8, ga.data_ptr(), 32, 0, acc1, gb.data_ptr(), 48, 16,
           acc2, L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(ga[:, 0:24], ea) and torch.equal(gb[:, 16:40], eb)
    assert torch.equal(ga[:, 24:], rest_a) and torch.equal(gb[:, :16], rest_b)
