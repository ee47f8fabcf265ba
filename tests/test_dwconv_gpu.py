"""Depthwise k x k conv kernels (YOLO-MS MS-Block IB_k mid conv) through the C-ABI
against fp32 PyTorch-CPU grouped convolution (groups = C) on the same dtype-rounded operands:
forward (folded BN + SiLU, and BN statistics: per-tile sum and centred M2), dgrad (store / accumulate), wgrad; plus the
branch-sum kernel yms_add_views.  Parity here is against torch's definition of a depthwise conv,
not against the reference (which has no MS-Block code: annotations.md:66-133)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from hiputil import DT, check_moments, merge_moments, nchw, nhwc, r8, split_stats, stats_buffer
from yms import _lib as L

pytestmark = pytest.mark.gpu

SHAPES = [(2, 20, 20, 64, 3), (1, 17, 33, 48, 5), (3, 40, 40, 32, 7), (2, 13, 9, 16, 9), (1, 80, 80, 64, 9),
          (2, 8, 70, 40, 5), (2, 24, 80, 32, 3), (2, 11, 45, 24, 7), (2, 40, 40, 128, 3), (1, 9, 23, 192, 3)]
TOL = {"f32": 2e-5, "bf16": 1e-2}


def _close(got, ref, tol):
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"max err {err:.3g} vs scale {scale:.3g} (tol {tol})"


# tile width of the forward / dgrad kernels: automatic (32 / 40 / 20 by the map width) or forced,
# with the end-of-tile wait that leaves the tile's stores in flight (default) or drains them ("w"),
# and 64-channel blocks for k = 3 (automatic when C % 64 == 0) or forced 32-channel blocks ("g4")
@pytest.mark.parametrize("tx", ["0", "32", "40", "20", "0w", "0g4", "40g4"])
@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("shp", SHAPES)
def test_dwconv_fwd_dgrad_wgrad(shp, dt, tx, monkeypatch):
    monkeypatch.setenv("YMS_DW_TX", tx.replace("g4", "").rstrip("w"))
    monkeypatch.setenv("YMS_DW_WAITALL", "1" if tx.endswith("w") else "0")
    monkeypatch.setenv("YMS_DW_G", "4" if tx.endswith("g4") else "0")
    # k = 3 weight gradient: strip walker (4 or 8 channel groups) or the tile kernel ("w" variant)
    monkeypatch.setenv("YMS_DW_WG3", "0" if tx.endswith("w") else "1")
    monkeypatch.setenv("YMS_DW_WGK", "0" if tx.endswith("w") else "1")   # k >= 5: opt-in rows-over-waves kernel
    monkeypatch.setenv("YMS_DW_WG3_G", "8" if tx == "0" else "4")
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
    _close(dw.cpu() - 0.5, wg.grad, 1e-4 if dt == "f32" else 2e-3)


@pytest.mark.parametrize("iters", ["0", "1", "2", "4"])
def test_add_views(iters, monkeypatch):
    monkeypatch.setenv("YMS_ADD_ITERS", iters)      # items per thread (read per call)
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


@pytest.mark.parametrize("iters", ["0", "1", "2", "4"])
@pytest.mark.parametrize("acc1,acc2", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_add_grad2_routes_into_both_addends(acc1, acc2, iters, monkeypatch):
    """yms_add_grad2: the MS-Block branch-sum backward, ga (+)= g and gb (+)= g in one pass."""
    monkeypatch.setenv("YMS_ADD_ITERS", iters)
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


# depthwise dgrad fused with the producer's BN + SiLU backward reduce (MS-Block IB: 1x1 expand ->
# BN -> SiLU -> depthwise): dx must equal the plain dgrad bit for bit, and the finalized
# (dgamma, dbeta, coefficients) must match the separate reduce + finalize on the same stored dx
@pytest.mark.parametrize("tx", ["0", "40", "20", "0g4"])
@pytest.mark.parametrize("shp", [(2, 20, 20, 64, 3), (2, 40, 40, 128, 3), (1, 17, 33, 48, 5), (2, 20, 20, 32, 9),
                                 (2, 9, 23, 192, 3), (1, 80, 80, 64, 7)])
@pytest.mark.parametrize("act", [1, 0])
def test_dwconv_dgrad_bnred_matches_separate_reduce(shp, act, tx, monkeypatch):
    monkeypatch.setenv("YMS_DW_TX", tx.replace("g4", ""))
    monkeypatch.setenv("YMS_DW_G", "4" if tx.endswith("g4") else "0")
    n, h, w, c, k = shp
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(sum(shp) + act)
    sh = L.DwShape(n, h, w, c, k, L.dtype_code(dtype))
    sp = ctypes.pointer(sh)
    st = L.stream_ptr()
    dz = nhwc(torch.randn(n, c, h, w, generator=g), dtype, ld=r8(c) + 8, off=8)
    wd = (torch.randn(c, 1, k, k, generator=g) / k).contiguous().cuda()
    rz = nhwc(torch.randn(n, c, h, w, generator=g) * 2 + 0.5, dtype, ld=r8(c) + 16, off=16)
    rsc = (torch.rand(c, generator=g) + 0.5).cuda()
    rsh = (torch.randn(c, generator=g) * 0.2).cuda()
    rmi = torch.cat([torch.randn(c, generator=g) * 0.3, torch.rand(c, generator=g) + 0.5]).cuda()
    npix = n * h * w
    # reference: plain dgrad, then the separate reduce over the stored dx
    dx0 = torch.zeros((n, h, w, r8(c)), dtype=dtype, device="cuda")
    L.call("yms_dwconv_dgrad", sp, dz.data_ptr(), dz.shape[-1], 8, wd.data_ptr(), dx0.data_ptr(), dx0.shape[-1], 0, 0, st)
    rows0 = L.lib().yms_bn_bwd_rows(npix, c)
    ws0 = torch.empty(rows0 * 2 * c, device="cuda")
    L.call("yms_bn_act_bwd_reduce", L.BF16, npix, c, rz.data_ptr(), rz.shape[-1], 16, dx0.data_ptr(), dx0.shape[-1], 0,
           rsc.data_ptr(), rsh.data_ptr(), rmi.data_ptr(), act, ws0.data_ptr(), st)
    # fused
    rows1 = L.lib().yms_dwconv_dgrad_rows(sp)
    assert rows1 >= 1
    ws1 = torch.full((rows1 * 2 * c + 64,), float("nan"), device="cuda")
    dx1 = torch.zeros_like(dx0)
    L.call("yms_dwconv_dgrad_bnred", sp, dz.data_ptr(), dz.shape[-1], 8, wd.data_ptr(), dx1.data_ptr(), dx1.shape[-1], 0,
           rz.data_ptr(), rz.shape[-1], 16, rsc.data_ptr(), rsh.data_ptr(), rmi.data_ptr(), act, ws1.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0)
    assert torch.isfinite(ws1[:rows1 * 2 * c]).all() and torch.isnan(ws1[rows1 * 2 * c:]).all()
    outs = []
    for ws, rows in ((ws0, rows0), (ws1, rows1)):
        dg, db, coef = torch.empty(c, device="cuda"), torch.empty(c, device="cuda"), torch.empty(2 * c, device="cuda")
        L.call("yms_bn_act_bwd_finalize", c, ws.data_ptr(), rows, npix, dg.data_ptr(), db.data_ptr(), coef.data_ptr(), st)
        outs.append(torch.cat([dg, db, coef]).double().cpu())
    ref = outs[0]
    assert ((outs[1] - ref).abs().max() / ref.abs().max()).item() < 1e-5


# depthwise forward / weight gradient with the producer's BN + act formed from its pre-BN z while
# staging (the MS-Block IB's expand conv output is never materialised in training): against
# yms_affine_act followed by the plain kernels.  Padding must stay zero (not act(shift)).
@pytest.mark.parametrize("tx", ["0", "40", "20", "0g4"])
@pytest.mark.parametrize("shp", [(2, 20, 20, 64, 3), (2, 40, 40, 128, 3), (1, 17, 33, 48, 5), (2, 20, 20, 32, 9),
                                 (2, 9, 23, 192, 3), (1, 80, 80, 64, 7), (3, 12, 70, 16, 3)])
@pytest.mark.parametrize("act", [1, 0])
def test_dwconv_bnin_matches_affine_then_conv(shp, act, tx, monkeypatch):
    monkeypatch.setenv("YMS_DW_TX", tx.replace("g4", ""))
    monkeypatch.setenv("YMS_DW_G", "4" if tx.endswith("g4") else "0")
    n, h, w, c, k = shp
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(sum(shp) * 3 + act)
    sh = L.DwShape(n, h, w, c, k, L.dtype_code(dtype))
    sp = ctypes.pointer(sh)
    st = L.stream_ptr()
    npix = n * h * w
    z = nhwc(torch.randn(n, c, h, w, generator=g) * 2 + 0.3, dtype, ld=r8(c) + 8, off=8)
    isc = (torch.rand(c, generator=g) + 0.5).cuda()
    ish = (torch.randn(c, generator=g) * 0.5 + 0.5).cuda()     # act(shift) != 0: padding must not see it
    wd = (torch.randn(c, 1, k, k, generator=g) / k).contiguous().cuda()
    dz = nhwc(torch.randn(n, c, h, w, generator=g), dtype)
    # reference: materialise x = act(z * isc + ish), then the plain kernels
    x = torch.zeros((n, h, w, r8(c)), dtype=dtype, device="cuda")
    L.call("yms_affine_act", L.BF16, npix, c, z.data_ptr(), z.shape[-1], 8, isc.data_ptr(), ish.data_ptr(), act,
           None, 0, 0, x.data_ptr(), x.shape[-1], 0, st)
    rows = L.lib().yms_dwconv_stats_rows(sp)
    outs = []
    for bnin in (False, True):
        buf = stats_buffer(rows, r8(c))
        y = torch.zeros((n, h, w, r8(c)), dtype=dtype, device="cuda")
        wsb = L.lib().yms_dwconv_wgrad_ws_bytes(sp)
        ws = torch.empty(wsb // 4, device="cuda")
        dw = torch.zeros((c, 1, k, k), device="cuda")
        if bnin:
            L.call("yms_dwconv_fwd_bnin", sp, z.data_ptr(), z.shape[-1], 8, isc.data_ptr(), ish.data_ptr(), act,
                   wd.data_ptr(), y.data_ptr(), y.shape[-1], 0, buf.data_ptr(), r8(c), st)
            L.call("yms_dwconv_wgrad_bnin", sp, z.data_ptr(), z.shape[-1], 8, isc.data_ptr(), ish.data_ptr(), act,
                   dz.data_ptr(), dz.shape[-1], 0, ws.data_ptr(), wsb, dw.data_ptr(), 0, st)
        else:
            L.call("yms_dwconv_fwd", sp, x.data_ptr(), x.shape[-1], 0, wd.data_ptr(), y.data_ptr(), y.shape[-1], 0,
                   None, None, 0, buf.data_ptr(), r8(c), st)
            L.call("yms_dwconv_wgrad", sp, x.data_ptr(), x.shape[-1], 0, dz.data_ptr(), dz.shape[-1], 0, ws.data_ptr(),
                   wsb, dw.data_ptr(), 0, st)
        torch.cuda.synchronize()
        s1, m2 = merge_moments(split_stats(buf, rows, r8(c)), c, npix)
        outs.append((y.float().cpu(), dw.cpu(), s1, m2))
    (y0, dw0, a0, b0), (y1, dw1, a1, b1) = outs
    _close(y1, y0, 1e-2)
    _close(dw1, dw0, 1e-5)
    assert ((a1 - a0).abs().max() / (a0.abs().max() + 1e-6)).item() < 1e-5
    assert ((b1 - b0).abs() / b0.clamp_min(1e-30)).max().item() < 1e-4
