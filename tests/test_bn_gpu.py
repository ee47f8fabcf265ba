"""BN(+SiLU) backward through the C-ABI (reduce -> finalize -> apply) against an fp64 torch
reference of nn.BatchNorm2d's training backward (components.py:73-74), at pixel counts where
the 256-row partial-sum cap applies and does not divide npix (B=7 / B=9 at 640^2
stride-8 layers), plus small and ragged counts.  The partial-sum scratch is pre-filled with NaN,
so a finalize that read rows the reduce did not write fails loudly."""
import ctypes

import pytest
import torch

from yms import _lib as L

pytestmark = pytest.mark.gpu


def _ref(z, gy, sc, sh, mu, istd, act):
    a = z * sc + sh
    if act:
        s = torch.sigmoid(a)
        da = gy * (s * (1 + a * (1 - s)))
    else:
        da = gy
    xh = (z - mu) * istd
    dbeta = da.sum(0)
    dgamma = (da * xh).sum(0)
    n = z.shape[0]
    dz = sc * (da - dbeta / n - xh * (dgamma / n))
    return dgamma, dbeta, dz


@pytest.mark.parametrize("npix,c,act", [(44800, 64, 1), (44801, 64, 1), (57600, 32, 1), (40001, 24, 0), (100, 16, 1),
                                        (7 * 80 * 80, 128, 1), (25600, 768, 1), (3000, 1152, 0)])
def test_bn_bwd_matches_fp64(npix, c, act):
    g = torch.Generator().manual_seed(npix + c)
    z = torch.randn(npix, c, generator=g, dtype=torch.float64)
    gy = torch.randn(npix, c, generator=g, dtype=torch.float64)
    sc = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(c, generator=g, dtype=torch.float64) * 0.2
    mu = z.mean(0)
    istd = 1.0 / (z.var(0, unbiased=False) + 1e-3).sqrt()
    dg, db, dz = _ref(z, gy, sc, sh, mu, istd, act)
    dev = "cuda"
    zd, gyd = z.float().to(dev), gy.float().to(dev)
    scd, shd = sc.float().to(dev), sh.float().to(dev)
    mi = torch.cat([mu, istd]).float().to(dev)
    rows = L.lib().yms_bn_bwd_rows(npix, c)
    assert rows >= 1
    st = L.stream_ptr()

    def rel(a, b):
        return ((a.double().cpu() - b).norm() / b.norm()).item()

    for fused in (False, True):
        ws = torch.full((rows + 16, 2, c), float("nan"), dtype=torch.float32, device=dev)   # NaN beyond `rows`
        cnt = torch.zeros(4, dtype=torch.int32, device=dev)
        dgd = torch.empty(c, device=dev)
        dbd = torch.empty(c, device=dev)
        coef = torch.empty(2 * c, device=dev)
        out = torch.empty_like(zd)
        if fused:
            L.call("yms_bn_act_bwd_reduce_finalize", L.F32, npix, c, zd.data_ptr(), c, 0, gyd.data_ptr(), c, 0,
                   scd.data_ptr(), shd.data_ptr(), mi.data_ptr(), act, ws.data_ptr(), cnt.data_ptr(), dgd.data_ptr(),
                   dbd.data_ptr(), coef.data_ptr(), st)
        else:
            L.call("yms_bn_act_bwd_reduce", L.F32, npix, c, zd.data_ptr(), c, 0, gyd.data_ptr(), c, 0,
                   scd.data_ptr(), shd.data_ptr(), mi.data_ptr(), act, ws.data_ptr(), st)
            L.call("yms_bn_act_bwd_finalize", c, ws.data_ptr(), rows, npix, dgd.data_ptr(), dbd.data_ptr(),
                   coef.data_ptr(), st)
        L.call("yms_bn_act_bwd_apply", L.F32, npix, c, zd.data_ptr(), c, 0, gyd.data_ptr(), c, 0, scd.data_ptr(),
               shd.data_ptr(), mi.data_ptr(), coef.data_ptr(), act, out.data_ptr(), c, 0, None, 0, 0, 0, st)
        torch.cuda.synchronize()
        # rows the reduce wrote lie in [0, rows): the NaN tail is untouched; the two-kernel reduce
        # writes exactly yms_bn_bwd_rows rows (the fused one may write fewer: <= 32768 / c)
        assert torch.isnan(ws[rows:]).all()
        if not fused:
            assert torch.isfinite(ws[:rows]).all()
        assert int(cnt[0]) == 0          # the fused finalize leaves its counter at zero
        assert rel(dgd, dg) < 1e-5, fused
        assert rel(dbd, db) < 1e-5, fused
        assert rel(out, dz) < 1e-5, fused


def test_bias_bwd_fused():
    g = torch.Generator().manual_seed(5)
    npix, c = 64 * 20 * 20, 80
    gy = torch.randn(npix, 88, generator=g, dtype=torch.float64)
    dev = "cuda"
    gyb = gy.to(torch.bfloat16).to(dev)
    ref = gyb.double().cpu()[:, :c].sum(0)
    rows = L.lib().yms_bn_bwd_rows(npix, c)
    ws = torch.empty((rows, 2, c), dtype=torch.float32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int32, device=dev)
    db = torch.empty(c, device=dev)
    for _ in range(2):      # the counter is reusable: it returns to zero
        L.call("yms_bias_bwd", L.BF16, npix, c, gyb.data_ptr(), 88, 0, ws.data_ptr(), cnt.data_ptr(), db.data_ptr(),
               L.stream_ptr())
        torch.cuda.synchronize()
        assert ((db.double().cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-5
        assert int(cnt[0]) == 0


def _finalize(buf, rows, ld, c, npix):
    gam = torch.rand(c, generator=torch.Generator().manual_seed(c)).cuda() + 0.5
    bet = torch.randn(c, generator=torch.Generator().manual_seed(c + 1)).cuda()
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    mi = torch.empty(2 * c, device="cuda")
    sc, sh = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    L.call("yms_bn_finalize", c, buf.data_ptr(), rows, ld, npix, gam.data_ptr(), bet.data_ptr(), rm.data_ptr(),
           rv.data_ptr(), ctypes.c_float(0.03), ctypes.c_float(1e-3), mi.data_ptr(), sc.data_ptr(), sh.data_ptr(),
           L.stream_ptr())
    torch.cuda.synchronize()
    return mi[:c].double().cpu(), mi[c:].double().cpu(), rv.double().cpu()


@pytest.mark.parametrize("b,h,w,offset,dt", [(2, 3, 2, 300.0, "f32"), (4, 40, 40, 1000.0, "f32"),
                                             (9, 80, 80, 50.0, "f32"), (16, 80, 80, 300.0, "bf16"),
                                             (3, 17, 23, 1000.0, "bf16")])
def test_bn_stats_large_mean_conv_and_dw(b, h, w, offset, dt):
    """Training BN statistics where |mean| / std ~ 4e2-8e3 (sum z^2 - n mean^2 in fp32 would lose
    every digit): conv (fp32: 128-pixel rows, > 1024 rows exercises the in-place pre-reduction;
    bf16: per-block slot rows) and depthwise (8x32 tile rows) against fp64 moments of the
    kernels' own z, through yms_bn_finalize and the producers' count tables."""
    from hiputil import DT, conv_fwd, nchw, nhwc, r8, ref_conv, shape, stats_buffer
    dtype = DT[dt]
    c = 64
    g = torch.Generator().manual_seed(b * h)
    x = offset + torch.randn(b, c, h, w, generator=g)
    wt = (torch.rand(c, c, 1, 1, generator=g) + 0.5) / c
    sp = shape(b, h, w, c, c, 1, 1, dtype)
    y, (st, cnt) = conv_fwd(nhwc(x, dtype), wt, sp, dtype, stats=True)
    n = b * h * w
    assert cnt.sum().item() == n
    # statistics come from the fp32 accumulators: compare with the fp32 conv of the same operands
    z = ref_conv(x, wt, 1, dtype).double() if dt == "bf16" else nchw(y, c).double().cpu()
    rows, ld = st.shape[0], st.shape[2]
    mean, istd, rv = _finalize(_flat(st, cnt), rows, ld, c, n)
    var = z.var((0, 2, 3), unbiased=False)
    tol = 1e-6 if dt == "f32" else 2e-6
    assert ((mean - z.mean((0, 2, 3))).abs() / z.mean((0, 2, 3)).abs()).max().item() < tol
    assert ((istd - 1 / (var + 1e-3).sqrt()).abs() * (var + 1e-3).sqrt()).max().item() < 1e-4
    assert ((rv - (0.97 + 0.03 * var * n / (n - 1))).abs() / rv).max().item() < 1e-5
    # depthwise 3x3 on the same large-offset input
    ds = L.DwShape(b, h, w, c, 3, L.dtype_code(dtype))
    dsp = ctypes.pointer(ds)
    wd = (torch.rand(c, 1, 3, 3, generator=g) + 0.5).cuda() / 9
    drows = L.lib().yms_dwconv_stats_rows(dsp)
    dbuf = stats_buffer(drows, r8(c))
    xb = nhwc(x, dtype)
    yd = torch.zeros((b, h, w, r8(c)), dtype=dtype, device="cuda")
    L.call("yms_dwconv_fwd", dsp, xb.data_ptr(), xb.shape[-1], 0, wd.data_ptr(), yd.data_ptr(), yd.shape[-1], 0,
           None, None, 0, dbuf.data_ptr(), r8(c), L.stream_ptr())
    torch.cuda.synchronize()
    assert dbuf[drows * 2 * r8(c):].sum().item() == n
    zd = torch.nn.functional.conv2d(x.to(dtype).double(), wd.double().cpu(), None, 1, 1, 1, c)
    mean, istd, _ = _finalize(dbuf, drows, r8(c), c, n)
    var = zd.var((0, 2, 3), unbiased=False)
    assert ((mean - zd.mean((0, 2, 3))).abs() / zd.mean((0, 2, 3)).abs()).max().item() < 1e-5
    assert ((istd - 1 / (var + 1e-3).sqrt()).abs() * (var + 1e-3).sqrt()).max().item() < 1e-4


def _flat(st, cnt):
    """the conv_fwd helper's statistics views -> their (contiguous) workspace"""
    base = st.reshape(-1)
    assert cnt.data_ptr() == base.data_ptr() + base.numel() * 4
    return torch.as_strided(base, (base.numel() + cnt.numel(),), (1,))


# SPPF pool backward (argmax + gather per pool, slot 3 -> 2 -> 1 -> 0) against torch's CPU
# max_pool2d backward on the kernel's own forward slots: PyTorch scan order with the first max and
# NaN-propagating comparisons -- ties (quantised values), NaNs, maps of every size class, channel
# counts not a multiple of 16; each slot's gradient rounded to the dtype before it feeds the next pool
@pytest.mark.parametrize("n,h,w,c", [(2, 20, 20, 64), (1, 13, 17, 40), (2, 24, 30, 48), (1, 40, 40, 24),
                                     (3, 5, 7, 16)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_sppf_pool_bwd_matches_torch(n, h, w, c, dt):
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(n * 100 + h + w + c)
    ld = 4 * c + 8
    # slots 0..3 of an NHWC concat buffer at channel offset 8; quantised values give many ties
    buf = torch.zeros(n, h, w, ld)
    x0 = (torch.randint(-4, 5, (n, h, w, c), generator=g).float() * 0.25)
    x0[0, 1, 2, :3] = float("nan")
    buf[..., 8:8 + c] = x0
    buf = buf.to(dt).cuda()
    L.call("yms_sppf_pool_fwd", L.dtype_code(dt), n, h, w, c, buf.data_ptr(), ld, 8, L.stream_ptr())
    g0 = torch.randn(n, h, w, ld, generator=g).to(dt).cuda()
    ws = torch.empty(n * h * w * ((c + 7) // 8) * 8, dtype=torch.uint8, device="cuda")
    gb = g0.clone()
    L.call("yms_sppf_pool_bwd", L.dtype_code(dt), n, h, w, c, buf.data_ptr(), ld, 8, gb.data_ptr(), ld, 8,
           ws.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    xs = buf.float().cpu()
    ref = g0.float().cpu()

    def slot(t, k):
        return t[..., 8 + k * c:8 + (k + 1) * c].permute(0, 3, 1, 2)

    for k in (3, 2, 1):
        xin = slot(xs, k - 1).contiguous().requires_grad_(True)
        y = F.max_pool2d(xin, 5, 1, 2)
        assert torch.equal(torch.isnan(y), torch.isnan(slot(xs, k)))
        y.backward(slot(ref, k).contiguous())
        ref[..., 8 + (k - 1) * c:8 + k * c] = (slot(ref, k - 1) + xin.grad).to(dt).float().permute(0, 2, 3, 1)
    got = gb.float().cpu()
    assert torch.equal(got[..., 8 + 3 * c:], ref[..., 8 + 3 * c:])      # slot 3 (the last pool's output)
    assert torch.equal(got[..., :8], ref[..., :8])
    # fp32 sums of the same addends in another order: one rounding step of the dtype at most
    tol = 2 ** -7 if dt == torch.bfloat16 else 2 ** -10
    d = (got - ref).abs()
    assert (d <= tol * ref.abs() + 1e-6).all(), d.max().item()


@pytest.mark.parametrize("npix,c,ld,off", [(44800, 64, 64, 0), (40001, 24, 40, 8), (100, 16, 16, 0),
                                           (25600, 768, 776, 8), (3001, 40, 48, 0), (999, 20, 32, 8),
                                           (7 * 80 * 80, 128, 256, 128)])
@pytest.mark.parametrize("dt", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("has_z", [True, False])
def test_bn_bwd_reduce_partial_rows(npix, c, ld, off, dt, has_z):
    """The software-pipelined reduce (unconditional loads with the tail pixels re-read and masked):
    exactly yms_bn_bwd_rows partial rows written, summing to the fp64 (sum da, sum da * xhat) of the
    same dtype-rounded pixels; without z the rows carry sum gy (bias gradient)."""
    tdt, code = {"bf16": (torch.bfloat16, L.BF16), "f16": (torch.float16, L.F16), "f32": (torch.float32, L.F32)}[dt]
    g = torch.Generator().manual_seed(npix * 7 + c)
    z = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    gy = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    sc = (torch.rand(c, generator=g) + 0.5).cuda()
    sh = (torch.randn(c, generator=g) * 0.2).cuda()
    mi = torch.cat([torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5]).cuda()
    rows = L.lib().yms_bn_bwd_rows(npix, c)
    ws = torch.full((rows + 4, 2, c), float("nan"), device="cuda")
    L.call("yms_bn_act_bwd_reduce", code, npix, c, z.data_ptr() if has_z else None, ld, off, gy.data_ptr(), ld,
           off, sc.data_ptr(), sh.data_ptr(), mi.data_ptr(), 1, ws.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.isnan(ws[rows:]).all() and torch.isfinite(ws[:rows]).all()
    tot = ws[:rows].double().sum(0).cpu()
    gg = gy[:, off:off + c].double().cpu()
    if not has_z:
        assert ((tot[0] - gg.sum(0)).norm() / gg.sum(0).norm()).item() < 1e-5
        return
    zz = z[:, off:off + c].double().cpu()
    a = zz * sc.double().cpu() + sh.double().cpu()
    s = torch.sigmoid(a)
    da = gg * (s * (1 + a * (1 - s)))
    xh = (zz - mi[:c].double().cpu()) * mi[c:].double().cpu()
    assert ((tot[0] - da.sum(0)).norm() / da.sum(0).norm()).item() < 1e-5
    assert ((tot[1] - (da * xh).sum(0)).norm() / (da * xh).sum(0).norm()).item() < 1e-5


@pytest.mark.parametrize("npix,c,ld", [(44801, 64, 64), (3001, 40, 48), (25600, 768, 776), (999, 24, 32)])
@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("gres_mode", [0, 1, 2])          # no residual gradient / store / accumulate
@pytest.mark.parametrize("inplace", [False, True])         # dz written over z (the plan's default)
def test_bn_bwd_apply_matches_fp64(npix, c, ld, dt, gres_mode, inplace):
    """The software-pipelined apply pass against fp64 of the same formula: dz = scale (da - coef0 -
    xhat coef1) and the residual gradient (gy, or r + gy), including dz over z in place and an
    accumulated residual gradient (masked stores: a clamped duplicate pixel is never written twice);
    the pad columns past c stay untouched."""
    tdt, code = {"bf16": (torch.bfloat16, L.BF16), "f32": (torch.float32, L.F32)}[dt]
    g = torch.Generator().manual_seed(npix + c + gres_mode)
    z0 = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    gy = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    r0 = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    sc = (torch.rand(c, generator=g) + 0.5).cuda()
    sh = (torch.randn(c, generator=g) * 0.2).cuda()
    mi = torch.cat([torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5]).cuda()
    coef = (torch.randn(2 * c, generator=g) * 0.1).cuda()
    z = z0.clone()
    dz = z if inplace else torch.full_like(z0, 7.0)
    r = r0.clone()
    L.call("yms_bn_act_bwd_apply", code, npix, c, z.data_ptr(), ld, 0, gy.data_ptr(), ld, 0, sc.data_ptr(),
           sh.data_ptr(), mi.data_ptr(), coef.data_ptr(), 1, dz.data_ptr(), ld, 0,
           r.data_ptr() if gres_mode else None, ld, 0, int(gres_mode == 2), L.stream_ptr())
    torch.cuda.synchronize()
    zz, gg = z0[:, :c].double().cpu(), gy[:, :c].double().cpu()
    scd, cf = sc.double().cpu(), coef.double().cpu()
    a = zz * scd + sh.double().cpu()
    s = torch.sigmoid(a)
    da = gg * (s * (1 + a * (1 - s)))
    xh = (zz - mi[:c].double().cpu()) * mi[c:].double().cpu()
    ref = scd * (da - cf[:c] - xh * cf[c:])
    got = dz.double().cpu()
    tol = 1e-5 if dt == "f32" else 1e-2
    assert ((got[:, :c] - ref).abs().max() <= tol * (1 + ref.abs().max())).item()
    pad = z0 if inplace else torch.full_like(z0, 7.0)
    assert torch.equal(dz[:, c:], pad[:, c:])
    rr = r.double().cpu()
    if gres_mode == 0:
        assert torch.equal(r, r0)
    else:
        want = gy[:, :c].double().cpu() + (r0[:, :c].double().cpu() if gres_mode == 2 else 0)
        assert torch.equal(rr[:, :c], want.to(tdt).double())
        assert torch.equal(r[:, c:], r0[:, c:])


@pytest.mark.parametrize("npix,c,ld", [(44801, 64, 64), (3001, 40, 48), (25600, 768, 776), (999, 24, 32)])
@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("res_mode", [0, 1, 2])            # no residual / residual / y written over the residual
def test_affine_act_matches_fp64(npix, c, ld, dt, res_mode):
    """The software-pipelined forward BN+SiLU(+res) pass against fp64 of the same formula, ragged
    pixel counts and an in-place residual included; pad columns untouched."""
    tdt, code = {"bf16": (torch.bfloat16, L.BF16), "f32": (torch.float32, L.F32)}[dt]
    g = torch.Generator().manual_seed(npix + c + res_mode)
    z = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    r0 = torch.randn(npix, ld, generator=g).to(tdt).cuda()
    sc = (torch.rand(c, generator=g) + 0.5).cuda()
    sh = (torch.randn(c, generator=g) * 0.2).cuda()
    r = r0.clone()
    y = r if res_mode == 2 else torch.full_like(z, 7.0)
    L.call("yms_affine_act", code, npix, c, z.data_ptr(), ld, 0, sc.data_ptr(), sh.data_ptr(), 1,
           r.data_ptr() if res_mode else None, ld, 0, y.data_ptr(), ld, 0, L.stream_ptr())
    torch.cuda.synchronize()
    ref = F_silu(z[:, :c].double().cpu() * sc.double().cpu() + sh.double().cpu())
    if res_mode:
        ref = ref + r0[:, :c].double().cpu()
    got = y.double().cpu()
    tol = 1e-6 if dt == "f32" else 1e-2
    assert ((got[:, :c] - ref).abs().max() <= tol * (1 + ref.abs().max())).item()
    pad = r0 if res_mode == 2 else torch.full_like(z, 7.0)
    assert torch.equal(y[:, c:], pad[:, c:])


def F_silu(a):
    return a * torch.sigmoid(a)
