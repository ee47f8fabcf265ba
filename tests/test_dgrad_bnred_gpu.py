"""The producer's BN + SiLU backward reduce fused into the direct 3x3 input gradient's epilogue
(yms_conv_dgrad_bnred, csrc/conv_direct.hip): the input gradient dx is the producer's output
gradient gy (components.py:69-77 Conv feeding the next Conv; autograd of BatchNorm2d + SiLU).

Against the separate path on the same operands: yms_conv_dgrad (store / accumulate) followed by
yms_bn_act_bwd_reduce over (z, dx) and yms_bn_act_bwd_finalize.  dx must be bit-identical (the same
MFMA sums and rounding); dgamma / dbeta / the apply coefficients agree to fp32 summation order, and
both match an fp64 evaluation of the reduce formula on the stored dx.  Shapes: the stride-1 kernel
(tile widths 32 / 16, 32 / 64 reduction channels, 8..32 dx channels, ragged heights, channel slices
of wider buffers; 33..64 dx channels report 0 rows: two fragments' sums exceed the registers) and the stride-2 parity-class kernel (the stem's 320^2 32 <- 64 layer at reduced
batch, odd maps)."""
import ctypes

import pytest
import torch

from hiputil import DT, pack, r8, shape
from yms import _lib as L

pytestmark = pytest.mark.gpu

# (n, cin = dx channels, h, w, cout = reduction channels, stride, accumulate)
CASES = [
    (2, 32, 32, 64, 32, 1, 0),
    (2, 32, 40, 32, 64, 1, 0),
    (2, 32, 40, 32, 64, 1, 1),
    (2, 32, 23, 48, 64, 1, 1),
    (1, 24, 37, 16, 32, 1, 0),
    (3, 16, 16, 16, 64, 1, 1),
    (4, 32, 80, 80, 32, 1, 1),
    (2, 32, 160, 160, 32, 1, 0),
    (2, 32, 320, 320, 64, 2, 0),
    (2, 32, 64, 64, 64, 2, 1),
    (1, 32, 33, 63, 64, 2, 0),
    (2, 8, 30, 64, 32, 2, 0),
]


def _run(case, dt, act):
    n, cin, h, w, cout, s, acc = case
    dtype = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(sum(case) + act)
    sh = shape(n, h, w, cin, cout, 3, s, dtype)
    sp = ctypes.pointer(sh)
    if L.lib().yms_conv_dgrad_bnred_rows(sp) <= 0:
        pytest.skip("not a direct-kernel input-gradient shape")
    wt = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) / (cout * 9) ** 0.5
    wpt = pack(wt, sh, dtype, 1)
    dzld = r8(cout) + 8                                   # channel slice of a wider dz buffer
    dz = torch.randn(n, sh.ho, sh.wo, dzld, device="cuda", generator=g).to(dtype)
    dxld, dxoff = r8(cin) + 16, 8                         # dx at channel offset 8 of a wider buffer
    base = torch.randn(n, h, w, dxld, device="cuda", generator=g).to(dtype)
    zld, zoff = r8(cin) + 8, 8
    z = (torch.randn(n, h, w, zld, device="cuda", generator=g) * 1.5 + 0.3).to(dtype)
    sc = torch.rand(cin, device="cuda", generator=g) + 0.5
    shf = torch.randn(cin, device="cuda", generator=g) * 0.3
    mi = torch.cat([torch.randn(cin, device="cuda", generator=g) * 0.2, torch.rand(cin, device="cuda", generator=g) + 0.4])
    st = L.stream_ptr()
    npix = n * h * w
    # separate path
    dx0 = base.clone()
    L.call("yms_conv_dgrad", sp, dz.data_ptr(), dzld, 0, wpt.data_ptr(), dx0.data_ptr(), dxld, dxoff, acc, st)
    rows0 = L.lib().yms_bn_bwd_rows(npix, cin)
    ws0 = torch.full((rows0 * 2 * cin,), float("nan"), device="cuda")
    L.call("yms_bn_act_bwd_reduce", L.dtype_code(dtype), npix, cin, z.data_ptr(), zld, zoff, dx0.data_ptr(), dxld, dxoff,
           sc.data_ptr(), shf.data_ptr(), mi.data_ptr(), act, ws0.data_ptr(), st)
    out0 = torch.empty(4 * cin, device="cuda")
    L.call("yms_bn_act_bwd_finalize", cin, ws0.data_ptr(), rows0, npix, out0.data_ptr(), out0[cin:].data_ptr(),
           out0[2 * cin:].data_ptr(), st)
    # fused
    dx1 = base.clone()
    rows1 = L.lib().yms_conv_dgrad_bnred_rows(sp)
    ws1 = torch.full((rows1 * 2 * cin,), float("nan"), device="cuda")
    L.call("yms_conv_dgrad_bnred", sp, dz.data_ptr(), dzld, 0, wpt.data_ptr(), dx1.data_ptr(), dxld, dxoff, acc,
           z.data_ptr(), zld, zoff, sc.data_ptr(), shf.data_ptr(), mi.data_ptr(), act, ws1.data_ptr(), st)
    out1 = torch.empty(4 * cin, device="cuda")
    L.call("yms_bn_act_bwd_finalize", cin, ws1.data_ptr(), rows1, npix, out1.data_ptr(), out1[cin:].data_ptr(),
           out1[2 * cin:].data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0)                          # padding / other channels untouched alike
    assert torch.isfinite(ws1).all(), "a partial row was not written"
    # fp64 reduce of the stored dx
    gy = dx0[..., dxoff:dxoff + cin].double()
    zz = z[..., zoff:zoff + cin].double()
    a = zz * sc.double() + shf.double()
    da = gy * (torch.sigmoid(a) * (1 + a * (1 - torch.sigmoid(a)))) if act == 1 else gy
    xh = (zz - mi[:cin].double()) * mi[cin:].double()
    ref = torch.cat([(da * xh).sum((0, 1, 2)), da.sum((0, 1, 2))]).float()
    for got in (out1, out0):
        err = ((got[:2 * cin] - ref).abs() / (ref.abs().max() + 1e-6)).max().item()
        assert err <= 2e-5, err
    err = ((out1 - out0).abs() / (out0.abs().max() + 1e-6)).max().item()
    assert err <= 2e-5, err


@pytest.mark.parametrize("act", [1, 0])
@pytest.mark.parametrize("case", CASES)
def test_dgrad_bnred_bf16(case, act):
    _run(case, "bf16", act)


@pytest.mark.parametrize("case", CASES[:6] + CASES[9:])
def test_dgrad_bnred_f16(case):
    _run(case, "f16", 1)


def test_dgrad_bnred_rows_and_refusals():
    """Rows = the direct kernel's persistent blocks; shapes outside it (fp32, 128 reduction channels,
    widths off the tile grid, 64 dx channels) report 0 rows and the call returns YMS_ERR_UNSUPPORTED."""
    ok = shape(64, 160, 160, 32, 32, 3, 1, torch.bfloat16)
    assert 1 <= L.lib().yms_conv_dgrad_bnred_rows(ctypes.pointer(ok)) <= 64 * 5 * 20
    for bad in (shape(2, 80, 80, 32, 64, 3, 1, torch.float32), shape(2, 40, 40, 32, 128, 3, 1, torch.bfloat16),
                shape(2, 40, 40, 32, 64, 3, 1, torch.bfloat16), shape(2, 80, 80, 64, 64, 3, 1, torch.bfloat16)):
        sp = ctypes.pointer(bad)
        assert L.lib().yms_conv_dgrad_bnred_rows(sp) == 0
        t = torch.zeros(16, device="cuda")
        p = t.data_ptr()
        assert L.lib().yms_conv_dgrad_bnred(sp, p, r8(bad.cout), 0, p, p, r8(bad.cin), 0, 0, p, r8(bad.cin), 0,
                                            p, p, p, 1, p, None) == 2
