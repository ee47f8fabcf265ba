"""Test helpers: drive single C-ABI ops of libyms.so on torch tensors (test infra only)."""
import ctypes

import torch
import torch.nn.functional as F

from yms import _lib as L

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def r8(c):
    return (c + 7) // 8 * 8


def nhwc(x, dtype, ld=None, off=0):
    """NCHW fp32 -> zero-padded NHWC [n,h,w,ld] buffer of dtype with x at channel offset off."""
    n, c, h, w = x.shape
    ld = ld or r8(off + c)
    buf = torch.zeros((n, h, w, ld), dtype=dtype, device="cuda")
    buf[..., off:off + c] = x.permute(0, 2, 3, 1).to(dtype)
    return buf


def nchw(buf, c, off=0):
    return buf[..., off:off + c].permute(0, 3, 1, 2).float()


def shape(n, h, w, cin, cout, k, s, dtype):
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    return L.ConvShape(n, h, w, cin, cout, k, s, p, ho, wo, L.dtype_code(dtype))


def pack(w, sh, dtype, for_dgrad):
    sp = ctypes.pointer(sh)
    out = torch.empty(L.lib().yms_conv_packed_elems(sp, for_dgrad), dtype=dtype, device="cuda")
    wc = w.float().contiguous().cuda()
    L.call("yms_conv_pack_weight", sp, wc.data_ptr(), out.data_ptr(), for_dgrad, L.stream_ptr())
    return out


def conv_fwd(xb, w, sh, dtype, scale=None, shift=None, act=0, res=None, stats=False, yld=None, yoff=0,
             xoff=0):
    sp = ctypes.pointer(sh)
    wp = pack(w, sh, dtype, 0)
    yld = yld or r8(yoff + sh.cout)
    y = torch.zeros((sh.n, sh.ho, sh.wo, yld), dtype=dtype, device="cuda")
    st, buf = None, None
    if stats:
        rows, ld = L.lib().yms_conv_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
        buf = stats_buffer(rows, ld)
        st = split_stats(buf, rows, ld)
    L.call("yms_conv_fwd", sp, xb.data_ptr(), xb.shape[-1], xoff, wp.data_ptr(), y.data_ptr(), yld, yoff,
           L.ptr(scale), L.ptr(shift), act, L.ptr(res), res.shape[-1] if res is not None else 0, 0,
           L.ptr(buf), L.stream_ptr())
    return y, st


def stats_buffer(rows, ld):
    """BN statistics workspace: [rows][2][ld] moments + [rows] pixel counts, NaN-filled so a row the
    producer did not write shows up."""
    return torch.full((rows * (2 * ld + 1),), float("nan"), dtype=torch.float32, device="cuda")


def split_stats(buf, rows, ld):
    """-> (moment rows [rows, 2, ld], counts [rows]) views of a statistics workspace."""
    return buf[:rows * 2 * ld].view(rows, 2, ld), buf[rows * 2 * ld:]


def merge_moments(st, c, npix):
    """BN statistics (moment rows [rows][2][ld] = (sum z, sum (z - row mean)^2) over n_r pixels,
    counts [rows] = n_r) -> (sum z, M2 about the global mean) per channel, fp64 on the host.  Every
    row must have been written, and the counts must add up to npix."""
    rows_, counts = st
    rows_, n = rows_.double().cpu(), counts.double().cpu().view(-1, 1)
    assert torch.isfinite(rows_[:, :, :c]).all() and torch.isfinite(n).all()
    assert n.sum().item() == npix, (n.sum().item(), npix)
    s1, m2 = rows_[:, 0, :c], rows_[:, 1, :c]
    mean = s1.sum(0) / npix
    keep = (n > 0).view(-1)
    s1, m2, n = s1[keep], m2[keep], n[keep]
    return s1.sum(0), (m2 + n * (s1 / n - mean) ** 2).sum(0)


def check_moments(st, z, tol):
    """Statistics (moment rows, counts) of the pre-BN tensor z (NCHW fp32) against its exact sum
    and centred M2."""
    c = z.shape[1]
    npix = z.numel() // c
    s1, m2 = merge_moments(st, c, npix)
    zd = z.double()                       # on z's device; only the per-channel sums come back
    ref1 = zd.sum((0, 2, 3)).cpu()
    ref2 = ((zd - zd.mean((0, 2, 3), keepdim=True)) ** 2).sum((0, 2, 3)).cpu()
    del zd
    e1 = ((s1 - ref1).abs().max() / (ref1.abs().max() + 1e-6)).item()
    e2 = ((m2 - ref2).abs() / ref2.clamp_min(1e-30)).max().item()
    assert e1 <= tol and e2 <= tol, (e1, e2)


def ref_conv(x, w, s, dtype):
    """fp32 conv on operands rounded to `dtype` (what the MFMA path multiplies)."""
    xr = x.to(dtype).float()
    wr = w.to(dtype).float()
    return F.conv2d(xr, wr, None, s, w.shape[-1] // 2)
