"""ctypes binding of libyms.so (C-ABI declared in include/yms.h).

The HIP library is mandatory: there is no CPU or eager-PyTorch fallback.  If the
shared object is missing or a call returns a non-zero status, a RuntimeError is
raised immediately.  torch must be imported before the library is loaded so that
libyms.so binds to the HIP runtime already loaded by torch (same soname).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the process' HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YMS_LIB") or os.path.join(_HERE, "libyms.so")   # YMS_LIB: dev A/B builds (tools/ab_lib.sh)

F32, BF16, F16 = 0, 1, 2
ACT_NONE, ACT_SILU = 0, 1

_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}


def dtype_code(dt):
    try:
        return _DT[dt]
    except KeyError:
        raise RuntimeError(f"yms: unsupported dtype {dt}; use float32, bfloat16 or float16") from None


class ConvShape(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in
                ("n", "h", "w", "cin", "cout", "k", "stride", "pad", "ho", "wo", "dtype")]


class DwShape(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("n", "h", "w", "c", "k", "dtype")]


class PackJob(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("packed", ctypes.c_void_p)] + [
        (k, ctypes.c_int) for k in ("cout", "cin", "ks", "rows", "kp_elems", "c8_in", "for_dgrad", "dtype")] + [
        ("w2", ctypes.c_void_p), ("split", ctypes.c_int)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_D = ctypes.c_double
_SZ = ctypes.c_size_t
_SP = ctypes.POINTER(ConvShape)
_DP = ctypes.POINTER(DwShape)

_SIGS = {
    "yms_version": (ctypes.c_char_p, []),
    "yms_status_string": (ctypes.c_char_p, [_I]),
    "yms_conv_packed_elems": (_SZ, [_SP, _I]),
    "yms_conv_pack_weight": (_I, [_SP, _P, _P, _I, _P]),
    "yms_pack_job_init": (_I, [_SP, _P, _P, _I, ctypes.POINTER(PackJob)]),
    "yms_conv_pack_weights_batched": (_I, [_I, _P, _P, _P]),
    "yms_conv_stats_rows": (_I, [_SP]),
    "yms_conv_stats_ld": (_I, [_SP]),
    "yms_conv_direct_set": (_I, [_I]),
    "yms_conv_fwd": (_I, [_SP, _P, _I, _I, _P, _P, _I, _I, _P, _P, _I, _P, _I, _I, _P, _P]),
    "yms_conv_stem_supported": (_I, [_SP]),
    "yms_conv_stem_stats_rows": (_I, [_SP]),
    "yms_conv_stem_fwd": (_I, [_SP, _P, _P, _P, _I, _I, _P, _P, _I, _P, _I, _P]),
    "yms_conv_stem_wgrad_ws_bytes": (_SZ, [_SP]),
    "yms_conv_stem_wgrad": (_I, [_SP, _P, _P, _I, _I, _P, _I, _I, _P, _P, _P, _P, _I, _P, _SZ, _P, _I, _P]),
    "yms_conv_dgrad": (_I, [_SP, _P, _I, _I, _P, _P, _I, _I, _I, _P]),
    "yms_conv_dgrad_bnred_rows": (_I, [_SP]),
    "yms_conv_dgrad_bnred": (_I, [_SP, _P, _I, _I, _P, _P, _I, _I, _I, _P, _I, _I, _P, _P, _P, _I, _P, _P]),
    "yms_conv_wgrad_ws_bytes": (_SZ, [_SP]),
    "yms_conv_wgrad": (_I, [_SP, _P, _I, _I, _P, _I, _I, _P, _SZ, _P, _I, _P]),
    "yms_bn_fold": (_I, [_I, _P, _P, _P, _P, _F, _P, _P, _P]),
    "yms_bn_finalize": (_I, [_I, _P, _I, _I, _L, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P]),
    "yms_bn_finalize_ld": (_I, [_I, _P, _I, _I, _L, _P, _P, _P, _P, _F, _F, _P, _I, _P, _P, _P]),
    "yms_affine_act": (_I, [_I, _L, _I, _P, _I, _I, _P, _P, _I, _P, _I, _I, _P, _I, _I, _P]),
    "yms_bn_bwd_rows": (_I, [_L, _I]),
    "yms_bn_act_bwd_reduce": (_I, [_I, _L, _I, _P, _I, _I, _P, _I, _I, _P, _P, _P, _I, _P, _P]),
    "yms_bn_act_bwd_finalize": (_I, [_I, _P, _I, _L, _P, _P, _P, _P]),
    "yms_bn_act_bwd_apply": (_I, [_I, _L, _I, _P, _I, _I, _P, _I, _I, _P, _P, _P, _P, _I, _P, _I, _I,
                                  _P, _I, _I, _I, _P]),
    "yms_bn_act_bwd_reduce_finalize": (_I, [_I, _L, _I, _P, _I, _I, _P, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P,
                                            _P, _P]),
    "yms_bias_bwd": (_I, [_I, _L, _I, _P, _I, _I, _P, _P, _P, _P]),
    "yms_sppf_ws_bytes": (_SZ, [_I, _I, _I, _I]),
    "yms_sppf_pool_fwd": (_I, [_I, _I, _I, _I, _I, _P, _I, _I, _P]),
    "yms_sppf_pool_bwd": (_I, [_I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _P]),
    "yms_upsample2x_fwd": (_I, [_I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P]),
    "yms_upsample2x_bwd": (_I, [_I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _I, _P]),
    "yms_pack_input": (_I, [_I, _I, _I, _I, _I, _P, _P, _I, _P]),
    "yms_nhwc_to_nchw": (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _P]),
    "yms_nchw_to_nhwc": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _I, _I, _I, _P]),
    "yms_cast": (_I, [_I, _I, _L, _P, _P, _P]),
    "yms_zero": (_I, [_P, _SZ, _P]),
    "yms_copy": (_I, [_P, _P, _SZ, _P]),
    "yms_dwconv_stats_rows": (_I, [_DP]),
    "yms_dwconv_fwd": (_I, [_DP, _P, _I, _I, _P, _P, _I, _I, _P, _P, _I, _P, _I, _P]),
    "yms_dwconv_dgrad": (_I, [_DP, _P, _I, _I, _P, _P, _I, _I, _I, _P]),
    "yms_dwconv_wgrad_ws_bytes": (_SZ, [_DP]),
    "yms_dwconv_wgrad": (_I, [_DP, _P, _I, _I, _P, _I, _I, _P, _SZ, _P, _I, _P]),
    "yms_add_views": (_I, [_I, _L, _I, _P, _I, _I, _P, _I, _I, _P, _I, _I, _I, _P]),
    "yms_add_grad2": (_I, [_I, _L, _I, _P, _I, _I, _P, _I, _I, _I, _P, _I, _I, _I, _P]),
    "yms_map_match": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "yms_map_accumulate": (_I, [_I, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "yms_det_loss_ws_bytes": (_SZ, [_I, _I, _I, _I]),
    "yms_stream_create_cu_subset": (_I, [_I, _I, ctypes.POINTER(ctypes.c_void_p)]),
    "yms_resize_normalize": (_I, [_I, _I, _P, _I, _I, _P, _P, _P, _P]),
    "yms_augment_image_bytes": (_SZ, []),
    "yms_augment_normalize": (_I, [_I, _I, _P, _I, _I, _P, _P, _P, _P]),
    "yms_det_loss": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _I, _F, _F, _I, _P, _P, _P, _SZ, _P, _P]),
    "yms_scale_by_device_scalar": (_I, [_I, _I, _P, _P, _P, _P]),
    "yms_head_decode": (_I, [_I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _F, _P, _P, _P, _P]),
    "yms_dfl": (_I, [_I, _I, _I, _I, _P, _P, _P]),
    "yms_nms_prep": (_I, [_I, _I, _I, _P, _F, _P, _P, _P, _P]),
    "yms_nms_ws_bytes": (_SZ, [_I, _I, _I]),
    "yms_nms_ws_bytes_min": (_SZ, [_I, _I, _I]),
    "yms_nms_classwise": (_I, [_I, _I, _I, _P, _P, _P, _D, _P, _P, _P, _P, _SZ, _P]),
    "yms_nms_single": (_I, [_I, _P, _P, _D, _P, _P, _P, _SZ, _P]),
}

EXPORTED = tuple(_SIGS)
_lib = None


def lib():
    """Load libyms.so (raises RuntimeError when the HIP extension has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"yms: HIP library {LIB_PATH} not found -- build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C yolo-ms_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, what):
    if status != 0:
        msg = lib().yms_status_string(status).decode()
        raise RuntimeError(f"yms: {what} failed: {msg} (status {status})")


_prof = None
_CONV = ("yms_conv_fwd", "yms_conv_dgrad", "yms_conv_dgrad_bnred", "yms_conv_wgrad", "yms_conv_stem_fwd")
_DW = ("yms_dwconv_fwd", "yms_dwconv_dgrad", "yms_dwconv_wgrad")
# launches whose hipStream_t is the last argument (status-returning entry points ending in a void*)
# (host-only entry points whose last pointer is a host buffer are listed out explicitly)
_HOST_ONLY = {"yms_map_accumulate", "yms_pack_job_init"}
_STREAM_LAST = {n for n, (res, args) in _SIGS.items()
                if res is _I and args and args[-1] is _P and n not in _HOST_ONLY}


_FN = {}


def _elt(dt):
    return 4 if dt == F32 else 2


def _work(name, args):
    """(algorithmic FLOPs, algorithmic HBM bytes) of one launch: every operand read or written once.
    Convs: input + output + weights (fp32 weight gradient); depthwise: the same with fp32 [C][k][k]
    weights (FLOPs = 2 n h w c k^2, VALU); BN / branch-sum elementwise passes: their streams."""
    if name in _CONV:
        sh = args[0].contents
        fl = 2 * sh.n * sh.ho * sh.wo * sh.cout * sh.cin * sh.k * sh.k
        es = _elt(sh.dtype)
        act = (sh.n * sh.h * sh.w * sh.cin + sh.n * sh.ho * sh.wo * sh.cout) * es
        if name == "yms_conv_dgrad_bnred":             # + the producer's z at the dx pixels
            act += sh.n * sh.h * sh.w * sh.cin * es
        return fl, act + sh.cout * sh.cin * sh.k * sh.k * (4 if name == "yms_conv_wgrad" else es)
    if name in _DW:
        d = args[0].contents
        vol = d.n * d.h * d.w * d.c
        return 2 * vol * d.k * d.k, 2 * vol * _elt(d.dtype) + 4 * d.c * d.k * d.k
    if name in ("yms_bn_act_bwd_reduce", "yms_affine_act", "yms_bn_act_bwd_apply", "yms_add_views",
                "yms_add_grad2"):
        vol = args[1] * args[2] * _elt(args[0])
        if name == "yms_bn_act_bwd_reduce":
            return 0, 2 * vol                                          # z, gy
        if name == "yms_affine_act":
            return 0, (2 + (args[9] is not None)) * vol                # z (+res) -> y
        if name == "yms_bn_act_bwd_apply":
            return 0, (3 + (args[17] is not None) * (1 + bool(args[20]))) * vol   # z, gy -> dz (+ gres)
        if name == "yms_add_views":
            return 0, (2 + (args[6] is not None) + bool(args[12])) * vol
        return 0, (3 + bool(args[9]) + bool(args[13])) * vol       # add_grad2: gy -> ga, gb
    return 0, 0


def call(name, *args):
    if _prof is None:
        fn = _FN.get(name)
        if fn is None:
            fn = _FN[name] = getattr(lib(), name)
        st = fn(*args)
        if st != 0:
            check(st, name)
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    # entry points take their hipStream_t last: time them on the stream they run on (weight
    # gradients run on the backward's side stream)
    st = torch.cuda.ExternalStream(args[-1]) if name in _STREAM_LAST and args[-1] else None
    s.record(st)
    check(getattr(lib(), name)(*args), name)
    e.record(st)
    fl, nb = _work(name, args)
    _prof.append((name, s, e, fl, nb))


def profile_begin():
    """Record a HIP event pair around every C-ABI launch (diagnostic): conv launches on the
    stream they are issued to, everything else on the current stream."""
    global _prof
    _prof = []


def profile_end(peak_tflops=2500.0, peak_gbs=8000.0, valu_tflops=157.3):
    """-> {name: [calls, total_ms, flops, bytes, roofline_ms, hbm_bound_calls]} for the launches
    since profile_begin().  roofline_ms sums, per launch, max(flops / peak, bytes / peak_gbs): the
    time the launch would take at the roofline of its own arithmetic intensity (peak = the dense
    MFMA rate for convs, the fp32 VALU rate for the depthwise kernels)."""
    global _prof
    torch.cuda.synchronize()
    out = {}
    for name, s, e, fl, nb in _prof:
        r = out.setdefault(name, [0, 0.0, 0, 0, 0.0, 0])
        r[0] += 1
        r[1] += s.elapsed_time(e)
        r[2] += fl
        r[3] += nb
        pk = valu_tflops if name in _DW else peak_tflops
        t_f, t_b = fl / (pk * 1e9), nb / (peak_gbs * 1e6)   # ms
        r[4] += max(t_f, t_b)
        r[5] += int(t_b > t_f)
    _prof = None
    return out


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()
