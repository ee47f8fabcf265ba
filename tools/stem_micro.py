"""Dev tool: stem conv in isolation -- yms_conv_stem_fwd (NCHW fp32 in) against the generic
yms_pack_input + yms_conv_fwd pair, B=32/64 at 640, bf16, eval (BN+SiLU) and train (stats)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import torch
from yms import _lib as L
from hiputil import shape, pack

st = L.stream_ptr()
for n in (32, 64):
    sh = shape(n, 640, 640, 3, 32, 3, 2, torch.bfloat16)
    sp = ctypes.pointer(sh)
    x = torch.randn(n, 3, 640, 640, device="cuda")
    w = torch.randn(32, 3, 3, 3, device="cuda") * 0.3
    xp = torch.zeros(n, 640, 640, 8, dtype=torch.bfloat16, device="cuda")
    wp = pack(w, sh, torch.bfloat16, 0)
    y = torch.empty(n, 320, 320, 32, dtype=torch.bfloat16, device="cuda")
    sc, sf = torch.ones(32, device="cuda"), torch.zeros(32, device="cuda")
    rows = max(L.lib().yms_conv_stem_stats_rows(sp), L.lib().yms_conv_stats_rows(sp))
    stats = torch.empty(rows * (2 * 128 + 1), device="cuda")
    ops = {
        "pack_input": lambda: L.call("yms_pack_input", L.BF16, n, 3, 640, 640, x.data_ptr(), xp.data_ptr(), 8, st),
        "conv_fwd eval": lambda: L.call("yms_conv_fwd", sp, xp.data_ptr(), 8, 0, wp.data_ptr(), y.data_ptr(), 32, 0,
                                        sc.data_ptr(), sf.data_ptr(), 1, None, 0, 0, None, st),
        "conv_fwd stats": lambda: L.call("yms_conv_fwd", sp, xp.data_ptr(), 8, 0, wp.data_ptr(), y.data_ptr(), 32, 0,
                                         None, None, 0, None, 0, 0, stats.data_ptr(), st),
        "stem eval": lambda: L.call("yms_conv_stem_fwd", sp, x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 0,
                                    sc.data_ptr(), sf.data_ptr(), 1, None, 0, st),
        "stem stats": lambda: L.call("yms_conv_stem_fwd", sp, x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 0,
                                     None, None, 0, stats.data_ptr(), 128, st),
    }
    for name, fn in ops.items():
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 50
        nb = n * 3 * 640 * 640 * 4 + n * 320 * 320 * 32 * 2
        print(f"B={n} {name:15s} {us:8.1f} us   (stem algorithmic {nb / us / 1e3:6.0f} GB/s)", flush=True)

# training backward of the stem layer: fused yms_conv_stem_wgrad vs apply + (pack) + generic wgrad
for n in (64,):
    sh = shape(n, 640, 640, 3, 32, 3, 2, torch.bfloat16)
    sp = ctypes.pointer(sh)
    x = torch.randn(n, 3, 640, 640, device="cuda")
    xp = torch.zeros(n, 640, 640, 8, dtype=torch.bfloat16, device="cuda")
    z = torch.randn(n, 320, 320, 32, device="cuda").to(torch.bfloat16)
    gy = torch.randn(n, 320, 320, 32, device="cuda").to(torch.bfloat16)
    dz = torch.empty_like(z)
    sc, sf = torch.rand(32, device="cuda") + 0.5, torch.randn(32, device="cuda")
    mi = torch.cat([torch.zeros(32, device="cuda"), torch.ones(32, device="cuda")])
    coef = torch.zeros(64, device="cuda")
    dw = torch.empty(32, 3, 3, 3, device="cuda")
    wsf = torch.empty(L.lib().yms_conv_stem_wgrad_ws_bytes(sp) // 4 + 1, device="cuda")
    wsg = torch.empty(L.lib().yms_conv_wgrad_ws_bytes(sp) // 4 + 1, device="cuda")
    npix = n * 320 * 320
    ops = {
        "stem_wgrad fused": lambda: L.call("yms_conv_stem_wgrad", sp, x.data_ptr(), gy.data_ptr(), 32, 0, z.data_ptr(), 32,
                                           0, sc.data_ptr(), sf.data_ptr(), mi.data_ptr(), coef.data_ptr(), 1,
                                           wsf.data_ptr(), wsf.numel() * 4, dw.data_ptr(), 0, st),
        "bn apply": lambda: L.call("yms_bn_act_bwd_apply", L.BF16, npix, 32, z.data_ptr(), 32, 0, gy.data_ptr(), 32, 0,
                                   sc.data_ptr(), sf.data_ptr(), mi.data_ptr(), coef.data_ptr(), 1, dz.data_ptr(), 32, 0,
                                   None, 0, 0, 0, st),
        "generic wgrad": lambda: L.call("yms_conv_wgrad", sp, xp.data_ptr(), 8, 0, dz.data_ptr(), 32, 0, wsg.data_ptr(),
                                        wsg.numel() * 4, dw.data_ptr(), 0, st),
    }
    for name, fn in ops.items():
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"B={n} {name:17s} {s.elapsed_time(e) * 50:8.1f} us", flush=True)
