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
