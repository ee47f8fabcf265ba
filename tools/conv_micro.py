"""Single-conv microbenchmark through the C-ABI (dev tool).
   python tools/conv_micro.py [reps]  -- prints us and TF/s per shape for fwd (affine), fwd (stats),
   dgrad and wgrad at bf16."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import torch
from yms import _lib as L
from hiputil import shape, pack, r8

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ONLY = sys.argv[2] if len(sys.argv) > 2 else ""
SHAPES = [  # n, h, w, cin, cout, k, s
    (64, 40, 40, 768, 256, 1, 1),
    (64, 40, 40, 128, 128, 3, 1),
    (64, 80, 80, 64, 64, 3, 1),
    (64, 160, 160, 32, 32, 3, 1),
    (64, 20, 20, 256, 256, 3, 1),
    (64, 80, 80, 128, 80, 3, 1),
    (64, 80, 80, 128, 64, 3, 1),
    (64, 40, 40, 256, 64, 3, 1),
    (64, 20, 20, 512, 80, 3, 1),
]
if os.environ.get("YMS_MICRO_SHAPES") == "ms":   # YOLO-MS-S MS-Block 1x1 convs (B=64)
    SHAPES = [(64, 160, 160, 64, 96, 1, 1), (64, 160, 160, 32, 64, 1, 1), (64, 160, 160, 64, 32, 1, 1),
              (64, 160, 160, 96, 64, 1, 1), (64, 80, 80, 128, 192, 1, 1), (64, 80, 80, 64, 128, 1, 1),
              (64, 80, 80, 128, 64, 1, 1), (64, 80, 80, 192, 128, 1, 1), (64, 40, 40, 128, 256, 1, 1),
              (64, 40, 40, 256, 128, 1, 1)]
if os.environ.get("YMS_MICRO_SHAPES") == "wg":   # every distinct 3x3 layer of YOLOv8-s at 640 (B=64)
    SHAPES = [(64, 640, 640, 3, 32, 3, 2), (64, 320, 320, 32, 64, 3, 2), (64, 160, 160, 32, 32, 3, 1),
              (64, 160, 160, 64, 128, 3, 2), (64, 80, 80, 64, 64, 3, 1), (64, 80, 80, 128, 256, 3, 2),
              (64, 40, 40, 128, 128, 3, 1), (64, 40, 40, 256, 512, 3, 2), (64, 20, 20, 256, 256, 3, 1),
              (64, 80, 80, 128, 128, 3, 2), (64, 40, 40, 256, 256, 3, 2), (64, 80, 80, 128, 64, 3, 1),
              (64, 80, 80, 128, 80, 3, 1), (64, 80, 80, 80, 80, 3, 1), (64, 40, 40, 256, 64, 3, 1),
              (64, 40, 40, 256, 80, 3, 1), (64, 20, 20, 512, 64, 3, 1), (64, 20, 20, 512, 80, 3, 1)]
if os.environ.get("YMS_MICRO_SHAPES") == "direct":   # the direct small-channel 3x3 kernel's layers
    SHAPES = [(64, 80, 80, 64, 64, 3, 1), (64, 160, 160, 32, 32, 3, 1), (8, 320, 320, 32, 32, 3, 1),
              (8, 160, 160, 64, 64, 3, 1), (64, 320, 320, 32, 64, 3, 2)]
dt = torch.bfloat16
st = L.stream_ptr()


def timeit(fn):
    for _ in range(3):
        fn()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / REPS


for (n, h, w, ci, co, k, s_) in SHAPES:
    sh = shape(n, h, w, ci, co, k, s_, dt)
    sp = ctypes.pointer(sh)
    x = torch.randn(n, h, w, r8(ci), device="cuda").to(dt)
    wt = torch.randn(co, ci, k, k, device="cuda") / (ci * k * k) ** 0.5
    wp = pack(wt, sh, dt, 0)
    wpt = pack(wt, sh, dt, 1)
    y = torch.empty(n, sh.ho, sh.wo, r8(co), device="cuda", dtype=dt)
    sc = torch.ones(co, device="cuda"); sf = torch.zeros(co, device="cuda")
    rows, ld = L.lib().yms_conv_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
    stt = torch.empty(rows * (2 * ld + 1), device="cuda")
    dz = torch.randn(n, sh.ho, sh.wo, r8(co), device="cuda").to(dt)
    dx = torch.empty_like(x)
    wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4 + 1, device="cuda")
    dw = torch.empty(co, ci, k, k, device="cuda")
    fl = 2.0 * n * sh.ho * sh.wo * co * ci * k * k
    ops = {
        "fwd": lambda: L.call("yms_conv_fwd", sp, x.data_ptr(), x.shape[-1], 0, wp.data_ptr(), y.data_ptr(),
                              y.shape[-1], 0, sc.data_ptr(), sf.data_ptr(), 1, None, 0, 0, None, st),
        "fwd_stats": lambda: L.call("yms_conv_fwd", sp, x.data_ptr(), x.shape[-1], 0, wp.data_ptr(), y.data_ptr(),
                                    y.shape[-1], 0, None, None, 0, None, 0, 0, stt.data_ptr(), st),
        "dgrad": lambda: L.call("yms_conv_dgrad", sp, dz.data_ptr(), dz.shape[-1], 0, wpt.data_ptr(), dx.data_ptr(),
                                dx.shape[-1], 0, 0, st),
        "wgrad": lambda: L.call("yms_conv_wgrad", sp, x.data_ptr(), x.shape[-1], 0, dz.data_ptr(), dz.shape[-1], 0,
                                ws.data_ptr(), wsb, dw.data_ptr(), 0, st),
    }
    for name, fn in ops.items():
        if ONLY and ONLY != name:
            continue
        us = timeit(fn)
        print(f"{name:9s} n{n} {h}x{w} {ci:4d}->{co:4d} k{k} s{s_}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
