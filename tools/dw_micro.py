"""Dev tool: depthwise k x k kernels in isolation (B=64 YOLO-MS-S shapes): us and GB/s."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import _lib as L

st = L.stream_ptr()
SHAPES = [(64, 160, 160, 64, 3), (64, 80, 80, 128, 5), (64, 40, 40, 256, 7), (64, 20, 20, 512, 9),
          (64, 80, 80, 64, 3), (64, 40, 40, 128, 3)]
if os.environ.get("YMS_MICRO_SHAPES") == "k9":
    SHAPES = [(64, 20, 20, 512, 9)]
if os.environ.get("YMS_MICRO_SHAPES") == "mss":   # YOLO-MS-S depthwise layers at B=64 (x2, x2, x2, x2, x4, x4)
    SHAPES = [(64, 160, 160, 64, 3), (64, 80, 80, 128, 5), (64, 40, 40, 256, 7), (64, 20, 20, 512, 9),
              (64, 80, 80, 384, 3), (64, 40, 40, 768, 3)]
if os.environ.get("YMS_MICRO_SHAPES") == "k79":   # VERDICT r04 item 6 shapes (YOLO-MS-S calibrated + round 3)
    SHAPES = [(64, 40, 40, 288, 7), (64, 20, 20, 288, 9), (64, 40, 40, 256, 7), (64, 20, 20, 512, 9)]
if os.environ.get("YMS_MICRO_SHAPES") == "mss4":   # round-4 YOLO-MS-S (calibrated) + the round-3 k >= 5 shapes
    SHAPES = [(64, 160, 160, 64, 3), (64, 80, 80, 160, 5), (64, 40, 40, 288, 7), (64, 20, 20, 288, 9),
              (64, 80, 80, 320, 3), (64, 40, 40, 576, 3), (64, 40, 40, 320, 3), (64, 20, 20, 576, 3),
              (64, 80, 80, 128, 5), (64, 40, 40, 256, 7), (64, 20, 20, 512, 9)]
if os.environ.get("YMS_MICRO_SHAPES") == "k3big":
    SHAPES = [(64, 160, 160, 64, 3)]
if os.environ.get("YMS_MICRO_SHAPES") == "msl":   # YOLO-MS-L backbone depthwise layers at B=64 (x4 each)
    SHAPES = [(64, 160, 160, 112, 3), (64, 80, 80, 224, 5), (64, 40, 40, 448, 7), (64, 20, 20, 384, 9),
              (64, 80, 80, 112, 3), (64, 40, 40, 224, 3), (64, 20, 20, 192, 3)]
# env variants timed side by side (each read per call): name=VAR:VAL,VAR:VAL;...
VARIANTS = [("default", {})]
if os.environ.get("YMS_DWM_VARIANTS"):
    VARIANTS = []
    for item in os.environ["YMS_DWM_VARIANTS"].split(";"):
        name, _, kv = item.partition("=")
        VARIANTS.append((name, dict(p.split(":") for p in kv.split(",") if p)))
if os.environ.get("YMS_DWM_OPS"):
    OPS = os.environ["YMS_DWM_OPS"].split(",")
else:
    OPS = None
for (n, h, w, c, k) in SHAPES:
    sh = L.DwShape(n, h, w, c, k, L.BF16)
    sp = ctypes.pointer(sh)
    x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    wt = torch.randn(c, 1, k, k, device="cuda")
    sc, sf = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    rows = L.lib().yms_dwconv_stats_rows(sp)
    stt = torch.empty(rows * (2 * c + 1), device="cuda")
    wsb = L.lib().yms_dwconv_wgrad_ws_bytes(sp)
    ws = torch.empty(wsb // 4 + 1, device="cuda")
    dw = torch.empty(c, 1, k, k, device="cuda")
    ops = {
        "dgrad0": lambda: L.call("yms_dwconv_dgrad", sp, x.data_ptr(), c, 0, wt.data_ptr(), y.data_ptr(), c, 0, 0, st),
        "fwd_noact": lambda: L.call("yms_dwconv_fwd", sp, x.data_ptr(), c, 0, wt.data_ptr(), y.data_ptr(), c, 0,
                                    None, None, 0, None, 0, st),
        "fwd": lambda: L.call("yms_dwconv_fwd", sp, x.data_ptr(), c, 0, wt.data_ptr(), y.data_ptr(), c, 0,
                              sc.data_ptr(), sf.data_ptr(), 1, None, 0, st),
        "fwd_stats": lambda: L.call("yms_dwconv_fwd", sp, x.data_ptr(), c, 0, wt.data_ptr(), y.data_ptr(), c, 0,
                                    None, None, 0, stt.data_ptr(), c, st),
        "dgrad": lambda: L.call("yms_dwconv_dgrad", sp, x.data_ptr(), c, 0, wt.data_ptr(), y.data_ptr(), c, 0, 0, st),
        "wgrad": lambda: L.call("yms_dwconv_wgrad", sp, x.data_ptr(), c, 0, y.data_ptr(), c, 0, ws.data_ptr(), wsb,
                                dw.data_ptr(), 0, st),
    }
    nb = x.numel() * 2 * 2
    for name, fn in ops.items():
        if OPS and name not in OPS:
            continue
        line = f"{name:9s} {n}x{h}x{w} c{c} k{k}:"
        for vname, env in VARIANTS:
            for a, b in env.items():
                os.environ[a] = b
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 100
            line += f"  {vname} {us:7.1f} us {nb / us / 1e3:5.0f} GB/s"
            for a in env:
                os.environ.pop(a, None)
        print(line, flush=True)
