"""Per-layer conv timing vs roofline for one forward (and optionally train step) (dev tool)."""
import os, sys, ctypes
os.environ.setdefault("YMS_WGRAD_STREAM", "0")   # events below are recorded on the current stream
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import _lib as L, set_compute_dtype
from yolov8.yolov8 import YOLOv8

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
mode = sys.argv[2] if len(sys.argv) > 2 else "infer"
m = YOLOv8("s", 80).cuda()
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(B, 3, 640, 640, device="cuda")
recs = []
orig = L.call
def call(name, *args):
    if name not in ("yms_conv_fwd", "yms_conv_dgrad", "yms_conv_wgrad"):
        return orig(name, *args)
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record(); orig(name, *args); e.record()
    sh = args[0].contents
    recs.append((name, sh.n, sh.h, sh.w, sh.cin, sh.cout, sh.k, sh.stride, sh.ho, sh.wo, s, e))
if mode == "infer":
    m.eval()
    for _ in range(3): m(x)
    L.call = call
    m(x)
else:
    m.train()
    for _ in range(2): sum((o.float()**2).mean() for o in m(x)).backward()
    L.call = call
    sum((o.float()**2).mean() for o in m(x)).backward()
torch.cuda.synchronize()
L.call = orig
tot_t = 0; tot_f = 0
print(f"{'op':6s} {'cin':>5s} {'cout':>5s} k s {'Ho':>4s} {'us':>8s} {'TF/s':>7s} {'GB/s':>7s} {'roof_us':>8s} {'eff':>5s}")
for r in recs:
    name, n, h, w, ci, co, k, st, ho, wo, s, e = r
    us = s.elapsed_time(e) * 1e3
    fl = 2 * n * ho * wo * co * ci * k * k
    by = 2 * (n * h * w * ci + n * ho * wo * co + co * ci * k * k)
    if name == "yms_conv_fwd" and mode == "train": by += 2 * n * ho * wo * co   # z store
    roof = max(fl / 2.5e15, by / 6.0e12) * 1e6
    tot_t += us; tot_f += fl
    print(f"{name[9:15]:6s} {ci:5d} {co:5d} {k} {st} {ho:4d} {us:8.1f} {fl/us/1e6:7.1f} {by/us/1e3:7.0f} {roof:8.1f} {roof/us:5.2f}")
print(f"total {tot_t/1e3:.2f} ms  {tot_f/tot_t/1e6:.1f} TF/s")
