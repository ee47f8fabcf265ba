"""Per-call timing of the BN / SiLU kernels of one training step (dev tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import _lib as L, set_compute_dtype
from yolov8.yolov8 import YOLOv8

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
m = YOLOv8("s", 80).cuda().train()
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(B, 3, 640, 640, device="cuda")
NAMES = ("yms_affine_act", "yms_bn_act_bwd_reduce", "yms_bn_act_bwd_apply", "yms_bn_finalize", "yms_bn_act_bwd_finalize")
recs = []
orig = L.call
def call(name, *args):
    if name not in NAMES:
        return orig(name, *args)
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record(); orig(name, *args); e.record()
    npix, c = (args[1], args[2]) if name != "yms_bn_finalize" and name != "yms_bn_act_bwd_finalize" else (args[4] if name == "yms_bn_finalize" else args[3], args[0])
    recs.append((name, npix, c, s, e))
for _ in range(2): sum((o.float()**2).mean() for o in m(x)).backward()
L.call = call
sum((o.float()**2).mean() for o in m(x)).backward()
torch.cuda.synchronize()
L.call = orig
EB = {"yms_affine_act": 4, "yms_bn_act_bwd_reduce": 4, "yms_bn_act_bwd_apply": 6, "yms_bn_finalize": 0, "yms_bn_act_bwd_finalize": 0}
agg = {}
for name, npix, c, s, e in recs:
    us = s.elapsed_time(e) * 1e3
    gb = EB[name] * npix * c / us / 1e3
    key = (name, npix * c > 20e6)
    a = agg.setdefault(key, [0, 0.0, 0.0])
    a[0] += 1; a[1] += us; a[2] += EB[name] * npix * c
    print(f"{name[4:]:22s} npix {npix:9d} c {c:4d} {us:8.1f} us {gb:7.0f} GB/s")
for (name, big), (n, us, by) in sorted(agg.items()):
    print(f"SUM {name[4:]:22s} {'big' if big else 'small'} calls {n:3d} {us/1e3:7.3f} ms  {by/us/1e3 if us else 0:6.0f} GB/s")
