"""Per-call timing of the training BN/SiLU kernels in one YOLOv8-s train step (dev tool).
   python tools/bn_layers.py [B]"""
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
NAMES = ("yms_affine_act", "yms_bn_act_bwd_reduce", "yms_bn_act_bwd_apply", "yms_bn_finalize",
         "yms_bn_act_bwd_finalize", "yms_sppf_pool_bwd", "yms_upsample2x_bwd", "yms_bias_bwd")
recs = []
orig = L.call
def call(name, *a):
    if name not in NAMES:
        return orig(name, *a)
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record(); orig(name, *a); e.record()
    recs.append((name, a, s, e))
for _ in range(2):
    sum((o.float() ** 2).mean() for o in m(x)).backward()
L.call = call
sum((o.float() ** 2).mean() for o in m(x)).backward()
torch.cuda.synchronize()
L.call = orig
tot = {}
print(f"{'op':24s} {'npix':>9s} {'c':>5s} {'us':>8s} {'GB/s':>7s}")
for name, a, s, e in recs:
    us = s.elapsed_time(e) * 1e3
    by = 0
    npix = c = 0
    if name == "yms_affine_act":
        npix, c = a[1], a[2]
        by = 2 * npix * c * (2 + (a[9] is not None and a[9] != 0))
    elif name == "yms_bn_act_bwd_reduce":
        npix, c = a[1], a[2]
        by = 2 * npix * c * 2
    elif name == "yms_bn_act_bwd_apply":
        npix, c = a[1], a[2]
        by = 2 * npix * c * 3
    tot.setdefault(name, [0, 0.0, 0])
    tot[name][0] += 1; tot[name][1] += us; tot[name][2] += by
    if by:
        print(f"{name[4:28]:24s} {npix:9d} {c:5d} {us:8.1f} {by / us / 1e3:7.0f}")
for k, (n, us, by) in tot.items():
    print(f"TOTAL {k:28s} calls {n:4d} {us / 1e3:8.3f} ms  {by / max(us, 1e-9) / 1e3:7.0f} GB/s")
