"""Class-segment size statistics of the bench's inference input (random-init YOLOv8-s).
Usage: nms_stats.py [size=640] [batch=32] [bf16|f16]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import set_compute_dtype
from yms import ops as yops
from yolov8.yolov8 import YOLOv8
torch.manual_seed(0)
m = YOLOv8("s", 80).cuda().eval()
m.head.stride = torch.tensor([8.0, 16.0, 32.0])
S = int(sys.argv[1]) if len(sys.argv) > 1 else 640
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
DT = torch.float16 if len(sys.argv) > 3 and sys.argv[3] == "f16" else torch.bfloat16
set_compute_dtype(m, DT)
x = torch.randn(B, 3, S, S, device="cuda", generator=torch.Generator(device="cuda").manual_seed(99))
y = m(x)
bxy, score, keep, klbl, counts = yops.batched_nms_indices(y, 0.25, 0.45)
sc, lab = y[..., 4:].max(-1)
lab[sc <= 0.25] = -1
for b in range(min(B, 4)):
    cnt = torch.bincount(lab[b][lab[b] >= 0], minlength=80)
    big = cnt[cnt > 1024]
    print(f"img {b}: cand {int((lab[b] >= 0).sum())} kept {int(counts[b])} max seg {int(cnt.max())} "
          f"big segs {big.tolist()} segs>0 {int((cnt > 0).sum())}")
tot = torch.stack([torch.bincount(lab[b][lab[b] >= 0], minlength=80) for b in range(B)])
print("sum of n^2 over segments per image (M pairs):", (tot.double() ** 2).sum(1).mean().item() / 1e6)
print("kept per image:", counts.float().mean().item())
