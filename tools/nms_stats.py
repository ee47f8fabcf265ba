"""Class-segment size statistics of the bench's inference input (random-init YOLOv8-s, B=32)."""
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
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(32, 3, 640, 640, device="cuda", generator=torch.Generator(device="cuda").manual_seed(99))
y = m(x)
bxy, score, keep, klbl, counts = yops.batched_nms_indices(y, 0.25, 0.45)
sc, lab = y[..., 4:].max(-1)
lab[sc <= 0.25] = -1
for b in range(4):
    cnt = torch.bincount(lab[b][lab[b] >= 0], minlength=80)
    big = cnt[cnt > 1024]
    print(f"img {b}: cand {int((lab[b] >= 0).sum())} kept {int(counts[b])} max seg {int(cnt.max())} "
          f"big segs {big.tolist()} segs>0 {int((cnt > 0).sum())}")
tot = torch.stack([torch.bincount(lab[b][lab[b] >= 0], minlength=80) for b in range(32)])
print("sum of n^2 over segments per image (M pairs):", (tot.double() ** 2).sum(1).mean().item() / 1e6)
print("kept per image:", counts.float().mean().item())
