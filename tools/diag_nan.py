"""Dev: which parameter gradients are non-finite after one bf16 train step (version, nc, size)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import set_compute_dtype
from yolov8.yolov8 import YOLOv8

for v, nc, size, dt in [("n", 3, 192, torch.bfloat16), ("n", 8, 192, torch.bfloat16), ("n", 80, 192, torch.bfloat16),
                        ("n", 3, 192, torch.float32), ("n", 3, 256, torch.bfloat16), ("s", 3, 192, torch.bfloat16)]:
    torch.manual_seed(0)
    m = YOLOv8(v, nc).cuda().train()
    if dt != torch.float32:
        set_compute_dtype(m, dt)
    x = torch.randn(2, 3, size, size, generator=torch.Generator().manual_seed(1)).cuda()
    outs = m(x)
    fin = [bool(torch.isfinite(o.float()).all()) for o in outs]
    g = torch.Generator(device="cuda").manual_seed(3)
    sum((o.float() * torch.randn(o.shape, device="cuda", generator=g)).sum() for o in outs).backward()
    torch.cuda.synchronize()
    bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    print(v, nc, size, dt, "outs finite", fin, "nonfinite grads", len(bad), bad[-6:], flush=True)
