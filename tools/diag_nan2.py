"""Dev: the sibling test's sequence (fp32 fused / unfused, then bf16) with NaN checks per step."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import set_compute_dtype
from yolov8.yolov8 import YOLOv8

v, nc, size = "n", 3, 192
torch.manual_seed(0)
sd = YOLOv8(v, nc).state_dict()
x = torch.randn(2, 3, size, size, generator=torch.Generator().manual_seed(1)).cuda()
for fuse, dt in [(1, torch.float32), (0, torch.float32), (1, torch.bfloat16), (0, torch.bfloat16), (1, torch.bfloat16)]:
    os.environ["YMS_HEAD_FUSE"] = str(fuse)
    m = YOLOv8(v, nc).cuda()
    m.load_state_dict(sd)
    m.train()
    if dt != torch.float32:
        set_compute_dtype(m, dt)
    outs = m(x)
    g = torch.Generator(device="cuda").manual_seed(3)
    sum((o.float() * torch.randn(o.shape, device="cuda", generator=g)).sum() for o in outs).backward()
    torch.cuda.synchronize()
    bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    mx = max(p.grad.abs().max().item() for p in m.named_parameters().__iter__().__next__()[1:] if p.grad is not None) if False else None
    big = sorted(((p.grad.float().abs().max().item(), k) for k, p in m.named_parameters() if p.grad is not None), reverse=True)[:3]
    print(fuse, dt, "outs finite", [bool(torch.isfinite(o.float()).all()) for o in outs], "nonfinite", len(bad), bad[:4], big, flush=True)
