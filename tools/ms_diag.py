"""Dev diagnostic: gradient drift vs fp64 of the GPU fp32 path and of the CPU fp32 oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from oracle import ms_ref as MS
from oracle import model_ref as MR
from yolov8.yolov8 import YOLOv8

v = sys.argv[1] if len(sys.argv) > 1 else "ms-xs"
h, w = int(sys.argv[2]), int(sys.argv[3])
BF16 = len(sys.argv) > 4 and sys.argv[4] == "bf16"
SEED = int(sys.argv[5]) if len(sys.argv) > 5 else 41
O = MS if v.startswith("ms-") else MR
sd = O.init_params(v, 80)
x = torch.randn(2, 3, h, w, generator=torch.Generator().manual_seed(SEED))


def cpu(dt, autocast=False):
    p = {k: (t.clone().to(dt).requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else (t.clone().to(dt) if t.is_floating_point() else t.clone())) for k, t in sd.items()}
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
        r = O.forward(p, v, 80, x.to(dt), True)
    sum((o.double() ** 2).mean() for o in r).backward()
    return {k: t.grad.double() for k, t in p.items() if t.grad is not None}


g64, g32 = cpu(torch.float64), cpu(torch.float32, BF16)
m = YOLOv8(v, 80).cuda()
m.load_state_dict(sd)
m.train()
with torch.autocast("cuda", dtype=torch.bfloat16, enabled=BF16):
    outs = m(x.cuda())
sum((o.double() ** 2).mean() for o in outs).backward()
pd = dict(m.named_parameters())
rel = lambda a, b: ((a.double().cpu() - b).norm() / (b.norm() + 1e-30)).item()
eg = sorted(rel(pd[k].grad, g64[k]) for k in g64)
ec = sorted(rel(g32[k], g64[k]) for k in g64)
n = len(eg)
tag = "bf16" if BF16 else "fp32"
print(f"{v} {h}x{w} seed {SEED}: GPU {tag} vs fp64 median {eg[n // 2]:.2e} p90 {eg[9 * n // 10]:.2e} max {eg[-1]:.2e} | "
      f"CPU {tag} vs fp64 median {ec[n // 2]:.2e} p90 {ec[9 * n // 10]:.2e} max {ec[-1]:.2e}")
