"""Per-parameter gradient error of the HIP training path vs an fp64 CPU oracle (dev tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from oracle import model_ref as M
from yolov8.yolov8 import YOLOv8

v, nc = sys.argv[1] if len(sys.argv) > 1 else "s", 80
dt = {"bf16": torch.bfloat16, "f32": torch.float32, "f16": torch.float16}[sys.argv[2] if len(sys.argv) > 2 else "bf16"]
H = int(sys.argv[3]) if len(sys.argv) > 3 else 128
sd = M.init_params(v, nc)
x = torch.randn(2, 3, H, H, generator=torch.Generator().manual_seed(1))

def oracle(dtype):
    p = {k: (t.clone().to(dtype).requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else (t.clone().to(dtype) if t.is_floating_point() else t.clone()))
         for k, t in sd.items()}
    r = M.forward(p, v, nc, x.to(dtype), True)
    sum((o.double() ** 2).mean() for o in r).backward()
    return {k: t.grad.double() for k, t in p.items() if t.grad is not None}, [o.detach().double() for o in r]

g64, o64 = oracle(torch.float64)
g32, o32 = oracle(torch.float32)
m = YOLOv8(v, nc).cuda()
m.load_state_dict(sd)
m.train()
if dt != torch.float32:
    with torch.autocast("cuda", dtype=dt):
        outs = m(x.cuda())
else:
    outs = m(x.cuda())
sum((o.double() ** 2).mean() for o in outs).backward()
pd = dict(m.named_parameters())
def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()
for i, (o, r, r32) in enumerate(zip(outs, o64, o32)):
    print(f"out{i}: gpu rel {rel(o.detach().double().cpu(), r):.2e}  cpu32 rel {rel(r32, r):.2e}")
rows = []
for k in g64:
    if k not in pd:
        continue
    rows.append((rel(pd[k].grad.double().cpu(), g64[k]), rel(g32[k], g64[k]), k, g64[k].norm().item()))
rows.sort(reverse=True)
for r in rows[:25]:
    print(f"{r[0]:.2e} (cpu32 {r[1]:.2e}) |g|={r[3]:.2e} {r[2]}")
print("median gpu rel", sorted(x[0] for x in rows)[len(rows)//2])
