"""Dev tool: host enqueue time of a training step vs the GPU step time (is the launch path the
bottleneck?).  python tools/host_overhead.py [version]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import set_compute_dtype
from yolov8.yolov8 import YOLOv8
from yolov8.tools.loss import ComputeLoss
sys.path.insert(0, ROOT)
from bench import synth_targets

v = sys.argv[1] if len(sys.argv) > 1 else "s"
torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
m = YOLOv8(v, 80).cuda().train()
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(64, 3, 640, 640, device="cuda")
opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.937, nesterov=True, foreach=True)
crit = ComputeLoss(m.head, 80, "cuda", (640, 640))
tg = synth_targets(64, 80, 8, 1, "cuda")


def step():
    opt.zero_grad(set_to_none=True)
    crit.loss_tensor(m(x), tg)[0].backward()
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
N = 20
t0 = time.perf_counter()
host = []
for _ in range(N):
    a = time.perf_counter()
    step()
    host.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue per step {sum(host) / N * 1e3:.2f} ms (min {min(host) * 1e3:.2f}), "
      f"wall per step {(t2 - t0) / N * 1e3:.2f} ms, queue drained {(t2 - t1) * 1e3:.1f} ms after the last enqueue")
