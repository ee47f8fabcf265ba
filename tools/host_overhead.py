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

# per phase: host time to enqueue, and GPU time between events recorded at the phase boundaries
ph = {k: [] for k in ("fwd", "loss", "bwd", "opt")}
gp = {k: [] for k in ph}
for _ in range(N):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    opt.zero_grad(set_to_none=True)
    a = time.perf_counter(); ev[0].record()
    outs = m(x)
    b = time.perf_counter(); ev[1].record()
    loss = crit.loss_tensor(outs, tg)[0]
    c = time.perf_counter(); ev[2].record()
    loss.backward()
    d = time.perf_counter(); ev[3].record()
    opt.step()
    e = time.perf_counter(); ev[4].record()
    for k, (u, v) in zip(ph, ((a, b), (b, c), (c, d), (d, e))):
        ph[k].append(v - u)
    torch.cuda.synchronize()
    for i, k in enumerate(ph):
        gp[k].append(ev[i].elapsed_time(ev[i + 1]))
print("phase   host_ms  gpu_ms (median of %d)" % N)
for k in ph:
    print(f"{k:5s} {sorted(ph[k])[N // 2] * 1e3:8.2f} {sorted(gp[k])[N // 2]:8.2f}")
