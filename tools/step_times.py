"""Dev tool: per-step wall times of the training step (synchronize after each step), to find
outlier steps.   python tools/step_times.py [version] [steps] [batch]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
import bench
from yms import set_compute_dtype
from yolov8.tools.loss import ComputeLoss
from yolov8.yolov8 import YOLOv8

v = sys.argv[1] if len(sys.argv) > 1 else "ms-l"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = YOLOv8(v, 80).to(dev)
m.head.stride = torch.tensor([8.0, 16.0, 32.0])
set_compute_dtype(m, torch.bfloat16)
m.train()
opt = bench.make_sgd(m.parameters())
x = torch.randn(B, 3, 640, 640, device=dev)
crit = ComputeLoss(m.head, 80, dev, (640, 640))
tg = bench.synth_targets(B, 80, 8, 4321, dev)
for i in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    crit.loss_tensor(m(x), tg)[0].backward()
    t1 = time.perf_counter()
    opt.step()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {i:2d}: host enqueue {1e3 * (t1 - t0):8.1f} ms, total {1e3 * (t2 - t0):8.1f} ms, "
          f"reserved {torch.cuda.memory_reserved() / 2**30:6.1f} GiB", flush=True)
