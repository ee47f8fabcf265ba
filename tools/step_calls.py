"""Dev tool: run S training steps of a graph (bench.py's step: GPU ComputeLoss, SGD) and write the
yms_* launches of the LAST step (entry point, conv / depthwise shape) as JSON lines, so per-dispatch
rocprofv3 counters (--pmc, whose dispatch order matches the call order per stream) can be mapped to
layers:  rocprofv3 --pmc FETCH_SIZE -d D -o run -- python3 tools/step_calls.py OUT.json [version] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch  # noqa: E402

from bench import make_sgd, synth_targets  # noqa: E402
from yms import _lib as L, set_compute_dtype  # noqa: E402
from yolov8.tools.loss import ComputeLoss  # noqa: E402
from yolov8.yolov8 import YOLOv8  # noqa: E402

out = sys.argv[1]
v = sys.argv[2] if len(sys.argv) > 2 else "s"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = YOLOv8(v, 80).to(dev).train()
m.head.stride = torch.tensor([8.0, 16.0, 32.0])
set_compute_dtype(m, torch.bfloat16)
opt = make_sgd(m.parameters())
x = torch.randn(64, 3, 640, 640, device=dev)
crit = ComputeLoss(m.head, 80, dev, (640, 640))
tg = synth_targets(64, 80, 8, 4321, dev)
orig = L.call
rec = []
on = [False]


def call(name, *args):
    if on[0]:
        e = {"name": name}
        if name.startswith("yms_conv") and args and hasattr(args[0], "contents"):
            sh = args[0].contents
            e["shape"] = [sh.n, sh.h, sh.w, sh.cin, sh.cout, sh.k, sh.stride]
        elif name.startswith("yms_dwconv") and args and hasattr(args[0], "contents"):
            sh = args[0].contents
            e["shape"] = [sh.n, sh.h, sh.w, sh.c, sh.k]
        rec.append(e)
    return orig(name, *args)


L.call = call
for i in range(steps):
    on[0] = i == steps - 1
    opt.zero_grad(set_to_none=True)
    crit.loss_tensor(m(x), tg)[0].backward()
    opt.step()
torch.cuda.synchronize()
with open(out, "w") as f:
    for e in rec:
        f.write(json.dumps(e) + "\n")
print(f"{len(rec)} calls recorded")
