"""NMS micro-benchmark on the SURVEY 8d input sets (dev tool)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from yms import ops
from test_nms_gpu import clustered

def timeit(pred, conf=0.25, iou=0.45, reps=20):
    d = torch.from_numpy(pred).cuda()
    for _ in range(3): ops.batched_nms_indices(d, conf, iou)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(reps): r = ops.batched_nms_indices(d, conf, iou)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, r[4].cpu().numpy()

rng = np.random.default_rng(1)
B, A, nc = 32, 8400, 80
dense = np.zeros((B, A, 4 + nc), np.float32)
dense[..., :2] = rng.uniform(0, 640, (B, A, 2)); dense[..., 2:4] = rng.uniform(10, 120, (B, A, 2))
dense[..., 4:] = rng.uniform(0.2, 0.6, (B, A, nc))
print("dense random-init-like (B=32, ~105/class): %.3f ms kept/img %s" % (timeit(dense)[0], timeit(dense)[1][:4]))
print("clustered (B=32, 20x30 boxes): %.3f ms" % timeit(clustered(B, nc))[0])
one = dense[..., :5].copy(); one[..., 4] = rng.uniform(0, 1, (B, A))
print("single class nc=1 (B=32, 8400 cand): %.3f ms" % timeit(one)[0])
from test_nms_gpu import _level_segments
lv = _level_segments(B, 5)
for win in ("1", "0"):
    os.environ["YMS_NMS_WINDOW"] = win
    t, k = timeit(lv)
    print("level segments 6400/1600/400 (B=32, bench regime) window=%s: %.3f ms kept/img %s" % (win, t, k[:4]))
    os.environ["YMS_NMS_WINDOW"] = "1"
