"""NMS micro-benchmark on the SURVEY 8d input sets (dev tool): wall time per batched_nms_indices
call (prep + class-wise NMS + Python glue) for each YMS_NMS_GRAPH_MIN in $YMS_NMSB_GMIN
(default "128,0": graph kernels on / off)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from yms import ops
from test_nms_gpu import clustered, _level_segments


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
one = dense[..., :5].copy(); one[..., 4] = rng.uniform(0, 1, (B, A))
sets = [("level segments 6400/1600/400 (B=32, bench regime)", _level_segments(B, 5)),
        ("dense random-init-like (B=32, ~105/class)", dense),
        ("clustered (B=32, 20x30 boxes)", clustered(B, nc)),
        ("single class nc=1 (B=32, 8400 cand)", one)]
for gmin in os.environ.get("YMS_NMSB_GMIN", "2048,0").split(","):
    os.environ["YMS_NMS_GRAPH_MIN"] = gmin
    for name, pred in sets:
        t, k = timeit(pred)
        print("graph_min=%-4s %-52s %.3f ms kept/img %s" % (gmin, name, t, k[:4]), flush=True)
