"""Dev: per-tensor bf16 gradient drift vs fp64 with the fused BN reduce on / off (conditioned fixture)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import torch
import test_train_conditioned_gpu as T

v, size = (sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else ("s", 640)
sd, x = T._fixture(v, size, 42)
g64, _, _ = T._cpu(v, sd, x, torch.float64)
res = {}
for mode in ("0", "1"):
    os.environ["YMS_BNRED"] = mode
    m, outs = T._gpu(v, sd, x, torch.bfloat16)
    pd = dict(m.named_parameters())
    res[mode] = {k: T._rel(pd[k].grad, g64[k]) for k in g64 if k in pd}
worst = sorted(res["1"], key=lambda k: -res["1"][k])[:12]
for k in worst:
    print(f"{k:50s} fused {res['1'][k]:.4f}  separate {res['0'][k]:.4f}")
