"""Dev tool: conditioning of the random-init training graphs -- CPU fp32 parameter-gradient drift
vs fp64 (median / p90 / max of per-tensor relative L2) under the closed-form init and under
oracle.model_ref.ordered_init.   python tools/cond_sweep.py <version> <size> [seed]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

from oracle import model_ref as M  # noqa: E402
from oracle import ms_ref as MS  # noqa: E402

v, size = sys.argv[1], int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 41
O = MS if v.startswith("ms-") else M
x = torch.randn(2, 3, size, size, generator=torch.Generator().manual_seed(seed))


def grads(sd, dt):
    p = {k: (t.clone().to(dt).requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else (t.clone().to(dt) if t.is_floating_point() else t.clone()))
         for k, t in sd.items()}
    r = O.forward(p, v, 80, x.to(dt), True)
    sum((o.double() ** 2).mean() for o in r).backward()
    return {k: t.grad.double() for k, t in p.items() if t.grad is not None}


for tag, sd in (("closed-form", O.init_params(v, 80)), ("ordered", M.ordered_init(O.init_params(v, 80)))):
    t0 = time.time()
    a, b = grads(sd, torch.float64), grads(sd, torch.float32)
    e = sorted(((b[k] - a[k]).norm() / (a[k].norm() + 1e-30)).item() for k in a)
    n = len(e)
    print(f"{v} {size} seed {seed} {tag:11s}: CPU fp32 vs fp64 median {e[n // 2]:.2e} p90 {e[9 * n // 10]:.2e} "
          f"max {e[-1]:.2e} ({time.time() - t0:.1f} s)")
