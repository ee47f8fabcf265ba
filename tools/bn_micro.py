"""Dev tool: elementwise BN kernels in isolation (B=64 YOLO-MS-S shapes, bf16): us and GB/s of
the forward affine+SiLU, the backward reduce (z, dy read) and the backward apply (z, dy read, dz write)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import _lib as L

st = L.stream_ptr()
BF = L.BF16
for (npix, c) in [(409600, 384), (409600, 576), (6553600, 32), (1638400, 128), (1638400, 64), (102400, 768)]:
    z = torch.randn(npix, c, device="cuda").to(torch.bfloat16)
    gy = torch.randn(npix, c, device="cuda").to(torch.bfloat16)
    dz = torch.empty_like(z)
    sc, sh = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")
    mi = torch.cat([torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")])
    rows = L.lib().yms_bn_bwd_rows(npix, c)
    ws = torch.empty(rows * 2 * c, device="cuda")
    coef = torch.zeros(2 * c, device="cuda")
    dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    P = lambda t: t.data_ptr()
    ops = {
        "affine": (lambda: L.call("yms_affine_act", BF, npix, c, P(z), c, 0, P(sc), P(sh), 1, None, 0, 0, P(dz), c, 0,
                                  st), 2),
        "reduce": (lambda: L.call("yms_bn_act_bwd_reduce", BF, npix, c, P(z), c, 0, P(gy), c, 0, P(sc), P(sh), P(mi), 1,
                                  P(ws), st), 2),
        "finalize": (lambda: L.call("yms_bn_act_bwd_finalize", c, P(ws), rows, npix, P(dg), P(db), P(coef), st), 0),
        "apply": (lambda: L.call("yms_bn_act_bwd_apply", BF, npix, c, P(z), c, 0, P(gy), c, 0, P(sc), P(sh), P(mi),
                                 P(coef), 1, P(dz), c, 0, None, 0, 0, 0, st), 3),
    }
    for name, (fn, ntens) in ops.items():
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 100
        nb = npix * c * 2 * ntens
        print(f"{name:9s} npix {npix:8d} c{c:4d}: {us:8.1f} us  {nb / us / 1e3:7.0f} GB/s", flush=True)
