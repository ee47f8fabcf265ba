"""Deterministic input vectors shared by the golden-fixture generators and the tests that read the
fixtures.  Large inputs (the 8400-anchor head maps) are regenerated from an integer hash instead of
being stored: the formula is exact in uint64 arithmetic and rounds once to fp32, so the generator
(build container) and the tests (CPU here, GPU box) see bit-identical values."""
from __future__ import annotations

import numpy as np


def hashed_uniform(shape, seed, lo=-1.0, hi=1.0):
    """fp32 array of ``shape`` with values in [lo, hi): Knuth multiplicative hash of the flat index."""
    n = int(np.prod(shape))
    idx = np.arange(n, dtype=np.uint64)
    h = (idx * np.uint64(2654435761) + np.uint64(seed) * np.uint64(40503) + np.uint64(12345)) % np.uint64(1 << 32)
    u = h.astype(np.float64) / float(1 << 32)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def bf16_round(a):
    """Round fp32 values to the nearest bf16 (ties to even), returned as fp32."""
    b = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return b.astype(np.uint32).view(np.float32)


def checksum_weights(n, seed=7):
    """fp64 weights for gradient checksums over ``n`` elements (flattened NCHW order)."""
    return hashed_uniform((n,), seed).astype(np.float64)


def loss_targets(B, nc, counts, seed, extra=(), wh_lo=0.05, wh_span=0.4):
    """[M, 6] fp32 targets [img, cls, cx, cy, w, h] (normalised), ``counts[b]`` random GTs per image."""
    rng = np.random.default_rng(seed)
    rows = []
    for b in range(B):
        n = counts[b] if isinstance(counts, (list, tuple)) else counts
        for _ in range(n):
            wh = rng.random(2) * wh_span + wh_lo
            c = rng.random(2) * (1 - wh) + wh / 2
            rows.append([b, int(rng.integers(0, nc)), c[0], c[1], wh[0], wh[1]])
    rows += [list(e) for e in extra]
    return np.asarray(rows, dtype=np.float32).reshape(-1, 6)


def loss_maps(B, nc, shapes, seed, scale, bf16):
    """The head maps of a loss fixture: per level [B, 64 + nc, h, w] fp32 (bf16-rounded if asked)."""
    out = []
    for i, (h, w) in enumerate(shapes):
        a = hashed_uniform((B, 64 + nc, h, w), seed * 10 + i, -scale, scale)
        out.append(bf16_round(a) if bf16 else a)
    return out


def load_loss_case(name):
    """-> dict: fixture arrays plus 'maps' (regenerated), 'B', 'nc', 'img', 'shapes', 'ious'."""
    import os
    z = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"loss_{name}.npz")))
    B, nc, ih, iw, mseed, _ = (int(v) for v in z["meta"])
    shapes = [tuple(int(v) for v in s) for s in z["shapes"]]
    z.update(B=B, nc=nc, img=(ih, iw), shapes=shapes,
             maps=loss_maps(B, nc, shapes, mseed, float(z["scale"][0]), bool(z["bf16"][0])),
             ious=sorted({k.split(":")[0] for k in z if k.endswith(":loss")}))
    return z
