"""Fit the lane layout of v_mfma_f32_4x4x4_16b_bf16 from tools/mfma4_probe output (dev tool).
   python tools/mfma4_probe.py < probe.txt"""
import itertools
import sys

import numpy as np

rows = np.array([[float(v) for v in line.split()] for line in sys.stdin if line.strip()])
A, B, D = rows[:, 0:4], rows[:, 4:8], rows[:, 8:12]
# candidate maps: lane -> (block, index) for the A row / B column / D column, D register -> row
maps = {"blk=l/4,idx=l%4": lambda l: (l // 4, l % 4), "blk=l%16,idx=l/16": lambda l: (l % 16, l // 16)}
for (na, fa), (nb, fb), (nd, fd) in itertools.product(maps.items(), repeat=3):
    Am = np.zeros((16, 4, 4)); Bm = np.zeros((16, 4, 4))
    for l in range(64):
        b, i = fa(l); Am[b, i, :] = A[l]
        b, j = fb(l); Bm[b, :, j] = B[l]
    C = np.einsum("bik,bkj->bij", Am, Bm)
    ok = True
    for l in range(64):
        b, j = fd(l)
        for r in range(4):
            ok &= abs(D[l, r] - C[b, r, j]) < 1e-3
    for l in range(64):        # alternative: D register = column, lane index = row
        pass
    print(f"A {na:18s} B {nb:18s} D(reg=row) {nd:18s}: {'MATCH' if ok else '-'}")
