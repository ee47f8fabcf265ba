"""CPU restatement of the dataset transform's Resize + Normalize + ToTensorV2 -- TEST INFRASTRUCTURE ONLY.

yolov8/tools/dataset.py:132-134 applies albumentations ``A.Resize(H, W, cv2.INTER_LINEAR)``,
``A.Normalize(mean, std)`` and ``ToTensorV2()`` per image (flips before, :124-127).  cv2 and
albumentations are not installed, so this restates the published cv2 INTER_LINEAR coordinate
mapping (half-pixel centres, edge clamp with zero weight) in float64 arithmetic with fp32
weights, as the GPU kernel does -- parity with cv2's 8-bit fixed-point rounding is UNPINNED.
Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np


def _coords(n_out, n_in):
    scale = np.float32(n_in) / np.float32(n_out)
    x = (np.arange(n_out, dtype=np.float32) + np.float32(0.5)) * scale - np.float32(0.5)
    s = np.floor(x).astype(np.int64)
    f = (x - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo], f[lo] = 0, 0.0
    hi = s >= n_in - 1
    s[hi], f[hi] = n_in - 1, 0.0
    s1 = np.minimum(s + 1, n_in - 1)
    return s, s1, f


def resize_normalize(img, out_h, out_w, mean, std, flags=0):
    """HWC uint8 -> CHW float32 (flip -> bilinear resize -> (v/255 - mean)/std)."""
    im = img
    if flags & 1:
        im = im[:, ::-1]
    if flags & 2:
        im = im[::-1]
    im = im.astype(np.float32)
    y0, y1, fy = _coords(out_h, im.shape[0])
    x0, x1, fx = _coords(out_w, im.shape[1])
    fx = fx[None, :, None]
    fy = fy[:, None, None]
    top = im[y0][:, x0] + fx * (im[y0][:, x1] - im[y0][:, x0])
    bot = im[y1][:, x0] + fx * (im[y1][:, x1] - im[y1][:, x0])
    v = top + fy * (bot - top)
    mean = np.asarray(mean, np.float32)
    std = np.asarray(std, np.float32)
    out = (v / np.float32(255.0) - mean) / std
    return out.transpose(2, 0, 1).astype(np.float32)
