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


# ------------------------------------------------------------------------------------------
# Training augmentation (dataset.py:84-131) -- the restated single-sample chain of
# yolo-ms_amd/csrc/preprocess.hip (augment_normalize_kernel), replayed in the same fp32 operations
# and order (the kernel is compiled without FMA contraction).  Parity with albumentations / cv2
# (sequential resampling, fixed-point HSV) is UNPINNED; this pins the GPU kernel to its stated
# semantics.
# ------------------------------------------------------------------------------------------
REFLECT101, CLAMP, CONSTANT = 0, 1, 2
F32 = np.float32


def _rgb2hsv8(r, g, b):
    mx = np.maximum(r, np.maximum(g, b))
    mn = np.minimum(r, np.minimum(g, b))
    d = mx - mn
    v = mx
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.where(mx > 0, np.rint(F32(255) * d / mx), F32(0)).astype(F32)
        hr = F32(60) * (g - b) / d
        hg = F32(120) + F32(60) * (b - r) / d
        hb = F32(240) + F32(60) * (r - g) / d
    hd = np.where(mx == r, hr, np.where(mx == g, hg, hb))
    hd = np.where(d > 0, hd, F32(0)).astype(F32)
    hd = np.where(hd < 0, hd + F32(360), hd).astype(F32)
    h = np.rint(hd * F32(0.5)).astype(F32)
    h = np.where(h >= 180, h - F32(180), h).astype(F32)
    return h, s, v


def _hsv2rgb8(h, s, v):
    sf = s * (F32(1) / F32(255))
    hh = h * F32(2) / F32(60)
    i = np.floor(hh)
    f = hh - i
    p = v * (F32(1) - sf)
    q = v * (F32(1) - sf * f)
    t = v * (F32(1) - sf * (F32(1) - f))
    sec = (i.astype(np.int64) % 6 + 6) % 6
    r = np.choose(sec, [v, q, p, p, t, v])
    g = np.choose(sec, [t, v, v, q, p, p])
    b = np.choose(sec, [p, p, t, v, v, q])
    clip = lambda a: np.minimum(np.maximum(np.rint(a), F32(0)), F32(255)).astype(F32)
    return clip(r), clip(g), clip(b)


def hsv_shift8(rgb, shift):
    """[..., 3] float32 0..255 RGB -> shifted RGB (cv2 8-bit HSV, albumentations LUT semantics)."""
    h, s, v = _rgb2hsv8(rgb[..., 0], rgb[..., 1], rgb[..., 2])
    h = h + F32(shift[0])
    h = h - F32(180) * np.floor(h / F32(180))
    h = np.floor(h)
    s = np.floor(np.minimum(np.maximum(s + F32(shift[1]), F32(0)), F32(255)))
    v = np.floor(np.minimum(np.maximum(v + F32(shift[2]), F32(0)), F32(255)))
    return np.stack(_hsv2rgb8(h.astype(F32), s.astype(F32), v.astype(F32)), -1)


def _reflect101(x, n):
    if n <= 1:
        return np.zeros_like(x)
    L = F32(n - 1)
    period = F32(2) * L
    x = np.abs(x)
    x = x - period * np.floor(x / period)
    return np.where(x > L, period - x, x).astype(F32)


def augment_normalize(img, hsv, stages, out_h, out_w, mean, std):
    """HWC uint8 source + (optional HSV shift, stages [(m float32[9] output -> input frame, in_w,
    in_h, border)] ordered first -> last) -> CHW float32 normalised image."""
    oy, ox = np.meshgrid(np.arange(out_h, dtype=F32), np.arange(out_w, dtype=F32), indexing="ij")
    x, y = ox.reshape(-1), oy.reshape(-1)
    blank = np.zeros(x.shape, bool)
    for m, in_w, in_h, border in reversed(stages):
        m = np.asarray(m, F32)
        X = m[0] * x + m[1] * y + m[2]
        Y = m[3] * x + m[4] * y + m[5]
        Z = m[6] * x + m[7] * y + m[8]
        with np.errstate(divide="ignore", invalid="ignore"):
            x, y = (X / Z).astype(F32), (Y / Z).astype(F32)
        bad = ~((np.abs(x) < F32(1e7)) & (np.abs(y) < F32(1e7)))
        blank |= bad
        x = np.where(bad, F32(0), x)
        y = np.where(bad, F32(0), y)
        if border == REFLECT101:
            x, y = _reflect101(x, in_w), _reflect101(y, in_h)
        else:
            if border == CONSTANT:
                blank |= (x < F32(-0.5)) | (y < F32(-0.5)) | (x > F32(in_w) - F32(0.5)) | (y > F32(in_h) - F32(0.5))
            x = np.minimum(np.maximum(x, F32(0)), F32(in_w - 1)).astype(F32)
            y = np.minimum(np.maximum(y, F32(0)), F32(in_h - 1)).astype(F32)
    h, w = img.shape[:2]
    x0 = np.minimum(np.floor(x).astype(np.int64), w - 1)
    y0 = np.minimum(np.floor(y).astype(np.int64), h - 1)
    fx = (x - x0.astype(F32)).astype(F32)[:, None]
    fy = (y - y0.astype(F32)).astype(F32)[:, None]
    x1, y1 = np.minimum(x0 + 1, w - 1), np.minimum(y0 + 1, h - 1)
    src = img.astype(F32)
    t = [src[y0, x0], src[y0, x1], src[y1, x0], src[y1, x1]]
    if hsv is not None:
        t = [hsv_shift8(q, hsv) for q in t]
    top = t[0] + fx * (t[1] - t[0])
    bot = t[2] + fx * (t[3] - t[2])
    v = top + fy * (bot - top)
    v = np.where(blank[:, None], F32(0), v).astype(F32)
    mean, std = np.asarray(mean, F32), np.asarray(std, F32)
    sc = F32(1) / (F32(255) * std)
    bb = -mean / std
    out = v * sc + bb
    return out.reshape(out_h, out_w, 3).transpose(2, 0, 1).astype(F32)
