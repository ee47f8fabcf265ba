"""The search-radius bound the graph and window-grid NMS kernels rely on (csrc/head_nms.hip,
gr_radius / gr_region): for an IoU threshold t >= 0, any pair that iou_gt_f accepts has its centres
within max(w(1-t'), w/2 + max(0, 1/2 - t') Wmax) (+ slack) of each other in x (same in y), t' the
lowered threshold the kernels use.  A fuzz over box scales from 1e-3 to 1e6, size mixes, equal
centres and thresholds up to 1, in fp32 exactly as the kernels evaluate it (numpy float32).  CPU
only; the GPU kernels' keep lists are checked against oracle/nms_ref.c in test_nms_gpu.py."""
import numpy as np

f32 = np.float32


def _iou_gt_f(i, j, thr):
    xx1 = np.maximum(i[..., 0], j[..., 0]); yy1 = np.maximum(i[..., 1], j[..., 1])
    xx2 = np.minimum(i[..., 2], j[..., 2]); yy2 = np.minimum(i[..., 3], j[..., 3])
    ok = (xx2 > xx1) & (yy2 > yy1)
    ia = (i[..., 2] - i[..., 0]) * (i[..., 3] - i[..., 1])
    ja = (j[..., 2] - j[..., 0]) * (j[..., 3] - j[..., 1])
    inter = np.maximum(f32(0), xx2 - xx1) * np.maximum(f32(0), yy2 - yy1)
    with np.errstate(all="ignore"):
        ovr = inter / (ia + ja - inter)
    return ok & (ovr > thr)


def _radius(w, wmax, c, tr):
    r = np.maximum(w * (f32(1) - tr), f32(0.5) * w + np.maximum(f32(0), f32(0.5) - tr) * wmax)
    return r * f32(1.00001) + f32(1e-5) * (np.abs(c) + wmax) + f32(1e-30)


def test_search_radius_contains_every_suppressing_pair():
    rng = np.random.default_rng(0)
    checked = 0
    for trial in range(120):
        n = 200
        kind = trial % 4
        scale = 10.0 ** rng.uniform(-3, 6)
        c = rng.uniform(0, 1, (n, 2)) * scale
        if kind == 0:
            wh = rng.uniform(0.01, 0.3, (n, 2)) * scale
        elif kind == 1:
            wh = np.exp(rng.uniform(-6, 1, (n, 2))) * scale
        elif kind == 2:
            wh = np.repeat(rng.uniform(0.05, 0.5, (n, 1)), 2, 1) * scale
        else:
            wh = rng.uniform(0.1, 0.2, (n, 2)) * scale
            c[:] = c[:1] + rng.normal(0, 1e-4, (n, 2)) * scale
        b = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(f32)
        w = b[:, 2] - b[:, 0]; h = b[:, 3] - b[:, 1]
        cx = f32(0.5) * (b[:, 0] + b[:, 2]); cy = f32(0.5) * (b[:, 1] + b[:, 3])
        for thr in (0.0, 0.1, 0.45, 0.5, 0.7, 0.95, 0.999999):
            thr_f = f32(thr)
            tr = max(f32(0), thr_f * f32(1 - 1e-4) - f32(1e-6))          # head_nms.hip's lowered t
            acc = _iou_gt_f(b[:, None, :], b[None, :, :], thr_f)
            np.fill_diagonal(acc, False)
            rx = _radius(w, w.max(), cx, tr); ry = _radius(h, h.max(), cy, tr)
            ii, jj = np.nonzero(acc)
            inside = ((cx[jj] >= cx[ii] - rx[ii]) & (cx[jj] <= cx[ii] + rx[ii]) &
                      (cy[jj] >= cy[ii] - ry[ii]) & (cy[jj] <= cy[ii] + ry[ii]))
            assert inside.all(), (trial, kind, thr, scale, int((~inside).sum()))
            checked += len(ii)
    assert checked > 10000
