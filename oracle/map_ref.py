"""CPU restatement of the mAP@0.5 the reference validates with -- TEST INFRASTRUCTURE ONLY.

The reference computes ``torchmetrics.detection.MeanAveragePrecision(box_format='xyxy',
iou_type='bbox', iou_thresholds=[0.5])`` over per-image {'boxes','scores','labels'} predictions
and {'boxes','labels'} targets and reads ``map_50`` (yolov8/tools/train.py:41-47, 146, 152-153).
torchmetrics and its pycocotools backend are third-party and NOT installed here, so this is a
restatement of the published COCOeval algorithm (pycocotools/cocoeval.py: evaluateImg +
accumulate; maskUtils.iou for boxes) at the settings that call uses -- parity unpinned:

  * per (image, class): detections stably sorted by descending score, the first maxDets = 100 kept;
    ground truths in their given order (no crowd, no ignore: area range 'all');
  * greedy matching in detection order at IoU >= 0.5: each detection takes the not-yet-matched
    ground truth with the highest IoU, a later ground truth winning a tie (``if iou < best:
    continue`` with best starting at min(0.5, 1 - 1e-10)); IoU in double, boxes xywh with
    area = w*h (no +1);
  * per class over the dataset: the kept detections concatenated image by image, stably sorted by
    descending score; tp / fp cumulative sums, recall = tp / n_gt, precision = tp / (tp + fp + eps)
    made non-increasing from the right, sampled at the 101 recall thresholds 0, 0.01, .., 1 by
    ``searchsorted(recall, thr, 'left')`` (0 past the end); AP = mean of the 101 samples;
  * mAP = mean AP over classes with at least one ground truth (classes with ground truth but no
    detection score 0; classes with detections only are excluded).
"""
from __future__ import annotations

import numpy as np

MAX_DETS = 100
REC_THRS = np.linspace(0.0, 1.00, int(np.round((1.00 - 0.0) / 0.01)) + 1, endpoint=True)
EPS = np.spacing(1)


def iou_xyxy(d, g):
    """maskUtils.iou for boxes (pycocotools bbox IoU, iscrowd = 0) on xyxy inputs, in double."""
    d = np.asarray(d, dtype=np.float32)
    g = np.asarray(g, dtype=np.float32)
    # xyxy -> xywh in fp32 (torchvision box_convert on fp32 tensors), then double (pycocotools)
    dx, dy = d[:, 0].astype(np.float64), d[:, 1].astype(np.float64)
    dw, dh = (d[:, 2] - d[:, 0]).astype(np.float64), (d[:, 3] - d[:, 1]).astype(np.float64)
    gx, gy = g[:, 0].astype(np.float64), g[:, 1].astype(np.float64)
    gw, gh = (g[:, 2] - g[:, 0]).astype(np.float64), (g[:, 3] - g[:, 1]).astype(np.float64)
    out = np.zeros((len(d), len(g)))
    for i in range(len(d)):
        for j in range(len(g)):
            w = min(dx[i] + dw[i], gx[j] + gw[j]) - max(dx[i], gx[j])
            h = min(dy[i] + dh[i], gy[j] + gh[j]) - max(dy[i], gy[j])
            if w <= 0 or h <= 0:
                continue
            inter = w * h
            union = dw[i] * dh[i] + gw[j] * gh[j] - inter
            out[i, j] = inter / union
    return out


def match_image(dboxes, dscores, dlabels, gboxes, glabels, iou_thr=0.5):
    """-> per detection (tp, kept) flags, in the input order."""
    nd = len(dscores)
    tp = np.zeros(nd, dtype=np.int8)
    kept = np.zeros(nd, dtype=np.int8)
    for c in np.unique(np.concatenate([dlabels, glabels]).astype(np.int64)) if nd or len(glabels) else []:
        di = np.nonzero(dlabels == c)[0]
        gi = np.nonzero(glabels == c)[0]
        order = di[np.argsort(-dscores[di], kind="mergesort")][:MAX_DETS]
        kept[order] = 1
        if len(gi) == 0 or len(order) == 0:
            continue
        ious = iou_xyxy(dboxes[order], gboxes[gi])
        gtm = np.zeros(len(gi), dtype=bool)
        for k in range(len(order)):
            best, m = min(iou_thr, 1 - 1e-10), -1
            for j in range(len(gi)):
                if gtm[j]:
                    continue
                if ious[k, j] < best:
                    continue
                best, m = ious[k, j], j
            if m >= 0:
                gtm[m] = True
                tp[order[k]] = 1
    return tp, kept


def accumulate(per_image, n_gt_per_class):
    """per_image: list of (scores, labels, tp, kept) in evaluation order -> (mAP, {class: AP})."""
    aps = {}
    for c, npig in sorted(n_gt_per_class.items()):
        if npig == 0:
            continue
        sc, tps = [], []
        for scores, labels, tp, kept in per_image:
            idx = np.nonzero((labels == c) & (kept == 1))[0]
            idx = idx[np.argsort(-scores[idx], kind="mergesort")]
            sc.append(scores[idx])
            tps.append(tp[idx])
        sc = np.concatenate(sc) if sc else np.zeros(0)
        tpv = np.concatenate(tps).astype(bool) if tps else np.zeros(0, dtype=bool)
        inds = np.argsort(-sc, kind="mergesort")
        tpv = tpv[inds]
        tp_sum = np.cumsum(tpv).astype(float)
        fp_sum = np.cumsum(~tpv).astype(float)
        rc = tp_sum / npig
        pr = (tp_sum / (fp_sum + tp_sum + EPS)).tolist()
        for i in range(len(pr) - 1, 0, -1):
            if pr[i] > pr[i - 1]:
                pr[i - 1] = pr[i]
        q = np.zeros(len(REC_THRS))
        ri = np.searchsorted(rc, REC_THRS, side="left")
        for k, pi in enumerate(ri):
            if pi < len(pr):
                q[k] = pr[pi]
        aps[c] = float(np.mean(q))
    m = float(np.mean(list(aps.values()))) if aps else -1.0
    return m, aps


def map50(preds, targets):
    """preds / targets: lists of dicts of numpy arrays ('boxes' xyxy, 'scores', 'labels')."""
    per_image, ngt = [], {}
    for p, t in zip(preds, targets):
        gl = np.asarray(t["labels"]).astype(np.int64)
        for c in gl:
            ngt[int(c)] = ngt.get(int(c), 0) + 1
        dl = np.asarray(p["labels"]).astype(np.int64)
        for c in dl:
            ngt.setdefault(int(c), 0)
        tp, kept = match_image(np.asarray(p["boxes"]).reshape(-1, 4), np.asarray(p["scores"]), dl,
                               np.asarray(t["boxes"]).reshape(-1, 4), gl)
        per_image.append((np.asarray(p["scores"]), dl, tp, kept))
    return accumulate(per_image, ngt)
