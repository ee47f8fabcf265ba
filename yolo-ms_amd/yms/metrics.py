"""mAP@0.5 on the MI355X path: the reference's validation metric,
``torchmetrics.detection.MeanAveragePrecision(box_format='xyxy', iou_type='bbox',
iou_thresholds=[0.5])`` read as ``map_50`` (yolov8/tools/train.py:41-47, 146, 152-153).

``update(preds, targets)`` takes the same per-image lists of dicts the reference builds
(``yms.ops.postprocess`` returns them for a batch) and runs the detection <-> ground-truth
matching on the GPU (``yms_map_match``, one wave per image); ``compute()`` runs the per-class
precision / recall accumulation and 101-point interpolation in the native host code
(``yms_map_accumulate``).  COCOeval semantics (maxDets 100, area 'all'); parity is against the
restatement oracle/map_ref.py (torchmetrics / pycocotools are not installed: unpinned)."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L


class MeanAveragePrecision:
    def __init__(self, box_format="xyxy", iou_type="bbox", iou_thresholds=(0.5,), **_ignored):
        if box_format != "xyxy" or iou_type != "bbox" or list(iou_thresholds) != [0.5]:
            raise ValueError("yms.metrics.MeanAveragePrecision implements box_format='xyxy', iou_type='bbox', "
                             "iou_thresholds=[0.5] (the reference's validation metric)")
        self.reset()

    def reset(self):
        self._scores, self._labels, self._image, self._tp, self._kept = [], [], [], [], []
        self._ngt = {}
        self._n_images = 0

    def to(self, device):      # torchmetrics-style no-op (state lives on the host)
        return self

    def update(self, preds, targets):
        if len(preds) != len(targets):
            raise ValueError("preds and targets must have the same length")
        if not preds:
            return
        dev = next((p["boxes"].device for p in preds if isinstance(p["boxes"], torch.Tensor)), None)
        if dev is None or dev.type != "cuda":
            raise RuntimeError("yms: mAP matching runs on ROCm GPU tensors only (no CPU fallback)")
        db = torch.cat([p["boxes"].reshape(-1, 4).float() for p in preds]).contiguous()
        ds = torch.cat([p["scores"].reshape(-1).float() for p in preds]).contiguous()
        dl = torch.cat([p["labels"].reshape(-1).to(torch.int32) for p in preds]).contiguous()
        gb = torch.cat([t["boxes"].reshape(-1, 4).float().to(dev) for t in targets]).contiguous()
        gl = torch.cat([t["labels"].reshape(-1).to(torch.int32).to(dev) for t in targets]).contiguous()
        nd = [int(p["scores"].numel()) for p in preds]
        ng = [int(t["labels"].numel()) for t in targets]
        doff = torch.tensor(np.concatenate([[0], np.cumsum(nd)]), dtype=torch.int32, device=dev)
        goff = torch.tensor(np.concatenate([[0], np.cumsum(ng)]), dtype=torch.int32, device=dev)
        D = max(int(sum(nd)), 1)
        tp = torch.zeros(D, dtype=torch.uint8, device=dev)
        kept = torch.zeros(D, dtype=torch.uint8, device=dev)
        rank = torch.empty(D, dtype=torch.int32, device=dev)
        L.call("yms_map_match", len(preds), L.ptr(db) if db.numel() else None, L.ptr(ds) if ds.numel() else None,
               L.ptr(dl) if dl.numel() else None, doff.data_ptr(), L.ptr(gb) if gb.numel() else None,
               L.ptr(gl) if gl.numel() else None, goff.data_ptr(), tp.data_ptr(), kept.data_ptr(), rank.data_ptr(),
               max(ng) if ng else 0, L.stream_ptr(dev))
        n = int(sum(nd))
        self._scores.append(ds.cpu().numpy())
        self._labels.append(dl.cpu().numpy())
        self._tp.append(tp[:n].cpu().numpy())
        self._kept.append(kept[:n].cpu().numpy())
        self._image.append(np.repeat(np.arange(self._n_images, self._n_images + len(preds), dtype=np.int32), nd))
        for c in gl.cpu().numpy().tolist():
            self._ngt[c] = self._ngt.get(c, 0) + 1
        self._n_images += len(preds)

    def compute(self):
        cat = (lambda xs, dt: np.ascontiguousarray(np.concatenate(xs).astype(dt)) if xs else np.zeros(0, dt))
        sc, lb = cat(self._scores, np.float32), cat(self._labels, np.int32)
        im, tp, kp = cat(self._image, np.int32), cat(self._tp, np.uint8), cat(self._kept, np.uint8)
        ncls = max([int(lb.max()) + 1 if lb.size else 0] + [c + 1 for c in self._ngt] + [1])
        ngt = np.zeros(ncls, dtype=np.int32)
        for c, k in self._ngt.items():
            if c >= 0:
                ngt[c] = k
        ap = np.zeros(ncls, dtype=np.float64)
        m = np.zeros(1, dtype=np.float64)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a.size else None
        L.check(L.lib().yms_map_accumulate(int(sc.size), p(sc), p(lb), p(im), p(tp), p(kp), ncls, p(ngt), p(ap), p(m)),
                "yms_map_accumulate")
        per = {c: float(ap[c]) for c in range(ncls) if ngt[c] > 0}
        mv = torch.tensor(float(m[0]), dtype=torch.float64)
        return {"map": mv, "map_50": mv.clone(), "map_per_class": per}
