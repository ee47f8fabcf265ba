"""GPU tier of mAP@0.5: the matching kernel (yms_map_match) and the full metric (yms.metrics) against
the COCOeval restatement (oracle/map_ref.py) -- identical tp / kept flags and bit-identical mAP --
on clustered synthetic detections with exact score ties and on the random-init model's own
post-processed output (train.py:63-113 -> validate_epoch's metric)."""
import numpy as np
import pytest
import torch

from oracle import map_ref as R
from yms.metrics import MeanAveragePrecision

pytestmark = pytest.mark.gpu


def _clustered(rng, n_img, nc=12):
    preds, targets = [], []
    for _ in range(n_img):
        k = int(rng.integers(0, 9))
        c = rng.uniform(40, 600, (k, 2))
        wh = rng.uniform(10, 120, (k, 2))
        gb = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
        gl = rng.integers(0, nc, k)
        boxes, scores, labels = [], [], []
        for j in range(k):
            m = int(rng.integers(0, 40))
            jit = rng.normal(0, 0.15, (m, 4)) * np.tile(wh[j], 2)
            boxes.append(gb[j] + jit)
            scores.append(np.round(rng.beta(2, 5, m) * 16) / 16)          # exact ties
            labels.append(np.where(rng.random(m) < 0.85, gl[j], rng.integers(0, nc, m)))
        fp = int(rng.integers(0, 30))
        boxes.append(rng.uniform(0, 640, (fp, 4)).cumsum(1)[:, [0, 1, 2, 3]] % 640)
        scores.append(rng.random(fp))
        labels.append(rng.integers(0, nc, fp))
        b = np.concatenate(boxes).astype(np.float32).reshape(-1, 4)
        b[:, 2:] = np.maximum(b[:, 2:], b[:, :2] + 1)
        preds.append({"boxes": b, "scores": np.concatenate(scores).astype(np.float32),
                      "labels": np.concatenate(labels).astype(np.int64)})
        targets.append({"boxes": gb.reshape(-1, 4), "labels": gl.astype(np.int64)})
    return preds, targets


def _torch(ds, dev="cuda"):
    return [{k: torch.from_numpy(np.asarray(v)).to(dev) for k, v in d.items()} for d in ds]


def test_map_matches_restatement_clustered():
    rng = np.random.default_rng(7)
    preds, targets = _clustered(rng, 40)
    metric = MeanAveragePrecision(iou_thresholds=[0.5])
    for i in range(0, 40, 16):                 # several update() batches
        metric.update(_torch(preds[i:i + 16]), _torch(targets[i:i + 16]))
    out = metric.compute()
    m_ref, ap_ref = R.map50(preds, targets)
    assert out["map_50"].item() == m_ref
    assert out["map_per_class"] == ap_ref
    # per-detection flags of the kernel equal the restatement's
    tp_all = np.concatenate(metric._tp)
    kept_all = np.concatenate(metric._kept)
    ref_tp, ref_kept = [], []
    for p, t in zip(preds, targets):
        a, b = R.match_image(p["boxes"], p["scores"], p["labels"], t["boxes"], t["labels"])
        ref_tp.append(a)
        ref_kept.append(b)
    assert np.array_equal(tp_all, np.concatenate(ref_tp))
    assert np.array_equal(kept_all, np.concatenate(ref_kept))


def test_map_on_model_postprocess_output():
    """The reference's validation flow: eval forward -> class-wise NMS post-process -> mAP@0.5, on
    the random-init model with ground truth taken from its own high-score detections (jittered)."""
    from oracle import model_ref as M
    from yms import ops
    from yolov8.yolov8 import YOLOv8
    torch.manual_seed(0)
    m = YOLOv8("n", 80).cuda().eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    x = torch.randn(4, 3, 256, 256, generator=torch.Generator().manual_seed(3)).cuda()
    dets = ops.postprocess(m(x), 0.25, 0.45)
    rng = np.random.default_rng(1)
    targets = []
    for d in dets:
        k = min(6, d["boxes"].shape[0])
        b = d["boxes"][:k].cpu().numpy() + rng.normal(0, 2, (k, 4)).astype(np.float32)
        targets.append({"boxes": b, "labels": d["labels"][:k].cpu().numpy()})
    metric = MeanAveragePrecision(iou_thresholds=[0.5])
    metric.update(dets, _torch(targets))
    got = metric.compute()["map_50"].item()
    ref = R.map50([{k: v.cpu().numpy() for k, v in d.items()} for d in dets], targets)[0]
    assert got == ref
    assert 0.0 <= got <= 1.0
    del M
