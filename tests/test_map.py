"""mAP@0.5 (the reference's torchmetrics call at train.py:41-47, 146, 152-153).
CPU tier: known-answer cases of the COCOeval restatement (oracle/map_ref.py; torchmetrics and
pycocotools are absent, so parity is unpinned beyond these hand-computed answers) and the native
host accumulation (yms_map_accumulate) bit-exact against the restatement's accumulate."""
import ctypes

import numpy as np
import pytest

from oracle import map_ref as R
from yms import _lib as L


def _d(boxes, scores, labels):
    return {"boxes": np.array(boxes, np.float32).reshape(-1, 4), "scores": np.array(scores, np.float32),
            "labels": np.array(labels, np.int64)}


def _t(boxes, labels):
    return {"boxes": np.array(boxes, np.float32).reshape(-1, 4), "labels": np.array(labels, np.int64)}


def test_known_answers():
    g = [[0, 0, 10, 10]]
    one = pytest.approx(1.0, abs=1e-12)      # precision = tp / (tp + fp + eps), as COCOeval
    assert R.map50([_d(g, [0.9], [1])], [_t(g, [1])])[0] == one
    # a higher-scored false positive first: P = [0, 1/2], R = [0, 1] -> 101 samples of 0.5
    m, ap = R.map50([_d([[50, 50, 60, 60], [0, 0, 10, 10]], [0.9, 0.8], [1, 1])], [_t(g, [1])])
    assert ap[1] == pytest.approx(0.5, abs=1e-12)
    # IoU exactly 0.5 matches (>=), just below does not
    half = [[0, 0, 10, 10]], [[0, 0, 10, 5]]           # IoU 0.5
    assert R.map50([_d(half[1], [1.0], [0])], [_t(half[0], [0])])[0] == one
    assert R.map50([_d([[0, 0, 10, 4.99]], [1.0], [0])], [_t(half[0], [0])])[0] == 0.0
    # wrong class, and a class with detections but no ground truth is excluded from the mean
    m, ap = R.map50([_d(g + g, [0.9, 0.8], [2, 3])], [_t(g, [3])])
    assert set(ap) == {3} and m == one
    # a class with ground truth and no detection scores 0
    m, ap = R.map50([_d(g, [0.9], [1])], [_t(g + g, [1, 4])])
    assert ap[1] == one and ap[4] == 0.0 and m == pytest.approx(0.5, abs=1e-12)
    # a ground truth is matched once: the duplicate is a false positive
    m, ap = R.map50([_d(g + g, [0.9, 0.8], [1, 1])], [_t(g, [1])])
    assert m == one     # precision at recall 1 is reached at the first detection
    # only the 100 best detections per (image, class) count
    dets = [[0, 0, 10, 10]] * 101
    m, _ = R.map50([_d([[50, 50, 51, 51]] * 100 + g, list(np.linspace(1, 0.5, 100)) + [0.1], [1] * 101)],
                   [_t(g, [1])])
    assert m == 0.0
    del dets


def test_host_accumulate_matches_restatement():
    rng = np.random.default_rng(0)
    per_image, ngt = [], {}
    scores, labels, image, tp, kept = [], [], [], [], []
    for i in range(25):
        n = int(rng.integers(0, 60))
        sc = rng.choice(np.linspace(0, 1, 17).astype(np.float32), n)     # many exact ties
        lb = rng.integers(0, 6, n)
        t = (rng.random(n) < 0.4).astype(np.int8)
        k = (rng.random(n) < 0.9).astype(np.int8)
        per_image.append((sc, lb, t, k))
        scores.append(sc); labels.append(lb); image.append(np.full(n, i)); tp.append(t); kept.append(k)
        for c in rng.integers(0, 7, int(rng.integers(0, 5))):
            ngt[int(c)] = ngt.get(int(c), 0) + 1
    for c in range(6):
        ngt.setdefault(c, 0)
    m_ref, ap_ref = R.accumulate(per_image, ngt)
    cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs).astype(dt))
    sc, lb, im, t, k = (cat(scores, np.float32), cat(labels, np.int32), cat(image, np.int32), cat(tp, np.uint8),
                        cat(kept, np.uint8))
    ncls = 8
    n_gt = np.array([ngt.get(c, 0) for c in range(ncls)], np.int32)
    ap = np.zeros(ncls)
    m = np.zeros(1)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert L.lib().yms_map_accumulate(sc.size, p(sc), p(lb), p(im), p(t), p(k), ncls, p(n_gt), p(ap), p(m)) == 0
    assert m[0] == m_ref                                     # bit-exact
    for c, v in ap_ref.items():
        assert ap[c] == v, c
