"""Known-answer tests pinning the C restatement of torchvision NMS + the reference's
class-wise post-process (oracle/nms_ref.c).  CPU tier.  (NMS parity is unpinned by
the reference: torchvision is absent, no reference test/fixture covers it.)"""
import numpy as np

from oracle import nms as onms


def test_basic_suppression():
    b = np.array([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30]], np.float32)
    s = np.array([0.9, 0.8, 0.7], np.float32)
    assert onms.nms(b, s, 0.5).tolist() == [0, 2]          # IoU(0,1)=81/119=0.68
    assert onms.nms(b, s, 0.7).tolist() == [0, 1, 2]


def test_stable_ties():
    b = np.array([[0, 0, 1, 1], [5, 5, 6, 6], [0, 0, 1, 1]], np.float32)
    s = np.array([0.5, 0.5, 0.5], np.float32)
    assert onms.nms(b, s, 0.5).tolist() == [0, 1]           # lower index wins the tie


def test_threshold_is_strict_and_double():
    b = np.array([[0, 0, 10, 10], [0, 0, 10, 5]], np.float32)  # IoU exactly 0.5
    s = np.array([0.9, 0.8], np.float32)
    assert onms.nms(b, s, 0.5).tolist() == [0, 1]           # 0.5 > 0.5 is false
    assert onms.nms(b, s, 0.4999).tolist() == [0]
    # a ratio of float(0.6) ~ 0.6000000238 exceeds the double threshold 0.6 (CPU kernel semantics)
    b = np.array([[0, 0, 10, 10], [0, 0, 10, 6]], np.float32)  # inter 60, union 100
    assert onms.nms(b, s, 0.6).tolist() == [0]


def test_empty_and_zero_area():
    assert onms.nms(np.zeros((0, 4), np.float32), np.zeros(0, np.float32), 0.5).tolist() == []
    b = np.array([[0, 0, 0, 0], [0, 0, 0, 0]], np.float32)
    s = np.array([0.3, 0.4], np.float32)
    # 0/0 = NaN -> never > thr -> both kept, score order
    assert onms.nms(b, s, 0.5).tolist() == [1, 0]


def test_postprocess_classwise_order():
    # 4 anchors, 2 classes; cxcywh boxes
    pred = np.array([
        [5, 5, 10, 10, 0.9, 0.1],
        [5.5, 5.5, 10, 10, 0.8, 0.2],   # overlaps anchor 0, same class -> suppressed
        [5, 5, 10, 10, 0.1, 0.6],       # class 1 (separate NMS)
        [50, 50, 4, 4, 0.2, 0.24],      # below conf 0.25 -> dropped
    ], np.float32)
    ki, kl, bx = onms.postprocess(pred, 0.25, 0.45)
    assert ki.tolist() == [0, 2] and kl.tolist() == [0, 1]
    np.testing.assert_array_equal(bx[0], [0, 0, 10, 10])


def test_argmax_first_index_on_ties():
    pred = np.array([[5, 5, 10, 10, 0.5, 0.5]], np.float32)
    ki, kl, _ = onms.postprocess(pred, 0.25, 0.45)
    assert kl.tolist() == [0]
