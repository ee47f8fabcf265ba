"""Training augmentation host half (yms/data.py: sample_augmentation, transform_boxes, the C-ABI record
layout) and known answers of its restatement (oracle/preprocess_ref.py augment_normalize), for the
reference's transform list dataset.py:84-131.  Parity with albumentations / cv2 is unpinned (neither
is installed); these pin the restated semantics."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import preprocess_ref as P
from yms import _lib as L
from yms import data as D

CFG = {"hsv_h": 0.015, "hsv_s": 0.7, "hsv_v": 0.4, "degrees": 0.0, "translate": 0.1, "scale": 0.5,
       "shear": 0.0, "perspective": 0.0, "flipud": 0.0, "fliplr": 0.5}       # config/coco_yolov8.yaml:44-56
MEAN, STD = D.IMAGENET_MEAN, D.IMAGENET_STD


def stages_of(plan):
    """(m float32[9], in_w, in_h, border) per stage, as plan_struct hands them to the kernel."""
    rec = D.plan_struct(plan, _FakeImage(plan.src_h, plan.src_w))
    return [(np.array(rec.st[k].m[:], np.float32), rec.st[k].in_w, rec.st[k].in_h, rec.st[k].border)
            for k in range(rec.nst)], (tuple(rec.hsv[:]) if rec.do_hsv else None)


class _FakeImage:
    def __init__(self, h, w):
        self.shape = (h, w, 3)

    def data_ptr(self):
        return 0

    def stride(self, d):
        return (self.shape[1] * 3, 3, 1)[d]


def test_record_layout_matches_library():
    assert ctypes.sizeof(D.AugImage) == L.lib().yms_augment_image_bytes()
    assert "yms_augment_normalize" in L.EXPORTED


def test_sampling_follows_the_reference_list():
    rng = np.random.default_rng(0)
    counts = {}
    for _ in range(2000):
        pl = D.sample_augmentation(rng, CFG, 480, 640, 640, 640)
        assert pl.frame == (640, 640) and pl.applied[-1] == "resize"
        order = [a for a in pl.applied if a != "resize"]
        assert order == sorted(order, key=["hsv", "rotate", "shift", "scale", "shear", "perspective",
                                           "fliplr", "flipud"].index)
        for a in pl.applied:
            counts[a] = counts.get(a, 0) + 1
        if pl.hsv is not None:
            dh, ds, dv = pl.hsv
            assert abs(dh) <= 1 and abs(ds) <= 70 and abs(dv) <= 40      # int(0.015*100), int(0.7*100), ...
    for a in ("hsv", "shift", "scale", "fliplr"):
        assert 900 < counts[a] < 1100, (a, counts[a])                  # p = 0.5 each
    assert "rotate" not in counts and "shear" not in counts and "perspective" not in counts   # 0 in the config
    # validation: only the Resize
    pl = D.sample_augmentation(rng, CFG, 480, 640, 320, 320, is_train=False)
    assert pl.applied == ["resize"] and pl.hsv is None


def test_identity_chain_is_the_plain_resize():
    img = np.random.default_rng(1).integers(0, 256, (37, 53, 3), dtype=np.uint8)
    pl = D.sample_augmentation(None, {}, 37, 53, 64, 96, is_train=False)
    st, hsv = stages_of(pl)
    a = P.augment_normalize(img, hsv, st, 64, 96, MEAN, STD)
    b = P.resize_normalize(img, 64, 96, MEAN, STD)
    assert np.abs(a - b).max() < 2e-5


def _plan(h, w, stages_fwd, out=None):
    pl = D.AugPlan(h, w)
    for F, ow, oh, border in stages_fwd:
        pl.add(F, ow, oh, border, "t")
    ow, oh = out or pl.frame
    fw, fh = pl.frame
    pl.add(D._resize_matrix(fw, fh, ow, oh), ow, oh, D.AUG_CLAMP, "resize")
    return pl


def test_rotate_90_and_flip_known_answers():
    img = np.random.default_rng(2).integers(0, 256, (24, 24, 3), dtype=np.uint8)
    ref = lambda im: P.resize_normalize(np.ascontiguousarray(im), 24, 24, MEAN, STD)
    rot = _plan(24, 24, [(D._rot_matrix(11.5, 11.5, 90.0), 24, 24, D.AUG_REFLECT101)])
    st, _ = stages_of(rot)
    assert np.abs(P.augment_normalize(img, None, st, 24, 24, MEAN, STD) - ref(np.rot90(img, 1))).max() < 1e-4
    flip = _plan(24, 24, [(np.array([[-1, 0, 23], [0, 1, 0], [0, 0, 1]]), 24, 24, D.AUG_CLAMP)])
    st, _ = stages_of(flip)
    assert np.abs(P.augment_normalize(img, None, st, 24, 24, MEAN, STD) - ref(img[:, ::-1])).max() < 1e-5


def test_shift_reflects_and_shear_blanks():
    img = np.random.default_rng(3).integers(0, 256, (16, 20, 3), dtype=np.uint8)
    # ShiftScaleRotate by +3 px in x, BORDER_REFLECT_101: out[:, x] = in[:, reflect(x - 3)]
    sh = _plan(16, 20, [(np.array([[1, 0, 3], [0, 1, 0], [0, 0, 1]]), 20, 16, D.AUG_REFLECT101)])
    st, _ = stages_of(sh)
    got = P.augment_normalize(img, None, st, 16, 20, MEAN, STD)
    idx = [abs(x - 3) for x in range(20)]
    assert np.abs(got - P.resize_normalize(np.ascontiguousarray(img[:, idx]), 16, 20, MEAN, STD)).max() < 1e-5
    # a constant-border stage that moves the image 100 px away: every pixel is 0 before Normalize
    far = _plan(16, 20, [(np.array([[1, 0, 100], [0, 1, 0], [0, 0, 1]]), 20, 16, D.AUG_CONSTANT)])
    st, _ = stages_of(far)
    got = P.augment_normalize(img, None, st, 16, 20, MEAN, STD)
    blank = (0.0 - np.asarray(MEAN, np.float32)) / np.asarray(STD, np.float32)
    assert np.abs(got - blank[:, None, None]).max() < 1e-6


def test_hsv_known_answers():
    rgb = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [128, 64, 32], [10, 10, 10]], np.float32)
    same = P.hsv_shift8(rgb, (0.0, 0.0, 0.0))
    assert np.abs(same - rgb).max() <= 2.0                  # 8-bit HSV round trip is within 2 levels
    grey = P.hsv_shift8(rgb, (0.0, -255.0, 0.0))            # saturation 0: r = g = b = v
    assert np.all(grey[:, 0] == grey[:, 1]) and np.all(grey[:, 1] == grey[:, 2])
    assert np.all(grey[:, 0] == rgb.max(1))
    bright = P.hsv_shift8(rgb, (0.0, 0.0, 255.0))           # value clipped at 255
    assert np.all(bright.max(1) == 255)
    hue = P.hsv_shift8(np.array([[255, 0, 0]], np.float32), (60.0, 0.0, 0.0))   # 120 degrees: red -> green
    assert hue.tolist() == [[0.0, 255.0, 0.0]]


def test_boxes_follow_the_stages():
    boxes, labels = [[10, 20, 30, 40], [0, 0, 4, 4]], [3, 7]
    # horizontal flip of a 100 x 80 (w x h) image, resize to 200 x 160
    flip = _plan(80, 100, [(np.array([[-1, 0, 99], [0, 1, 0], [0, 0, 1]]), 100, 80, D.AUG_CLAMP)], out=(200, 160))
    t = D.transform_boxes(boxes, labels, flip)
    assert t.shape == (2, 5)
    assert torch.allclose(t[0], torch.tensor([3.0, 1 - 25 / 100, 40 / 80, 30 / 100, 40 / 80]), atol=1e-6)
    # a shift that pushes box 1 to 99% outside the frame: dropped by min_visibility 0.1
    sh = _plan(80, 100, [(np.array([[1, 0, -3.96], [0, 1, 0], [0, 0, 1]]), 100, 80, D.AUG_REFLECT101)])
    t = D.transform_boxes(boxes, labels, sh)
    assert t.shape == (1, 5) and t[0, 0] == 3
    # RandomScale changes the frame, not the normalised boxes
    sc = _plan(80, 100, [(D._resize_matrix(100, 80, 150, 120), 150, 120, D.AUG_CLAMP)], out=(64, 64))
    t = D.transform_boxes(boxes, labels, sc)
    assert torch.allclose(t[0, 1:], torch.tensor([25 / 100, 40 / 80, 30 / 100, 40 / 80]), atol=1e-5)
    # rotation by 90 degrees about the centre of a square frame swaps the box's width and height
    rot = _plan(100, 100, [(D._rot_matrix(49.5, 49.5, 90.0), 100, 100, D.AUG_REFLECT101)])
    t = D.transform_boxes(boxes[:1], labels[:1], rot)
    assert torch.allclose(t[0, 3:], torch.tensor([40 / 100, 30 / 100]), atol=1e-5)
    # min_area = 1 px: a 0.5 x 0.5 px box vanishes
    assert D.transform_boxes([[5, 5, 0.5, 0.5]], [1], sc).shape == (0, 5)


@pytest.mark.parametrize("cfg", [CFG, dict(CFG, degrees=15.0, shear=5.0, perspective=0.05, flipud=0.5)])
def test_dataset_items_and_collate(tmp_path, cfg):
    import json

    from PIL import Image
    rng = np.random.default_rng(4)
    imgs = []
    for i, (h, w) in enumerate([(48, 64), (40, 40), (33, 71)]):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / f"{i}.png")
        imgs.append({"id": i + 1, "file_name": f"{i}.png", "height": h, "width": w})
    anns = [{"id": 1, "image_id": 1, "category_id": 5, "bbox": [4, 6, 20, 18], "area": 360, "iscrowd": 0},
            {"id": 2, "image_id": 2, "category_id": 9, "bbox": [10, 10, 15, 12], "area": 180, "iscrowd": 0},
            {"id": 3, "image_id": 3, "category_id": 5, "bbox": [1, 2, 60, 25], "area": 1500, "iscrowd": 0}]
    cats = [{"id": 5, "name": "a"}, {"id": 9, "name": "b"}]
    (tmp_path / "a.json").write_text(json.dumps({"images": imgs, "annotations": anns, "categories": cats}))
    ds = D.COCODataset(str(tmp_path), str(tmp_path / "a.json"), cfg, True, (64, 64), 2)
    items = [ds[i] for i in range(3)]
    for im, t, pl in items:
        assert isinstance(pl, D.AugPlan) and pl.frame == (64, 64)
        assert t.dim() == 2 and t.shape[1] == 5 and torch.all((t[:, 1:] >= 0) & (t[:, 1:] <= 1))
    images, plans, tg = D.collate_targets(items)
    assert len(plans) == 3 and tg.shape[1] == 6
    with pytest.raises(TypeError):
        ds["0"]
