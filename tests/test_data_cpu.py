"""Input pipeline host half (yms/data.py; reference yolov8/tools/dataset.py:12-267): COCO json
parsing in pycocotools' orders and the dataset's filters, target conversion, collate format, and
known answers of the resize / normalize restatement (oracle/preprocess_ref.py)."""
import json

import numpy as np
import pytest
import torch

from oracle import preprocess_ref as P
from yms import data as D


def _coco(tmp_path, sizes):
    from PIL import Image
    rng = np.random.default_rng(0)
    imgs = []
    for i, (h, w) in enumerate(sizes):
        fn = f"im{i}.png"
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / fn)
        imgs.append({"id": 10 - i, "file_name": fn, "height": h, "width": w})
    imgs.append({"id": 99, "file_name": "missing.png", "height": 8, "width": 8})   # filtered out
    cats = [{"id": 7, "name": "b"}, {"id": 3, "name": "a"}, {"id": 5, "name": "c"}]   # file order, not sorted
    anns = [
        {"id": 1, "image_id": 10, "category_id": 3, "bbox": [2, 4, 10, 6], "area": 60, "iscrowd": 0},
        {"id": 2, "image_id": 10, "category_id": 7, "bbox": [0, 0, 5, 5], "area": 25, "iscrowd": 1},   # crowd
        {"id": 3, "image_id": 10, "category_id": 5, "bbox": [1, 1, 4, 4], "area": 0, "iscrowd": 0},    # zero area
        {"id": 4, "image_id": 9, "category_id": 5, "bbox": [3, 3, 0, 4], "area": 5, "iscrowd": 0},     # w = 0
        {"id": 5, "image_id": 9, "category_id": 7, "bbox": [1, 2, 20, 10], "area": 200, "iscrowd": 0},
        {"id": 6, "image_id": 9, "category_id": 42, "bbox": [1, 2, 3, 4], "area": 12, "iscrowd": 0},   # unknown cat
    ]
    p = tmp_path / "ann.json"
    p.write_text(json.dumps({"images": imgs, "annotations": anns, "categories": cats}))
    return p


def test_coco_parsing_filters_and_targets(tmp_path):
    ann = _coco(tmp_path, [(32, 48), (40, 40)])
    ds = D.COCODetection(str(tmp_path), str(ann), img_size=(64, 64), num_classes=2)
    assert ds.image_ids == [9, 10]                      # sorted ids, missing file dropped
    assert ds.cat_ids == [7, 3] and ds.cat2label == {7: 0, 3: 1}   # first num_classes in file order
    img, t, flags = ds[1]                               # image id 10: 32 x 48
    assert img.shape == (32, 48, 3) and img.dtype == np.uint8 and flags == 0
    assert t.shape == (1, 5)
    exp = [1, (2 + 5) / 48, (4 + 3) / 32, 10 / 48, 6 / 32]
    assert torch.allclose(t[0], torch.tensor(exp, dtype=torch.float32))
    _, t9, _ = ds[0]                                    # id 9: w=0 and unknown category dropped
    assert t9.shape == (1, 5) and t9[0, 0] == 0
    images, fl, tg = D.collate_targets([ds[0], ds[1]])
    assert tg.shape == (2, 6) and tg[:, 0].tolist() == [0.0, 1.0] and fl == [0, 0]


def test_target_filters_and_flips():
    # a 0.5 x 0.5 px box becomes < 1 px^2 after a downscale: dropped (A.BboxParams min_area = 1)
    t = D.coco_boxes_to_targets([[10, 10, 0.5, 0.5], [0, 0, 100, 50]], [0, 1], 200, 100, 100, 50)
    assert t.shape == (1, 5) and t[0, 0] == 1
    assert torch.allclose(t[0, 1:], torch.tensor([0.25, 0.25, 0.5, 0.5]))
    f = D.flip_targets(t, 3)
    assert torch.allclose(f[0, 1:], torch.tensor([0.75, 0.75, 0.5, 0.5]))


def test_resize_reference_known_answers():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (5, 7, 3), dtype=np.uint8)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    same = P.resize_normalize(img, 5, 7, mean, std)      # identity size: the normalised pixels
    exp = ((img.astype(np.float32) / 255 - np.float32(mean)) / np.float32(std)).transpose(2, 0, 1)
    assert np.allclose(same, exp, atol=1e-6)
    const = np.full((9, 11, 3), 77, np.uint8)
    out = P.resize_normalize(const, 4, 6, (0, 0, 0), (1, 1, 1))
    assert np.allclose(out, 77 / 255, atol=1e-6)
    # 2x upscale of a 2x2 image: half-pixel centres -> weights 0, 0.25, 0.75, clamped at the edges
    g = np.array([[[0, 0, 0], [100, 100, 100]], [[200, 200, 200], [40, 40, 40]]], np.uint8)
    up = P.resize_normalize(g, 4, 4, (0, 0, 0), (1, 1, 1))[0] * 255
    row0 = [0, 25, 75, 100]
    assert np.allclose(up[0], row0, atol=1e-4)
    assert np.allclose(up[:, 0], [0, 50, 150, 200], atol=1e-4)
    # flips act before the resize
    fl = P.resize_normalize(g, 4, 4, (0, 0, 0), (1, 1, 1), flags=1)[0] * 255
    assert np.allclose(fl[0], row0[::-1], atol=1e-4)


def test_flip_streams_differ_across_workers_and_epochs(tmp_path):
    """Each DataLoader worker (and each epoch of non-persistent workers) draws its own flip stream:
    a Generator built in __init__ would be forked identically into every worker."""
    ann = _coco(tmp_path, [(8, 8)] * 2)
    ds = D.COCODetection(str(tmp_path), str(ann), img_size=(8, 8), num_classes=2, fliplr=0.5, flipud=0.5)
    idx = [0, 1] * 32
    sub = torch.utils.data.Subset(ds, idx)

    def epoch(seed):
        torch.manual_seed(seed)
        dl = torch.utils.data.DataLoader(sub, batch_size=16, num_workers=2, collate_fn=ds.collate_fn,
                                         multiprocessing_context="fork")
        return [tuple(f) for _, f, _ in dl]

    e1 = epoch(0)
    assert len(e1) == 4
    # batches 0 and 2 come from worker 0, 1 and 3 from worker 1: same indices, different draws
    assert e1[0] != e1[1] and e1[2] != e1[3]
    assert epoch(1) != e1                    # a new epoch (new base seed) draws anew
    assert epoch(0) == e1                    # and the stream is reproducible from torch's seed
