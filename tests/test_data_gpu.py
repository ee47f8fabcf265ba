"""GPU input pipeline (csrc/preprocess.hip via yms.data) against the resize / normalize
restatement (oracle/preprocess_ref.py; dataset.py:124-134 + collate :235-267): variable-size
uint8 images batched into one launch, up- and down-scaling, odd sizes, flips, bf16 output, and
the end-to-end COCO json -> GPU batch path."""
import numpy as np
import pytest
import torch

from oracle import preprocess_ref as P
from yms import data as D

pytestmark = pytest.mark.gpu
MEAN, STD = D.IMAGENET_MEAN, D.IMAGENET_STD


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_resize_normalize_vs_reference(dtype, tol):
    rng = np.random.default_rng(3)
    sizes = [(480, 640), (640, 480), (333, 517), (1280, 960), (64, 64), (17, 1000)]
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]
    flags = [0, 1, 2, 3, 0, 1]
    dev = D.to_device(imgs, "cuda")
    out = D.resize_normalize(dev, (320, 352), MEAN, STD, flags, dtype).float().cpu().numpy()
    for i, im in enumerate(imgs):
        ref = P.resize_normalize(im, 320, 352, MEAN, STD, flags[i])
        err = np.abs(out[i] - ref).max()
        assert err <= tol * max(1.0, np.abs(ref).max()), (sizes[i], flags[i], err)


def test_coco_to_gpu_batch(tmp_path):
    from test_data_cpu import _coco
    ann = _coco(tmp_path, [(32, 48), (40, 40)])
    ds = D.COCODetection(str(tmp_path), str(ann), img_size=(64, 96), num_classes=3)
    batch = [ds[i] for i in range(len(ds))]
    x, tg = D.collate_to_gpu(batch, (64, 96), "cuda")
    assert x.shape == (2, 3, 64, 96) and tg.device.type == "cuda" and tg.shape[1] == 6
    for i, (img, t, f) in enumerate(batch):
        ref = P.resize_normalize(img, 64, 96, MEAN, STD, f)
        assert np.abs(x[i].cpu().numpy() - ref).max() < 2e-5
    _, _, t_host = D.collate_targets(batch)
    assert torch.equal(tg.cpu(), t_host)


AUG_FULL = {"hsv_h": 0.015, "hsv_s": 0.7, "hsv_v": 0.4, "degrees": 20.0, "translate": 0.1, "scale": 0.5,
            "shear": 8.0, "perspective": 0.08, "flipud": 0.5, "fliplr": 0.5}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_augment_normalize_vs_restatement(dtype):
    """yms_augment_normalize (one launch over a batch of variable-size images, every transform of
    dataset.py:91-127 drawn -- rotate, shift, random scale, shear, perspective, flips, HSV) against
    oracle/preprocess_ref.augment_normalize on the same sampled chains: the kernel evaluates the
    same fp32 operations in the same order (no FMA contraction), so fp32 outputs agree to the last
    bit on all but isolated pixels and bf16 within its rounding."""
    from test_augment_cpu import stages_of
    rng = np.random.default_rng(11)
    sizes = [(480, 640), (333, 517), (64, 64), (17, 200), (640, 480), (250, 250), (90, 120), (300, 40)]
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]
    prng = np.random.default_rng(5)
    plans = [D.sample_augmentation(prng, AUG_FULL, h, w, 160, 192) for h, w in sizes]
    # force coverage: every transform appears at least once over the batch
    applied = set(a for p in plans for a in p.applied)
    assert {"hsv", "rotate", "shift", "scale", "shear", "perspective", "fliplr", "flipud"} <= applied, applied
    dev = D.to_device(imgs, "cuda")
    out = D.augment_normalize(dev, plans, (160, 192), MEAN, STD, dtype).float().cpu().numpy()
    for i, (im, pl) in enumerate(zip(imgs, plans)):
        st, hsv = stages_of(pl)
        ref = P.augment_normalize(im, hsv, st, 160, 192, MEAN, STD)
        if dtype == torch.bfloat16:
            ref = torch.from_numpy(ref).to(torch.bfloat16).float().numpy()
        diff = np.abs(out[i] - ref)
        level = 1.0 / (255.0 * min(STD))                  # one intensity step after Normalize
        assert (diff > 1e-6).mean() < 1e-3, (i, pl.applied, (diff > 1e-6).mean())
        assert diff.max() <= 2 * level, (i, pl.applied, diff.max())


def test_augmented_dataset_to_gpu_batch(tmp_path):
    """COCODataset(transform_params, is_train) -> collate_to_gpu: the augmented batch equals the
    restatement of each sample's plan; targets are in the augmented frame."""
    from test_augment_cpu import stages_of
    from test_data_cpu import _coco
    ann = _coco(tmp_path, [(32, 48), (40, 40)])
    ds = D.COCODataset(str(tmp_path), str(ann), AUG_FULL, True, (64, 96), 3)
    batch = [ds[i] for i in range(len(ds))]
    x, tg = D.collate_to_gpu(batch, (64, 96), "cuda")
    assert x.shape == (2, 3, 64, 96) and tg.shape[1] == 6
    for i, (img, t, pl) in enumerate(batch):
        st, hsv = stages_of(pl)
        ref = P.augment_normalize(img, hsv, st, 64, 96, MEAN, STD)
        assert np.abs(x[i].cpu().numpy() - ref).max() <= 2.0 / (255.0 * min(STD))
