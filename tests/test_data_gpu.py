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
