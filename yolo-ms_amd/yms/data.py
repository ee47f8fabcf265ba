"""Input pipeline: the reference's COCO dataset + collate (yolov8/tools/dataset.py)
with the per-sample Resize / Normalize / ToTensorV2 moved to the GPU.

The reference decodes each image with PIL, transforms it on the host with albumentations (cv2
bilinear resize, normalize, HWC -> CHW fp32) and stacks fp32 tensors in ``collate_fn``
(dataset.py:143-267).  Here the host only decodes (PIL) and parses the annotations; the uint8 RGB
images travel to the GPU as decoded (a quarter of the fp32 bytes over PCIe, pinned + async), and
one ``yms_resize_normalize`` launch produces the whole ``[B, 3, H, W]`` batch (csrc/preprocess.hip).
Targets keep the reference's format: per image ``[n, 5]`` = (class, cx, cy, w, h) normalised,
collated to ``[M, 6]`` with the batch index first (dataset.py:235-267).

Annotations are read with the ``json`` module in pycocotools' orders (image ids sorted, category
ids in file order, annotations per image in file order); pycocotools, albumentations and cv2 are
not installed here.  Training colour / geometric augmentations other than the flips
(dataset.py:92-127) are not reproduced.
"""
from __future__ import annotations

import ctypes
import json
import os
from collections import defaultdict

import numpy as np
import torch

from . import _lib as L

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class PrepImage(ctypes.Structure):
    """csrc/preprocess.hip PrepImage: one decoded HWC uint8 image on the device."""
    _fields_ = [("src", ctypes.c_void_p), ("h", ctypes.c_int), ("w", ctypes.c_int), ("pitch", ctypes.c_int),
                ("flags", ctypes.c_int)]


def to_device(images, device, pin=True):
    """uint8 HWC numpy / torch images -> device uint8 tensors (pinned host staging, async copies)."""
    out = []
    for im in images:
        t = torch.as_tensor(np.ascontiguousarray(im)) if not isinstance(im, torch.Tensor) else im.contiguous()
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
            raise ValueError(f"yms: expected HWC uint8 RGB images, got {tuple(t.shape)} {t.dtype}")
        if t.device.type != "cuda":
            if pin:
                t = t.pin_memory()
            t = t.to(device, non_blocking=True)
        out.append(t)
    return out


def resize_normalize(images, size, mean=IMAGENET_MEAN, std=IMAGENET_STD, flips=None, dtype=torch.float32):
    """Device HWC uint8 images (any sizes) -> [B, 3, H, W] normalised batch on the GPU
    (A.Resize(INTER_LINEAR) + A.Normalize + ToTensorV2 + torch.stack).  flips: per-image bit 0 =
    horizontal, bit 1 = vertical (applied before the resize, as in the training transform)."""
    if not images:
        raise ValueError("yms: empty batch")
    dev = images[0].device
    if dev.type != "cuda":
        raise RuntimeError("yms: resize_normalize runs on ROCm GPU tensors only (no CPU fallback)")
    H, W = size
    n = len(images)
    tab = (PrepImage * n)()
    for i, im in enumerate(images):
        if im.device != dev or im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3 or im.stride(2) != 1 \
                or im.stride(1) != 3:
            raise ValueError("yms: images must be contiguous HWC uint8 RGB tensors on one device")
        tab[i] = PrepImage(im.data_ptr(), im.shape[0], im.shape[1], im.stride(0), int(flips[i]) if flips else 0)
    tab_dev = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(dev, non_blocking=False)
    out = torch.empty((n, 3, H, W), dtype=dtype, device=dev)
    L.call("yms_resize_normalize", L.dtype_code(dtype), n, tab_dev.data_ptr(), H, W,
           (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std), out.data_ptr(), L.stream_ptr(dev))
    # keep the images and the table alive until the kernel has read them (stream-ordered frees)
    for im in images:
        im.record_stream(torch.cuda.current_stream(dev))
    tab_dev.record_stream(torch.cuda.current_stream(dev))
    return out


def flip_targets(t, flags):
    """[n, 5] (class, cx, cy, w, h) normalised targets of a flipped image."""
    t = t.clone()
    if flags & 1:
        t[:, 1] = 1.0 - t[:, 1]
    if flags & 2:
        t[:, 2] = 1.0 - t[:, 2]
    return t


def coco_boxes_to_targets(boxes, labels, img_w, img_h, out_w, out_h):
    """COCO [x, y, w, h] pixel boxes of an (img_w x img_h) image -> [n, 5] targets after the resize to
    (out_w x out_h), with the reference's filters (A.BboxParams min_area = 1 px in the output
    image, dataset.py:85-88; final checks :218-228)."""
    rows = []
    for (x, y, w, h), c in zip(boxes, labels):
        sx, sy = out_w / img_w, out_h / img_h
        xr, yr, wr, hr = x * sx, y * sy, w * sx, h * sy
        if wr * hr < 1.0:
            continue
        cx, cy, wn, hn = (xr + wr / 2) / out_w, (yr + hr / 2) / out_h, wr / out_w, hr / out_h
        if wn > 1e-3 and hn > 1e-3 and 0 <= cx <= 1 and 0 <= cy <= 1 and 0 <= wn <= 1 and 0 <= hn <= 1:
            rows.append([c, cx, cy, wn, hn])
    return torch.tensor(rows, dtype=torch.float32) if rows else torch.empty(0, 5)


class COCODetection(torch.utils.data.Dataset):
    """dataset.py COCODataset's data source (image list, category map, annotation filters) without
    pycocotools; ``__getitem__`` returns (decoded HWC uint8 image, [n, 5] targets for ``img_size``),
    and ``collate_fn`` (or :func:`collate_to_gpu`) builds the GPU batch."""

    def __init__(self, images_dir, annotations_file, img_size=(640, 640), num_classes=80, fliplr=0.0, flipud=0.0,
                 seed=0):
        if not os.path.exists(annotations_file):
            raise FileNotFoundError(f"Annotations file not found: {annotations_file}")
        if not os.path.isdir(images_dir):
            raise NotADirectoryError(f"Images directory not found: {images_dir}")
        self.images_dir = images_dir
        self.img_h, self.img_w = img_size
        self.num_classes = num_classes
        self.fliplr, self.flipud = fliplr, flipud
        self.seed = int(seed)
        self._draws = 0
        d = json.load(open(annotations_file))
        self.imgs = {im["id"]: im for im in d.get("images", [])}
        self.img_to_anns = defaultdict(list)
        for a in d.get("annotations", []):
            self.img_to_anns[a["image_id"]].append(a)
        self.image_ids = [i for i in sorted(self.imgs)
                          if os.path.exists(os.path.join(images_dir, self.imgs[i]["file_name"]))]
        self.cat_ids = [c["id"] for c in d.get("categories", [])][:num_classes]
        self.cat2label = {c: i for i, c in enumerate(self.cat_ids)}
        self.label2cat = {i: c for i, c in enumerate(self.cat_ids)}

    def __len__(self):
        return len(self.image_ids)

    def annotations(self, idx):
        """-> (COCO [x, y, w, h] boxes, labels) kept by dataset.py:159-172's filters."""
        boxes, labels = [], []
        for a in self.img_to_anns[self.image_ids[idx]]:
            if a.get("iscrowd", 0) != 0 or not a.get("area", 0) > 0:
                continue
            lab = self.cat2label.get(a["category_id"])
            if lab is None:
                continue
            x, y, w, h = a["bbox"]
            if w <= 0 or h <= 0:
                continue
            boxes.append([x, y, w, h])
            labels.append(lab)
        return boxes, labels

    def __getitem__(self, idx):
        from PIL import Image
        info = self.imgs[self.image_ids[idx]]
        image = np.array(Image.open(os.path.join(self.images_dir, info["file_name"])).convert("RGB"))
        boxes, labels = self.annotations(idx)
        h0, w0 = image.shape[:2]
        t = coco_boxes_to_targets(boxes, labels, w0, h0, self.img_w, self.img_h)
        rng = self.sample_rng(idx)
        flags = (int(rng.random() < self.fliplr) if self.fliplr > 0 else 0) | \
                ((int(rng.random() < self.flipud) << 1) if self.flipud > 0 else 0)
        if flags:
            t = flip_targets(t, flags)
        return image, t, flags

    def sample_rng(self, idx):
        """Generator for one sample's random draws, seeded from (dataset seed, process stream, idx,
        draw count).  In a DataLoader worker the stream is torch's per-worker seed (base seed drawn
        anew for every epoch's iterator + worker id), so workers and epochs draw different streams;
        in the main process it is torch.initial_seed() and the draw counter moves epochs apart.  A
        Generator created once in __init__ would be forked unchanged into every worker instead."""
        info = torch.utils.data.get_worker_info()
        stream = info.seed if info is not None else torch.initial_seed()
        self._draws += 1
        return np.random.default_rng([self.seed, stream & 0xFFFFFFFFFFFFFFFF, int(idx), self._draws])

    def collate_fn(self, batch):
        """Host half of the collate: images stay decoded uint8; targets -> [M, 6] (dataset.py:235-267)."""
        return collate_targets(batch)


def collate_targets(batch):
    """[(image, [n, 5] targets, flags)] -> (images, flags, [M, 6] targets with the batch index first)."""
    images, flags, rows = [], [], []
    for i, (img, t, f) in enumerate(batch):
        images.append(img)
        flags.append(f)
        if t.shape[0] > 0:
            rows.append(torch.cat([torch.full((t.shape[0], 1), float(i)), t], 1))
    targets = torch.cat(rows, 0) if rows else torch.empty(0, 6)
    return images, flags, targets


def collate_to_gpu(batch, img_size, device, dtype=torch.float32, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """dataset.py collate_fn output on the GPU: ([B, 3, H, W] normalised images, [M, 6] targets)."""
    images, flags, targets = collate_targets(batch)
    dev_images = to_device(images, device)
    x = resize_normalize(dev_images, img_size, mean, std, flags, dtype)
    return x, targets.to(device, non_blocking=True)
