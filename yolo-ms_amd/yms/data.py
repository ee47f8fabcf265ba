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
not installed here.

Training augmentation (dataset.py:84-131, the albumentations chain HueSaturationValue -> Rotate ->
ShiftScaleRotate -> RandomScale -> Affine(shear) -> Perspective -> HorizontalFlip / VerticalFlip ->
Resize -> Normalize with BboxParams(coco, min_visibility 0.1, min_area 1)) is restated:
``sample_augmentation`` draws each image's transforms on the host in that order with
albumentations' probabilities and parameter distributions, composes them into a chain of
pixel-coordinate stages, and ``augment_normalize`` applies the whole chain plus Normalize in ONE
GPU launch (csrc/preprocess.hip: one bilinear sample per output pixel instead of one resampling
per transform); ``transform_boxes`` moves the COCO boxes through the same stages (corner
envelopes, clipped once at the end, then the visibility / area filters).  albumentations and cv2
are not installed, so parity with them is UNPINNED; the GPU kernel is pinned
to the restatement in oracle/preprocess_ref.py.
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


# ------------------------------------------------------------------------------------------
# training augmentation (dataset.py:84-131)
# ------------------------------------------------------------------------------------------
AUG_REFLECT101, AUG_CLAMP, AUG_CONSTANT = 0, 1, 2
AUG_MAX_STAGES = 8


class AugStage(ctypes.Structure):
    """One geometric stage: m maps OUTPUT pixel-index coordinates to the input frame (in_w x in_h)."""
    _fields_ = [("m", ctypes.c_float * 9), ("in_w", ctypes.c_int), ("in_h", ctypes.c_int),
                ("border", ctypes.c_int), ("pad_", ctypes.c_int)]


class AugImage(ctypes.Structure):
    """csrc/preprocess.hip AugImage (checked against yms_augment_image_bytes())."""
    _fields_ = [("src", ctypes.c_void_p), ("h", ctypes.c_int), ("w", ctypes.c_int), ("pitch", ctypes.c_int),
                ("nst", ctypes.c_int), ("hsv", ctypes.c_float * 3), ("do_hsv", ctypes.c_int),
                ("st", AugStage * AUG_MAX_STAGES)]


class AugPlan:
    """One image's sampled transform: optional HSV shift (LUT units) and geometric stages, each
    (F, in_w, in_h, out_w, out_h, border) with F the 3x3 FORWARD map of pixel-index coordinates
    (input -> output; homogeneous)."""

    def __init__(self, h, w):
        self.src_h, self.src_w = h, w
        self.hsv = None
        self.stages = []
        self.applied = []          # names of the transforms drawn (diagnostics / tests)

    @property
    def frame(self):
        if self.stages:
            return self.stages[-1][3], self.stages[-1][4]
        return self.src_w, self.src_h

    def add(self, F, out_w, out_h, border, name):
        in_w, in_h = self.frame
        self.stages.append((np.asarray(F, np.float64), in_w, in_h, int(out_w), int(out_h), border))
        self.applied.append(name)


def _rot_matrix(cx, cy, deg, scale=1.0):
    """cv2.getRotationMatrix2D(center, angle, scale) as a 3x3 (positive angle = counter-clockwise)."""
    a = np.deg2rad(deg)
    al, be = scale * np.cos(a), scale * np.sin(a)
    return np.array([[al, be, (1 - al) * cx - be * cy], [-be, al, be * cx + (1 - al) * cy], [0, 0, 1]])


def _resize_matrix(in_w, in_h, out_w, out_h):
    """cv2.resize INTER_LINEAR pixel-centre map, input index -> output index."""
    sx, sy = in_w / out_w, in_h / out_h
    return np.array([[1 / sx, 0, 0.5 / sx - 0.5], [0, 1 / sy, 0.5 / sy - 0.5], [0, 0, 1]])


def _homography(src, dst):
    """cv2.getPerspectiveTransform: the 3x3 H with dst ~ H src for four point pairs."""
    A, b = [], []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y])
        b += [u, v]
    h = np.linalg.solve(np.asarray(A, np.float64), np.asarray(b, np.float64))
    return np.append(h, 1.0).reshape(3, 3)


def sample_augmentation(rng, tp, h, w, out_h, out_w, is_train=True):
    """dataset.py:89-131 for one image of h x w pixels: each transform of the training list is
    drawn with albumentations' probability (p = 0.5; the flips p = fliplr / flipud) and parameter
    distribution, in list order, from the numpy Generator ``rng``; then the final Resize.
    tp: the config's augmentation dict (hsv_h/s/v, degrees, translate, scale, shear, perspective,
    fliplr, flipud)."""
    tp = tp or {}
    plan = AugPlan(h, w)
    if is_train:
        hl, sl, vl = (int(tp.get(k, 0) * 100) for k in ("hsv_h", "hsv_s", "hsv_v"))
        if tp.get("hsv_h", 0) > 0 or tp.get("hsv_s", 0) > 0 or tp.get("hsv_v", 0) > 0:
            if rng.random() < 0.5:     # A.HueSaturationValue(hue_shift_limit, sat_shift_limit, val_shift_limit)
                plan.hsv = (rng.uniform(-hl, hl), rng.uniform(-sl, sl), rng.uniform(-vl, vl))
                plan.applied.append("hsv")
        if tp.get("degrees", 0) > 0 and rng.random() < 0.5:       # A.Rotate(limit=degrees), reflect-101
            fw, fh = plan.frame
            ang = rng.uniform(-tp["degrees"], tp["degrees"])
            plan.add(_rot_matrix((fw - 1) / 2, (fh - 1) / 2, ang), fw, fh, AUG_REFLECT101, "rotate")
        if tp.get("translate", 0) > 0 and rng.random() < 0.5:     # A.ShiftScaleRotate(shift only), reflect-101
            fw, fh = plan.frame
            t = tp["translate"]
            dx, dy = rng.uniform(-t, t), rng.uniform(-t, t)
            plan.add(np.array([[1, 0, dx * fw], [0, 1, dy * fh], [0, 0, 1]]), fw, fh, AUG_REFLECT101, "shift")
        if tp.get("scale", 0) > 0 and rng.random() < 0.5:         # A.RandomScale(scale_limit): resized frame
            fw, fh = plan.frame
            sc = rng.uniform(1 - tp["scale"], 1 + tp["scale"])
            nw, nh = max(1, int(fw * sc)), max(1, int(fh * sc))
            plan.add(_resize_matrix(fw, fh, nw, nh), nw, nh, AUG_CLAMP, "scale")
        if tp.get("shear", 0) > 0 and rng.random() < 0.5:         # A.Affine(shear x / y in degrees), constant 0
            fw, fh = plan.frame
            shx, shy = (np.tan(np.deg2rad(rng.uniform(-tp["shear"], tp["shear"]))) for _ in range(2))
            cx, cy = (fw - 1) / 2, (fh - 1) / 2
            Sm = np.array([[1, shx, 0], [shy, 1, 0], [0, 0, 1]])
            T0 = np.array([[1, 0, -cx], [0, 1, -cy], [0, 0, 1]])
            T1 = np.array([[1, 0, cx], [0, 1, cy], [0, 0, 1]])
            plan.add(T1 @ Sm @ T0, fw, fh, AUG_CONSTANT, "shear")
        if tp.get("perspective", 0) > 0 and rng.random() < 0.5:   # A.Perspective(scale=(0, p)), keep_size
            fw, fh = plan.frame
            sc = rng.uniform(0, tp["perspective"])
            j = np.mod(np.abs(rng.normal(0, sc, (4, 2))), 0.32)
            quad = [(j[0, 0] * fw, j[0, 1] * fh), ((1 - j[1, 0]) * fw, j[1, 1] * fh),
                    ((1 - j[2, 0]) * fw, (1 - j[2, 1]) * fh), (j[3, 0] * fw, (1 - j[3, 1]) * fh)]
            quad = [(x - 0.5, y - 0.5) for x, y in quad]
            rect = [(0, 0), (fw - 1, 0), (fw - 1, fh - 1), (0, fh - 1)]
            plan.add(_homography(quad, rect), fw, fh, AUG_CONSTANT, "perspective")
        if tp.get("fliplr", 0) > 0 and rng.random() < tp["fliplr"]:
            fw, fh = plan.frame
            plan.add(np.array([[-1, 0, fw - 1], [0, 1, 0], [0, 0, 1]]), fw, fh, AUG_CLAMP, "fliplr")
        if tp.get("flipud", 0) > 0 and rng.random() < tp["flipud"]:
            fw, fh = plan.frame
            plan.add(np.array([[1, 0, 0], [0, -1, fh - 1], [0, 0, 1]]), fw, fh, AUG_CLAMP, "flipud")
    fw, fh = plan.frame
    plan.add(_resize_matrix(fw, fh, out_w, out_h), out_w, out_h, AUG_CLAMP, "resize")
    if len(plan.stages) > AUG_MAX_STAGES:
        raise RuntimeError("yms: augmentation chain longer than AUG_MAX_STAGES")
    return plan


def plan_struct(plan, image):
    """AugImage record of one plan over a device HWC uint8 image tensor."""
    rec = AugImage()
    rec.src = image.data_ptr()
    rec.h, rec.w, rec.pitch = image.shape[0], image.shape[1], image.stride(0)
    if (rec.h, rec.w) != (plan.src_h, plan.src_w):
        raise ValueError("yms: augmentation plan sampled for another image size")
    rec.nst = len(plan.stages)
    if plan.hsv is not None:
        rec.do_hsv = 1
        rec.hsv[:] = [float(v) for v in plan.hsv]
    for k, (F, in_w, in_h, _, _, border) in enumerate(plan.stages):
        M = np.linalg.inv(F)
        M = M / M[2, 2] if abs(M[2, 2]) > 1e-12 else M
        rec.st[k].m[:] = [float(v) for v in M.reshape(-1)]
        rec.st[k].in_w, rec.st[k].in_h, rec.st[k].border = in_w, in_h, border
    return rec


def augment_normalize(images, plans, size, mean=IMAGENET_MEAN, std=IMAGENET_STD, dtype=torch.float32):
    """Device HWC uint8 images + their sampled plans -> [B, 3, H, W] augmented, resized, normalised
    batch in one launch (yms_augment_normalize)."""
    if not images or len(images) != len(plans):
        raise ValueError("yms: one augmentation plan per image")
    dev = images[0].device
    if dev.type != "cuda":
        raise RuntimeError("yms: augment_normalize runs on ROCm GPU tensors only (no CPU fallback)")
    if L.lib().yms_augment_image_bytes() != ctypes.sizeof(AugImage):
        raise RuntimeError("yms: AugImage layout differs from the library's")
    H, W = size
    n = len(images)
    tab = (AugImage * n)()
    for i, (im, pl) in enumerate(zip(images, plans)):
        if im.device != dev or im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3 or im.stride(2) != 1 \
                or im.stride(1) != 3:
            raise ValueError("yms: images must be contiguous HWC uint8 RGB tensors on one device")
        if pl.frame != (W, H):
            raise ValueError("yms: plan's final Resize does not produce the batch size")
        tab[i] = plan_struct(pl, im)
    tab_dev = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(dev, non_blocking=False)
    out = torch.empty((n, 3, H, W), dtype=dtype, device=dev)
    L.call("yms_augment_normalize", L.dtype_code(dtype), n, tab_dev.data_ptr(), H, W,
           (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std), out.data_ptr(), L.stream_ptr(dev))
    for im in images:
        im.record_stream(torch.cuda.current_stream(dev))
    tab_dev.record_stream(torch.cuda.current_stream(dev))
    return out


def transform_boxes(boxes, labels, plan, min_visibility=0.1, min_area=1.0):
    """COCO [x, y, w, h] pixel boxes of the plan's source image -> [n, 5] targets (class, cx, cy, w, h
    normalised to the final frame).  Each box's corners go through every stage (continuous pixel
    coordinates, X = index + 0.5); the box is the envelope of its transformed corners, clipped to
    the final frame once; BboxParams(min_visibility=0.1, min_area=1) then drop boxes whose clipped
    area is below 10% of the unclipped one or below 1 px, and the reference's final checks apply
    (dataset.py:84-88, :218-228)."""
    out_w, out_h = plan.frame
    rows = []
    for (x, y, w, h), c in zip(boxes, labels):
        P = np.array([[x, y], [x + w, y], [x + w, y + h], [x, y + h]], np.float64) - 0.5
        for F, *_ in plan.stages:
            q = np.c_[P, np.ones(4)] @ F.T
            P = q[:, :2] / q[:, 2:3]
        P = P + 0.5
        x0, y0 = P.min(0)
        x1, y1 = P.max(0)
        area = (x1 - x0) * (y1 - y0)
        cx0, cy0 = min(max(x0, 0.0), out_w), min(max(y0, 0.0), out_h)
        cx1, cy1 = min(max(x1, 0.0), out_w), min(max(y1, 0.0), out_h)
        carea = max(cx1 - cx0, 0.0) * max(cy1 - cy0, 0.0)
        if area <= 0 or carea / area < min_visibility or carea < min_area:
            continue
        bw, bh = cx1 - cx0, cy1 - cy0
        cxn, cyn, wn, hn = (cx0 + bw / 2) / out_w, (cy0 + bh / 2) / out_h, bw / out_w, bh / out_h
        if wn > 1e-3 and hn > 1e-3 and 0 <= cxn <= 1 and 0 <= cyn <= 1 and 0 <= wn <= 1 and 0 <= hn <= 1:
            rows.append([c, cxn, cyn, wn, hn])
    return torch.tensor(rows, dtype=torch.float32) if rows else torch.empty(0, 5)


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


class COCODataset(COCODetection):
    """dataset.py:12-233 ``COCODataset(images_dir, annotations_file, transform_params=None,
    is_train=True, img_size=(640, 640), num_classes=80)``: the training transform of
    ``transform_params`` (the config's ``augmentation`` dict) is sampled per sample on the host
    (``sample_augmentation``) and applied on the GPU by the collate (``collate_to_gpu``);
    ``is_train=False`` keeps only the Resize.  ``__getitem__`` -> (decoded HWC uint8 image,
    [n, 5] targets in the augmented frame, AugPlan)."""

    def __init__(self, images_dir, annotations_file, transform_params=None, is_train=True, img_size=(640, 640),
                 num_classes=80, seed=0):
        super().__init__(images_dir, annotations_file, img_size=img_size, num_classes=num_classes, seed=seed)
        self.transform_params = dict(transform_params or {})
        self.is_train = is_train

    def __getitem__(self, idx):
        from PIL import Image
        if torch.is_tensor(idx):
            idx = idx.item()
        if not isinstance(idx, int):
            raise TypeError(f"Index should be an integer, got {type(idx).__name__} instead.")
        info = self.imgs[self.image_ids[idx]]
        image = np.array(Image.open(os.path.join(self.images_dir, info["file_name"])).convert("RGB"))
        boxes, labels = self.annotations(idx)
        h0, w0 = image.shape[:2]
        plan = sample_augmentation(self.sample_rng(idx), self.transform_params, h0, w0, self.img_h, self.img_w,
                                   self.is_train)
        return image, transform_boxes(boxes, labels, plan), plan


def collate_targets(batch):
    """[(image, [n, 5] targets, flags or AugPlan)] -> (images, flags / plans, [M, 6] targets with the
    batch index first)."""
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
    images, extra, targets = collate_targets(batch)
    dev_images = to_device(images, device)
    if extra and isinstance(extra[0], AugPlan):
        x = augment_normalize(dev_images, extra, img_size, mean, std, dtype)
    else:
        x = resize_normalize(dev_images, img_size, mean, std, extra, dtype)
    return x, targets.to(device, non_blocking=True)
