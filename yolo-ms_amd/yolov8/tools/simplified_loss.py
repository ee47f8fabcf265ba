"""``SimplifiedYOLOLoss`` drop-in: the training loss ``train.py`` imports (train.py:14) and builds
(train.py:321-330), with the reference's constructor (simplified_loss.py:12-22) and call
``criterion(predictions_from_head, targets) -> (loss, loss_items)``, computed on the MI355X by the
fused detection-loss kernels of csrc/det_loss.hip.

What it computes.  The reference's own ``SimplifiedYOLOLoss.forward`` cannot run on the head it is
paired with: it views a ``[B, 64 + nc, H, W]`` map as ``[B, -1, 4 + nc]``
(simplified_loss.py:44), which raises for nc = 80 at every resolution, and reads the anchor index
as the class (:52-53 vs :104-112).  There is no defined result to reproduce, so this class runs the
reference's legacy ``ComputeLoss`` semantics (loss.py:94-677: top-10 IoU assigner, BCE, CIoU, DFL)
-- the loss whose values ``tests/golden/loss_*.npz`` pin from the reference's own code -- with the
constructor's weights mapped onto its terms:

  box_weight -> lambda_box (ComputeLoss's 7.5),  cls_weight -> lambda_cls (0.5),
  DFL weight -> 1.5 (ComputeLoss's; the simplified loss has no DFL term to configure).

``alpha`` and ``gamma`` (the focal terms of simplified_loss.py:128-143) are accepted and stored but
not used: the classification term is ComputeLoss's BCE.  ``img_size`` and ``strides`` are used as
ComputeLoss uses them (grid of each level, anchor scale).

``loss_items`` carries the keys ``train.py:376-390`` reads (``loss_box``, ``loss_cls``,
``loss_dfl``) plus ``total_loss``, as Python floats.  ``loss`` is differentiable: the kernels
produce d(loss)/d(head maps) with the value, so ``loss.backward()`` drives the plan's backward.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from yolov8.tools.loss import ComputeLoss as _FusedComputeLoss

__all__ = ["SimplifiedYOLOLoss", "ComputeLoss", "bbox_iou"]


class SimplifiedYOLOLoss(nn.Module):
    """simplified_loss.py:6-22 constructor; ComputeLoss semantics on the GPU (module docstring)."""

    def __init__(self, num_classes, device, img_size=(640, 640), strides=[8, 16, 32],
                 alpha=0.25, gamma=1.5, box_weight=7.5, cls_weight=0.5):
        super().__init__()
        self.num_classes = num_classes
        self.device = device
        self.img_size = img_size
        self.alpha = alpha          # accepted, unused (module docstring)
        self.gamma = gamma          # accepted, unused
        self.box_weight = box_weight
        self.cls_weight = cls_weight
        self._loss = _FusedComputeLoss(None, num_classes, device, img_size,
                                       strides=tuple(float(s) for s in strides))
        self._loss.lambda_box = float(box_weight)
        self._loss.lambda_cls = float(cls_weight)
        self.strides = self._loss.strides

    def forward(self, predictions, targets):
        """predictions: the train-mode head maps ``[B, 64 + nc, H_i, W_i]``; targets ``[M, 6]`` =
        (image, class, cx, cy, w, h) normalised, as collate_fn emits them (dataset.py:235-267)."""
        return self._loss(predictions, targets)

    def loss_tensor(self, predictions, targets):
        """-> (total, [box, cls, dfl]) device tensors without a host sync (see ComputeLoss)."""
        return self._loss.loss_tensor(predictions, targets)


def ComputeLoss(model_head=None, num_classes=80, device='cpu', img_size=(640, 640),
                strides=[8, 16, 32], dfl_ch=16, reg_max=16, iou_type='ciou'):
    """The factory simplified_loss.py:156-167 keeps for backwards compatibility: returns a
    ``SimplifiedYOLOLoss`` over ``num_classes`` / ``img_size`` / ``strides``."""
    return SimplifiedYOLOLoss(num_classes=num_classes, device=device, img_size=img_size, strides=strides)


def _pairwise_iou(b1, b2):
    """[N,4] x [M,4] xyxy -> (iou [N,M], union [N,M]), torchvision ``box_iou``'s arithmetic."""
    a1 = (b1[:, 2] - b1[:, 0]) * (b1[:, 3] - b1[:, 1])
    a2 = (b2[:, 2] - b2[:, 0]) * (b2[:, 3] - b2[:, 1])
    lt = torch.max(b1[:, None, :2], b2[None, :, :2])
    rb = torch.min(b1[:, None, 2:], b2[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = a1[:, None] + a2[None, :] - inter
    return inter / union, union


def bbox_iou(box1, box2, xywh=True, GIoU=False, DIoU=False, CIoU=False, eps=1e-7):
    """The validation helper simplified_loss.py:170-185 defines (imported by train.py:14): the
    PAIRWISE [N, M] IoU matrix of box1 [N,4] and box2 [M,4] -- torchvision ``box_iou``, or
    ``complete_box_iou`` (eps 1e-7) when CIoU -- restated in torch ops on the boxes' device
    (torchvision is absent here: parity with it is unpinned; tests/test_simplified_loss_cpu.py).
    GIoU / DIoU are accepted and, as in the reference, ignored."""
    if xywh:
        box1 = torch.cat((box1[..., :2] - box1[..., 2:] / 2, box1[..., :2] + box1[..., 2:] / 2), dim=-1)
        box2 = torch.cat((box2[..., :2] - box2[..., 2:] / 2, box2[..., :2] + box2[..., 2:] / 2), dim=-1)
    iou, _ = _pairwise_iou(box1, box2)
    if not CIoU:
        return iou
    # torchvision complete_box_iou: DIoU term over the enclosing box diagonal, then the aspect term
    lti = torch.min(box1[:, None, :2], box2[None, :, :2])
    rbi = torch.max(box1[:, None, 2:], box2[None, :, 2:])
    whi = (rbi - lti).clamp(min=0)
    diag = whi[..., 0] ** 2 + whi[..., 1] ** 2 + eps
    c1 = (box1[:, :2] + box1[:, 2:]) / 2
    c2 = (box2[:, :2] + box2[:, 2:]) / 2
    cdist = ((c1[:, None, :] - c2[None, :, :]) ** 2).sum(-1)
    diou = iou - cdist / diag
    w1, h1 = box1[:, 2] - box1[:, 0], box1[:, 3] - box1[:, 1]
    w2, h2 = box2[:, 2] - box2[:, 0], box2[:, 3] - box2[:, 1]
    v = (4 / (math.pi ** 2)) * (torch.atan(w1 / h1)[:, None] - torch.atan(w2 / h2)[None, :]) ** 2
    with torch.no_grad():
        alpha = v / (1 - iou + v + eps)
    return diou - alpha * v
