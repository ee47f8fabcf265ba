"""Detection loss on the MI355X: the reference's ``ComputeLoss`` (yolov8/tools/loss.py:94-677)
behind its own constructor and call, computed by the HIP kernels of csrc/det_loss.hip.

``ComputeLoss(head, nc, device, img_size)(preds_from_head, targets_collated) -> (loss, items)``:
``preds_from_head`` are the training head maps ([B, 64 + nc, H, W], as the yolov8 modules return
them: channels-last views of the plan's NHWC buffers), ``targets_collated`` the dataloader's
[M, 6] (image, class, cx, cy, w, h) normalised rows.  The returned ``loss`` is differentiable: the
kernels produce d(loss)/d(maps) together with the value (analytic gradients of BCE, CIoU / GIoU /
DIoU / IoU through the DFL decode, and the two-bin DFL cross entropy), so ``loss.backward()``
feeds them straight into the plan's backward.  ``items`` holds Python floats like the
reference's (``.item()`` synchronises; ``det_loss`` returns the device tensors instead).

Semantics are the reference's, including its quirks (oracle/loss_ref.py lists them): decoded
offsets in grid units, top-10 IoU assignment with later GTs overwriting, the BCE mean counted twice
for images with foreground, NaN box / DFL terms replaced by 0.  Only ``dfl_ch = reg_max = 16`` and
the fixed assigner are supported, as in the reference's training configuration.
"""
from __future__ import annotations

import ctypes
import math

import torch
from torch import nn

from yms import _lib as L

IOU_TYPES = {"iou": 0, "giou": 1, "diou": 2, "ciou": 3}
DFL_CH = 16


def bbox_iou(box1, box2, xywh=True, GIoU=False, DIoU=False, CIoU=False, eps=1e-7):
    """IoU / GIoU / DIoU / CIoU of broadcastable boxes (loss.py:9-91), elementwise torch ops on the
    boxes' device (a utility of the reference's API; the loss itself uses the fused kernels)."""
    if xywh:
        b1 = torch.cat((box1[..., :2] - box1[..., 2:] / 2, box1[..., :2] + box1[..., 2:] / 2), -1)
        b2 = torch.cat((box2[..., :2] - box2[..., 2:] / 2, box2[..., :2] + box2[..., 2:] / 2), -1)
    else:
        b1, b2 = box1, box2
    b1 = b1.to(b2.device).float()
    b2 = b2.float()
    iw = (torch.min(b1[..., 2], b2[..., 2]) - torch.max(b1[..., 0], b2[..., 0])).clamp(min=0)
    ih = (torch.min(b1[..., 3], b2[..., 3]) - torch.max(b1[..., 1], b2[..., 1])).clamp(min=0)
    inter = iw * ih
    union = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1]) + \
        (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1]) - inter + eps
    iou = inter / union
    if not (GIoU or DIoU or CIoU):
        return iou
    cw = (torch.max(b1[..., 2], b2[..., 2]) - torch.min(b1[..., 0], b2[..., 0])).clamp(min=0)
    ch = (torch.max(b1[..., 3], b2[..., 3]) - torch.min(b1[..., 1], b2[..., 1])).clamp(min=0)
    if GIoU:
        ca = cw * ch + eps
        return iou - (ca - union) / ca
    rho2 = ((b1[..., 0] + b1[..., 2]) / 2 - (b2[..., 0] + b2[..., 2]) / 2) ** 2 + \
        ((b1[..., 1] + b1[..., 3]) / 2 - (b2[..., 1] + b2[..., 3]) / 2) ** 2
    d = rho2 / (cw ** 2 + ch ** 2)
    if DIoU:
        return iou - d
    w1, h1 = b1[..., 2] - b1[..., 0], b1[..., 3] - b1[..., 1]
    w2, h2 = b2[..., 2] - b2[..., 0], b2[..., 3] - b2[..., 1]
    v = (4 / math.pi ** 2) * (torch.atan(w2 / (h2 + eps)) - torch.atan(w1 / (h1 + eps))) ** 2
    alpha = (v / (1 - iou + v + eps)).detach()
    return iou - d - alpha * v


def _nhwc(p):
    """[B, C, H, W] head map -> (NHWC base tensor [B, H, W, ld], ld) without a copy when it already is
    a channels-last view with a channel stride that is a multiple of 8."""
    B, C, H, W = p.shape
    s = p.stride()
    if s[1] == 1 and s[3] % 8 == 0 and s[3] >= C and s[2] == W * s[3] and s[0] == H * W * s[3]:
        base = torch.as_strided(p, (B, H, W, s[3]), (s[0], s[2], s[3], 1))
        return base, s[3]
    ld = (C + 7) // 8 * 8
    base = torch.zeros((B, H, W, ld), dtype=p.dtype, device=p.device)
    base[..., :C] = p.permute(0, 2, 3, 1)
    return base, ld


def _storage_elems(g):
    """Elements of the NHWC buffer under a channels-last gradient view (its padding channels, zero,
    scale to zero)."""
    B, C, H, W = g.shape
    return B * H * W * g.stride(2) // W if g.stride(1) == 1 else g.numel()


def det_loss(preds, targets, nc, img_size, strides=(8.0, 16.0, 32.0), iou_type="ciou", pos_weight=None,
             lambdas=(7.5, 0.5, 1.5), need_grad=True):
    """-> (out [4] fp32 device tensor = total, box, cls, dfl; list of gradient maps shaped like
    ``preds`` (channels-last, same dtype) or None)."""
    if not preds or any(p.device.type != "cuda" for p in preds):
        raise RuntimeError("yms: the detection loss runs on ROCm GPU tensors only (no CPU fallback)")
    if len(preds) > 4 or len(strides) < len(preds):
        raise ValueError("yms: 1-4 head levels with one stride each")
    dt = preds[0].dtype
    B = preds[0].shape[0]
    C = 4 * DFL_CH + nc
    for p in preds:
        if p.dim() != 4 or p.shape[0] != B or p.shape[1] != C or p.dtype != dt:
            raise ValueError(f"yms: head maps must be [B, {C}, H, W] of one dtype, got {tuple(p.shape)} {p.dtype}")
    bases = [_nhwc(p) for p in preds]
    ld = bases[0][1]
    if any(b[1] != ld for b in bases):          # one channel stride for every level: repack
        ld = (C + 7) // 8 * 8
        bases = []
        for p in preds:
            t = torch.zeros((B, p.shape[2], p.shape[3], ld), dtype=dt, device=p.device)
            t[..., :C] = p.permute(0, 2, 3, 1)
            bases.append((t, ld))
    dev = preds[0].device
    tg = targets.to(device=dev, dtype=torch.float32).reshape(-1, 6).contiguous()
    M = tg.shape[0]
    hs = [p.shape[2] for p in preds]
    ws = [p.shape[3] for p in preds]
    A = sum(h * w for h, w in zip(hs, ws))
    grads = None
    if need_grad:
        mk = torch.zeros if ld != C else torch.empty
        grads = [mk((B, h, w, ld), dtype=dt, device=dev) for h, w in zip(hs, ws)]
    pw = None
    if pos_weight is not None:
        pw = torch.as_tensor(pos_weight, dtype=torch.float32, device=dev).expand(nc).contiguous()
    wsb = L.lib().yms_det_loss_ws_bytes(B, A, nc, M)
    ws_t = torch.empty(wsb, dtype=torch.uint8, device=dev)
    out = torch.empty(4, dtype=torch.float32, device=dev)
    n = len(preds)
    maps = (ctypes.c_void_p * n)(*[b[0].data_ptr() for b in bases])
    gptr = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads]) if grads is not None else None
    img_h, img_w = img_size
    L.call("yms_det_loss", L.dtype_code(dt), B, nc, n, maps, gptr, (ctypes.c_int * n)(*hs), (ctypes.c_int * n)(*ws),
           (ctypes.c_float * n)(*[float(s) for s in strides[:n]]), ld, tg.data_ptr() if M else None, M,
           ctypes.c_float(float(img_w)), ctypes.c_float(float(img_h)), IOU_TYPES[iou_type], L.ptr(pw),
           (ctypes.c_float * 3)(*[float(x) for x in lambdas]), ws_t.data_ptr(), wsb, out.data_ptr(),
           L.stream_ptr(dev))
    if grads is not None:
        grads = [g[..., :C].permute(0, 3, 1, 2) for g in grads]
    return out, grads


class _DetLossFn(torch.autograd.Function):
    """-> (total [], terms [3] = box, cls, dfl).  The kernel produces d(total)/d(maps) only, so the
    terms are marked non-differentiable: backward through one of them raises instead of dropping it
    (the reference returns the terms as floats, loss.py:666-672)."""

    @staticmethod
    def forward(ctx, cfg, targets, *preds):
        out, grads = det_loss(list(preds), targets, *cfg, need_grad=any(p.requires_grad for p in preds))
        ctx.grads = grads
        ctx.n_preds = len(preds)
        terms = out[1:].clone()
        ctx.mark_non_differentiable(terms)
        return out[0].clone(), terms

    @staticmethod
    def backward(ctx, g, _gterms):
        grads = ctx.grads
        ctx.grads = None
        if grads is None:
            return (None, None) + (None,) * ctx.n_preds
        # grads *= g in place on the device (a no-op launch for the 1.0 seed of loss.backward()):
        # no elementwise pass over the head gradients, no host sync to test g
        gf = g.detach().to(torch.float32).contiguous()
        n = len(grads)
        L.call("yms_scale_by_device_scalar", L.dtype_code(grads[0].dtype), n,
               (ctypes.c_void_p * n)(*[gr.data_ptr() for gr in grads]),
               (ctypes.c_long * n)(*[_storage_elems(gr) for gr in grads]), gf.data_ptr(), L.stream_ptr(gf.device))
        return (None, None, *grads)


class ComputeLoss(nn.Module):
    """loss.py:94-677 interface: ``ComputeLoss(model_head, num_classes, device, img_size, strides,
    dfl_ch, reg_max, iou_type, bce_pos_weight)``; ``forward(preds_from_head, targets_collated) ->
    (total_loss, {"loss_box", "loss_cls", "loss_dfl", "total_loss"})``."""

    def __init__(self, model_head, num_classes, device, img_size, strides=(8.0, 16.0, 32.0), dfl_ch=16,
                 reg_max=16, iou_type="ciou", bce_pos_weight=None):
        super().__init__()
        if dfl_ch != DFL_CH or reg_max != DFL_CH:
            raise ValueError("yms: the fused loss supports dfl_ch = reg_max = 16 (the YOLOv8 head's)")
        self.iou_type = iou_type.lower()
        assert self.iou_type in IOU_TYPES, f"Unsupported iou_type: {iou_type}"
        self.model_head = model_head
        self.num_classes = num_classes
        self.device = device
        self.img_size_h, self.img_size_w = img_size[0], img_size[1]
        self.strides = torch.tensor(list(strides), device=device)
        self._strides = tuple(float(s) for s in strides)
        self.dfl_ch = dfl_ch
        self.reg_max = reg_max
        self.bce_pos_weight = bce_pos_weight
        self.lambda_box, self.lambda_cls, self.lambda_dfl = 7.5, 0.5, 1.5

    def forward(self, preds_from_head, targets_collated):
        total, terms = self.loss_tensor(preds_from_head, targets_collated)
        vals = torch.cat([total.detach().view(1), terms]).cpu().tolist()
        items = {"loss_box": vals[1], "loss_cls": vals[2], "loss_dfl": vals[3], "total_loss": vals[0]}
        return total, items

    def loss_tensor(self, preds_from_head, targets_collated):
        """-> (total [] device tensor, differentiable; terms [3] device tensor (box, cls, dfl), not
        differentiable); no host sync."""
        cfg = (self.num_classes, (self.img_size_h, self.img_size_w), self._strides, self.iou_type,
               self.bce_pos_weight, (self.lambda_box, self.lambda_cls, self.lambda_dfl))
        return _DetLossFn.apply(cfg, targets_collated, *preds_from_head)
