"""CPU restatement of the reference's detection loss ``ComputeLoss`` -- TEST INFRASTRUCTURE ONLY.

Follows yolov8/tools/loss.py (rafaelghiorzi/YOLO-MS) line by line in semantics:

  * bbox_iou (loss.py:9-91): xywh -> xyxy, IoU with ``union + eps`` (eps 1e-7), GIoU / DIoU / CIoU
    with the enclosing box; CIoU's alpha is detached; the enclosing diagonal has NO eps.
  * anchors (loss.py:414-438): per level, grid-cell centres ((w + 0.5) * stride, (h + 0.5) * stride),
    levels concatenated in head order, row-major over (h, w).
  * decode (loss.py:127-206): softmax over each side's 16 bins, expected bin index e_s (in GRID units,
    not multiplied by the stride -- the reference's own choice), x1 = ax - e0, y1 = ay - e1,
    x2 = ax + e2, y2 = ay + e3, returned as (cx, cy, w, h).
  * default_assigner (loss.py:221-373): plain IoU of every decoded prediction with every GT; per GT in
    target order: k = min(10, #(IoU > 0.1)); the k highest-IoU anchors become foreground, their
    target box / l-t-r-b distances are OVERWRITTEN by later GTs, their one-hot class bits ACCUMULATE.
  * forward (loss.py:376-677): per image, GT boxes (cx, cy, w, h) x (img_w, img_h); with foreground:
    the mean BCE over all anchors x classes is added TWICE (loss.py:530 and :551), box loss
    mean(1 - CIoU) over foreground (NaN -> 0), DFL: targets / stride, two-bin cross entropy with
    weights (1 - frac, frac), indices clamped to [0, 15], mean over foreground x 4 (NaN -> 0);
    without foreground: the BCE mean once.  Each term / batch, total = 7.5 box + 0.5 cls + 1.5 dfl.

Parity is PINNED: tests/golden/make_loss_golden.py runs the reference's own ComputeLoss in the build
container (its unused torchvision imports at loss.py:4 resolve to a stub module whose functions raise
if called) and tests/test_loss_golden.py requires this restatement to reproduce those fixtures
bit-for-bit in fp32 (values and every gradient element): all four IoU types, images without GT, a GT
without foreground, shared anchors, pos_weight, bf16-rounded maps, the 640 grid at nc = 80.  Top-k
ties are broken towards the lower anchor index (torch.topk's order for equal values is unspecified;
continuous IoUs do not tie).
Only tests/ may import this module.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

LAMBDA_BOX, LAMBDA_CLS, LAMBDA_DFL = 7.5, 0.5, 1.5
TOPK, IOU_MIN = 10, 0.1


def bbox_iou(box1, box2, xywh=True, GIoU=False, DIoU=False, CIoU=False, eps=1e-7):
    """IoU / GIoU / DIoU / CIoU of broadcastable boxes (loss.py:9-91)."""
    if xywh:
        b1 = torch.cat((box1[..., :2] - box1[..., 2:] / 2, box1[..., :2] + box1[..., 2:] / 2), -1)
        b2 = torch.cat((box2[..., :2] - box2[..., 2:] / 2, box2[..., :2] + box2[..., 2:] / 2), -1)
    else:
        b1, b2 = box1, box2
    iw = (torch.min(b1[..., 2], b2[..., 2]) - torch.max(b1[..., 0], b2[..., 0])).clamp(min=0)
    ih = (torch.min(b1[..., 3], b2[..., 3]) - torch.max(b1[..., 1], b2[..., 1])).clamp(min=0)
    inter = iw * ih
    a1 = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1])
    a2 = (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1])
    union = a1 + a2 - inter + eps
    iou = inter / union
    if not (GIoU or DIoU or CIoU):
        return iou
    cw = (torch.max(b1[..., 2], b2[..., 2]) - torch.min(b1[..., 0], b2[..., 0])).clamp(min=0)
    ch = (torch.max(b1[..., 3], b2[..., 3]) - torch.min(b1[..., 1], b2[..., 1])).clamp(min=0)
    if GIoU:
        c_area = cw * ch + eps
        return iou - (c_area - union) / c_area
    rho2 = ((b1[..., 0] + b1[..., 2]) / 2 - (b2[..., 0] + b2[..., 2]) / 2) ** 2 + \
           ((b1[..., 1] + b1[..., 3]) / 2 - (b2[..., 1] + b2[..., 3]) / 2) ** 2
    c2 = cw ** 2 + ch ** 2
    d = rho2 / c2
    if DIoU:
        return iou - d
    w1, h1 = b1[..., 2] - b1[..., 0], b1[..., 3] - b1[..., 1]
    w2, h2 = b2[..., 2] - b2[..., 0], b2[..., 3] - b2[..., 1]
    v = (4 / math.pi ** 2) * (torch.atan(w2 / (h2 + eps)) - torch.atan(w1 / (h1 + eps))) ** 2
    alpha = (v / (1 - iou + v + eps)).detach()
    return iou - d - alpha * v


def anchors(shapes, strides, dtype=torch.float32):
    """-> (A, 2) pixel centres and (A,) strides over the levels' (H, W) grids."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        sy, sx = torch.meshgrid(torch.arange(h, dtype=dtype) + 0.5, torch.arange(w, dtype=dtype) + 0.5,
                                indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2) * s)
        st.append(torch.full((h * w,), float(s), dtype=dtype))
    return torch.cat(pts), torch.cat(st)


def decode(dist, anc, dfl=16):
    """(A, 4*dfl) logits -> (A, 4) boxes (cx, cy, w, h) in pixels (grid-unit offsets, loss.py:127-206)."""
    p = F.softmax(dist.view(-1, 4, dfl), dim=2)
    e = (p * torch.arange(dfl, dtype=dist.dtype)).sum(2)
    x1, y1 = anc[:, 0] - e[:, 0], anc[:, 1] - e[:, 1]
    x2, y2 = anc[:, 0] + e[:, 2], anc[:, 1] + e[:, 3]
    return torch.stack(((x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1), -1)


def assign(pbox, gbox, glab, anc, nc):
    """loss.py:221-373 -> (target boxes, target scores, fg mask, target l-t-r-b), all (A, .)."""
    A = pbox.shape[0]
    tb = torch.zeros((A, 4), dtype=pbox.dtype)
    ts = torch.zeros((A, nc), dtype=pbox.dtype)
    fg = torch.zeros(A, dtype=torch.bool)
    tl = torch.zeros((A, 4), dtype=pbox.dtype)
    if gbox.shape[0] == 0:
        return tb, ts, fg, tl
    with torch.no_grad():
        ious = bbox_iou(pbox.unsqueeze(1), gbox.unsqueeze(0), xywh=True)        # (A, G)
    for i in range(gbox.shape[0]):
        col = ious[:, i]
        k = min(TOPK, int((col > IOU_MIN).sum()))
        if k == 0:
            continue
        idx = torch.tensor(_topk_lower_index(col, k), dtype=torch.long)   # ties -> lower anchor index
        fg[idx] = True
        g = gbox[i]
        tb[idx] = g
        ts[idx, int(glab[i])] = 1.0
        x1, y1, x2, y2 = g[0] - g[2] / 2, g[1] - g[3] / 2, g[0] + g[2] / 2, g[1] + g[3] / 2
        a = anc[idx]
        tl[idx] = torch.stack((a[:, 0] - x1, a[:, 1] - y1, x2 - a[:, 0], y2 - a[:, 1]), 1)
    return tb, ts, fg, tl


def _topk_lower_index(col, k):
    # stable descending sort: equal values keep ascending index order
    order = torch.sort(-col, stable=True).indices
    return order[:k].tolist()


def compute_loss(preds, targets, nc, img_size, strides=(8.0, 16.0, 32.0), dfl=16, iou_type="ciou",
                 pos_weight=None):
    """preds: list of (B, 4*dfl + nc, H, W) head maps (any float dtype; autograd-capable),
    targets: (M, 6) [img, cls, cx, cy, w, h] normalised.  -> (total, dict of the three terms)."""
    dt = preds[0].dtype
    B = preds[0].shape[0]
    img_h, img_w = img_size
    flat = torch.cat([p.reshape(B, p.shape[1], -1).permute(0, 2, 1) for p in preds], 1)
    anc, st = anchors([(p.shape[2], p.shape[3]) for p in preds], strides, dt)
    dist, cls = flat[..., :4 * dfl], flat[..., 4 * dfl:]
    bce = torch.nn.BCEWithLogitsLoss(pos_weight=pos_weight, reduction="none")
    lbox = torch.zeros((), dtype=dt)
    lcls = torch.zeros((), dtype=dt)
    ldfl = torch.zeros((), dtype=dt)
    for b in range(B):
        m = targets[:, 0] == b
        glab = targets[m, 1]
        gbox = targets[m, 2:].clone().to(dt)
        gbox[:, 0::2] *= img_w
        gbox[:, 1::2] *= img_h
        pb = decode(dist[b], anc, dfl)
        tb, ts, fg, tl = assign(pb.detach(), gbox, glab, anc, nc)
        nfg = int(fg.sum())
        if nfg > 0:
            lc = bce(cls[b], ts).mean()
            lcls = lcls + lc + lc
            iou = bbox_iou(pb[fg], tb[fg], xywh=True, CIoU=iou_type == "ciou", GIoU=iou_type == "giou",
                           DIoU=iou_type == "diou")
            lb = (1.0 - iou).mean()
            if torch.isnan(lb):
                lb = torch.zeros((), dtype=dt)
            lbox = lbox + lb
            t = (tl[fg] / st[fg].unsqueeze(1)).view(-1)
            left = t.floor().long()
            right = (t + 1.0).floor().long()
            wr = t - left.to(dt)
            wl = 1.0 - wr
            left, right = left.clamp(0, dfl - 1), right.clamp(0, dfl - 1)
            pd = dist[b][fg].reshape(-1, dfl)
            ld = (F.cross_entropy(pd, left, reduction="none") * wl +
                  F.cross_entropy(pd, right, reduction="none") * wr).mean()
            if torch.isnan(ld):
                ld = torch.zeros((), dtype=dt)
            ldfl = ldfl + ld
        else:
            lcls = lcls + bce(cls[b], ts).mean()
    lbox, lcls, ldfl = lbox / B, lcls / B, ldfl / B
    total = LAMBDA_BOX * lbox + LAMBDA_CLS * lcls + LAMBDA_DFL * ldfl
    return total, {"loss_box": lbox, "loss_cls": lcls, "loss_dfl": ldfl}
