"""Known-answer tests of the ComputeLoss restatement (oracle/loss_ref.py; yolov8/tools/loss.py:9-677).
The restatement is pinned to the reference's own outputs by tests/test_loss_golden.py; these add
hand-computed known answers for the semantics it claims."""
import math

import torch

from oracle import loss_ref as R


def test_bbox_iou_known_values():
    a = torch.tensor([[10.0, 10.0, 4.0, 4.0]])          # xywh: [8, 8, 12, 12]
    b = torch.tensor([[12.0, 10.0, 4.0, 4.0]])          # [10, 8, 14, 12]: overlap 2 x 4
    iou = R.bbox_iou(a, b, xywh=True)
    assert abs(iou.item() - 8.0 / (16 + 16 - 8 + 1e-7)) < 1e-7
    # identical boxes: IoU = 16 / (16 + eps); CIoU adds no distance / aspect terms
    c = R.bbox_iou(a, a, xywh=True, CIoU=True)
    assert abs(c.item() - 16.0 / (16.0 + 1e-7)) < 1e-7
    # DIoU of the shifted pair: centre distance 2^2, enclosing box 6 x 4 -> diagonal^2 52
    d = R.bbox_iou(a, b, xywh=True, DIoU=True)
    assert abs(d.item() - (iou.item() - 4.0 / 52.0)) < 1e-6
    # GIoU of disjoint boxes: 0 - (enclosing - union) / enclosing
    e = torch.tensor([[20.0, 10.0, 4.0, 4.0]])          # [18, 8, 22, 12]
    g = R.bbox_iou(a, e, xywh=True, GIoU=True)
    ca = 14.0 * 4.0 + 1e-7
    assert abs(g.item() - (0.0 - (ca - (32.0 + 1e-7)) / ca)) < 1e-6
    # CIoU aspect term for a 4x4 prediction vs an 8x2 target with the same centre
    f = torch.tensor([[10.0, 10.0, 8.0, 2.0]])
    ci = R.bbox_iou(a, f, xywh=True, CIoU=True)
    iou_af = 8.0 / (16 + 16 - 8 + 1e-7)
    v = 4 / math.pi ** 2 * (math.atan(8 / (2 + 1e-7)) - math.atan(4 / (4 + 1e-7))) ** 2
    alpha = v / (1 - iou_af + v + 1e-7)
    assert abs(ci.item() - (iou_af - 0.0 - alpha * v)) < 1e-6


def test_anchor_grid_and_decode():
    anc, st = R.anchors([(2, 3), (1, 1)], (8.0, 16.0))
    assert anc.tolist() == [[4, 4], [12, 4], [20, 4], [4, 12], [12, 12], [20, 12], [8, 8]]
    assert st.tolist() == [8, 8, 8, 8, 8, 8, 16]
    # one-hot-ish logits: side s concentrated on bin 2 -> offsets 2 (grid units, NOT x stride)
    dist = torch.full((1, 64), -1e4)
    for s in range(4):
        dist[0, s * 16 + 2] = 0.0
    box = R.decode(dist, torch.tensor([[100.0, 50.0]]))
    assert torch.allclose(box, torch.tensor([[100.0, 50.0, 4.0, 4.0]]))


def test_assignment_overwrite_and_class_accumulation():
    # 12 predictions along x; GT 1 (another class) overlaps GT 0 and shares 8 of its top-10 anchors
    A = 12
    pbox = torch.tensor([[50.0 + 0.01 * i, 50.0, 20.0, 20.0] for i in range(A)])
    anc = torch.tensor([[50.0 + 0.01 * i, 50.0] for i in range(A)])
    gbox = torch.tensor([[50.0, 50.0, 20.0, 20.0], [50.11, 50.0, 20.0, 20.0]])
    glab = torch.tensor([3.0, 1.0])
    tb, ts, fg, tl = R.assign(pbox, gbox, glab, anc, nc=5)
    both = fg.clone()
    ious0 = R.bbox_iou(pbox, gbox[0:1])
    top0 = set(torch.sort(-ious0, stable=True).indices[:10].tolist())
    ious1 = R.bbox_iou(pbox, gbox[1:2])
    top1 = set(torch.sort(-ious1, stable=True).indices[:10].tolist())
    assert int(fg.sum()) == len(top0 | top1) and top0 != top1   # top-10 of each GT, union of both
    for a in range(A):
        assert bool(both[a]) == (a in top0 or a in top1)
        # class bits accumulate; box / l-t-r-b come from the LAST GT that picked the anchor
        assert ts[a, 3].item() == (1.0 if a in top0 else 0.0)
        assert ts[a, 1].item() == (1.0 if a in top1 else 0.0)
        if a in top1:
            assert torch.equal(tb[a], gbox[1])
        elif a in top0:
            assert torch.equal(tb[a], gbox[0])


def test_assignment_needs_iou_above_threshold():
    pbox = torch.tensor([[0.0, 0.0, 1.0, 1.0], [100.0, 100.0, 10.0, 10.0]])
    anc = pbox[:, :2].clone()
    tb, ts, fg, tl = R.assign(pbox, torch.tensor([[300.0, 300.0, 5.0, 5.0]]), torch.tensor([0.0]), anc, nc=2)
    assert not fg.any() and ts.sum() == 0


def test_loss_terms_structure():
    """BCE mean counted twice with foreground, once without; image without GT; weights."""
    torch.manual_seed(0)
    nc = 3
    preds = [torch.randn(2, 64 + nc, 4, 4), torch.randn(2, 64 + nc, 2, 2)]
    img = (32, 32)
    targets = torch.tensor([[0, 1, 0.5, 0.5, 0.6, 0.6]])       # image 1 has no GT
    total, items = R.compute_loss(preds, targets, nc, img, strides=(8.0, 16.0))
    flat = torch.cat([p.reshape(2, 64 + nc, -1).permute(0, 2, 1) for p in preds], 1)
    bce1 = torch.nn.functional.binary_cross_entropy_with_logits(flat[1, :, 64:], torch.zeros(20, nc))
    anc, st = R.anchors([(4, 4), (2, 2)], (8.0, 16.0))
    pb0 = R.decode(flat[0, :, :64], anc)
    tb, ts, fg, tl = R.assign(pb0, torch.tensor([[16.0, 16.0, 19.2, 19.2]]), torch.tensor([1.0]), anc, nc)
    assert fg.any()
    bce0 = torch.nn.functional.binary_cross_entropy_with_logits(flat[0, :, 64:], ts)
    assert abs(items["loss_cls"].item() - (2 * bce0.item() + bce1.item()) / 2) < 1e-6
    assert abs(total.item() - (7.5 * items["loss_box"] + 0.5 * items["loss_cls"] + 1.5 * items["loss_dfl"]).item()) < 1e-5
