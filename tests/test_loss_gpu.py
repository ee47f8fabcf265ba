"""GPU detection loss (csrc/det_loss.hip via yolov8.tools.loss.ComputeLoss) against the CPU
restatement of the reference's ComputeLoss (oracle/loss_ref.py; loss.py:94-677): the three terms
and d(total)/d(head maps) (autograd through the restatement), on random head maps with targets
covering the reference's edge cases -- images without GT, a GT no prediction overlaps (no
foreground), GTs of different classes sharing anchors (overwritten boxes, accumulated class bits),
every IoU variant, BCE pos_weight, bf16 maps, the full 640x640 anchor grid at nc = 80.  The
restatement is pinned bit-for-bit to the reference's own ComputeLoss by the fixtures of
tests/golden/make_loss_golden.py (tests/test_loss_golden.py); test_loss_vs_reference_fixtures checks
the GPU kernels against those fixtures directly."""
import numpy as np
import pytest
import torch

import vectors as V
from oracle import loss_ref as R
from test_loss_golden import CASES, check_against_fixture
from yolov8.tools.loss import ComputeLoss, det_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _maps(B, nc, shapes, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(B, 64 + nc, h, w, generator=g) * scale for h, w in shapes]


def _channels_last(p, dtype):
    """NCHW-shaped channels-last view of an NHWC buffer, like the plan's head outputs."""
    return p.to(DEV, dtype).permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)


def _targets(B, nc, n_per_img, seed, extra=()):
    g = torch.Generator().manual_seed(seed)
    rows = []
    for b in range(B):
        for _ in range(n_per_img[b] if isinstance(n_per_img, (list, tuple)) else n_per_img):
            wh = torch.rand(2, generator=g) * 0.4 + 0.05
            c = torch.rand(2, generator=g) * (1 - wh) + wh / 2
            rows.append([b, int(torch.randint(0, nc, (1,), generator=g)), c[0], c[1], wh[0], wh[1]])
    rows += list(extra)
    return torch.tensor(rows, dtype=torch.float32).reshape(-1, 6)


def _check(preds_cpu, targets, nc, img, strides, dtype=torch.float32, iou_type="ciou", pos_weight=None,
           tol=2e-5, gtol=2e-4):
    # oracle on the dtype-rounded maps, fp64 arithmetic, autograd gradients
    ref_in = [p.to(dtype).double().requires_grad_(True) for p in preds_cpu]
    pw = None if pos_weight is None else torch.as_tensor(pos_weight, dtype=torch.float64)
    total, items = R.compute_loss(ref_in, targets.double(), nc, img, strides, iou_type=iou_type, pos_weight=pw)
    total.backward()
    preds = [_channels_last(p, dtype).requires_grad_(True) for p in preds_cpu]
    out, grads = det_loss(preds, targets.to(DEV), nc, img, strides, iou_type=iou_type,
                          pos_weight=pos_weight)
    o = out.cpu().double()
    ref = torch.stack([total.detach(), items["loss_box"].detach(), items["loss_cls"].detach(),
                       items["loss_dfl"].detach()])
    assert torch.isfinite(o).all()
    err = ((o - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
    assert err < tol, (o.tolist(), ref.tolist())
    for g, r in zip(grads, ref_in):
        gg = g.float().cpu().double()
        rel = ((gg - r.grad).norm() / r.grad.norm().clamp_min(1e-30)).item()
        assert rel < gtol, rel
    return o


@pytest.mark.parametrize("name", CASES)
def test_loss_vs_reference_fixtures(name):
    """det_loss vs the reference ComputeLoss's own outputs (fp32 maps; bf16 for the bf16-rounded case,
    whose gradient is stored in bf16: half-ulp 2^-9 relative per element)."""
    z = V.load_loss_case(name)
    bf16 = bool(z["bf16"][0])
    dtype = torch.bfloat16 if bf16 else torch.float32
    vtol, gtol = (1e-4, 4e-3) if bf16 else (2e-5, 2e-4)
    for iou in z["ious"]:
        preds = [_channels_last(torch.from_numpy(m), dtype).requires_grad_(True) for m in z["maps"]]
        pw = None if "pos_weight" not in z else torch.from_numpy(z["pos_weight"])
        out, grads = det_loss(preds, torch.from_numpy(z["targets"]).to(DEV), z["nc"], z["img"],
                              iou_type=iou, pos_weight=pw)
        vals = out.cpu().double().numpy()
        assert np.isfinite(vals).all()
        check_against_fixture(z, iou, vals, [g.float().cpu().double().numpy() for g in grads], vtol, gtol)


@pytest.mark.parametrize("iou_type", ["ciou", "giou", "diou", "iou"])
def test_loss_small_vs_oracle(iou_type):
    B, nc, img, strides = 3, 5, (64, 96), (8.0, 16.0, 32.0)
    shapes = [(8, 12), (4, 6), (2, 3)]
    preds = _maps(B, nc, shapes, 1, scale=2.0)
    extra = [[1, 2, 0.9, 0.9, 0.001, 0.001],       # tiny GT far from every prediction: no foreground
             [0, 4, 0.5, 0.5, 0.5, 0.5], [0, 1, 0.52, 0.5, 0.5, 0.5]]   # two classes, shared anchors
    targets = _targets(B, nc, [3, 0, 4], 2, extra)    # image 1: only the tiny GT -> no foreground
    _check(preds, targets, nc, img, strides, iou_type=iou_type)


def test_loss_no_targets_and_pos_weight():
    B, nc, img, strides = 2, 7, (64, 64), (8.0, 16.0, 32.0)
    preds = _maps(B, nc, [(8, 8), (4, 4), (2, 2)], 3)
    _check(preds, torch.zeros((0, 6)), nc, img, strides)
    pw = torch.linspace(0.5, 3.0, nc)
    _check(preds, _targets(B, nc, 5, 4), nc, img, strides, pos_weight=pw)


def test_loss_bf16_maps():
    B, nc, img, strides = 2, 80, (128, 128), (8.0, 16.0, 32.0)
    preds = _maps(B, nc, [(16, 16), (8, 8), (4, 4)], 5, scale=1.5)
    # gradients are stored in bf16 (half-ulp 2^-9 ~ 2e-3 relative per element)
    _check(preds, _targets(B, nc, 6, 6), nc, img, strides, dtype=torch.bfloat16, tol=1e-4, gtol=4e-3)


def test_loss_640_full_grid_nc80():
    """The bench's anchor grid (8400 anchors, three levels) with 8 GTs per image."""
    B, nc, img, strides = 2, 80, (640, 640), (8.0, 16.0, 32.0)
    preds = _maps(B, nc, [(80, 80), (40, 40), (20, 20)], 7, scale=3.0)
    _check(preds, _targets(B, nc, 8, 8), nc, img, strides, tol=5e-5, gtol=5e-4)


def test_compute_loss_module_backward_through_model():
    """ComputeLoss (reference constructor / call) on the yolov8 model's training head maps:
    loss.backward() reaches every parameter through the plan's backward."""
    from yolov8.yolov8 import YOLOv8
    torch.manual_seed(0)
    m = YOLOv8("n", 80).to(DEV).train()
    crit = ComputeLoss(m.head, 80, DEV, (128, 128))
    x = torch.randn(2, 3, 128, 128, device=DEV)
    tg = _targets(2, 80, 4, 9).to(DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        outs = m(x)
    loss, items = crit(outs, tg)
    assert set(items) == {"loss_box", "loss_cls", "loss_dfl", "total_loss"}
    assert abs(items["total_loss"] - (7.5 * items["loss_box"] + 0.5 * items["loss_cls"] +
                                      1.5 * items["loss_dfl"])) < 1e-4 * abs(items["total_loss"])
    loss.backward()
    grads = [p.grad for p in m.parameters() if p.requires_grad]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)
    assert sum(float(g.abs().sum()) > 0 for g in grads) >= len(grads) - 1   # DFL projection excluded


def test_loss_terms_are_reported_not_differentiable():
    """loss_tensor -> (total, terms): total carries d(total)/d(maps); the terms are values, and a
    backward through one of them raises instead of being dropped silently."""
    B, nc = 2, 7
    preds = [_channels_last(p, torch.float32).requires_grad_(True)
             for p in _maps(B, nc, [(8, 8), (4, 4), (2, 2)], 3)]
    crit = ComputeLoss(None, nc, DEV, (64, 64))
    total, terms = crit.loss_tensor(preds, _targets(B, nc, 4, 5).to(DEV))
    assert terms.shape == (3,) and not terms.requires_grad
    with pytest.raises(RuntimeError):
        terms[0].backward()
    total.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in preds)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("gscale", [1.0, 2.5, 0.3, 0.0])
def test_loss_backward_scales_by_incoming_grad(dtype, gscale):
    """The loss's autograd backward multiplies its map gradients by the incoming d(out)/d(total) on
    the device (yms_scale_by_device_scalar; a no-op launch for the 1.0 seed): bit-identical to
    torch's `grad * g.to(grad.dtype)` on the g = 1 gradients, padding channels included."""
    B, nc = 2, 7                                      # 64 + 7 = 71 channels: NHWC ld 72 (a padding lane)
    maps = _maps(B, nc, [(8, 8), (4, 4), (2, 2)], 11)
    tg = _targets(B, nc, 4, 12).to(DEV)
    crit = ComputeLoss(None, nc, DEV, (64, 64))
    ref_preds = [_channels_last(p, dtype).requires_grad_(True) for p in maps]
    crit.loss_tensor(ref_preds, tg)[0].backward()
    preds = [_channels_last(p, dtype).requires_grad_(True) for p in maps]
    total = crit.loss_tensor(preds, tg)[0]
    (total * gscale).backward()
    g = torch.tensor(gscale, device=DEV)
    for p, r in zip(preds, ref_preds):
        want = r.grad * g.to(dtype)
        assert p.grad.dtype == dtype and torch.equal(p.grad, want)


@pytest.mark.parametrize("name", [c for c in CASES if c != "posw"])
def test_simplified_loss_dropin_vs_reference_fixtures(name):
    """yolov8.tools.simplified_loss.SimplifiedYOLOLoss built with train.py:321-330's exact keyword set
    (the reference's defaults for alpha / gamma / box_weight / cls_weight) runs ComputeLoss's CIoU
    semantics: its total and terms and d(total)/d(maps) match the reference-generated fixtures."""
    from yolov8.tools.simplified_loss import SimplifiedYOLOLoss
    z = V.load_loss_case(name)
    if "ciou" not in z["ious"]:
        pytest.skip("fixture has no CIoU case")
    bf16 = bool(z["bf16"][0])
    dtype = torch.bfloat16 if bf16 else torch.float32
    vtol, gtol = (1e-4, 4e-3) if bf16 else (2e-5, 2e-4)
    img_h, img_w = z["img"]
    crit = SimplifiedYOLOLoss(num_classes=z["nc"], device=DEV, img_size=(img_h, img_w),
                              strides=[8., 16., 32.], alpha=0.25, gamma=1.5, box_weight=7.5, cls_weight=0.5)
    preds = [_channels_last(torch.from_numpy(m), dtype).requires_grad_(True) for m in z["maps"]]
    loss, items = crit(preds, torch.from_numpy(z["targets"]).to(DEV))
    assert set(items) >= {"loss_box", "loss_cls", "loss_dfl"}
    loss.backward()
    vals = np.array([items["total_loss"], items["loss_box"], items["loss_cls"], items["loss_dfl"]])
    assert abs(float(loss) - vals[0]) <= 1e-6 * max(1.0, abs(vals[0]))
    check_against_fixture(z, "ciou", vals, [p.grad.float().cpu().double().numpy() for p in preds], vtol, gtol)


def test_simplified_loss_weights_map_onto_terms():
    """box_weight / cls_weight scale the box and classification terms (DFL keeps ComputeLoss's 1.5);
    the terms themselves do not depend on the weights."""
    from yolov8.tools.simplified_loss import SimplifiedYOLOLoss
    z = V.load_loss_case("small")
    img = z["img"]
    tg = torch.from_numpy(z["targets"]).to(DEV)
    outs = []
    for bw, cw in ((7.5, 0.5), (2.0, 3.0)):
        crit = SimplifiedYOLOLoss(z["nc"], DEV, img_size=img, box_weight=bw, cls_weight=cw)
        preds = [_channels_last(torch.from_numpy(m), torch.float32).requires_grad_(True) for m in z["maps"]]
        loss, items = crit(preds, tg)
        loss.backward()
        assert abs(items["total_loss"] - (bw * items["loss_box"] + cw * items["loss_cls"] + 1.5 * items["loss_dfl"])) \
            <= 1e-5 * abs(items["total_loss"])
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in preds)
        outs.append(items)
    a, b = outs
    for k in ("loss_box", "loss_cls", "loss_dfl"):
        assert abs(a[k] - b[k]) <= 1e-6 * max(abs(a[k]), 1e-3)
