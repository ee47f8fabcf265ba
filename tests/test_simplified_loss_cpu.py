"""CPU tier of the SimplifiedYOLOLoss drop-in (train.py:14,321-330): the import train.py does resolves
to this package (not the reference's broken, torchvision-importing file), the constructor takes the
reference's signature and defaults (simplified_loss.py:12-22), and the weights land on ComputeLoss's
lambdas.  The numerics are GPU tests (tests/test_loss_gpu.py)."""
import inspect

import torch

import yolov8.tools.simplified_loss as S


def test_train_py_import_resolves_here():
    from yolov8.tools.simplified_loss import SimplifiedYOLOLoss, bbox_iou  # train.py:14
    assert "yolo-ms_amd" in inspect.getsourcefile(SimplifiedYOLOLoss)
    assert callable(bbox_iou)


def test_constructor_signature_and_defaults():
    sig = inspect.signature(S.SimplifiedYOLOLoss.__init__)
    assert list(sig.parameters)[1:] == ["num_classes", "device", "img_size", "strides", "alpha", "gamma",
                                        "box_weight", "cls_weight"]
    d = {k: p.default for k, p in sig.parameters.items() if p.default is not inspect.Parameter.empty}
    assert d == {"img_size": (640, 640), "strides": [8, 16, 32], "alpha": 0.25, "gamma": 1.5,
                 "box_weight": 7.5, "cls_weight": 0.5}


def test_train_py_keyword_set_and_weight_mapping():
    crit = S.SimplifiedYOLOLoss(num_classes=80, device="cpu", img_size=(512, 640), strides=[8., 16., 32.],
                                alpha=0.3, gamma=2.0, box_weight=5.0, cls_weight=1.0)
    inner = crit._loss
    assert (inner.lambda_box, inner.lambda_cls, inner.lambda_dfl) == (5.0, 1.0, 1.5)
    assert (inner.img_size_h, inner.img_size_w) == (512, 640)
    assert torch.equal(crit.strides, torch.tensor([8., 16., 32.]))
    assert (crit.alpha, crit.gamma) == (0.3, 2.0)
    f = S.ComputeLoss(None, num_classes=3, device="cpu")      # simplified_loss.py:156-167 factory
    assert isinstance(f, S.SimplifiedYOLOLoss) and f.num_classes == 3


def test_cpu_tensors_fail_loudly():
    crit = S.SimplifiedYOLOLoss(3, "cpu", img_size=(64, 64))
    preds = [torch.zeros(1, 67, s, s) for s in (8, 4, 2)]
    try:
        crit(preds, torch.zeros(0, 6))
    except RuntimeError as e:
        assert "GPU" in str(e)
    else:
        raise AssertionError("CPU tensors must raise (no CPU fallback)")


def test_bbox_iou_is_pairwise_like_torchvision():
    """simplified_loss.py:170-185 returns torchvision's PAIRWISE [N, M] box_iou / complete_box_iou
    (the elementwise loss.py helper gave [N] or a broadcast error).  Known answers;
    parity with torchvision itself is unpinned (not installed)."""
    b1 = torch.tensor([[5.0, 5.0, 10.0, 10.0], [20.0, 20.0, 4.0, 4.0], [5.0, 5.0, 2.0, 2.0]])   # xywh
    b2 = torch.tensor([[5.0, 5.0, 10.0, 10.0], [10.0, 5.0, 10.0, 10.0]])
    iou = S.bbox_iou(b1, b2)
    assert iou.shape == (3, 2)
    assert torch.allclose(iou[0], torch.tensor([1.0, 1.0 / 3.0]))      # identical; half-overlap 50/150
    assert torch.all(iou[1] == 0)                                        # disjoint
    assert torch.isclose(iou[2, 0], torch.tensor(4.0 / 100.0))          # contained 2x2 in 10x10
    xyxy = S.bbox_iou(torch.tensor([[0.0, 0.0, 10.0, 10.0]]), torch.tensor([[0.0, 0.0, 10.0, 5.0]]), xywh=False)
    assert xyxy.shape == (1, 1) and torch.isclose(xyxy[0, 0], torch.tensor(0.5))
    ciou = S.bbox_iou(b1, b2, CIoU=True)
    assert ciou.shape == (3, 2) and torch.isclose(ciou[0, 0], torch.tensor(1.0))
    # CIoU <= IoU (centre-distance and aspect penalties are non-negative); equal aspect ratios leave
    # only the centre term: (10-5)^2 / (15^2 + 10^2 + eps)
    assert torch.all(ciou <= iou + 1e-6)
    assert torch.isclose(ciou[0, 1], torch.tensor(1.0 / 3.0 - 25.0 / 325.0), atol=1e-6)
