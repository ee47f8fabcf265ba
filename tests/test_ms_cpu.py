"""CPU tier for the YOLO-MS family (MS-Block / HKS; NOT reference-pinned -- the
reference has no MS-Block code): version registry and the reference's ValueError contract, the
product module's state_dict keys equal the independent oracle's, and plans build for every
version (heterogeneous depthwise kernel sizes 3/5/7/9 in the backbone)."""
import pytest
import torch

from oracle import ms_ref as MS
from yms import runner
from yms.plan import DWConvOp
from yolov8.model.components import yolo_params
from yolov8.model.yolo_ms import ms_params
from yolov8.yolov8 import YOLOv8


def test_versions_and_reference_error_contract():
    for v in ("ms-xs", "ms-s", "ms-l"):
        ms_params(v)
        with pytest.raises(ValueError, match=f"Unknown YOLOv8 version: {v}"):
            yolo_params(v)              # the reference's table is untouched
    with pytest.raises(ValueError, match="Unknown YOLO-MS version"):
        ms_params("xs")
    with pytest.raises(ValueError, match="Unknown YOLOv8 version: xs"):
        YOLOv8("xs", 80)


@pytest.mark.parametrize("v", ["ms-xs", "ms-s", "ms-l"])
def test_state_dict_matches_oracle(v):
    m = YOLOv8(v, 80)
    assert [(k, tuple(t.shape)) for k, t in m.state_dict().items()] == [(k, tuple(s)) for k, s in MS.state_keys(v, 80)]
    m.load_state_dict(MS.init_params(v, 80))


@pytest.mark.parametrize("v", ["ms-xs", "ms-s", "ms-l"])
def test_plan_has_hks_depthwise_stages(v):
    m = YOLOv8(v, 80).train()
    p = runner.get_plan(m, [torch.empty(2, 3, 640, 640, device="meta")], torch.bfloat16, True)
    ks = sorted({op.dshape.k for op in p.ops if isinstance(op, DWConvOp)})
    assert ks == [3, 5, 7, 9]
    L = ms_params(v)[3]
    assert sum(isinstance(op, DWConvOp) for op in p.ops) == 8 * 2 * L     # 8 MSBlocks x 2 branches x L


def test_oracle_forward_shapes():
    v, nc = "ms-xs", 80
    sd = MS.init_params(v, nc)
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        y = MS.forward(dict(sd), v, nc, x, False)
    assert y.shape == (1, 84, 84)
