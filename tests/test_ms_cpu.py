"""CPU tier for the YOLO-MS family (MS-Block / HKS; NOT reference-pinned -- the
reference has no MS-Block code): version registry and the reference's ValueError contract, the
product module's state_dict keys equal the independent oracle's, plans build for every version
(heterogeneous depthwise kernel sizes 3/5/7/9 in the backbone), and the graphs are the size of the
published family: parameters and forward MACs at 640x640 against the reference-held model-zoo
table (model_zoos.md:21-53), the one reference-held pin for these models."""
import pytest
import torch

from oracle import ms_ref as MS
from yms import runner
from yms.plan import DWConvOp
from yolov8.model.components import yolo_params
from yolov8.model.yolo_ms import MODEL_ZOO, ms_complexity, ms_params
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
    L = ms_params(v)[1]
    assert sum(isinstance(op, DWConvOp) for op in p.ops) == 8 * 2 * L     # 8 MSBlocks x 2 branches x L


def test_oracle_forward_shapes():
    v, nc = "ms-xs", 80
    sd = MS.init_params(v, nc)
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        y = MS.forward(dict(sd), v, nc, x, False)
    assert y.shape == (1, 84, 84)


# model_zoos.md:21-53, verbatim: YOLO-MS-XS 5.1M / 8.7G, YOLO-MS-S 8.7M / 15.0G, YOLO-MS 23.3M / 38.8G
ZOO_TABLE = {"ms-xs": (5.1e6, 8.7e9), "ms-s": (8.7e6, 15.0e9), "ms-l": (23.3e6, 38.8e9)}


@pytest.mark.parametrize("v", ["ms-xs", "ms-s", "ms-l"])
def test_sizes_match_model_zoo_table(v):
    """Parameters within 3% and forward conv MACs (the table's "FLOPs": mmengine / fvcore count a
    multiply-add as one FLOP) within 5% at 640x640, counted twice: from the product modules and by
    tracing the independent oracle restatement's convolutions.  The build's calibration lands within
    2% on every entry."""
    tp, tm = ZOO_TABLE[v]
    assert MODEL_ZOO[v] == (tp / 1e6, tm / 1e9)
    n_par, macs, elems = ms_complexity(v)
    o_par, o_macs = MS.complexity(v)
    assert (n_par, macs) == (o_par, o_macs)
    m = YOLOv8(v, 80)
    assert n_par == sum(p.numel() for p in m.parameters()) - 16        # all but the frozen DFL arange
    assert abs(n_par / tp - 1) < 0.02, n_par
    assert abs(macs / tm - 1) < 0.02, macs
    # with fvcore's one op per batch-norm / upsample output element the total stays within 3%
    assert abs((macs + elems) / tm - 1) < 0.03, macs + elems
