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


def test_msblock_concat_aliases_input_conv_output():
    """[X_1 | X_2 | X_3] becomes [Y_1 | Y_2 | Y_3] in place: no Y_1 = X_1 copy, the IB outputs are
    written over X_2 / X_3 after the branch sums read them, out_conv reads the in_conv's buffer;
    the gradient tracker stores (not accumulates) dX_{i+1} over the consumed dY_{i+1}."""
    from yms.plan import AddOp, ConvOp
    m = YOLOv8("ms-s", 80).train()
    p = runner.get_plan(m, [torch.empty(2, 3, 128, 128, device="meta")], torch.bfloat16, True)
    blk = m.backbone.ms_4
    ops = {id(getattr(op, "mod", None)): op for op in p.ops if isinstance(op, ConvOp)}
    cin, cout = ops[id(blk.in_conv)], ops[id(blk.out_conv)]
    assert cout.x.buf is cin.y.buf and cout.x.off == cin.y.off and cout.x.c == cin.y.c
    adds = [op for op in p.ops if isinstance(op, AddOp) and op.a.buf is cin.y.buf]
    assert len(adds) == 2 and all(op.b is not None for op in adds)          # X_2 + Y_1, X_3 + Y_2 only
    last = [ops[id(br[-1].out_conv)] for br in blk.branches]
    mid = blk.mid
    assert [(v.y.buf is cin.y.buf, v.y.off) for v in last] == [(True, mid), (True, 2 * mid)]
    # backward: each branch-sum backward stores dX_{i+1} (the slice's dY_{i+1} was taken by the IB)
    assert [op.acc[0] for op in adds] == [0, 0]
    # ... and accumulates dY_i into the slice out_conv's dgrad stored
    assert [op.acc[1] for op in adds] == [1, 1]


def test_grad_tracker_release():
    from yms.plan import Buf, GradTracker, View
    b = Buf(0, 1, 4, 4, 24, "t", False)
    T = GradTracker()
    whole, s1 = View(b, 0, 24), View(b, 8, 8)
    assert T.write(whole) == 0          # out_conv dgrad: [dY1|dY2|dY3]
    T.read(s1)                          # the IB's backward takes dY2 ...
    T.release(s1)                       # ... and the slice is dead
    assert T.write(s1) == 0             # dX2 stored
    assert T.write(View(b, 0, 8)) == 1  # dY1 += ...
