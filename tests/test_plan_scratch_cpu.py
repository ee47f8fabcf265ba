"""CPU tier for the plan's scratch ownership and the depthwise fusion selection (plans built on
meta tensors, no GPU): every backward scratch region is its own range of the grad arena -- the
side stream's weight gradients use only "wgrad", the main stream the others -- and the opt-in
MS-Block IB fusions (YMS_DW_BNIN / YMS_DW_BNRED, yms/plan.py Plan._find_dw_bnred) pick exactly the
expand-conv -> depthwise pairs of yolov8/model/yolo_ms.py MSBlockLayer."""
import pytest
import torch

from yms import runner
from yms.plan import ConvOp, DWConvOp
from yolov8.yolov8 import YOLOv8


def _plan(v, dt=torch.bfloat16, training=True, size=64):
    m = YOLOv8(v, 80).train(training)
    x = torch.empty(2, 3, size, size, device="meta")
    return runner.get_plan(m, [x], dt, training)


@pytest.mark.parametrize("v", ["s", "l", "ms-s"])
def test_grad_scratch_regions_are_disjoint_and_sized(v):
    p = _plan(v)
    regions = sorted((p.gscratch[k], p.gscratch[k] + p.scratch_req.get(k, 0), k)
                     for k in ("bwd", "coef", "wgrad", "sppf", "stemwg"))
    assert regions[0][0] >= p.act_bytes                  # after the activation-gradient layout
    for (a0, a1, ka), (b0, b1, kb) in zip(regions, regions[1:]):
        assert a1 <= b0, (ka, kb)
    assert regions[-1][1] <= p.gscratch["cnt"] <= p.garena_bytes
    # every op's weight-gradient workspace fits the shared side-stream region
    for op in p.ops:
        if isinstance(op, ConvOp) and type(op) is ConvOp and op.stem_input is None:
            assert op.wg_ws <= p.scratch_req["wgrad"]


def test_dw_fusions_off_by_default():
    p = _plan("ms-s")
    for op in p.ops:
        if type(op) is DWConvOp:
            assert op.bnin is None and op.bnred is None
        if type(op) is ConvOp:
            assert op.bnin_by is None and op.red_rows == 0


@pytest.mark.parametrize("which", ["YMS_DW_BNIN", "YMS_DW_BNRED"])
def test_dw_fusion_pairs(which, monkeypatch):
    monkeypatch.setenv(which, "1")
    p = _plan("ms-s")
    pairs = 0
    for i, op in enumerate(p.ops):
        if type(op) is not DWConvOp:
            continue
        prod = op.bnin if which == "YMS_DW_BNIN" else op.bnred
        assert prod is p.ops[i - 1] and type(prod) is ConvOp and prod.y.buf is op.x.buf
        readers = [o for o in p.ops if o is not prod and any(getattr(a, "buf", None) is op.x.buf
                                                             for a in vars(o).values())]
        assert readers == [op]
        if which == "YMS_DW_BNIN":
            assert prod.bnin_by is op
        else:
            assert prod.red_rows > 0 and 4 * 2 * prod.c * prod.red_rows <= p.scratch_req["bwd"]
        pairs += 1
    assert pairs == sum(1 for op in p.ops if type(op) is DWConvOp) > 0
