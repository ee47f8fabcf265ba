"""CPU tier for the stem path's host logic (plan selection and scratch layout; the kernels are
covered by tests/test_stem_gpu.py): plans are built on meta tensors, no GPU needed.  Reference
layer: yolov8/model/yolov8_backbone.py:30-40 (the backbone's first Conv(3, c1, 3, 2, 1))."""
import pytest
import torch

from yms import runner
from yms.plan import ConvOp
from yolov8.yolov8 import YOLOv8


def _plan(v, dt, training, requires_grad=False, size=64):
    m = YOLOv8(v, 80).train(training)
    x = torch.empty(2, 3, size, size, device="meta", requires_grad=requires_grad)
    return runner.get_plan(m, [x], dt, training)


@pytest.mark.parametrize("v", ["n", "s", "ms-xs"])
@pytest.mark.parametrize("training", [False, True])
def test_stem_selected_for_16bit_plans(v, training):
    p = _plan(v, torch.bfloat16, training)
    assert list(p.stem_inputs) == [0]
    op = p.stem_inputs[0]
    assert op is p.ops[0] and type(op) is ConvOp and op.stem_input == 0
    assert (op.shape.k, op.shape.stride, op.shape.cin) == (3, 2, 3)
    # exactly one op reads the input buffer
    readers = [o for o in p.ops if any(getattr(a, "buf", None) is p.inputs[0].buf for a in vars(o).values())]
    assert readers == [op]


def test_stem_not_selected_for_fp32_or_input_grad(monkeypatch):
    assert _plan("s", torch.float32, True).stem_inputs == {}
    assert _plan("s", torch.bfloat16, True, requires_grad=True).stem_inputs == {}
    monkeypatch.setenv("YMS_STEM", "0")
    assert _plan("n", torch.bfloat16, False).stem_inputs == {}


@pytest.mark.parametrize("v", ["s", "ms-s"])
def test_stem_wgrad_scratch_is_not_the_side_stream_scratch(v):
    """The stem's weight gradient runs on the main stream while the side stream may still run
    earlier layers' wgrads in the shared "wgrad" scratch: its own region, disjoint from it."""
    p = _plan(v, torch.bfloat16, True)
    a0, a1 = p.gscratch["stemwg"], p.gscratch["stemwg"] + p.scratch_req["stemwg"]
    b0, b1 = p.gscratch["wgrad"], p.gscratch["wgrad"] + p.scratch_req["wgrad"]
    assert p.scratch_req["stemwg"] > 0 and (a1 <= b0 or b1 <= a0)
    assert p.stem_inputs[0].wg_ws <= p.scratch_req["stemwg"]
