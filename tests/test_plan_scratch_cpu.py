"""CPU tier for the plan's scratch ownership (plans built on meta tensors, no GPU): every backward
scratch region is its own range of the grad arena -- the side stream's weight gradients use only
"wgrad", the main stream the others."""
import pytest
import torch

from yms import runner
from yms.plan import ConvOp
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
