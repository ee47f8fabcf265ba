"""CPU tier for the fused BN-backward reduce routing (Plan._find_bnred; the kernels are covered by
tests/test_dgrad_bnred_gpu.py): plans are built on meta tensors, no GPU needed.  A Conv whose input
gradient is the LAST writer of its producer Conv's output gradient computes the producer's BN + SiLU
backward partial sums (components.py:69-77 Conv feeding Conv) into a grad-scratch region of the pair's
own, which the producer's finalize reads."""
import pytest
import torch

from yms import runner
from yms.plan import ConvOp
from yolov8.yolov8 import YOLOv8


def _plan(v, size=640):
    m = YOLOv8(v, 80).train()
    x = torch.empty(2, 3, size, size, device="meta")
    return runner.get_plan(m, [x], torch.bfloat16, True)


@pytest.mark.parametrize("v", ["s", "ms-s"])
def test_pairs_have_their_own_rows_region(v):
    p = _plan(v)
    cons = [op for op in p.ops if type(op) is ConvOp and op.bnred_for is not None]
    assert cons, "no fused pair"
    keys = set()
    for c in cons:
        q = c.bnred_for
        assert q.bnred_by is c and c.bnred_wkey == q.bnred_key
        assert p.ops.index(q) < p.ops.index(c)          # the producer's backward runs after the consumer's
        assert q.bnred_key not in keys
        keys.add(q.bnred_key)
        assert p.scratch_req[q.bnred_key] >= 4 * q.bnred_rows * 2 * q.c
    # regions are disjoint
    spans = sorted((p.gscratch[k], p.gscratch[k] + p.scratch_req[k]) for k in keys)
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))


class _EveryShapeFuses:
    """The library with every 16-bit input gradient reporting fused-reduce rows (the routing of a
    kernel that took them all), so the plan forms chains of pairs."""

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        if name == "yms_conv_dgrad_bnred_rows":
            return lambda sp: 256 if sp.contents.dtype != 0 else 0
        return getattr(self._real, name)


def test_chained_pairs_keep_both_regions(monkeypatch):
    """A conv that is the consumer of one pair and the producer of the next (Bottleneck cv1 -> cv2
    chains, downsample -> C2f cv1) writes its producer's rows and reads its own from different
    regions (one shared attribute sent the consumer's rows into its own producer-side region)."""
    from yms import _lib as L
    real = L.lib()
    monkeypatch.setattr(L, "lib", lambda: _EveryShapeFuses(real))
    p = _plan("s")
    both = [op for op in p.ops if type(op) is ConvOp and op.bnred_for is not None and op.bnred_by is not None]
    assert both
    for op in both:
        assert op.bnred_wkey != op.bnred_key
        assert op.bnred_wkey == op.bnred_for.bnred_key


def test_disabled_by_env(monkeypatch):
    monkeypatch.setenv("YMS_BNRED", "0")
    p = _plan("s")
    assert not any(getattr(op, "bnred_for", None) is not None for op in p.ops)
