"""The head's sibling first convs (yolov8_head.py:84-85, 99-100: box[i][0] and cls[i][0] both read
x_i) run as one SiblingConvOp (yms/plan.py): outputs in the slots of one buffer, one BN backward
pass, one input gradient and one weight gradient over both.  Checked against the unfused plan
(YMS_HEAD_FUSE=0, one ConvOp per module) on the same weights and batch: the forward maps and the BN
running buffers are bit-identical (each member's conv, statistics and finalize are unchanged; the
affine pass is elementwise), and the parameter gradients agree to the accumulation-order rounding
(fp32: the reduce's per-block pixel order differs with the channel count; 16-bit: the unfused
input gradient rounds dx twice, store then accumulate; checked through the drift from fp32).  The
fused fp32 path is also covered by every fp32 oracle / golden model test, which run it by default."""
import pytest
import torch

from yms import set_compute_dtype
from yms.plan import SiblingConvOp
from yolov8.yolov8 import YOLOv8

pytestmark = pytest.mark.gpu


def _step(fuse, dtype, version, nc, x, sd, monkeypatch):
    monkeypatch.setenv("YMS_HEAD_FUSE", "1" if fuse else "0")
    m = YOLOv8(version, nc).cuda()
    m.load_state_dict(sd)
    m.train()
    if dtype != torch.float32:
        set_compute_dtype(m, dtype)
    outs = m(x)
    plans = list(m.__dict__["_yms_plans"].values())
    assert any(isinstance(op, SiblingConvOp) for op in plans[0].ops) == fuse
    g = torch.Generator(device="cuda").manual_seed(3)
    loss = sum((o.float() * torch.randn(o.shape, device="cuda", generator=g)).sum() for o in outs)
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().float().clone() for k, p in m.named_parameters() if p.grad is not None}
    bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
    return [o.detach().float().clone() for o in outs], grads, bufs


@pytest.mark.parametrize("version,nc,size", [("s", 80, 256), ("n", 3, 192), ("ms-s", 80, 256)])
def test_sibling_head_convs_match_unfused(version, nc, size, monkeypatch):
    torch.manual_seed(0)
    sd = YOLOv8(version, nc).state_dict()
    x = torch.randn(2, 3, size, size, generator=torch.Generator().manual_seed(1)).cuda()
    # fp32: the fused and unfused plans agree to accumulation-order rounding
    o1, g32, b1 = _step(True, torch.float32, version, nc, x, sd, monkeypatch)
    o0, g0, b0 = _step(False, torch.float32, version, nc, x, sd, monkeypatch)
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    for k in b0:
        assert torch.equal(b1[k], b0[k]), k
    assert g32.keys() == g0.keys() and any(k.startswith("head.cls.0.0") for k in g0)
    for k in g0:
        d = ((g32[k] - g0[k]).norm() / (g0[k].norm() + 1e-30)).item()
        assert d <= 2e-5, (k, d)
    # bf16: forward and running buffers still bit-identical; the gradients' drift from the fp32
    # gradients is no larger fused than unfused (random-init graphs amplify any rounding difference
    # on its way back through the BN layers, so the two bf16 runs are compared through their drift)
    o1, g1, b1 = _step(True, torch.bfloat16, version, nc, x, sd, monkeypatch)
    o0, g0, b0 = _step(False, torch.bfloat16, version, nc, x, sd, monkeypatch)
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    for k in b0:
        assert torch.equal(b1[k], b0[k]), k
    # (nc = 3: the z buffers' padding channels start zeroed -- arena garbage there used to turn the
    # input gradient NaN through zero weight rows, fused or not)
    for gg in (g1, g0):
        bad = [k for k, t in gg.items() if not torch.isfinite(t).all()]
        assert not bad, bad[:5]
    d1 = torch.tensor([((g1[k] - g32[k]).norm() / (g32[k].norm() + 1e-30)).item() for k in g32])
    d0 = torch.tensor([((g0[k] - g32[k]).norm() / (g32[k].norm() + 1e-30)).item() for k in g32])
    assert d1.median() <= 1.2 * d0.median() and d1.max() <= 1.5 * d0.max(), (d1.median(), d0.median(), d1.max(), d0.max())
