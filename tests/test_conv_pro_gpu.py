"""Training-forward convolution with the producer's BN + SiLU as an A-operand prologue
(yms_conv_fwd_pro): bit-identical to the separate path it replaces -- the producer's affine pass
(yms_affine_act: x = act(z * scale + shift), rounded once to bf16) followed by yms_conv_fwd with
statistics -- in the conv output z', its statistics rows, and the x it stores for the later readers
(components.py:72-77 applied twice: the producer's BN + SiLU, then the consumer's conv).  Covers
1x1 consumers (3x3 ones are refused), channel counts on the uniform (cin % 64 == 0) and per-lane
loader paths, more than one output-column tile (x stored once), channel-offset
views, and a whole training step of the plans with the prologue on / off (YMS_PRO)."""
import ctypes

import pytest
import torch

from hiputil import pack, r8, shape, stats_buffer
from yms import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(n, h, w, cin, cout, k, act, dt=torch.bfloat16, zld=None, xld=None, xoff=0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    zld = zld or r8(cin)
    xld = xld or r8(xoff + cin)
    z = torch.zeros((n, h, w, zld), dtype=dt, device=DEV)
    z[..., :cin] = (torch.randn(n, h, w, cin, device=DEV, generator=g) * 2).to(dt)
    z[0, 0, 0, :cin] = 0.0          # exact zeros inside the image must still become act(shift)
    sc = torch.rand(cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(cin, device=DEV, generator=g)
    wt = torch.randn(cout, cin, k, k, device=DEV, generator=g) / (cin * k * k) ** 0.5
    sp = ctypes.pointer(shape(n, h, w, cin, cout, k, 1, dt))
    assert L.lib().yms_conv_fwd_pro_supported(sp)
    wp = pack(wt, sp.contents, dt, 0)
    rows, ld = L.lib().yms_conv_stats_rows(sp), L.lib().yms_conv_stats_ld(sp)
    st = L.stream_ptr()
    # reference: affine pass + conv
    x_ref = torch.zeros((n, h, w, xld), dtype=dt, device=DEV)
    L.call("yms_affine_act", L.dtype_code(dt), n * h * w, cin, z.data_ptr(), zld, 0, sc.data_ptr(), sh.data_ptr(), act,
           None, 0, 0, x_ref.data_ptr(), xld, xoff, st)
    y_ref = torch.zeros((n, h, w, r8(cout)), dtype=dt, device=DEV)
    b_ref = stats_buffer(rows, ld)
    L.call("yms_conv_fwd", sp, x_ref.data_ptr(), xld, xoff, wp.data_ptr(), y_ref.data_ptr(), r8(cout), 0, None, None,
           0, None, 0, 0, b_ref.data_ptr(), st)
    # prologue
    x = torch.zeros((n, h, w, xld), dtype=dt, device=DEV)
    y = torch.zeros_like(y_ref)
    b = stats_buffer(rows, ld)
    L.call("yms_conv_fwd_pro", sp, z.data_ptr(), zld, 0, sc.data_ptr(), sh.data_ptr(), act, x.data_ptr(), xld, xoff,
           wp.data_ptr(), y.data_ptr(), r8(cout), 0, b.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref), (x.float() - x_ref.float()).abs().max().item()
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
    assert torch.equal(b.nan_to_num(7.0), b_ref.nan_to_num(7.0))


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 80), (40, 96), (256, 192), (96, 160), (576, 288)])
def test_pro_matches_affine_then_conv(cin, cout):
    _run(2, 12, 20, cin, cout, 1, L.ACT_SILU)


def test_pro_identity_act_views_and_large_maps():
    _run(3, 17, 9, 64, 64, 1, L.ACT_NONE)
    _run(2, 10, 14, 48, 72, 1, L.ACT_SILU, zld=56, xld=128, xoff=64)     # x into a concat slot
    _run(4, 40, 40, 160, 80, 1, L.ACT_SILU)
    _run(2, 80, 80, 64, 64, 1, L.ACT_SILU)


def test_pro_rejects_unsupported():
    dt = torch.bfloat16
    for sh_ in (shape(2, 8, 8, 64, 64, 3, 2, dt), shape(2, 8, 8, 1032, 64, 1, 1, dt),
                shape(2, 8, 8, 64, 64, 1, 1, torch.float32), shape(2, 8, 8, 64, 64, 3, 1, dt)):
        assert not L.lib().yms_conv_fwd_pro_supported(ctypes.pointer(sh_))


@pytest.mark.parametrize("version,size", [("s", 128), ("ms-s", 128)])
def test_training_step_bit_identical_with_and_without_prologue(monkeypatch, version, size):
    """A bf16 training step (forward, loss, backward) of the YOLOv8-s / YOLO-MS-S plans: the
    prologue convs (about a third of the affine passes gone) give exactly the same head maps,
    parameter gradients and running statistics as the separate affine passes."""
    from yolov8.yolov8 import YOLOv8
    from yms import runner
    torch.manual_seed(0)
    base = YOLOv8(version, 80)
    x = torch.randn(2, 3, size, size, generator=torch.Generator().manual_seed(1))
    res = []
    for pro in ("0", "1"):
        monkeypatch.setenv("YMS_PRO", pro)
        m = YOLOv8(version, 80)
        m.load_state_dict(base.state_dict())
        m = m.to(DEV).train()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            outs = m(x.to(DEV))
        sum((o.float() ** 2).mean() for o in outs).backward()
        plan = next(iter(m.__dict__[runner._CACHE_ATTR].values()))
        n_pro = sum(getattr(op, "pro", None) is not None for op in plan.ops)
        assert (n_pro > 0) == (pro == "1"), n_pro
        res.append(([o.detach().float().cpu() for o in outs],
                    {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None},
                    {k: b.detach().cpu() for k, b in m.named_buffers()}))
    (o0, g0, b0), (o1, g1, b1) = res
    assert all(torch.equal(a, b) for a, b in zip(o0, o1))
    assert g0.keys() == g1.keys() and all(torch.equal(g0[k], g1[k]) for k in g0)
    assert all(torch.equal(b0[k], b1[k]) for k in b0)
