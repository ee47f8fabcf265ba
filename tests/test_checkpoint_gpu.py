"""GPU tier: resuming from a yms checkpoint continues the HIP training run exactly (same params
after step 3 whether or not the run was interrupted after step 2) -- optimizer momentum, BN
running buffers and num_batches_tracked all restored."""
import pytest
import torch

from oracle import model_ref as M
from yms import checkpoint as C
from yolov8.yolov8 import YOLOv8

pytestmark = pytest.mark.gpu


def _run(m, opt, steps, seed0):
    for s in range(steps):
        x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(seed0 + s)).cuda()
        opt.zero_grad(set_to_none=True)
        loss = sum((o.float() ** 2).mean() for o in m(x))
        loss.backward()
        opt.step()


def _new(sd):
    m = YOLOv8("n", 80).cuda()
    m.load_state_dict(sd)
    m.train()
    return m, torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.937, nesterov=True, weight_decay=5e-4)


def test_resume_is_exact(tmp_path):
    sd = M.init_params("n", 80)
    m, opt = _new(sd)
    _run(m, opt, 2, 0)
    f = str(tmp_path / "ck.pt")
    C.save_checkpoint(f, m, opt, epoch=1)
    _run(m, opt, 1, 2)                       # uninterrupted run: step 3
    m2, opt2 = _new(M.init_params("n", 80))
    info = C.load_checkpoint(f, m2, opt2)
    assert info["epoch"] == 1 and info["has_optimizer"]
    _run(m2, opt2, 1, 2)                     # resumed run: step 3
    torch.cuda.synchronize()
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a.cpu(), b.cpu()), k
