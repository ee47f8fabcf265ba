"""Checkpoint save / resume: reference checkpoint formats (train.py:263-285,
410-425; tools/utils.py:45-82) load into the MI355X model, and a full yms checkpoint restores
optimizer + scheduler + epoch.  CPU tier (no forward needed); the GPU resume test is in
test_checkpoint_gpu.py."""
import os

import pytest
import torch

from oracle import model_ref as M
from yms import checkpoint as C
from yolov8.yolov8 import YOLOv8


def _fake_step(model, opt, seed):
    g = torch.Generator().manual_seed(seed)
    for p in model.parameters():
        if p.requires_grad:
            p.grad = torch.randn(p.shape, generator=g)
    opt.step()


def test_reference_formats_load_strictly(tmp_path):
    sd = M.init_params("n", 80)               # reference key set (pinned by tests/golden/state_keys.json)
    plain = tmp_path / "last.pt"
    torch.save(sd, plain)                                           # train.py:425 format
    wrapped = tmp_path / "dp.pt"
    torch.save({"module." + k: v for k, v in sd.items()}, wrapped)  # DataParallel-saved
    nested = tmp_path / "nested.pt"
    torch.save({"state_dict": sd}, nested)                          # utils.py:55-56 format
    for f in (plain, wrapped, nested):
        m = YOLOv8("n", 80)
        info = C.load_checkpoint(str(f), m, strict=True)
        assert info["missing"] == [] and info["unexpected"] == []
        got = m.state_dict()
        assert all(torch.equal(got[k], sd[k]) for k in sd)


def test_full_checkpoint_roundtrip_restores_optimizer_scheduler_epoch(tmp_path):
    torch.manual_seed(0)
    m = YOLOv8("n", 80)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.937, nesterov=True, weight_decay=5e-4)
    sch = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    for s in range(2):
        _fake_step(m, opt, s)
        sch.step()
    f = str(tmp_path / "ck.pt")
    C.save_checkpoint(f, m, opt, sch, epoch=2, best_val_metric=0.125)
    m2 = YOLOv8("n", 80)
    opt2 = torch.optim.SGD(m2.parameters(), lr=0.01, momentum=0.937, nesterov=True, weight_decay=5e-4)
    sch2 = torch.optim.lr_scheduler.StepLR(opt2, step_size=1, gamma=0.5)
    info = C.load_checkpoint(f, m2, opt2, sch2)
    assert info["epoch"] == 2 and info["best_val_metric"] == 0.125 and info["has_optimizer"]
    assert sch2.last_epoch == sch.last_epoch and opt2.param_groups[0]["lr"] == opt.param_groups[0]["lr"]
    # one more identical step on both: bit-identical parameters (momentum buffers restored)
    _fake_step(m, opt, 7)
    _fake_step(m2, opt2, 7)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    # the 'model' key is what the reference's own load_pretrained_weights reads (utils.py:54-56)
    obj = torch.load(f, weights_only=True)
    assert set(obj["model"]) == set(m.state_dict())


def test_load_pretrained_weights_reference_behaviour(tmp_path, capsys):
    m = YOLOv8("n", 80)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    C.load_pretrained_weights(m, str(tmp_path / "missing.pt"))
    assert "training from scratch" in capsys.readouterr().out
    # a different num_classes: strict=False still raises on shape mismatch inside load_state_dict,
    # which the reference reports and swallows (utils.py:77-79); the model is left usable
    f = tmp_path / "nc1.pt"
    torch.save(M.init_params("n", 1), f)
    C.load_pretrained_weights(m, str(f), strict=False)
    assert "Error loading pretrained weights" in capsys.readouterr().out
    assert set(m.state_dict()) == set(before)


def test_save_state_dict_is_reference_plain_format(tmp_path):
    m = YOLOv8("n", 80)
    f = str(tmp_path / "best.pt")
    C.save_state_dict(f, m)
    obj = torch.load(f, weights_only=True)
    assert list(obj) == list(m.state_dict())
    assert not any(k.startswith("module.") for k in obj)
