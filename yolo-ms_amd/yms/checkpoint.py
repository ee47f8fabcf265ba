"""Checkpoint save / resume for the MI355X model.

The reference saves plain ``model.state_dict()`` files (``best.pt``, ``epoch_N.pt``, ``last.pt``:
yolov8/tools/train.py:410-425) and loads them with ``module.`` stripping and ``strict=False``
(train.py:263-285; tools/utils.py:45-82 also accepts ``{'model': sd}`` / ``{'state_dict': sd}``).
It keeps no optimizer, scheduler or epoch state, so training cannot resume.

Here:

* ``save_checkpoint`` writes ``{'model', 'optimizer', 'scheduler', 'epoch', 'best_val_metric',
  'yms': {...}}``.  The ``'model'`` key is the format the reference's own
  ``load_pretrained_weights`` (utils.py:54-56) already reads, so a file written here loads in the
  reference unchanged; ``save_state_dict`` writes the reference's plain format.
* ``load_checkpoint`` reads every format the reference reads (plain state_dict, ``'model'``,
  ``'state_dict'``, ``module.`` prefixes from DataParallel / ``yms.dist.DataParallel``) with
  ``torch.load(weights_only=True)`` -- nothing in the file is executed -- and restores optimizer /
  scheduler / epoch when present, so ``resume`` continues bit-for-bit (tests/test_checkpoint*.py).

The state_dict key set is the reference's (355 keys for 's', 595 for 'l'; tests/golden/state_keys.json),
so the same file moves between the reference CPU path and this GPU path in both directions.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

FORMAT_VERSION = 1


def _strip_module(sd):
    """train.py:270-276 / utils.py:65-67: drop the DataParallel ``module.`` prefix."""
    if any(k.startswith("module.") for k in sd):
        return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())
    return sd


def _unwrap(model):
    return model.module if hasattr(model, "module") and isinstance(model.module, torch.nn.Module) else model


def model_state(obj):
    """The model state_dict inside any checkpoint format the reference reads (utils.py:51-62)."""
    if isinstance(obj, dict):
        if "model" in obj and isinstance(obj["model"], dict):
            return _strip_module(obj["model"])
        if "state_dict" in obj and isinstance(obj["state_dict"], dict):
            return _strip_module(obj["state_dict"])
        return _strip_module(obj)
    raise RuntimeError(f"yms: unrecognised checkpoint object of type {type(obj).__name__}")


def save_state_dict(path, model):
    """The reference's own format (train.py:410-425): a plain state_dict, no wrapper prefix."""
    _atomic_save(_unwrap(model).state_dict(), path)


def save_checkpoint(path, model, optimizer=None, scheduler=None, epoch=None, best_val_metric=None, extra=None):
    """Full training state.  ``epoch`` is the number of completed epochs (resume starts there)."""
    ck = {"model": _unwrap(model).state_dict(), "epoch": epoch, "best_val_metric": best_val_metric,
          "yms": {"format": FORMAT_VERSION}}
    if optimizer is not None:
        ck["optimizer"] = optimizer.state_dict()
    if scheduler is not None:
        ck["scheduler"] = scheduler.state_dict()
    if extra:
        ck["extra"] = dict(extra)
    _atomic_save(ck, path)


def _atomic_save(obj, path):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, model, optimizer=None, scheduler=None, strict=True, map_location="cpu"):
    """Load any reference-format or yms checkpoint into ``model`` (and the optimizer / scheduler when
    the file has them).  -> dict(epoch, best_val_metric, missing, unexpected, has_optimizer)."""
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    obj = torch.load(path, map_location=map_location, weights_only=True)
    sd = model_state(obj)
    target = _unwrap(model)
    res = target.load_state_dict(sd, strict=strict)
    info = {"epoch": None, "best_val_metric": None, "missing": list(res.missing_keys),
            "unexpected": list(res.unexpected_keys), "has_optimizer": False}
    if isinstance(obj, dict) and "yms" in obj:
        info["epoch"] = obj.get("epoch")
        info["best_val_metric"] = obj.get("best_val_metric")
        if optimizer is not None and "optimizer" in obj:
            optimizer.load_state_dict(obj["optimizer"])
            info["has_optimizer"] = True
        if scheduler is not None and "scheduler" in obj:
            scheduler.load_state_dict(obj["scheduler"])
    return info


def load_pretrained_weights(model, pretrained_path, strict=False):
    """Same name, arguments and behaviour as the reference's tools/utils.py:45-82 (missing file:
    train from scratch; any load error is reported and training continues from scratch)."""
    if not pretrained_path or not os.path.exists(pretrained_path):
        print("No pretrained weights found, training from scratch")
        return model
    try:
        info = load_checkpoint(pretrained_path, model, strict=strict)
        if info["missing"]:
            print(f"Missing keys: {info['missing']}")
        if info["unexpected"]:
            print(f"Unexpected keys: {info['unexpected']}")
        print(f"Successfully loaded pretrained weights from {pretrained_path}")
    except Exception as e:  # the reference swallows load errors the same way (utils.py:77-79)
        print(f"Error loading pretrained weights: {e}")
        print("Training from scratch")
    return model
