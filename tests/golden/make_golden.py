"""Generate golden fixtures by importing the REFERENCE model (build container only).

Run:  python tests/golden/make_golden.py      (needs /root/reference; never on the GPU box)

The reference package (/root/reference/yolov8, torch-only imports) is loaded with
the oracle's closed-form weights (oracle/model_ref.init_params), driven on seeded
inputs, and its outputs / gradients / updated BN buffers are written as small
.npz fixtures (inputs + expected outputs only -- no reference source is stored).
tests/test_oracle_golden.py then pins the oracle restatement against them.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import model_ref as M  # noqa: E402

REF = "/root/reference"


def _ref():
    sys.path.insert(0, REF)
    from yolov8.yolov8 import YOLOv8
    from yolov8.model import components as C
    from yolov8.model.yolov8_head import Head
    return YOLOv8, C, Head


def closed_form_into(module, prefix=""):
    """Load deterministic weights into a reference module by key name."""
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        key = prefix + k
        if k.endswith("num_batches_tracked"):
            new[k] = torch.zeros_like(v)
        elif k.endswith("dfl.conv.weight"):
            new[k] = v.clone()
        elif v.dim() == 4:
            fan_in = v.shape[1] * v.shape[2] * v.shape[3]
            new[k] = M._closed_form(key, tuple(v.shape), (3.0 / fan_in) ** 0.5 * 1.2)
        elif k.endswith("bn.weight"):
            new[k] = M._closed_form(key, tuple(v.shape), 0.25, base=1.0)
        elif k.endswith("bn.bias"):
            new[k] = M._closed_form(key, tuple(v.shape), 0.2)
        elif k.endswith("running_mean"):
            new[k] = M._closed_form(key, tuple(v.shape), 0.1)
        elif k.endswith("running_var"):
            new[k] = M._closed_form(key, tuple(v.shape), 0.3, base=1.2)
        elif k.endswith("bias"):
            new[k] = M._closed_form(key, tuple(v.shape), 0.5)
        else:
            raise KeyError(k)
    module.load_state_dict(new)


def run_block(name, module, x, prefix, cot_seed):
    """Eval forward, then train forward + backward with a fixed cotangent."""
    out = {"x": x.numpy()}
    closed_form_into(module, prefix)
    module.eval()
    with torch.no_grad():
        y = module(x.clone())
    if isinstance(y, (list, tuple)):
        for i, t in enumerate(y):
            out[f"eval_y{i}"] = t.numpy()
    else:
        out["eval_y"] = y.numpy()
    module.train()
    xg = x.clone().requires_grad_(True)
    y = module(xg)
    ys = list(y) if isinstance(y, (list, tuple)) else [y]
    g = torch.Generator().manual_seed(cot_seed)
    loss = 0
    for i, t in enumerate(ys):
        cot = torch.randn(t.shape, generator=g)
        out[f"train_y{i}"] = t.detach().numpy()
        out[f"cot{i}"] = cot.numpy()
        loss = loss + (t * cot).sum()
    loss.backward()
    out["dx"] = xg.grad.numpy()
    for k, p in module.named_parameters():
        if p.grad is not None:
            out[f"grad:{k}"] = p.grad.numpy()
    for k, b in module.named_buffers():
        out[f"buf:{k}"] = b.numpy()
    np.savez_compressed(os.path.join(HERE, f"block_{name}.npz"), **out)


def main():
    YOLOv8, C, Head = _ref()
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1234)

    def rnd(*s):
        return torch.randn(*s, generator=g)

    # --- state_dict key/shape sets (the checkpoint API) ---
    keys = {}
    for v, nc in (("n", 80), ("s", 80), ("l", 80), ("n", 1)):
        m = YOLOv8(v, nc)
        keys[f"{v}_{nc}"] = [[k, list(t.shape)] for k, t in m.state_dict().items()]
    try:
        YOLOv8("xs", 80)
        keys["xs_error"] = None
    except ValueError as e:
        keys["xs_error"] = str(e)
    with open(os.path.join(HERE, "state_keys.json"), "w") as f:
        json.dump(keys, f)

    # --- block fixtures (prefix '' : weights keyed by the block's own names) ---
    run_block("conv1x1", C.Conv(16, 24, 1, 1, 0), rnd(2, 16, 9, 7), "", 1)
    run_block("conv3x3s1", C.Conv(8, 16, 3, 1, 1), rnd(2, 8, 9, 11), "", 2)
    run_block("conv3x3s2", C.Conv(3, 16, 3, 2, 1), rnd(2, 3, 13, 10), "", 3)
    run_block("conv3x3s2_c24", C.Conv(24, 32, 3, 2, 1), rnd(1, 24, 8, 8), "", 4)
    run_block("bottleneck", C.Bottleneck(16, 16), rnd(2, 16, 6, 5), "", 5)
    run_block("c2f_n1", C.C2f(32, 32, 1), rnd(2, 32, 8, 6), "", 6)
    run_block("c2f_n2", C.C2f(24, 48, 2), rnd(1, 24, 7, 9), "", 7)
    run_block("sppf", C.SPPF(32, 32), rnd(2, 32, 9, 8), "", 8)
    up = C.Upsample()
    x = rnd(2, 8, 3, 5)
    np.savez_compressed(os.path.join(HERE, "block_upsample.npz"), x=x.numpy(), y=up(x).numpy())
    dflm = C.DFL()
    x = rnd(2, 64, 37)
    np.savez_compressed(os.path.join(HERE, "block_dfl.npz"), x=x.numpy(), y=dflm(x).numpy())

    # --- full-model fixtures ---
    for (v, nc, B, H, W) in (("n", 80, 2, 64, 64), ("n", 80, 1, 128, 96), ("n", 1, 2, 64, 64)):
        m = YOLOv8(v, nc)
        closed_form_into(m)
        x = rnd(B, 3, H, W)
        out = {"x": x.numpy()}
        m.eval()
        m.head.stride = torch.tensor([8.0, 16.0, 32.0])
        with torch.no_grad():
            out["eval_y"] = m(x.clone()).numpy()
        m.train()
        ys = m(x.clone())
        loss = 0
        gc = torch.Generator().manual_seed(99)
        for i, t in enumerate(ys):
            cot = torch.randn(t.shape, generator=gc)
            out[f"train_y{i}"] = t.detach().numpy()
            out[f"cot{i}"] = cot.numpy()
            loss = loss + (t * cot).sum()
        loss.backward()
        for k, p in m.named_parameters():
            if p.grad is None:
                continue
            gnp = p.grad.numpy().astype(np.float64)
            out[f"gsum:{k}"] = np.array([gnp.sum(), np.abs(gnp).sum()])
        for k in ("backbone.conv0.conv.weight", "backbone.c2f_4.m.0.conv2.conv.weight",
                  "neck.c2f_2.conv1.conv.weight", "head.cls.0.2.weight", "head.box.2.2.bias",
                  "backbone.sppf.conv1.bn.weight"):
            out[f"grad:{k}"] = dict(m.named_parameters())[k].grad.numpy()
        for k, b in m.named_buffers():
            if "running" in k and ("conv0" in k or "sppf.conv2" in k or "head.cls.2.1" in k):
                out[f"buf:{k}"] = b.numpy()
        np.savez_compressed(os.path.join(HERE, f"model_{v}{nc}_{B}x{H}x{W}.npz"), **out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
