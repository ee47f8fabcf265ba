"""CPU restatement of the YOLO-MS family (MS-Block / HKS) -- TEST INFRASTRUCTURE ONLY.

Parity for this family is NOT reference-pinned: the reference repository contains no MS-Block
code (annotations.md:66-133 is a diagram, model_zoos.md:21-53 the upstream size
table).  The structure restated here is the one SURVEY 7.4 specifies (YOLO-MS paper, arXiv
2308.05480) on the diagram's topology, written independently of the product module
(yolo-ms_amd/yolov8/model/yolo_ms.py) as plain functional torch-CPU fp32:

  IB_k(x)      = SiLU(BN(conv1x1)) -> SiLU(BN(depthwise kxk, groups=2c)) -> SiLU(BN(conv1x1))
  MSBlock(x)   = conv1x1(cat[Y1, Y2, Y3]);  [X1|X2|X3] = conv1x1(x),  Y1 = X1,  Yi = IB^L(Xi + Y(i-1))
  backbone     = conv0 s2, conv1 s2, MSBlock(k3), conv3 s2, MSBlock(k5) -> P3, conv5 s2,
                 MSBlock(k7) -> P4, conv7 s2, MSBlock(k9), SPPF ("MS-SPPF") -> P5
  neck         = PAFPN with MSFusion = 1x1 reduce of the deeper map, nearest x2, concat:
                 r5 = reduce_5(P5); td4 = MSBlock(cat[up r5, P4]); r4 = reduce_4(td4);
                 out1 = MSBlock(cat[up r4, P3]); out2 = MSBlock(cat[conv1 s2 out1, r4]);
                 out3 = MSBlock(cat[conv2 s2 out2, r5])          (neck MSBlocks k = 3)
  head         = the reference head (model_ref.head_raw / decode, reference-pinned) on the neck widths

Widths per version (stem c1, stage c2..c5; IB layers per branch) are the build's calibration to
model_zoos.md:21-53 (params / MACs at 640); ``complexity`` recounts both from this restatement.

Only tests/ may import this module.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

from oracle import model_ref as M

# version -> ((c1, c2, c3, c4, c5), IB layers per branch)
VERSIONS = {"ms-xs": ((24, 48, 112, 224, 192), 1),
            "ms-s": ((32, 64, 160, 288, 288), 1),
            "ms-l": ((56, 112, 224, 448, 384), 2)}
HKS = (3, 5, 7, 9)


def params(version):
    return VERSIONS[version]


def _conv_keys(name, cin, cout, k, groups=1):
    out = [(f"{name}.conv.weight", (cout, cin // groups, k, k))]
    for s in ("weight", "bias", "running_mean", "running_var"):
        out.append((f"{name}.bn.{s}", (cout,)))
    out.append((f"{name}.bn.num_batches_tracked", ()))
    return out


def _msblock_keys(name, cin, cout, k, L):
    hidden = int(cin * 3) // 2
    mid = hidden // 3
    out = _conv_keys(f"{name}.in_conv", cin, hidden, 1)
    for b in range(2):
        for j in range(L):
            pre = f"{name}.branches.{b}.{j}"
            out += _conv_keys(f"{pre}.in_conv", mid, 2 * mid, 1)
            out += _conv_keys(f"{pre}.mid_conv", 2 * mid, 2 * mid, k, groups=2 * mid)
            out += _conv_keys(f"{pre}.out_conv", 2 * mid, mid, 1)
    out += _conv_keys(f"{name}.out_conv", hidden, cout, 1)
    return out


def _head_keys(lvl_c, nc):
    """yolov8_head.py:83-113 for explicit level widths (box hidden 64, cls hidden nc)."""
    out = []
    for br, hid in (("box", 64), ("cls", nc)):
        for lv, c in enumerate(lvl_c):
            out += _conv_keys(f"head.{br}.{lv}.0", c, hid, 3)
            out += _conv_keys(f"head.{br}.{lv}.1", hid, hid, 3)
            out += [(f"head.{br}.{lv}.2.weight", (hid, hid, 1, 1)), (f"head.{br}.{lv}.2.bias", (hid,))]
    out.append(("head.dfl.conv.weight", (1, 16, 1, 1)))
    return out


def state_keys(version, nc):
    (c1, c2, c3, c4, c5), L = params(version)
    keys = []
    for name, ci, co in (("conv0", 3, c1), ("conv1", c1, c2), ("conv3", c2, c3), ("conv5", c3, c4), ("conv7", c4, c5)):
        keys += _conv_keys(f"backbone.{name}", ci, co, 3)
    for name, c, k in (("ms_2", c2, HKS[0]), ("ms_4", c3, HKS[1]), ("ms_6", c4, HKS[2]), ("ms_8", c5, HKS[3])):
        keys += _msblock_keys(f"backbone.{name}", c, c, k, L)
    keys += _conv_keys("backbone.sppf.conv1", c5, c5 // 2, 1)
    keys += _conv_keys("backbone.sppf.conv2", (c5 // 2) * 4, c5, 1)
    keys += _conv_keys("neck.reduce_5", c5, c4, 1)
    keys += _conv_keys("neck.reduce_4", c4, c3, 1)
    keys += _msblock_keys("neck.ms_1", 2 * c4, c4, 3, L)
    keys += _msblock_keys("neck.ms_2", 2 * c3, c3, 3, L)
    keys += _msblock_keys("neck.ms_3", 2 * c3, c4, 3, L)
    keys += _msblock_keys("neck.ms_4", 2 * c4, c5, 3, L)
    keys += _conv_keys("neck.conv1", c3, c3, 3)
    keys += _conv_keys("neck.conv2", c4, c4, 3)
    keys += _head_keys((c3, c4, c5), nc)
    return keys


def complexity(version, nc=80, size=640):
    """-> (parameters excluding the frozen DFL projection, conv MACs per image at size x size),
    counted by tracing this restatement's F.conv2d calls on the meta device."""
    n_par = sum(math.prod(s) for k, s in state_keys(version, nc)
                if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))
                and k != "head.dfl.conv.weight")
    macs = 0
    orig = F.conv2d

    def hook(x, wt, b=None, stride=1, padding=0, dilation=1, groups=1):
        nonlocal macs
        y = orig(x, wt, b, stride, padding, dilation, groups)
        if wt.shape[0] != 1 or wt.shape[1] != 16:      # not the DFL projection
            macs += y.shape[1] * y.shape[2] * y.shape[3] * wt.shape[1] * wt.shape[2] * wt.shape[3]
        return y

    sd = {k: torch.zeros(s, device="meta") if len(s) else torch.zeros((), device="meta")
          for k, s in state_keys(version, nc)}
    F.conv2d = hook
    try:
        forward(sd, version, nc, torch.zeros(1, 3, size, size, device="meta"), True)
    finally:
        F.conv2d = orig
    return n_par, macs


def init_params(version, nc):
    """Closed-form deterministic weights (model_ref._closed_form), non-identity BN statistics."""
    sd = OrderedDict()
    for key, shape in state_keys(version, nc):
        if key.endswith("num_batches_tracked"):
            sd[key] = torch.tensor(0, dtype=torch.long)
        elif key == "head.dfl.conv.weight":
            sd[key] = torch.arange(16, dtype=torch.float32).view(1, 16, 1, 1)
        elif key.endswith("conv.weight") or (key.startswith("head.") and key.endswith(".2.weight")):
            fan_in = shape[1] * shape[2] * shape[3]
            sd[key] = M._closed_form(key, shape, math.sqrt(3.0 / fan_in) * 1.2)
        elif key.endswith(".2.bias"):
            sd[key] = M._closed_form(key, shape, 0.5)
        elif key.endswith("bn.weight"):
            sd[key] = M._closed_form(key, shape, 0.25, base=1.0)
        elif key.endswith("bn.bias"):
            sd[key] = M._closed_form(key, shape, 0.2)
        elif key.endswith("running_mean"):
            sd[key] = M._closed_form(key, shape, 0.1)
        elif key.endswith("running_var"):
            sd[key] = M._closed_form(key, shape, 0.3, base=1.2)
        else:
            raise KeyError(key)
    return sd


def calibrate(sd, version, nc, x):
    """Running statistics := the batch statistics of one training-mode forward of x (momentum 1),
    so that eval-mode activations keep their training scale through the deep MS stacks (the
    closed-form running buffers compound to ~1e6 activations in ms-l's 3-layer IB chains)."""
    p = {k: t.clone() for k, t in sd.items()}
    saved = M.BN_MOMENTUM
    M.BN_MOMENTUM = 1.0
    try:
        with torch.no_grad():
            forward(p, version, nc, x, True)
    finally:
        M.BN_MOMENTUM = saved
    out = OrderedDict(sd)
    for k in sd:
        if "running_" in k:
            out[k] = p[k]
    return out


def conv_block(p, name, x, k, s, training, groups=1):
    y = F.conv2d(x, p[f"{name}.conv.weight"], None, s, k // 2, 1, groups)
    y = F.batch_norm(y, p[f"{name}.bn.running_mean"], p[f"{name}.bn.running_var"],
                     p[f"{name}.bn.weight"], p[f"{name}.bn.bias"], training, M.BN_MOMENTUM, M.BN_EPS)
    if training:
        p[f"{name}.bn.num_batches_tracked"] += 1
    return F.silu(y)


def ib_layer(p, name, x, k, training):
    y = conv_block(p, f"{name}.in_conv", x, 1, 1, training)
    y = conv_block(p, f"{name}.mid_conv", y, k, 1, training, groups=y.shape[1])
    return conv_block(p, f"{name}.out_conv", y, 1, 1, training)


def msblock(p, name, x, k, L, training):
    t = conv_block(p, f"{name}.in_conv", x, 1, 1, training)
    mid = t.shape[1] // 3
    ys = [t[:, :mid]]
    for b in range(2):
        s = t[:, (b + 1) * mid:(b + 2) * mid] + ys[-1]
        for j in range(L):
            s = ib_layer(p, f"{name}.branches.{b}.{j}", s, k, training)
        ys.append(s)
    return conv_block(p, f"{name}.out_conv", torch.cat(ys, 1), 1, 1, training)


def backbone(p, version, x, training):
    L = params(version)[1]
    x = conv_block(p, "backbone.conv0", x, 3, 2, training)
    x = conv_block(p, "backbone.conv1", x, 3, 2, training)
    x = msblock(p, "backbone.ms_2", x, HKS[0], L, training)
    x = conv_block(p, "backbone.conv3", x, 3, 2, training)
    out1 = msblock(p, "backbone.ms_4", x, HKS[1], L, training)
    x = conv_block(p, "backbone.conv5", out1, 3, 2, training)
    out2 = msblock(p, "backbone.ms_6", x, HKS[2], L, training)
    x = conv_block(p, "backbone.conv7", out2, 3, 2, training)
    x = msblock(p, "backbone.ms_8", x, HKS[3], L, training)
    out3 = M.sppf(p, "backbone.sppf", x, training)
    return out1, out2, out3


def neck(p, version, p3, p4, p5, training):
    L = params(version)[1]
    r5 = conv_block(p, "neck.reduce_5", p5, 1, 1, training)
    td4 = msblock(p, "neck.ms_1", torch.cat([M.upsample(r5), p4], 1), 3, L, training)
    r4 = conv_block(p, "neck.reduce_4", td4, 1, 1, training)
    out1 = msblock(p, "neck.ms_2", torch.cat([M.upsample(r4), p3], 1), 3, L, training)
    x = conv_block(p, "neck.conv1", out1, 3, 2, training)
    out2 = msblock(p, "neck.ms_3", torch.cat([x, r4], 1), 3, L, training)
    x = conv_block(p, "neck.conv2", out2, 3, 2, training)
    out3 = msblock(p, "neck.ms_4", torch.cat([x, r5], 1), 3, L, training)
    return out1, out2, out3


def forward(p, version, nc, x, training, strides=(8.0, 16.0, 32.0)):
    f = backbone(p, version, x, training)
    raw = M.head_raw(p, neck(p, version, *f, training), training)
    if training:
        return raw
    return M.decode(raw, nc, strides)
