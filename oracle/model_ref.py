"""CPU restatement of the reference YOLOv8 graph -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for the HIP path.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it,
and only as the checker / the timed CPU baseline -- never as the product.

It restates, as plain functional PyTorch-CPU fp32 code (F.conv2d,
F.batch_norm, F.silu, F.max_pool2d, torch.cat, F.interpolate), the graph
defined by the reference (paths relative to /root/reference):

  yolo_params            yolov8/model/components.py:193-209
  Conv                   yolov8/model/components.py:69-77
  Bottleneck             yolov8/model/components.py:80-93  (residual always on)
  C2f                    yolov8/model/components.py:96-122 (front-insert concat)
  SPPF                   yolov8/model/components.py:125-150
  Upsample               yolov8/model/components.py:153-160
  DFL                    yolov8/model/components.py:162-191
  Backbone               yolov8/model/yolov8_backbone.py:30-73
  Neck                   yolov8/model/yolov8_neck.py:54-94
  Head (+decode)         yolov8/model/yolov8_head.py:72-144
  Head.make_anchors      yolov8/model/yolov8_head.py:146-158
  YOLOv8                 yolov8/yolov8.py:7-32

Parity pinning: the restatement is checked against golden vectors produced
by importing the reference model in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz, tests/test_oracle_golden.py).
Gradients are those of torch-CPU autograd over this restated graph.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import torch
import torch.nn.functional as F

BN_EPS = 1e-3        # components.py:72  nn.BatchNorm2d(eps=0.001, momentum=0.03)
BN_MOMENTUM = 0.03


def yolo_params(version):
    """components.py:193-209 -- (depth, width, ratio); ValueError otherwise."""
    if version == 'n':
        return 1 / 3, 1 / 4, 2.0
    if version == 's':
        return 1 / 3, 1 / 2, 2.0
    if version == 'm':
        return 2 / 3, 3 / 4, 1.5
    if version == 'l':
        return 1.0, 1.0, 1.0
    if version == 'x':
        return 1.0, 1.25, 1.0
    raise ValueError(f"Unknown YOLOv8 version: {version}")


# ----------------------------------------------------------------------------
# Architecture table (names == reference state_dict keys)
# ----------------------------------------------------------------------------

def _c2f_convs(prefix, cin, cout, n):
    """C2f layer list, components.py:96-107 (conv1 1x1, n bottlenecks, conv2 1x1)."""
    mid = cout // 2
    out = [(f"{prefix}.conv1", cin, cout, 1, 1)]
    for i in range(n):
        out.append((f"{prefix}.m.{i}.conv1", mid, mid, 3, 1))
        out.append((f"{prefix}.m.{i}.conv2", mid, mid, 3, 1))
    out.append((f"{prefix}.conv2", (n + 2) * cout // 2, cout, 1, 1))
    return out


def arch(version, nc):
    """Every Conv block as (name, cin, cout, k, stride), in state_dict order,
    plus the head's plain 1x1 Conv2d(+bias) layers as ('name', cin, cout, 1, 1, 'bias')."""
    d, w, r = yolo_params(version)
    i = int
    convs = []
    # Backbone registration order: conv0, conv1, conv3, conv5, conv7, c2f_2, c2f_4, c2f_6, c2f_8, sppf
    convs += [("backbone.conv0", 3, i(64 * w), 3, 2),
              ("backbone.conv1", i(64 * w), i(128 * w), 3, 2),
              ("backbone.conv3", i(128 * w), i(256 * w), 3, 2),
              ("backbone.conv5", i(256 * w), i(512 * w), 3, 2),
              ("backbone.conv7", i(512 * w), i(512 * w * r), 3, 2)]
    convs += _c2f_convs("backbone.c2f_2", i(128 * w), i(128 * w), i(3 * d))
    convs += _c2f_convs("backbone.c2f_4", i(256 * w), i(256 * w), i(6 * d))
    convs += _c2f_convs("backbone.c2f_6", i(512 * w), i(512 * w), i(6 * d))
    convs += _c2f_convs("backbone.c2f_8", i(512 * w * r), i(512 * w * r), i(3 * d))
    p5 = i(512 * w * r)
    convs += [("backbone.sppf.conv1", p5, p5 // 2, 1, 1),
              ("backbone.sppf.conv2", (p5 // 2) * 4, p5, 1, 1)]
    # Neck: c2f_1..c2f_4, conv1, conv2 (yolov8_neck.py:58-65)
    convs += _c2f_convs("neck.c2f_1", i(512 * w * (1 + r)), i(512 * w), i(3 * d))
    convs += _c2f_convs("neck.c2f_2", i(768 * w), i(256 * w), i(3 * d))
    convs += _c2f_convs("neck.c2f_3", i(768 * w), i(512 * w), i(3 * d))
    convs += _c2f_convs("neck.c2f_4", i(512 * w * (1 + r)), i(512 * w * r), i(3 * d))
    convs += [("neck.conv1", i(256 * w), i(256 * w), 3, 2),
              ("neck.conv2", i(512 * w), i(512 * w), 3, 2)]
    # Head (yolov8_head.py:83-110)
    lvl_c = [i(256 * w), i(512 * w), i(512 * w * r)]
    for br, hid in (("box", 64), ("cls", nc)):
        for lv in range(3):
            convs.append((f"head.{br}.{lv}.0", lvl_c[lv], hid, 3, 1))
            convs.append((f"head.{br}.{lv}.1", hid, hid, 3, 1))
            convs.append((f"head.{br}.{lv}.2", hid, hid, 1, 1, "bias"))
    return convs


def state_keys(version, nc):
    """Ordered (key, shape) list identical to the reference model's state_dict."""
    out = []
    for spec in arch(version, nc):
        name, cin, cout, k = spec[0], spec[1], spec[2], spec[3]
        if len(spec) == 6:      # plain nn.Conv2d with bias
            out.append((f"{name}.weight", (cout, cin, k, k)))
            out.append((f"{name}.bias", (cout,)))
        else:
            out.append((f"{name}.conv.weight", (cout, cin, k, k)))
            for s in ("weight", "bias", "running_mean", "running_var"):
                out.append((f"{name}.bn.{s}", (cout,)))
            out.append((f"{name}.bn.num_batches_tracked", ()))
    out.append(("head.dfl.conv.weight", (1, 16, 1, 1)))
    # reorder to module registration order (box/cls ModuleLists registered before dfl)
    return out


def _closed_form(name, shape, amp, base=0.0, freq=0.7071):
    n = 1
    for s in shape:
        n *= s
    ph = (zlib.crc32(name.encode()) % 1000) / 1000.0 * 2 * math.pi
    idx = torch.arange(n, dtype=torch.float64)
    v = base + amp * torch.sin(freq * idx + ph)
    return v.to(torch.float32).reshape(shape)


def init_params(version, nc):
    """Deterministic closed-form weights (no RNG), so fixtures need not carry weights.

    Conv weights ~ sin(), scaled by sqrt(3/fan_in) (unit-gain uniform-like); BN affine
    and running stats are deliberately non-identity so BN folding is exercised."""
    sd = OrderedDict()
    for key, shape in state_keys(version, nc):
        if key.endswith("num_batches_tracked"):
            sd[key] = torch.tensor(0, dtype=torch.long)
        elif key == "head.dfl.conv.weight":
            sd[key] = torch.arange(16, dtype=torch.float32).view(1, 16, 1, 1)  # components.py:167-171
        elif key.endswith("conv.weight") or (key.startswith("head.") and key.endswith(".2.weight")):
            fan_in = shape[1] * shape[2] * shape[3]
            sd[key] = _closed_form(key, shape, math.sqrt(3.0 / fan_in) * 1.2)
        elif key.endswith(".2.bias"):
            sd[key] = _closed_form(key, shape, 0.5)
        elif key.endswith("bn.weight"):
            sd[key] = _closed_form(key, shape, 0.25, base=1.0)
        elif key.endswith("bn.bias"):
            sd[key] = _closed_form(key, shape, 0.2)
        elif key.endswith("running_mean"):
            sd[key] = _closed_form(key, shape, 0.1)
        elif key.endswith("running_var"):
            sd[key] = _closed_form(key, shape, 0.3, base=1.2)
        else:
            raise KeyError(key)
    return sd


def ordered_init(sd, seed=0, gamma=0.3):
    """Well-conditioned variant of a closed-form state dict (tests only): conv weights He-normal
    from a seeded generator, BN gammas around ``gamma`` (closed form, +-25%).

    The closed-form sin() weights are strongly correlated along the flattened index, and with BN
    gammas ~1 the deep graphs sit in a chaotic regime where forward rounding differences grow
    ~2x per 10 BN layers: torch's own CPU fp32 gradients then miss fp64 by up to 1e-1 (ms-l at
    640: median 0.56), so a gradient gate measures the graph, not the kernels.  With these
    weights the CPU fp32 gradients sit within ~6e-5 of fp64 on every graph the tests train (n, s,
    l, ms-xs, ms-s, ms-l; tools/cond_sweep.py), and absolute / 1.3x-of-CPU-bf16 gates apply."""
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for k, t in sd.items():
        if k.endswith("conv.weight") and k != "head.dfl.conv.weight" or (k.startswith("head.") and k.endswith(".2.weight")):
            fan = t.shape[1] * t.shape[2] * t.shape[3]
            out[k] = torch.randn(tuple(t.shape), generator=g) * math.sqrt(2.0 / fan)
        elif k.endswith("bn.weight"):
            out[k] = _closed_form(k, tuple(t.shape), 0.25 * gamma, base=gamma)
        else:
            out[k] = t.clone()
    return out


# ----------------------------------------------------------------------------
# Functional graph
# ----------------------------------------------------------------------------

def conv_block(p, name, x, k, s, training):
    """components.py:69-77: SiLU(BN(Conv2d(x, bias=False, stride s, pad k//2)))."""
    y = F.conv2d(x, p[f"{name}.conv.weight"], None, s, k // 2)
    y = F.batch_norm(y, p[f"{name}.bn.running_mean"], p[f"{name}.bn.running_var"],
                     p[f"{name}.bn.weight"], p[f"{name}.bn.bias"], training, BN_MOMENTUM, BN_EPS)
    if training:
        p[f"{name}.bn.num_batches_tracked"] += 1
    return F.silu(y)


def bottleneck(p, name, x, training):
    """components.py:80-93 -- residual is always applied (C2f never forwards shortcut)."""
    y = conv_block(p, f"{name}.conv1", x, 3, 1, training)
    y = conv_block(p, f"{name}.conv2", y, 3, 1, training)
    return y + x


def c2f(p, name, x, n, training):
    """components.py:108-122: outputs = [y_n, ..., y_1, x1, x2] then 1x1 conv."""
    x = conv_block(p, f"{name}.conv1", x, 1, 1, training)
    c = x.shape[1] // 2
    x1, x2 = x[:, :c], x[:, c:]
    outs = [x1, x2]
    for i in range(n):
        x1 = bottleneck(p, f"{name}.m.{i}", x1, training)
        outs.insert(0, x1)
    return conv_block(p, f"{name}.conv2", torch.cat(outs, 1), 1, 1, training)


def maxpool5(x):
    return F.max_pool2d(x, 5, 1, 2)


def sppf(p, name, x, training):
    """components.py:138-150."""
    x = conv_block(p, f"{name}.conv1", x, 1, 1, training)
    x1 = maxpool5(x)
    x2 = maxpool5(x1)
    x3 = maxpool5(x2)
    return conv_block(p, f"{name}.conv2", torch.cat([x, x1, x2, x3], 1), 1, 1, training)


def upsample(x):
    """components.py:159-160: nearest x2."""
    return F.interpolate(x, scale_factor=2, mode="nearest")


def backbone(p, version, x, training):
    """yolov8_backbone.py:54-73."""
    d, _, _ = yolo_params(version)
    x = conv_block(p, "backbone.conv0", x, 3, 2, training)
    x = conv_block(p, "backbone.conv1", x, 3, 2, training)
    x = c2f(p, "backbone.c2f_2", x, int(3 * d), training)
    x = conv_block(p, "backbone.conv3", x, 3, 2, training)
    out1 = c2f(p, "backbone.c2f_4", x, int(6 * d), training)
    x = conv_block(p, "backbone.conv5", out1, 3, 2, training)
    out2 = c2f(p, "backbone.c2f_6", x, int(6 * d), training)
    x = conv_block(p, "backbone.conv7", out2, 3, 2, training)
    x = c2f(p, "backbone.c2f_8", x, int(3 * d), training)
    out3 = sppf(p, "backbone.sppf", x, training)
    return out1, out2, out3


def neck(p, version, x_res_1, x_res_2, x, training):
    """yolov8_neck.py:67-94."""
    d, _, _ = yolo_params(version)
    n = int(3 * d)
    res_1 = x
    x = torch.cat([upsample(x), x_res_2], 1)
    res_2 = c2f(p, "neck.c2f_1", x, n, training)
    x = torch.cat([upsample(res_2), x_res_1], 1)
    out1 = c2f(p, "neck.c2f_2", x, n, training)
    x = conv_block(p, "neck.conv1", out1, 3, 2, training)
    x = torch.cat([x, res_2], 1)
    out2 = c2f(p, "neck.c2f_3", x, n, training)
    x = conv_block(p, "neck.conv2", out2, 3, 2, training)
    x = torch.cat([x, res_1], 1)
    out3 = c2f(p, "neck.c2f_4", x, n, training)
    return out1, out2, out3


def head_raw(p, feats, training):
    """yolov8_head.py:115-122: per level cat(box_i(x), cls_i(x))."""
    outs = []
    for lv, x in enumerate(feats):
        br = []
        for b in ("box", "cls"):
            y = conv_block(p, f"head.{b}.{lv}.0", x, 3, 1, training)
            y = conv_block(p, f"head.{b}.{lv}.1", y, 3, 1, training)
            y = F.conv2d(y, p[f"head.{b}.{lv}.2.weight"], p[f"head.{b}.{lv}.2.bias"])
            br.append(y)
        outs.append(torch.cat(br, 1))
    return outs


def make_anchors(feats, strides, offset=0.5):
    """yolov8_head.py:146-158 (dtype follows the features)."""
    anchors, stride_t = [], []
    dtype = feats[0].dtype
    for i, st in enumerate(strides):
        _, _, h, w = feats[i].shape
        sx = torch.arange(w, dtype=dtype) + offset
        sy = torch.arange(h, dtype=dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        anchors.append(torch.stack((sx, sy), -1).view(-1, 2))
        stride_t.append(torch.full((h * w, 1), float(st), dtype=dtype))
    return torch.cat(anchors), torch.cat(stride_t)


def dfl(box):
    """components.py:186-191: softmax over 16 bins (coord-major channels) . arange(16)."""
    b, c, a = box.shape
    x = box.view(b, 4, 16, a).transpose(1, 2).softmax(1)
    w = torch.arange(16, dtype=box.dtype).view(1, 16, 1, 1)
    return F.conv2d(x, w).view(b, 4, a)


def decode(raw, nc, strides):
    """yolov8_head.py:127-144 -> [B, A, 4+nc] (cx, cy, w, h)*stride, sigmoid(cls)."""
    no = 64 + nc
    anchors, st = (t.transpose(0, 1) for t in make_anchors(raw, strides))
    x = torch.cat([t.reshape(raw[0].shape[0], no, -1) for t in raw], 2)
    box, cls = x.split((64, nc), 1)
    a, b = dfl(box).chunk(2, 1)
    a = anchors.unsqueeze(0) - a
    b = anchors.unsqueeze(0) + b
    box = torch.cat(((a + b) / 2, b - a), 1)
    return torch.cat((box * st, cls.sigmoid()), 1).transpose(1, 2)


def forward(p, version, nc, x, training, strides=(8.0, 16.0, 32.0)):
    """yolov8.py:23-32.  Train mode -> list of [B, 64+nc, H, W]; eval -> [B, A, 4+nc]."""
    f = backbone(p, version, x, training)
    raw = head_raw(p, neck(p, version, *f, training), training)
    if training:
        return raw
    return decode(raw, nc, strides)


def count_conv_flops(version, nc, h, w):
    """Algorithmic conv FLOPs per image (2*MAC) for the forward graph."""
    flops = 0
    shapes = conv_shapes(version, nc, h, w)
    for (_, cin, cout, k, s, ho, wo) in shapes:
        flops += 2 * ho * wo * cout * cin * k * k
    return flops


def conv_shapes(version, nc, h, w):
    """(name, cin, cout, k, stride, Hout, Wout) per conv in forward order, obtained by
    tracing the functional graph with hooks on F.conv2d (meta device, no compute)."""
    rec = []
    orig = F.conv2d

    def hook(x, wt, b=None, stride=1, padding=0, *a, **kw):
        y = orig(x, wt, b, stride, padding, *a, **kw)
        s = stride if isinstance(stride, int) else stride[0]
        if wt.shape[0] != 1:
            rec.append((None, wt.shape[1], wt.shape[0], wt.shape[2], s, y.shape[2], y.shape[3]))
        return y

    sd = {k: torch.zeros(s, device="meta") if len(s) else torch.zeros((), device="meta")
          for k, s in state_keys(version, nc)}
    F.conv2d = hook
    try:
        forward(sd, version, nc, torch.zeros(1, 3, h, w, device="meta"), True)
    finally:
        F.conv2d = orig
    return rec
