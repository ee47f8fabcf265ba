"""YOLO-MS model family (MS-Block, heterogeneous-kernel-size backbone) on the MI355X plan runtime.

The reference repository implements YOLOv8 only; YOLO-MS appears there as a diagram
(annotations.md:66-133: C2f -> MSBlock in backbone and neck, SPPF -> "MS-SPPF", Concat ->
"MSFusion") and the upstream model-zoo table (model_zoos.md:21-53: YOLO-MS-XS 5.1 M params /
8.7 G FLOPs, YOLO-MS-S 8.7 M / 15.0 G, YOLO-MS 23.3 M / 38.8 G).  BASELINE.json's north star names
the MS-Block and the heterogeneous-kernel-size stages, so they are built here as SURVEY 7.4
describes them (YOLO-MS paper, arXiv 2308.05480; unverifiable offline), on the reference diagram's
topology, with widths calibrated to the model-zoo table (parity for this family is against the
build's own CPU restatement oracle/ms_ref.py, NOT reference-pinned):

  MSBlock(x)   = out_conv_1x1(cat[Y_1, Y_2, Y_3]),  [X_1 | X_2 | X_3] = in_conv_1x1(x)
                 Y_1 = X_1,  Y_i = IB_k^L(X_i + Y_{i-1})          (hidden = 3*in // 2 channels)
  IB_k         = Conv1x1(c -> 2c) -> depthwise Conv k x k (2c) -> Conv1x1(2c -> c)
                 every Conv = Conv2d(bias=False) -> BN(eps 1e-3, mom 0.03) -> SiLU (components.py:69-77)
  backbone     = the diagram's "Conv -> Conv" stem (two stride-2 3x3 Convs, as YOLOv8's), then
                 MSBlock(k = 3) | Conv s2, MSBlock(k = 5) -> P3 | Conv s2, MSBlock(k = 7) -> P4 |
                 Conv s2, MSBlock(k = 9), MS-SPPF -> P5   (HKS: the kernel grows with depth)
  MS-SPPF      = SPPF with the reference's cascade of three MaxPool2d(5, 1, 2): its concat holds the
                 5/9/13 pooling windows of one map, a multi-scale pool (components.py:125-150)
  MSFusion     = the PAFPN fusion of YOLO-MS's RTMDet lineage: the deeper map is reduced to the
                 lateral width by a 1x1 Conv ("reduce") before the top-down upsample, and the
                 bottom-up path concatenates with those reduced maps:
                   r5 = reduce_5(P5);  td4 = MSBlock(cat[up(r5), P4]);  r4 = reduce_4(td4)
                   out1 = MSBlock(cat[up(r4), P3])
                   out2 = MSBlock(cat[conv1_s2(out1), r4]);  out3 = MSBlock(cat[conv2_s2(out2), r5])
                 (neck MSBlocks k = 3; each concat is a channel-slot placement, no copy)
  head         = the reference's decoupled head and DFL decode on (out1, out2, out3), unchanged

Sizes (``MS_ARCH``): the stage widths and the IB depth are calibrated so that parameters and
forward multiply-accumulates at 640x640 match the model-zoo table (its "FLOPs" are MACs, the
mmengine / fvcore convention; see ``ms_complexity`` and tests/test_ms_cpu.py).  IB layers per
branch: one for XS / S, two for YOLO-MS (the paper's three-layer depth scaled by 1/3 and 2/3);
among the width tables that land within 2% of both figures, the one with the fewest activation
elements was taken (the training step is bound by the BN passes over them).  The reference's ``yolo_params`` keeps raising ValueError for every
string outside 'n'..'x', 'ms-*' included.
"""
from torch import nn

from yolov8.model.components import Conv, SPPF, Upsample, _YmsModule

# version -> ((stem c1, stage widths c2 (stride 4), c3 (P3), c4 (P4), c5 (P5)), IB layers per branch)
MS_ARCH = {
    "ms-xs": ((24, 48, 112, 224, 192), 1),
    "ms-s": ((32, 64, 160, 288, 288), 1),
    "ms-l": ((56, 112, 224, 448, 384), 2),
}
# model_zoos.md:21-53 (params in M, FLOPs = MACs in G at 640x640) of the upstream YOLO-MS family
MODEL_ZOO = {"ms-xs": (5.1, 8.7), "ms-s": (8.7, 15.0), "ms-l": (23.3, 38.8)}
HKS_KERNELS = (3, 5, 7, 9)        # backbone MS stages 1..4
NECK_KERNEL = 3


def ms_params(version):
    """-> (widths (c1..c5), ib_layers) of a YOLO-MS version; ValueError otherwise."""
    if version not in MS_ARCH:
        raise ValueError(f"Unknown YOLO-MS version: {version}")
    return MS_ARCH[version]


def ms_head_channels(version):
    """Channels of the three maps the neck hands to the head (P3, P4, P5 levels)."""
    c = ms_params(version)[0]
    return c[2], c[3], c[4]


def is_ms_version(version):
    return isinstance(version, str) and version in MS_ARCH


class MSBlockLayer(_YmsModule):
    """Inverted bottleneck IB_k: 1x1 expand (x2) -> depthwise k x k -> 1x1 project."""

    def __init__(self, channels, kernel_size):
        super().__init__()
        hid = 2 * channels
        self.in_conv = Conv(channels, hid, kernel_size=1, stride=1, padding=0)
        self.mid_conv = Conv(hid, hid, kernel_size=kernel_size, stride=1, padding=kernel_size // 2, groups=hid)
        self.out_conv = Conv(hid, channels, kernel_size=1, stride=1, padding=0)

    def emit(self, b, x, out=None):
        t = self.in_conv.emit(b, x)
        t = self.mid_conv.emit(b, t)
        return self.out_conv.emit(b, t, out=out)

    def forward(self, x):
        return self._yms_run(x)[0]


class MSBlock(_YmsModule):
    """Multi-scale block: three channel groups, the 2nd and 3rd through IB_k stacks, each fed the
    previous group's output (hierarchical residual), then a 1x1 fusion conv."""

    def __init__(self, in_channels, out_channels, kernel_size=3, layers=1):
        super().__init__()
        hidden = int(in_channels * 3) // 2
        if hidden % 3 or (hidden // 3) % 8:
            raise ValueError(f"MSBlock: hidden width {hidden} must split into 3 groups of a multiple of 8 channels")
        self.mid = hidden // 3
        self.kernel_size = kernel_size
        self.in_conv = Conv(in_channels, hidden, kernel_size=1, stride=1, padding=0)
        self.branches = nn.ModuleList([nn.Sequential(*[MSBlockLayer(self.mid, kernel_size) for _ in range(layers)])
                                       for _ in range(2)])
        self.out_conv = Conv(hidden, out_channels, kernel_size=1, stride=1, padding=0)

    @property
    def out_channels(self):
        return self.out_conv.conv.out_channels

    def emit(self, b, x, out=None):
        mid = self.mid
        # one buffer holds [X_1 | X_2 | X_3] and becomes the concat [Y_1 | Y_2 | Y_3] in place:
        # Y_1 = X_1 needs no copy, and Y_{i+1} is written over X_{i+1} once X_{i+1} + Y_i has been
        # formed (the gradient tracker releases a slice when its producer's backward has taken it)
        t = self.in_conv.emit(b, x)                           # [X_1 | X_2 | X_3]
        prev = t.slot(0, mid)                                 # Y_1 = X_1
        for i, br in enumerate(self.branches):
            s = b.add(t.slot((i + 1) * mid, mid), prev)       # X_{i+1} + Y_i
            for j, layer in enumerate(br):
                s = layer.emit(b, s, out=t.slot((i + 1) * mid, mid) if j == len(br) - 1 else None)
            prev = s
        return self.out_conv.emit(b, t, out=out)             # [Y_1 | Y_2 | Y_3]

    def forward(self, x):
        return self._yms_run(x)[0]


class MSBackbone(_YmsModule):
    """Two stride-2 stem Convs, heterogeneous-kernel-size MS stages (k = 3, 5, 7, 9), MS-SPPF."""

    def __init__(self, version, in_channels=3):
        super().__init__()
        (c1, c2, c3, c4, c5), L = ms_params(version)
        self.conv0 = Conv(in_channels, c1, kernel_size=3, stride=2, padding=1)
        self.conv1 = Conv(c1, c2, kernel_size=3, stride=2, padding=1)
        self.conv3 = Conv(c2, c3, kernel_size=3, stride=2, padding=1)
        self.conv5 = Conv(c3, c4, kernel_size=3, stride=2, padding=1)
        self.conv7 = Conv(c4, c5, kernel_size=3, stride=2, padding=1)
        k = HKS_KERNELS
        self.ms_2 = MSBlock(c2, c2, k[0], L)
        self.ms_4 = MSBlock(c3, c3, k[1], L)
        self.ms_6 = MSBlock(c4, c4, k[2], L)
        self.ms_8 = MSBlock(c5, c5, k[3], L)
        self.sppf = SPPF(c5, c5, kernel_size=5)               # MS-SPPF (module docstring)

    def out_channels(self):
        return self.ms_4.out_channels, self.ms_6.out_channels, self.sppf.conv2.conv.out_channels

    def emit(self, b, x, outs=(None, None, None)):
        x = self.conv0.emit(b, x)
        x = self.conv1.emit(b, x)
        x = self.ms_2.emit(b, x)
        x = self.conv3.emit(b, x)
        p3 = self.ms_4.emit(b, x, out=outs[0])
        x = self.conv5.emit(b, p3)
        p4 = self.ms_6.emit(b, x, out=outs[1])
        x = self.conv7.emit(b, p4)
        x = self.ms_8.emit(b, x)
        p5 = self.sppf.emit(b, x, out=outs[2])
        return p3, p4, p5

    def forward(self, x):
        return tuple(self._yms_run(x))


class MSNeck(_YmsModule):
    """PAFPN with MSFusion (1x1 reduce of the deeper map, upsample, concat) and MSBlock(k = 3)
    fusion blocks (module docstring).  Same plan interface as the YOLOv8 Neck (alloc_cats / emit)."""

    def __init__(self, version):
        super().__init__()
        (_, _, c3, c4, c5), L = ms_params(version)
        self.up = Upsample()
        self.reduce_5 = Conv(c5, c4, kernel_size=1, stride=1, padding=0)
        self.reduce_4 = Conv(c4, c3, kernel_size=1, stride=1, padding=0)
        self.ms_1 = MSBlock(2 * c4, c4, NECK_KERNEL, L)       # top-down P4
        self.ms_2 = MSBlock(2 * c3, c3, NECK_KERNEL, L)       # top-down P3 -> out1
        self.ms_3 = MSBlock(2 * c3, c4, NECK_KERNEL, L)       # bottom-up P4 -> out2
        self.ms_4 = MSBlock(2 * c4, c5, NECK_KERNEL, L)       # bottom-up P5 -> out3
        self.conv1 = Conv(c3, c3, kernel_size=3, stride=2, padding=1)
        self.conv2 = Conv(c4, c4, kernel_size=3, stride=2, padding=1)

    def alloc_cats(self, b, h3, w3, c3, h4, w4, c4, h5, w5, c5):
        """The four concat buffers; returns them and the slots P3 / P4 occupy (P5 is read by
        reduce_5 only and gets a buffer of its own)."""
        r4 = self.reduce_4.conv.out_channels
        r5 = self.reduce_5.conv.out_channels
        d1, d2 = self.conv1.conv.out_channels, self.conv2.conv.out_channels
        cat1 = b.new(h4, w4, r5 + c4, name="neck_cat1")      # [up(r5), P4]
        cat2 = b.new(h3, w3, r4 + c3, name="neck_cat2")      # [up(r4), P3]
        cat3 = b.new(h4, w4, d1 + r4, name="neck_cat3")      # [conv1(out1), r4]
        cat4 = b.new(h5, w5, d2 + r5, name="neck_cat4")      # [conv2(out2), r5]
        return (cat1, cat2, cat3, cat4), (cat2.slot(r4, c3), cat1.slot(r5, c4), None)

    def emit(self, b, p3, p4, p5, cats=None, outs=(None, None, None)):
        if cats is None:
            raise RuntimeError("yms: MSNeck.emit needs its concat buffers (use alloc_cats)")
        cat1, cat2, cat3, cat4 = cats
        r4c = self.reduce_4.conv.out_channels
        r5c = self.reduce_5.conv.out_channels
        d1, d2 = self.conv1.conv.out_channels, self.conv2.conv.out_channels
        r5 = self.reduce_5.emit(b, p5, out=cat4.slot(d2, r5c))
        self.up.emit(b, r5, out=cat1.slot(0, r5c))
        td4 = self.ms_1.emit(b, cat1)
        r4 = self.reduce_4.emit(b, td4, out=cat3.slot(d1, r4c))
        self.up.emit(b, r4, out=cat2.slot(0, r4c))
        out1 = self.ms_2.emit(b, cat2, out=outs[0])
        self.conv1.emit(b, out1, out=cat3.slot(0, d1))
        out2 = self.ms_3.emit(b, cat3, out=outs[1])
        self.conv2.emit(b, out2, out=cat4.slot(0, d2))
        out3 = self.ms_4.emit(b, cat4, out=outs[2])
        return out1, out2, out3

    def _yms_plan(self, b, inputs):
        x3, x4, x5 = inputs
        cats, slots = self.alloc_cats(b, x3.shape[2], x3.shape[3], x3.shape[1], x4.shape[2], x4.shape[3],
                                      x4.shape[1], x5.shape[2], x5.shape[3], x5.shape[1])
        p5 = b.new(x5.shape[2], x5.shape[3], x5.shape[1])
        ins = [slots[0], slots[1], p5]
        return ins, list(self.emit(b, *ins, cats=cats)), "maps"

    def forward(self, x_res_1, x_res_2, x):
        return tuple(self._yms_run(x_res_1, x_res_2, x))


def ms_complexity(version, nc=80, size=640):
    """-> (parameters, conv MACs per image at size x size, BN + upsample elements per image) of the
    YOLO-MS graph, computed from the module shapes (no tensors).  The model-zoo "FLOPs" are MACs
    (mmengine / fvcore count a multiply-add as one); fvcore also counts one op per batch-norm and
    nearest-upsample output element, reported as the third value."""
    from yolov8.yolov8 import YOLOv8
    m = YOLOv8(version, nc)
    params = sum(p.numel() for p in m.parameters()) - m.head.dfl.conv.weight.numel()
    macs, elems = 0, 0
    (c1, c2, c3, c4, c5), _ = ms_params(version)

    def conv(mod, h, w):
        nonlocal macs, elems
        cv = mod.conv if hasattr(mod, "conv") and isinstance(mod.conv, nn.Conv2d) else mod
        s = cv.stride[0]
        ho, wo = (h + 2 * cv.padding[0] - cv.kernel_size[0]) // s + 1, (w + 2 * cv.padding[0] - cv.kernel_size[0]) // s + 1
        macs += ho * wo * cv.out_channels * (cv.in_channels // cv.groups) * cv.kernel_size[0] * cv.kernel_size[1]
        if cv is not mod:
            elems += ho * wo * cv.out_channels
        return ho, wo

    def msblock(blk, h, w):
        conv(blk.in_conv, h, w)
        for br in blk.branches:
            for layer in br:
                for c in (layer.in_conv, layer.mid_conv, layer.out_conv):
                    conv(c, h, w)
        conv(blk.out_conv, h, w)

    bb, nk, hd = m.backbone, m.neck, m.head
    h = w = size
    h, w = conv(bb.conv0, h, w)
    h, w = conv(bb.conv1, h, w)
    msblock(bb.ms_2, h, w)
    for cv, blk in ((bb.conv3, bb.ms_4), (bb.conv5, bb.ms_6), (bb.conv7, bb.ms_8)):
        h, w = conv(cv, h, w)
        msblock(blk, h, w)
    conv(bb.sppf.conv1, h, w)
    conv(bb.sppf.conv2, h, w)
    s3, s4, s5 = size // 8, size // 16, size // 32
    conv(nk.reduce_5, s5, s5)
    elems += s4 * s4 * c4                                   # upsample
    msblock(nk.ms_1, s4, s4)
    conv(nk.reduce_4, s4, s4)
    elems += s3 * s3 * c3
    msblock(nk.ms_2, s3, s3)
    conv(nk.conv1, s3, s3)
    msblock(nk.ms_3, s4, s4)
    conv(nk.conv2, s4, s4)
    msblock(nk.ms_4, s5, s5)
    for i, s in enumerate((s3, s4, s5)):
        for br in (hd.box[i], hd.cls[i]):
            for mod in br:
                conv(mod, s, s)
    return params, macs, elems
