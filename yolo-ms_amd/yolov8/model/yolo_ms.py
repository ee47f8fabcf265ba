"""YOLO-MS model family (MS-Block, heterogeneous-kernel-size backbone) on the MI355X plan runtime.

The reference repository implements YOLOv8 only; YOLO-MS appears there as a diagram
(annotations.md:66-133: C2f -> MSBlock in backbone and neck, SPPF -> "MS-SPPF", Concat ->
"MSFusion") and the upstream model-zoo table (model_zoos.md).  BASELINE.json's north star names
the MS-Block and the heterogeneous-kernel-size stages, so they are built here as SURVEY 7.4
describes them (from the YOLO-MS paper, arXiv 2308.05480; unverifiable offline, so parity for
this family is against the build's own CPU restatement oracle/ms_ref.py, NOT reference-pinned):

  MSBlock(x)   = out_conv_1x1(cat[Y_1, Y_2, Y_3]),  [X_1 | X_2 | X_3] = in_conv_1x1(x)
                 Y_1 = X_1,  Y_i = IB_k^L(X_i + Y_{i-1})          (hidden = 3*in // 2 channels)
  IB_k         = Conv1x1(c -> 2c) -> depthwise Conv k x k (2c) -> Conv1x1(2c -> c)
                 every Conv = Conv2d(bias=False) -> BN(eps 1e-3, mom 0.03) -> SiLU (components.py:69-77)
  backbone     = the YOLOv8 stem / stride-2 convs with C2f stage i replaced by MSBlock(k = 3, 5, 7, 9)
                 (HKS: the kernel grows with depth), SPPF kept as the "MS-SPPF" slot
  neck         = the YOLOv8 PAFPN with every C2f replaced by MSBlock(k = 3); MSFusion = the
                 concatenation (a channel-slot placement here, as for YOLOv8)
  head         = the reference's decoupled head and DFL decode, unchanged

Versions 'ms-xs' / 'ms-s' / 'ms-l' take the widths and depth of the reference's 'n' / 's' / 'l'
rows (components.py:193-209; IB layers per branch = max(1, round(3 * depth))).  The reference's
``yolo_params`` keeps raising ValueError for every string outside 'n'..'x', 'ms-*' included.
"""
from torch import nn

from yolov8.model.components import Conv, SPPF, Upsample, yolo_params, _YmsModule
from yolov8.model.yolov8_neck import Neck

MS_VERSIONS = {"ms-xs": "n", "ms-s": "s", "ms-l": "l"}
HKS_KERNELS = (3, 5, 7, 9)        # backbone MS stages 1..4
NECK_KERNEL = 3


def ms_params(version):
    """-> (depth, width, ratio, ib_layers, base_version) of a YOLO-MS version; ValueError otherwise."""
    if version not in MS_VERSIONS:
        raise ValueError(f"Unknown YOLO-MS version: {version}")
    base = MS_VERSIONS[version]
    d, w, r = yolo_params(base)
    return d, w, r, max(1, round(3 * d)), base


def is_ms_version(version):
    return isinstance(version, str) and version in MS_VERSIONS


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
        t = self.in_conv.emit(b, x)                           # [X_1 | X_2 | X_3]
        cat = b.new(t.h, t.w, 3 * mid, name="ms_cat")         # [Y_1 | Y_2 | Y_3]
        b.add(t.slot(0, mid), None, out=cat.slot(0, mid))     # Y_1 = X_1
        prev = cat.slot(0, mid)
        for i, br in enumerate(self.branches):
            s = b.add(t.slot((i + 1) * mid, mid), prev)       # X_{i+1} + Y_i
            for j, layer in enumerate(br):
                s = layer.emit(b, s, out=cat.slot((i + 1) * mid, mid) if j == len(br) - 1 else None)
            prev = s
        return self.out_conv.emit(b, cat, out=out)

    def forward(self, x):
        return self._yms_run(x)[0]


class MSBackbone(_YmsModule):
    """YOLOv8 stem with heterogeneous-kernel-size MS stages (k = 3, 5, 7, 9) and SPPF."""

    def __init__(self, version, in_channels=3):
        super().__init__()
        d, w, r, L, _ = ms_params(version)
        c1, c2, c3, c4, c5 = int(64 * w), int(128 * w), int(256 * w), int(512 * w), int(512 * w * r)
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
        self.sppf = SPPF(c5, c5, kernel_size=5)

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


class MSNeck(Neck):
    """The YOLOv8 PAFPN (yolov8_neck.py:54-94) with MSBlock(k=3) in place of every C2f."""

    def __init__(self, version):
        nn.Module.__init__(self)
        d, w, r, L, _ = ms_params(version)
        self.up = Upsample()
        self.ms_1 = MSBlock(int(512 * w * (1 + r)), int(512 * w), NECK_KERNEL, L)
        self.ms_2 = MSBlock(int(768 * w), int(256 * w), NECK_KERNEL, L)
        self.ms_3 = MSBlock(int(768 * w), int(512 * w), NECK_KERNEL, L)
        self.ms_4 = MSBlock(int(512 * w * (1 + r)), int(512 * w * r), NECK_KERNEL, L)
        self.conv1 = Conv(int(256 * w), int(256 * w), kernel_size=3, stride=2, padding=1)
        self.conv2 = Conv(int(512 * w), int(512 * w), kernel_size=3, stride=2, padding=1)

    def _stage(self, i):
        return getattr(self, f"ms_{i}")
