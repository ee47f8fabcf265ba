"""YOLOv8 building blocks -- MI355X-native drop-in for the reference's
yolov8/model/components.py (rafaelghiorzi/YOLO-MS).

Same class names, constructor signatures, sub-module names (hence identical
state_dict keys) and forward contracts as the reference:

  Conv        components.py:69-77   Conv2d(bias=False) -> BatchNorm2d(eps=1e-3, momentum=0.03) -> SiLU
  Bottleneck  components.py:80-93   two 3x3 Conv, residual when shortcut
  C2f         components.py:96-122  1x1 -> split -> n bottlenecks (front-inserted) -> cat -> 1x1
  SPPF        components.py:125-150 1x1 -> 3 chained MaxPool2d(5,1,2) -> cat -> 1x1
  Upsample    components.py:153-160 nearest x2
  DFL         components.py:162-191 softmax over 16 bins . arange(16)
  yolo_params components.py:193-209

Execution is NOT eager PyTorch: ``forward`` hands the module tree to yms.runner,
which builds a static NHWC plan (concatenations become channel-offset placements)
and runs hand-written HIP kernels (implicit-GEMM MFMA convolutions with fused
BN/SiLU/residual epilogues, fused SPPF pooling, ...) as one autograd node.
"""
import torch
from torch import nn

from yms import runner as _runner
from yms import ops as _ops


class _YmsModule(nn.Module):
    """Default plan construction: one fresh NHWC buffer per input, ``emit`` the body."""

    def _yms_plan(self, b, inputs):
        ins = [b.new(x.shape[2], x.shape[3], x.shape[1]) for x in inputs]
        outs = self.emit(b, *ins)
        if not isinstance(outs, (list, tuple)):
            outs = [outs]
        return ins, list(outs), "maps"

    def _yms_run(self, *inputs):
        _, outs = _runner.run(self, list(inputs))
        return outs


class Conv(_YmsModule):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, groups=1,
                 activation=True) -> None:
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False, groups=groups)
        self.bn = nn.BatchNorm2d(out_channels, eps=0.001, momentum=0.03)
        self.activation = nn.SiLU(inplace=True) if activation else nn.Identity()

    def emit(self, b, x, out=None, res=None):
        return b.conv(self, x, out=out, res=res)

    def forward(self, x):
        return self._yms_run(x)[0]


class Bottleneck(_YmsModule):
    def __init__(self, in_channels, out_channels, shortcut=True) -> None:
        super().__init__()
        self.conv1 = Conv(in_channels, out_channels, kernel_size=3, stride=1, padding=1)
        self.conv2 = Conv(in_channels, out_channels, kernel_size=3, stride=1, padding=1)
        self.shortcut = shortcut

    def emit(self, b, x, out=None):
        y = self.conv1.emit(b, x)
        return self.conv2.emit(b, y, out=out, res=x if self.shortcut else None)

    def forward(self, x):
        return self._yms_run(x)[0]


class C2f(_YmsModule):
    def __init__(self, in_channels, out_channels, num_bottlenecks, shortcut=True) -> None:
        super().__init__()
        self.mid_channels = out_channels // 2
        self.num_bottlenecks = num_bottlenecks
        self.conv1 = Conv(in_channels, out_channels, kernel_size=1, stride=1, padding=0)
        # the reference never forwards `shortcut` to the bottlenecks (components.py:104)
        self.m = nn.ModuleList([Bottleneck(self.mid_channels, self.mid_channels) for _ in range(num_bottlenecks)])
        self.conv2 = Conv((num_bottlenecks + 2) * out_channels // 2, out_channels, kernel_size=1, stride=1, padding=0)

    def emit(self, b, x, out=None):
        n, cout = self.num_bottlenecks, self.conv1.conv.out_channels
        half = cout // 2
        ho = (x.h + 2 * self.conv1.conv.padding[0] - 1) // self.conv1.conv.stride[0] + 1
        wo = (x.w + 2 * self.conv1.conv.padding[0] - 1) // self.conv1.conv.stride[0] + 1
        # concat buffer [y_n, ..., y_1, x1, x2]  (front insertion, components.py:115-119)
        cat = b.new(ho, wo, n * half + cout, name="c2f_cat")
        xs = self.conv1.emit(b, x, out=cat.slot(n * half, cout))
        prev = cat.slot(n * half, half)            # x1
        for j in range(n):
            prev = self.m[j].emit(b, prev, out=cat.slot((n - 1 - j) * half, half))
        return self.conv2.emit(b, cat, out=out)

    def forward(self, x):
        return self._yms_run(x)[0]


class SPPF(_YmsModule):
    def __init__(self, in_channels, out_channels, kernel_size=5) -> None:
        super().__init__()
        hidden_channels = in_channels // 2
        self.conv1 = Conv(in_channels, hidden_channels, kernel_size=1, stride=1, padding=0)
        self.conv2 = Conv(hidden_channels * 4, out_channels, kernel_size=1, stride=1, padding=0)
        self.m = nn.MaxPool2d(kernel_size=kernel_size, stride=1, padding=kernel_size // 2, dilation=1, ceil_mode=False)

    def emit(self, b, x, out=None):
        if self.m.kernel_size not in (5, (5, 5)) or self.m.stride not in (1, (1, 1)):
            raise RuntimeError("yms: SPPF is implemented for the reference's MaxPool2d(5, 1, 2)")
        hid = self.conv1.conv.out_channels
        cat = b.new(x.h, x.w, 4 * hid, name="sppf_cat")   # [x, m(x), m(m(x)), m(m(m(x)))]
        self.conv1.emit(b, x, out=cat.slot(0, hid))
        b.sppf_pool(cat, hid)
        return self.conv2.emit(b, cat, out=out)

    def forward(self, x):
        return self._yms_run(x)[0]


class Upsample(_YmsModule):
    def __init__(self, scale_factor=2, mode='nearest') -> None:
        super().__init__()
        self.scale_factor = scale_factor
        self.mode = mode

    def emit(self, b, x, out=None):
        if self.scale_factor != 2 or self.mode != 'nearest':
            raise RuntimeError("yms: Upsample implements scale_factor=2, mode='nearest' (the reference's use)")
        return b.upsample(x, out=out)

    def forward(self, x):
        return self._yms_run(x)[0]


class DFL(nn.Module):
    """Distribution Focal Loss integral (components.py:162-191)."""

    def __init__(self, ch=16) -> None:
        super().__init__()
        self.ch = ch
        self.conv = nn.Conv2d(in_channels=ch, out_channels=1, kernel_size=1, bias=False).requires_grad_(False)
        x = torch.arange(ch, dtype=torch.float).view(1, ch, 1, 1)
        self.conv.weight.data[:] = torch.nn.Parameter(x)

    def forward(self, x):
        """x: [B, ch*4, A] -> [B, 4, A] (HIP kernel; weights fixed to arange(ch))."""
        return _ops.dfl(x, self.ch)


_SCALES = {  # version -> (depth multiple, width multiple, P5 width ratio)
    'n': (1 / 3, 1 / 4, 2.0),
    's': (1 / 3, 1 / 2, 2.0),
    'm': (2 / 3, 3 / 4, 1.5),
    'l': (1.0, 1.0, 1.0),
    'x': (1.0, 1.25, 1.0),
}


def yolo_params(version):
    """(depth, width, ratio) scaling of a model size; same table and ValueError as the reference."""
    if version not in _SCALES:
        raise ValueError(f"Unknown YOLOv8 version: {version}")
    return _SCALES[version]
