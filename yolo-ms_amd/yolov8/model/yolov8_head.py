"""Decoupled detection head + DFL decode -- MI355X-native drop-in for
yolov8/model/yolov8_head.py:72-158.

Per level i the box branch (Conv3x3, Conv3x3, 1x1 Conv2d+bias -> 4*ch) and the cls
branch (same, -> num_classes) write into the two channel slots of ONE NHWC buffer
[B, H, W, 4*ch+nc] (the reference's torch.cat at :122 is a placement).  Train mode
returns the three maps as [B, 4*ch+nc, H, W] tensors (channels-last views); eval mode
runs the fused decode kernel (anchors, DFL, ltrb->cxcywh, x stride, sigmoid) and
returns [B, A, 4+nc] fp32.  ``head.stride`` keeps the reference semantics: it
defaults to zeros(3) and callers set it to [8, 16, 32].
"""
import torch
from torch import nn

from yolov8.model.components import Conv, DFL, yolo_params, _YmsModule


class Head(_YmsModule):
    def __init__(self, version, ch=16, num_classes=80) -> None:
        super().__init__()
        self.ch = ch
        self.coordinates = self.ch * 4
        self.num_classes = num_classes
        self.no = self.coordinates + num_classes
        self.stride = torch.zeros(3)
        if isinstance(version, str) and version.startswith("ms-"):
            # YOLO-MS family (yolo_ms.py): the neck's calibrated widths, not yolo_params'
            from yolov8.model.yolo_ms import ms_head_channels
            in_c = list(ms_head_channels(version))
        else:
            d, w, r = yolo_params(version)
            in_c = [int(256 * w), int(512 * w), int(512 * w * r)]
        co, nc = self.coordinates, num_classes

        def branch(cin, hid):
            return nn.Sequential(Conv(cin, hid, kernel_size=3, stride=1, padding=1),
                                 Conv(hid, hid, kernel_size=3, stride=1, padding=1),
                                 nn.Conv2d(hid, hid, kernel_size=1, stride=1))

        self.box = nn.ModuleList([branch(c, co) for c in in_c])
        self.cls = nn.ModuleList([branch(c, nc) for c in in_c])
        self.dfl = DFL()   # the reference ignores `ch` here (yolov8_head.py:113)

    def emit(self, b, x0, x1, x2):
        if self.ch != 16:
            raise RuntimeError("yms: the DFL decode is built for ch=16 (as the reference's DFL())")
        outs = []
        for i, x in enumerate((x0, x1, x2)):
            o = b.new(x.h, x.w, self.no, name=f"head_out{i}")
            # the two branches' first convs read the same x_i: one SiblingConvOp (one buffer
            # [box | cls], one BN backward pass, one input and one weight gradient for both)
            firsts = b.sibling_convs([self.box[i][0], self.cls[i][0]], x)
            for br, t, off, c in ((self.box[i], firsts[0], 0, self.coordinates),
                                  (self.cls[i], firsts[1], self.coordinates, self.num_classes)):
                t = br[1].emit(b, t)
                b.conv2d_bias(br[2], t, out=o.slot(off, c))
            outs.append(o)
        return outs

    def yms_decode_info(self):
        st = self.stride
        if isinstance(st, torch.Tensor):
            key = (st.data_ptr(), st._version, st.device)
            cached = getattr(self, "_yms_stride_cache", None)
            if cached is None or cached[0] != key:
                self._yms_stride_cache = (key, [float(v) for v in st.detach().float().cpu().tolist()])
            vals = self._yms_stride_cache[1]
        else:
            vals = [float(v) for v in st]
        return {"nc": self.num_classes, "strides": vals}

    def _yms_plan(self, b, inputs):
        ins = [b.new(x.shape[2], x.shape[3], x.shape[1]) for x in inputs]
        outs = self.emit(b, *ins)
        return ins, outs, ("maps" if b.training else ("decode", self))

    def forward(self, x):
        outs = self._yms_run(*x)
        if self.training:
            for i, o in enumerate(outs):
                x[i] = o            # the reference overwrites the input list in place (:122)
            return x
        return outs[0]

    def make_anchors(self, x, stride, offset=0.5):
        """Anchor centres / per-anchor strides (yolov8_head.py:146-158); small host-side
        helper kept for API compatibility (the fused decode kernel computes them itself)."""
        assert x is not None
        anchor_tensor, stride_tensor = [], []
        dtype, device = x[0].dtype, x[0].device
        for i, s in enumerate(stride):
            _, _, h, w = x[i].shape
            sx = torch.arange(end=w, device=device, dtype=dtype) + offset
            sy = torch.arange(end=h, device=device, dtype=dtype) + offset
            sy, sx = torch.meshgrid(sy, sx, indexing='ij')
            anchor_tensor.append(torch.stack((sx, sy), -1).view(-1, 2))
            stride_tensor.append(torch.full((h * w, 1), s, dtype=dtype, device=device))
        return torch.cat(anchor_tensor), torch.cat(stride_tensor)
