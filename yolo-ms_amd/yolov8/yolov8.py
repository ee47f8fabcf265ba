"""YOLOv8 detector -- MI355X-native drop-in for the reference's yolov8/yolov8.py:7-32.

``YOLOv8(version, num_classes, dfl_ch=16)`` keeps the reference constructor, the
backbone/neck/head attributes (identical state_dict keys) and the output contract:
train mode -> list of 3 maps [B, 64+nc, H_i, W_i]; eval mode -> [B, A, 4+nc].

The whole forward (and, in training, backward) is ONE static plan of HIP kernels on
MI355X: the backbone writes P3/P4/P5 directly into the neck's concatenation buffers,
the neck writes into the head, the head's box/cls branches share one output buffer.
"""
from torch import nn

from yolov8.model.yolov8_backbone import Backbone
from yolov8.model.yolov8_neck import Neck
from yolov8.model.yolov8_head import Head
from yolov8.model.yolo_ms import MSBackbone, MSNeck, is_ms_version
from yms import runner as _runner


class YOLOv8(nn.Module):
    def __init__(self, version: str, num_classes: int, dfl_ch: int = 16) -> None:
        super().__init__()
        if is_ms_version(version):
            # YOLO-MS family ('ms-xs', 'ms-s', 'ms-l'): MS-Block / HKS backbone and neck, the
            # reference head (yolov8/model/yolo_ms.py; not in the reference's code)
            self.backbone = MSBackbone(version)
            self.neck = MSNeck(version)
            self.head = Head(version=version, num_classes=num_classes, ch=dfl_ch)
            return
        self.backbone = Backbone(version)
        self.neck = Neck(version)
        self.head = Head(version=version, num_classes=num_classes, ch=dfl_ch)

    def _yms_plan(self, b, inputs):
        (x,) = inputs
        H, W = x.shape[2], x.shape[3]
        if H % 32 or W % 32:
            raise RuntimeError(f"yms: input size must be a multiple of 32, got {H}x{W}")
        xin = b.new(H, W, x.shape[1], name="input")
        bb, nk = self.backbone, self.neck
        c3, c4, c5 = bb.out_channels()
        cats, slots = nk.alloc_cats(b, H // 8, W // 8, c3, H // 16, W // 16, c4, H // 32, W // 32, c5)
        p3, p4, p5 = bb.emit(b, xin, outs=slots)
        f = nk.emit(b, p3, p4, p5, cats=cats)
        outs = self.head.emit(b, *f)
        return [xin], outs, ("maps" if b.training else ("decode", self.head))

    def forward(self, x):
        _, outs = _runner.run(self, [x])
        if self.training:
            return list(outs)
        return outs[0]
