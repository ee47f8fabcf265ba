"""Backbone -- MI355X-native drop-in for yolov8/model/yolov8_backbone.py:30-73.

Stem of five stride-2 3x3 Conv blocks interleaved with four C2f stages, then SPPF;
emits P3 (stride 8), P4 (stride 16), P5 (stride 32).  Same attribute names as the
reference so checkpoints load unchanged.  When embedded in YOLOv8 the three
outputs are written straight into the neck's concatenation buffers.
"""
from yolov8.model.components import Conv, C2f, SPPF, yolo_params, _YmsModule


class Backbone(_YmsModule):
    def __init__(self, version, in_channels=3, shortcut=True) -> None:
        super().__init__()
        d, w, r = yolo_params(version)
        c1, c2, c3, c4, c5 = int(64 * w), int(128 * w), int(256 * w), int(512 * w), int(512 * w * r)
        self.conv0 = Conv(in_channels, c1, kernel_size=3, stride=2, padding=1)
        self.conv1 = Conv(c1, c2, kernel_size=3, stride=2, padding=1)
        self.conv3 = Conv(c2, c3, kernel_size=3, stride=2, padding=1)
        self.conv5 = Conv(c3, c4, kernel_size=3, stride=2, padding=1)
        self.conv7 = Conv(c4, c5, kernel_size=3, stride=2, padding=1)
        self.c2f_2 = C2f(c2, c2, num_bottlenecks=int(3 * d), shortcut=True)
        self.c2f_4 = C2f(c3, c3, num_bottlenecks=int(6 * d), shortcut=True)
        self.c2f_6 = C2f(c4, c4, num_bottlenecks=int(6 * d), shortcut=True)
        self.c2f_8 = C2f(c5, c5, num_bottlenecks=int(3 * d), shortcut=True)
        self.sppf = SPPF(c5, c5, kernel_size=5)

    def out_channels(self):
        """(P3, P4, P5) channels."""
        return (self.c2f_4.conv2.conv.out_channels, self.c2f_6.conv2.conv.out_channels,
                self.sppf.conv2.conv.out_channels)

    def emit(self, b, x, outs=(None, None, None)):
        x = self.conv0.emit(b, x)
        x = self.conv1.emit(b, x)
        x = self.c2f_2.emit(b, x)
        x = self.conv3.emit(b, x)
        p3 = self.c2f_4.emit(b, x, out=outs[0])
        x = self.conv5.emit(b, p3)
        p4 = self.c2f_6.emit(b, x, out=outs[1])
        x = self.conv7.emit(b, p4)
        x = self.c2f_8.emit(b, x)
        p5 = self.sppf.emit(b, x, out=outs[2])
        return p3, p4, p5

    def forward(self, x):
        return tuple(self._yms_run(x))
