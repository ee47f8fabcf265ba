"""Neck (FPN top-down + PAN bottom-up) -- MI355X-native drop-in for
yolov8/model/yolov8_neck.py:54-94.

Every torch.cat of the reference ([up(P5), P4], [up(res_2), P3], [conv1(out1), res_2],
[conv2(out2), P5]; yolov8_neck.py:79,83,88,91) is a pre-allocated NHWC buffer whose
channel slots are written directly by their producers (upsample kernel, strided conv
epilogues, and -- inside YOLOv8 -- the backbone's last layers).
"""
from yolov8.model.components import Conv, C2f, Upsample, yolo_params, _YmsModule


class Neck(_YmsModule):
    def __init__(self, version):
        super().__init__()
        d, w, r = yolo_params(version)
        n = int(3 * d)
        self.up = Upsample()
        self.c2f_1 = C2f(int(512 * w * (1 + r)), int(512 * w), num_bottlenecks=n, shortcut=False)
        self.c2f_2 = C2f(int(768 * w), int(256 * w), num_bottlenecks=n, shortcut=False)
        self.c2f_3 = C2f(int(768 * w), int(512 * w), num_bottlenecks=n, shortcut=False)
        self.c2f_4 = C2f(int(512 * w * (1 + r)), int(512 * w * r), num_bottlenecks=n, shortcut=False)
        self.conv1 = Conv(int(256 * w), int(256 * w), kernel_size=3, stride=2, padding=1)
        self.conv2 = Conv(int(512 * w), int(512 * w), kernel_size=3, stride=2, padding=1)

    def _stage(self, i):
        """Fusion block i (1..4): C2f here, MSBlock in the YOLO-MS neck (yolo_ms.MSNeck)."""
        return getattr(self, f"c2f_{i}")

    def _stage_out(self, i):
        m = self._stage(i)
        return m.conv2.conv.out_channels if hasattr(m, "conv2") else m.out_channels

    def alloc_cats(self, b, h3, w3, c3, h4, w4, c4, h5, w5, c5):
        """The four concat buffers; returns them and the slots P3/P4/P5 must occupy."""
        cr2 = self._stage_out(1)                           # res_2 channels
        cc1 = self.conv1.conv.out_channels
        cc2 = self.conv2.conv.out_channels
        cat1 = b.new(h4, w4, c5 + c4, name="neck_cat1")     # [up(P5), P4]
        cat2 = b.new(h3, w3, cr2 + c3, name="neck_cat2")    # [up(res_2), P3]
        cat3 = b.new(h4, w4, cc1 + cr2, name="neck_cat3")   # [conv1(out1), res_2]
        cat4 = b.new(h5, w5, cc2 + c5, name="neck_cat4")    # [conv2(out2), P5]
        cats = (cat1, cat2, cat3, cat4)
        return cats, (cat2.slot(cr2, c3), cat1.slot(c5, c4), cat4.slot(cc2, c5))

    def emit(self, b, p3, p4, p5, cats=None, outs=(None, None, None)):
        if cats is None:
            raise RuntimeError("yms: Neck.emit needs its concat buffers (use alloc_cats)")
        cat1, cat2, cat3, cat4 = cats
        c5, c4, c3 = p5.c, p4.c, p3.c
        cr2 = self._stage_out(1)
        cc1 = self.conv1.conv.out_channels
        cc2 = self.conv2.conv.out_channels
        self.up.emit(b, p5, out=cat1.slot(0, c5))
        res_2 = self._stage(1).emit(b, cat1, out=cat3.slot(cc1, cr2))
        self.up.emit(b, res_2, out=cat2.slot(0, cr2))
        out1 = self._stage(2).emit(b, cat2, out=outs[0])
        self.conv1.emit(b, out1, out=cat3.slot(0, cc1))
        out2 = self._stage(3).emit(b, cat3, out=outs[1])
        self.conv2.emit(b, out2, out=cat4.slot(0, cc2))
        out3 = self._stage(4).emit(b, cat4, out=outs[2])
        return out1, out2, out3

    def _yms_plan(self, b, inputs):
        x3, x4, x5 = inputs
        cats, slots = self.alloc_cats(b, x3.shape[2], x3.shape[3], x3.shape[1], x4.shape[2], x4.shape[3],
                                      x4.shape[1], x5.shape[2], x5.shape[3], x5.shape[1])
        outs = self.emit(b, *slots, cats=cats)
        return list(slots), list(outs), "maps"

    def forward(self, x_res_1, x_res_2, x):
        return tuple(self._yms_run(x_res_1, x_res_2, x))
