"""configs[1] end to end, exactly as bench.py times it: the random-init YOLOv8-s (and the YOLO-MS-S
graph of the `ms_family` line) at 640x640 bf16, B=32, forward + decode on the GPU, then class-wise
NMS (train.py:63-113) -- once on the compute stream and once as the serving pipeline (batch k's NMS
on a second stream while batch k+1's forward runs, bench.py `infer_step`).  Every image's keep
indices and labels are compared bit-exact with the C oracle (oracle/nms_ref.c, torchvision's CPU
algorithm restated; parity with torchvision itself is unpinned) on the same decoded tensor.

Reference: yolov8/tools/train.py:57-113 (validate_epoch: model(x) -> post-process + per-class
torchvision nms), yolov8/model/yolov8_head.py:127-144 (eval decode)."""
import numpy as np
import pytest
import torch

from oracle import nms as onms
from yms import ops, set_compute_dtype
from yolov8.yolov8 import YOLOv8

pytestmark = pytest.mark.gpu

CONF, IOU, B, SIZE = 0.25, 0.45, 32, 640


def _bench_model(version):
    # bench.py main(): torch.manual_seed(0) before the inference model is built
    torch.manual_seed(0)
    m = YOLOv8(version, 80).cuda().eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    set_compute_dtype(m, torch.bfloat16)
    return m


def _check_batch(det, keep, klbl, cnt):
    pred = np.ascontiguousarray(det.cpu().numpy())
    keep, klbl, cnt = keep.cpu().numpy(), klbl.cpu().numpy(), cnt.cpu().numpy()
    total = 0
    for b in range(pred.shape[0]):
        ki, kl, _ = onms.postprocess(pred[b], CONF, IOU)
        assert cnt[b] == len(ki), (b, int(cnt[b]), len(ki))
        assert np.array_equal(keep[b, :cnt[b]], ki), b
        assert np.array_equal(klbl[b, :cnt[b]], kl), b
        total += len(ki)
    return total


@pytest.mark.parametrize("version", ["s", "ms-s"])
def test_configs1_bench_path_single_and_overlapped(version):
    dev = torch.device("cuda", 0)
    main = torch.cuda.Stream(device=dev, priority=-1)      # bench.py --priority 1 (default)
    side = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(main):
        m = _bench_model(version)
        xs = [torch.randn(B, 3, SIZE, SIZE, device=dev, generator=torch.Generator(device=dev).manual_seed(99 + k))
              for k in range(3)]
        # single stream: decode output and NMS on the compute stream
        dets, single = [], []
        for x in xs:
            y = m(x)
            assert y.shape == (B, 8400, 84) and y.dtype == torch.float32
            dets.append(y.clone())
            single.append([t.clone() for t in ops.batched_nms_indices(y, CONF, IOU)[2:]])
        # serving pipeline: each batch's NMS on the side stream overlapping the next forward
        piped = []
        for k, x in enumerate(xs):
            y = m(x)
            side.wait_stream(main)
            y.record_stream(side)
            with torch.cuda.stream(side):
                piped.append(ops.batched_nms_indices(y, CONF, IOU)[2:])
        main.wait_stream(side)
    torch.cuda.synchronize()
    for k in range(len(xs)):
        kept = _check_batch(dets[k], *single[k])
        assert kept > B, (k, kept)                          # random-init regime: hundreds kept per image
        _check_batch(dets[k], *piped[k])
