"""yms -- MI355X-native (gfx950) runtime for the YOLO-MS / YOLOv8 detector hot path.

Layers:  libyms.so (hand-written HIP kernels behind the C-ABI of include/yms.h)
      -> yms._lib (ctypes binding) -> yms.plan (static NHWC execution plans)
      -> yms.runner (autograd bridge) -> yolov8.* (the reference's module API)
      -> yms.dist (data-parallel training over RCCL/xGMI)."""
from . import _lib
from .runner import compute_dtype, set_compute_dtype

__all__ = ["compute_dtype", "set_compute_dtype", "_lib"]
