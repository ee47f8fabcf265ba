"""NMS greedy phase profile (dev tool): needs `make -C yolo-ms_amd/csrc nmsprof`.
Usage: nms_prof_run.py SIZE BATCH  (random-init YOLOv8-s, fp16 at 1280 else bf16)"""
import os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
from yms import _lib
_lib.LIB_PATH = os.path.join(ROOT, "yolo-ms_amd", "yms", "libyms_nmsprof.so")
import torch
from yms import set_compute_dtype
from yms import ops as yops
from yolov8.yolov8 import YOLOv8
S = int(sys.argv[1]); B = int(sys.argv[2])
torch.manual_seed(0)
m = YOLOv8("s", 80).cuda().eval()
m.head.stride = torch.tensor([8.0, 16.0, 32.0])
set_compute_dtype(m, torch.float16 if S == 1280 else torch.bfloat16)
x = torch.randn(B, 3, S, S, device="cuda", generator=torch.Generator(device="cuda").manual_seed(99))
with torch.no_grad():
    y = m(x)
    torch.cuda.synchronize()
    print("---", S, flush=True)
    yops.batched_nms_indices(y, 0.25, 0.45)
    torch.cuda.synchronize()
