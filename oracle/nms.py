"""ctypes wrapper of the C restatement of post-process + class-wise NMS (oracle/nms_ref.c).

TEST INFRASTRUCTURE ONLY -- see nms_ref.c for the reference citations
(train.py:63-113, tools/test.py:166-218; torchvision nms semantics, parity unpinned)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "lib", "libyms_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(_HERE, "nms_ref.c")):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.yms_ref_nms.restype = ctypes.c_int64
        L.yms_ref_nms.argtypes = [P, P, ctypes.c_int64, ctypes.c_double, P]
        L.yms_ref_postprocess.restype = ctypes.c_int64
        L.yms_ref_postprocess.argtypes = [P, ctypes.c_int64, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_double, P, P, P]
        _lib = L
    return _lib


def nms(boxes, scores, iou):
    """torchvision.ops.nms semantics on numpy float32 arrays -> int64 keep."""
    b = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 4)
    s = np.ascontiguousarray(scores, dtype=np.float32).reshape(-1)
    keep = np.empty(max(len(s), 1), dtype=np.int64)
    n = lib().yms_ref_nms(b.ctypes.data, s.ctypes.data, len(s), float(iou), keep.ctypes.data)
    return keep[:n].copy()


def postprocess(pred, conf, iou):
    """One image: pred [A, 4+nc] -> (anchor_idx int64[K], label int32[K], boxes_xyxy[A,4])."""
    p = np.ascontiguousarray(pred, dtype=np.float32)
    A, no = p.shape
    ki = np.empty(max(A, 1), dtype=np.int64)
    kl = np.empty(max(A, 1), dtype=np.int32)
    bx = np.empty((max(A, 1), 4), dtype=np.float32)
    n = lib().yms_ref_postprocess(p.ctypes.data, A, no - 4, float(conf), float(iou),
                                  ki.ctypes.data, kl.ctypes.data, bx.ctypes.data)
    return ki[:n].copy(), kl[:n].copy(), bx[:A]


def postprocess_batch(pred, conf, iou):
    return [postprocess(pred[b], conf, iou)[:2] for b in range(pred.shape[0])]
