"""Functional HIP ops outside the module graph: torchvision-compatible NMS, the
reference's batched post-process (train.py:63-113 / tools/test.py:166-218) and the
standalone DFL integral.  GPU tensors only; every call goes through libyms.so."""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import _lib as L


def _cuda(*ts):
    for t in ts:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError("yms: ops run on ROCm GPU tensors only (no CPU fallback)")


def dfl(x, ch=16):
    """DFL (components.py:186-191): x [B, 4*ch, A] -> [B, 4, A]."""
    _cuda(x)
    b, c, a = x.shape
    if c != 4 * ch:
        raise RuntimeError(f"yms: DFL expects {4 * ch} channels, got {c}")
    xc = x.contiguous()
    out = torch.empty((b, 4, a), dtype=x.dtype, device=x.device)
    L.call("yms_dfl", L.dtype_code(x.dtype), b, a, ch, xc.data_ptr(), out.data_ptr(), L.stream_ptr(x.device))
    return out


_TLS = threading.local()


def _nms_ws(dev, B, A, nc, iou):
    """NMS scratch reused across calls, one buffer per (host thread, device, stream): one
    yms_nms_classwise call is a chain of launches on its stream (memset, route / sort, greedy,
    compact), so two threads sharing a stream would interleave their chains over one buffer
     -- a thread's own calls on a stream are ordered, so its buffer is safe to reuse.
    The cache lives in thread-local storage and goes with the thread."""
    # graph NMS (csrc/head_nms.hip) runs on segments of at least YMS_NMS_GRAPH_MIN boxes (default
    # 2048, 0 = off, at least 32, the C side's rule); without it the workspace leaves out the graph
    # kernels' suppressee lists (~530 B per anchor) and every segment takes the other exact routes
    gmin = int(os.environ.get("YMS_NMS_GRAPH_MIN", "2048"))
    full = iou >= 0.0 and gmin > 0 and A >= max(gmin, 32)
    nbytes = (L.lib().yms_nms_ws_bytes if full else L.lib().yms_nms_ws_bytes_min)(B, A, nc)
    cache = getattr(_TLS, "nms_ws", None)
    if cache is None:
        cache = _TLS.nms_ws = {}
    key = (dev.index, L.stream_ptr(dev))
    ws = cache.get(key)
    if ws is None or ws.numel() < nbytes:
        if len(cache) >= 8:            # a thread cycling through many streams: keep a few
            cache.pop(next(iter(cache)))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        cache[key] = ws
    return ws, nbytes


def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms(boxes [N,4] xyxy, scores [N], iou) -> int64 keep (score-descending)."""
    _cuda(boxes, scores)
    n = boxes.shape[0]
    dev = boxes.device
    if n == 0:
        return torch.empty(0, dtype=torch.int64, device=dev)
    b = boxes.detach().float().contiguous()
    s = scores.detach().float().contiguous()
    keep = torch.empty(n, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    ws, wsb = _nms_ws(dev, 1, n, 1, float(iou_threshold))
    L.call("yms_nms_single", n, b.data_ptr(), s.data_ptr(), ctypes.c_double(float(iou_threshold)),
           keep.data_ptr(), cnt.data_ptr(), ws.data_ptr(), wsb, L.stream_ptr(dev))
    return keep[:int(cnt.item())]


def batched_nms_indices(pred, conf_thresh=0.25, iou_thresh=0.45):
    """Class-wise NMS for a batch of decoded predictions [B, A, 4+nc] (fp32).

    Returns (boxes_xyxy [B,A,4], scores [B,A], keep_idx [B,A] int64, keep_lbl [B,A] int32,
    counts [B] int32): for image b the first counts[b] entries of keep_idx/keep_lbl are
    the kept anchors, ordered by class ascending then score descending -- the order the
    reference's per-class loop concatenates them in (train.py:85-101)."""
    _cuda(pred)
    B, A, no = pred.shape
    nc = no - 4
    dev = pred.device
    p = pred.detach().float().contiguous()
    st = L.stream_ptr(dev)
    bxy = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    score = torch.empty((B, A), dtype=torch.float32, device=dev)
    label = torch.empty((B, A), dtype=torch.int32, device=dev)
    L.call("yms_nms_prep", B, A, nc, p.data_ptr(), ctypes.c_float(float(conf_thresh)), bxy.data_ptr(),
           score.data_ptr(), label.data_ptr(), st)
    keep = torch.empty((B, A), dtype=torch.int64, device=dev)
    klbl = torch.empty((B, A), dtype=torch.int32, device=dev)
    counts = torch.empty(B, dtype=torch.int32, device=dev)
    ws, wsb = _nms_ws(dev, B, A, nc, float(iou_thresh))
    L.call("yms_nms_classwise", B, A, nc, bxy.data_ptr(), score.data_ptr(), label.data_ptr(),
           ctypes.c_double(float(iou_thresh)), keep.data_ptr(), klbl.data_ptr(), counts.data_ptr(),
           ws.data_ptr(), wsb, st)
    return bxy, score, keep, klbl, counts


def postprocess(pred, conf_thresh=0.25, iou_thresh=0.45):
    """Per image {'boxes' [K,4] xyxy, 'scores' [K], 'labels' [K] int64} -- the dicts the
    reference builds for torchmetrics (train.py:103-113)."""
    bxy, score, keep, klbl, counts = batched_nms_indices(pred, conf_thresh, iou_thresh)
    cnt = counts.cpu().tolist()
    out = []
    for b, k in enumerate(cnt):
        idx = keep[b, :k]
        out.append({"boxes": bxy[b].index_select(0, idx), "scores": score[b].index_select(0, idx),
                    "labels": klbl[b, :k].long()})
    return out
