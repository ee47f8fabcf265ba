"""Bit-exact parity of the HIP class-wise NMS against the C oracle (oracle/nms_ref.c),
on identical decoded inputs.  NMS parity is UNPINNED by the reference itself (torchvision
is a dependency absent from the reference tree and this image); the oracle restates
torchvision's CPU algorithm and is pinned by known-answer tests (test_nms_oracle.py)."""
import numpy as np
import pytest
import torch

from oracle import nms as onms
from yms import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["default", "graph", "nograph", "legacy"], autouse=True)
def nms_route(request, monkeypatch):
    """Every case runs four ways: the default routing (graph kernels for segments of >= 2048 finite
    boxes with few expected overlaps, the rest of the big segments sorted and resolved by the
    window-grid greedy when finite and <= 7168 boxes, else by the kept-list greedy); the graph
    kernels on every segment of >= 128 finite boxes (YMS_NMS_GRAPH_MIN=128, YMS_NMS_GRAPH_MAXC=0);
    no graph kernels (YMS_NMS_GRAPH_MIN=0: every big segment to the window-grid / kept-list
    greedy); and the round-3 kernels only (also YMS_NMS_WGRID=0, YMS_NMS_CAP=1024: segments of up
    to 1024 boxes in the class kernel, not the default 256)."""
    for k in ("YMS_NMS_GRAPH_MIN", "YMS_NMS_GRAPH_MAXC", "YMS_NMS_WGRID", "YMS_NMS_CAP"):
        monkeypatch.delenv(k, raising=False)
    if request.param == "graph":
        monkeypatch.setenv("YMS_NMS_GRAPH_MIN", "128")
        monkeypatch.setenv("YMS_NMS_GRAPH_MAXC", "0")
    elif request.param in ("nograph", "legacy"):
        monkeypatch.setenv("YMS_NMS_GRAPH_MIN", "0")
        if request.param == "legacy":
            monkeypatch.setenv("YMS_NMS_WGRID", "0")
            monkeypatch.setenv("YMS_NMS_CAP", "1024")
    return request.param


def clustered(B, nc, K=20, J=30, A=8400, seed=0):
    """SURVEY 8d input set 2: K objects x J jittered boxes, Beta(2,5) scores, uniform labels."""
    rng = np.random.default_rng(seed)
    pred = np.zeros((B, A, 4 + nc), np.float32)
    pred[..., 4:] = rng.uniform(0, 0.2, (B, A, nc)).astype(np.float32)
    for b in range(B):
        for k in range(K):
            cx, cy = rng.uniform(40, 600, 2)
            w, h = rng.uniform(20, 200, 2)
            lab = rng.integers(0, nc)
            for j in range(J):
                a = rng.integers(0, A)
                pred[b, a, :4] = [cx + rng.normal(0, 4), cy + rng.normal(0, 4), w * rng.uniform(0.8, 1.2),
                                  h * rng.uniform(0.8, 1.2)]
                pred[b, a, 4 + lab] = rng.beta(2, 5) + 0.25
        # background anchors: random boxes
        bg = pred[b, :, 2] == 0
        pred[b, bg, :2] = rng.uniform(0, 640, (bg.sum(), 2))
        pred[b, bg, 2:4] = rng.uniform(4, 100, (bg.sum(), 2))
    return pred


def _check(pred, conf, iou):
    d = torch.from_numpy(pred).cuda()
    bxy, score, keep, klbl, cnt = ops.batched_nms_indices(d, conf, iou)
    cnt = cnt.cpu().numpy()
    keep = keep.cpu().numpy()
    klbl = klbl.cpu().numpy()
    total = 0
    for b in range(pred.shape[0]):
        ki, kl, _ = onms.postprocess(pred[b], conf, iou)
        assert cnt[b] == len(ki), (b, cnt[b], len(ki))
        assert np.array_equal(keep[b, :cnt[b]], ki)
        assert np.array_equal(klbl[b, :cnt[b]], kl)
        total += len(ki)
    return total


@pytest.mark.parametrize("iou", [0.45, 0.5, 0.6])
def test_clustered_detections(iou):
    assert _check(clustered(4, 80), 0.25, iou) > 0


def test_dense_random_init_like():
    """~all anchors above conf, ~105 per class (random-init model regime)."""
    rng = np.random.default_rng(1)
    A, nc = 8400, 80
    pred = np.zeros((2, A, 4 + nc), np.float32)
    pred[..., :2] = rng.uniform(0, 640, (2, A, 2))
    pred[..., 2:4] = rng.uniform(10, 120, (2, A, 2))
    pred[..., 4:] = rng.uniform(0.2, 0.6, (2, A, nc))
    _check(pred, 0.25, 0.45)


def test_single_class_large_segment():
    """nc=1: one class holds all 8400 candidates (global-memory sort path)."""
    rng = np.random.default_rng(2)
    A = 8400
    pred = np.zeros((1, A, 5), np.float32)
    pred[..., :2] = rng.uniform(0, 640, (1, A, 2))
    pred[..., 2:4] = rng.uniform(10, 80, (1, A, 2))
    pred[..., 4] = rng.uniform(0.0, 1.0, (1, A))
    _check(pred, 0.25, 0.5)


def test_min_workspace_same_keep_lists():
    """A caller holding only yms_nms_ws_bytes_min bytes on segments of >= YMS_NMS_GRAPH_MIN boxes
    (sparse overlaps: the graph route's regime) gets the other exact routes: the keep lists and
    counts equal those of a call with the full yms_nms_ws_bytes workspace, and the oracle's."""
    import ctypes
    from yms import _lib as L
    rng = np.random.default_rng(21)
    B, A, nc = 2, 8400, 1
    pred = np.zeros((B, A, 4 + nc), np.float32)
    pred[..., :2] = rng.uniform(0, 640, (B, A, 2))
    pred[..., 2:4] = rng.uniform(4, 24, (B, A, 2))
    pred[..., 4] = rng.uniform(0.3, 1.0, (B, A))
    d = torch.from_numpy(pred).cuda()
    st = L.stream_ptr(d.device)
    bxy = torch.empty((B, A, 4), dtype=torch.float32, device="cuda")
    score = torch.empty((B, A), dtype=torch.float32, device="cuda")
    label = torch.empty((B, A), dtype=torch.int32, device="cuda")
    L.call("yms_nms_prep", B, A, nc, d.data_ptr(), ctypes.c_float(0.25), bxy.data_ptr(), score.data_ptr(),
           label.data_ptr(), st)
    outs = []
    for fn in (L.lib().yms_nms_ws_bytes, L.lib().yms_nms_ws_bytes_min):
        nb = fn(B, A, nc)
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        keep = torch.full((B, A), -7, dtype=torch.int64, device="cuda")
        klbl = torch.empty((B, A), dtype=torch.int32, device="cuda")
        cnt = torch.empty(B, dtype=torch.int32, device="cuda")
        L.call("yms_nms_classwise", B, A, nc, bxy.data_ptr(), score.data_ptr(), label.data_ptr(),
               ctypes.c_double(0.5), keep.data_ptr(), klbl.data_ptr(), cnt.data_ptr(), ws.data_ptr(), nb, st)
        c = cnt.cpu().numpy()
        outs.append((c, [keep[b, :c[b]].cpu().numpy() for b in range(B)]))
    assert L.lib().yms_nms_ws_bytes_min(B, A, nc) < L.lib().yms_nms_ws_bytes(B, A, nc)
    (c_full, k_full), (c_min, k_min) = outs
    assert np.array_equal(c_full, c_min)
    for b in range(B):
        assert np.array_equal(k_full[b], k_min[b])
        ki = onms.postprocess(pred[b], 0.25, 0.5)[0]
        assert np.array_equal(k_min[b], ki)


def test_ties_and_duplicates():
    """Exact score ties keep anchor order; identical boxes suppress; empty classes skipped."""
    A, nc = 64, 3
    pred = np.zeros((1, A, 4 + nc), np.float32)
    pred[0, :, :4] = [100, 100, 20, 20]
    pred[0, :, 4] = 0.5          # all tie on class 0
    pred[0, ::2, 5] = 0.7        # even anchors -> class 1, tied
    _check(pred, 0.25, 0.45)
    pred[0, :, 4:] = 0.1         # nothing above conf
    _check(pred, 0.25, 0.45)


def test_iou_exactly_at_threshold():
    # two boxes with IoU exactly 0.5: area 100 each, inter 100/3? use inter = 2/3 * area -> IoU 0.5
    b = np.array([[0, 0, 10, 10], [0, 0, 10, 5], [0, 0, 10, 7.5]], np.float32)   # IoU(0,1)=0.5
    s = np.array([0.9, 0.8, 0.7], np.float32)
    for thr in (0.45, 0.5, 0.6, 0.75):
        ref = onms.nms(b, s, thr)
        got = ops.nms(torch.from_numpy(b).cuda(), torch.from_numpy(s).cuda(), thr).cpu().numpy()
        assert np.array_equal(got, ref), (thr, got, ref)


def test_nms_single_matches_oracle_random():
    rng = np.random.default_rng(5)
    for n in (1, 7, 64, 65, 300, 1500):
        xy = rng.uniform(0, 100, (n, 2)).astype(np.float32)
        wh = rng.uniform(1, 40, (n, 2)).astype(np.float32)
        b = np.concatenate([xy, xy + wh], 1)
        s = rng.uniform(0, 1, n).astype(np.float32)
        s[::5] = 0.5   # ties
        ref = onms.nms(b, s, 0.5)
        got = ops.nms(torch.from_numpy(b).cuda(), torch.from_numpy(s).cuda(), 0.5).cpu().numpy()
        assert np.array_equal(got, ref), n


def test_postprocess_dicts():
    pred = clustered(2, 80, seed=3)
    res = ops.postprocess(torch.from_numpy(pred).cuda(), 0.25, 0.45)
    for b, r in enumerate(res):
        ki, kl, bx = onms.postprocess(pred[b], 0.25, 0.45)
        assert np.array_equal(r["labels"].cpu().numpy(), kl)
        assert np.array_equal(r["boxes"].cpu().numpy(), bx[ki])
        assert np.array_equal(r["scores"].cpu().numpy(), pred[b, ki, 4:].max(1))


# ---- configs[4]: 1280x1280 inputs, A = 33600 anchors ---------------------------------------

def test_1280_single_class_beyond_lds_sort():
    """nc=1 at A=33600: ~25k candidates in one segment, past the 16384-key LDS sort (global
    bitonic path) and the kept-list greedy over a long list."""
    rng = np.random.default_rng(7)
    A = 33600
    pred = np.zeros((1, A, 5), np.float32)
    pred[..., :2] = rng.uniform(0, 1280, (1, A, 2))
    pred[..., 2:4] = rng.uniform(10, 160, (1, A, 2))
    pred[..., 4] = rng.uniform(0.0, 1.0, (1, A))
    pred[0, ::97, 4] = 0.625     # exact score ties across far-apart anchors
    assert _check(pred, 0.25, 0.5) > 0


def test_1280_dense_multiclass():
    """80 classes, ~all 33600 anchors above conf (~420 per class), two images."""
    rng = np.random.default_rng(8)
    A, nc = 33600, 80
    pred = np.zeros((2, A, 4 + nc), np.float32)
    pred[..., :2] = rng.uniform(0, 1280, (2, A, 2))
    pred[..., 2:4] = rng.uniform(10, 240, (2, A, 2))
    pred[..., 4:] = rng.uniform(0.2, 0.6, (2, A, nc))
    _check(pred, 0.25, 0.45)


def test_s1280_fp16_model_decode_nms_end_to_end():
    """configs[4] path end to end: random-init YOLO-MS-S, 1280x1280 fp16 forward + decode on the
    GPU, then class-wise NMS on the GPU vs the C oracle on the same decoded tensor (bit-exact)."""
    from yolov8.yolov8 import YOLOv8
    torch.manual_seed(0)
    m = YOLOv8("s", 80).cuda().eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    x = torch.randn(2, 3, 1280, 1280, generator=torch.Generator().manual_seed(9))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        det = m(x.cuda())
    assert det.shape == (2, 33600, 84) and det.dtype == torch.float32
    assert _check(np.ascontiguousarray(det.cpu().numpy()), 0.25, 0.45) > 0


def test_big_segment_grid_edge_cases():
    """Big-segment greedy paths: wide boxes (> 64 grid cells, the wide-box list), zero-area and
    inverted boxes, kept lists beyond the LDS mirror / link pool (fallback to the full kept
    list), a non-finite coordinate (whole-list path) and a negative threshold."""
    rng = np.random.default_rng(11)
    A = 8400
    def seg(wlo, whi):
        p = np.zeros((1, A, 5), np.float32)
        p[..., :2] = rng.uniform(0, 640, (1, A, 2))
        p[..., 2:4] = rng.uniform(wlo, whi, (1, A, 2))
        p[..., 4] = rng.uniform(0.3, 1.0, (1, A))
        return p
    p = seg(8, 40)
    p[0, ::50, 2:4] = rng.uniform(300, 900, (len(p[0, ::50]), 2))    # wide boxes
    p[0, 1::97, 2] = 0.0                                               # zero width
    p[0, 2::89, 3] = -5.0                                              # inverted (negative h)
    assert _check(p, 0.25, 0.5) > 0
    p = seg(0.5, 3.0)                     # tiny, nearly disjoint: ~all kept (> 4096)
    assert _check(p, 0.25, 0.5) > 4096
    p = seg(8, 40)
    p[0, 123, 0] = np.nan
    _check(p, 0.25, 0.5)
    # NaN coordinates on the top-scoring box (the kept box i of the std::max/min restatement)
    # and scattered NaN widths / heights: the oracle uses std::max/min, the GPU IEEE max/min
    p = seg(8, 40)
    p[0, int(np.argmax(p[0, :, 4])), 2] = np.nan
    p[0, 5::61, 3] = np.nan
    p[0, 9::83, 1] = np.nan
    _check(p, 0.25, 0.5)
    p = seg(8, 40)
    p[0, 77, 1] = np.inf
    _check(p, 0.25, 0.5)
    _check(seg(8, 40), 0.25, -0.5)


def test_nms_on_side_stream_overlapping_next_forward():
    """The serving pipeline of bench.py (--nms-overlap): batch k's NMS on a second stream while
    batch k+1's forward runs on the main stream gives the same keep lists as one stream."""
    from yms import set_compute_dtype
    from yolov8.yolov8 import YOLOv8

    torch.manual_seed(0)
    m = YOLOv8("n", 80).cuda().eval()
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    set_compute_dtype(m, torch.bfloat16)
    xs = [torch.randn(2, 3, 128, 128, device="cuda", generator=torch.Generator(device="cuda").manual_seed(s))
          for s in range(3)]
    ref = []
    for x in xs:
        _, _, keep, klbl, cnt = ops.batched_nms_indices(m(x), 0.25, 0.45)
        ref.append((keep.clone(), klbl.clone(), cnt.clone()))
    side = torch.cuda.Stream()
    got = []
    for x in xs:
        y = m(x)
        side.wait_stream(torch.cuda.current_stream())
        y.record_stream(side)
        with torch.cuda.stream(side):
            got.append(ops.batched_nms_indices(y, 0.25, 0.45)[2:])
    torch.cuda.synchronize()
    for (k0, l0, c0), (k1, l1, c1) in zip(ref, got):
        assert torch.equal(c0, c1)
        for b in range(c0.numel()):
            n = int(c0[b])
            assert torch.equal(k0[b, :n], k1[b, :n]) and torch.equal(l0[b, :n], l1[b, :n])


def _level_segments(B, seed, jitter=20.0, size=160.0):
    """The bench's regime (random-init YOLOv8-s / YOLO-MS at 640): every anchor of a pyramid level
    carries the same arg-max class, so each image has three segments of 6400 / 1600 / 400
    candidates, with ~160-px boxes centred on the anchor grid."""
    rng = np.random.default_rng(seed)
    A, nc = 8400, 80
    pred = np.zeros((B, A, 4 + nc), np.float32)
    a0 = 0
    for s, cls in ((8, 3), (16, 7), (32, 11)):
        g = 640 // s
        ys, xs = np.meshgrid(np.arange(g), np.arange(g), indexing="ij")
        cx, cy = (xs.ravel() + 0.5) * s, (ys.ravel() + 0.5) * s
        sl = slice(a0, a0 + g * g)
        for b in range(B):
            pred[b, sl, 0] = cx + rng.normal(0, 2, g * g)
            pred[b, sl, 1] = cy + rng.normal(0, 2, g * g)
            pred[b, sl, 2:4] = size + rng.uniform(-jitter, jitter, (g * g, 2))
            pred[b, sl, 4:] = rng.uniform(0.0, 0.2, (g * g, nc))
            pred[b, sl, 4 + cls] = rng.uniform(0.3, 0.7, g * g)
        a0 += g * g
    return pred


def test_big_segment_greedy_bit_exact():
    """Big segments <= 8192 boxes on the big-segment kernels (window-grid / kept-list grid greedy,
    per the routing fixture): bit-exact against the oracle on the bench's level segments, on dense
    single-class segments, at thresholds 0.45 / 0.5 / 0.6 / 0 / negative, and with NaN / inf /
    zero-area boxes."""
    for thr in (0.45, 0.5, 0.6):
        assert _check(_level_segments(3, 21), 0.25, thr) > 0
    rng = np.random.default_rng(23)
    A = 8400
    p = np.zeros((1, A, 5), np.float32)
    p[..., :2] = rng.uniform(0, 640, (1, A, 2))
    p[..., 2:4] = rng.uniform(5, 60, (1, A, 2))
    p[..., 4] = rng.uniform(0.3, 1.0, (1, A))
    assert _check(p, 0.25, 0.5) > 64
    _check(p, 0.25, 0.0)
    _check(p, 0.25, -0.25)
    p[0, 1::97, 2] = 0.0
    p[0, 5::61, 3] = np.nan
    p[0, int(np.argmax(p[0, :, 4])), 2] = np.nan
    p[0, 77, 1] = np.inf
    _check(p, 0.25, 0.5)


def _single(b, s, thr):
    ref = onms.nms(b, s, thr)
    got = ops.nms(torch.from_numpy(b).cuda(), torch.from_numpy(s).cuda(), thr).cpu().numpy()
    assert np.array_equal(got, ref), (thr, len(got), len(ref))
    return len(ref)


def test_graph_nms_edge_cases(monkeypatch, nms_route):
    """The graph kernels on every segment of >= 32 boxes (YMS_NMS_GRAPH_MIN=32): suppressee lists
    beyond their 254-entry capacity (identical boxes: the full-rectangle rescan), long suppression
    chains (one decision round per link), mixed tiny / huge boxes (search rectangles spanning the
    grid), degenerate boxes mixed in, all centres equal, thresholds 0 / 0.999 / 1, exact ties."""
    if nms_route in ("nograph", "legacy"):
        pytest.skip("graph kernels forced on below")
    monkeypatch.setenv("YMS_NMS_GRAPH_MIN", "32")
    # "graph": every segment on the graph kernels; "default": dense ones (the identical boxes, the
    # clusters) routed by the build kernel to the big-segment kernels, down to 32 boxes
    monkeypatch.setenv("YMS_NMS_GRAPH_MAXC", "0" if nms_route == "graph" else "256")
    rng = np.random.default_rng(31)
    # identical boxes, distinct and tied scores
    b = np.tile(np.array([[10, 20, 50, 70]], np.float32), (2000, 1))
    s = rng.uniform(0, 1, 2000).astype(np.float32)
    s[::7] = 0.5
    assert _single(b, s, 0.5) == 1
    # a chain: box k overlaps k-1 and k+1 only (IoU 0.54; k+-2: 0.25), scores decreasing along the chain
    n = 700
    x = np.arange(n, dtype=np.float32) * 3.0
    b = np.stack([x, np.zeros(n, np.float32), x + 10.0, np.full(n, 10.0, np.float32)], 1)
    s = np.linspace(1.0, 0.1, n).astype(np.float32)
    assert _single(b, s, 0.5) == n // 2
    _single(b, s[::-1].copy(), 0.5)
    # mixed scales, degenerate boxes, equal centres
    for trial in range(6):
        n = int(rng.integers(40, 3000))
        c = rng.uniform(0, 640, (n, 2))
        wh = np.exp(rng.uniform(-3, 6, (n, 2)))
        if trial == 1:
            c[:] = c[0]
        b = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
        if trial == 2:
            b[::13, 2] = b[::13, 0]                 # zero width
            b[1::17, 3] = b[1::17, 1] - 1.0         # inverted
        s = rng.uniform(0, 1, n).astype(np.float32)
        s[::11] = 0.25
        for thr in (0.0, 0.3, 0.45, 0.5, 0.7, 0.999, 1.0):
            _single(b, s, thr)
    # class-wise: clustered detections with every class segment >= 32 on the graph kernels
    for iou in (0.45, 0.6):
        assert _check(clustered(3, 4, K=30, J=40, seed=4), 0.25, iou) > 0
    # exact-threshold pairs inside a larger segment
    base = np.array([[0, 0, 10, 10], [0, 0, 10, 5], [0, 0, 10, 7.5]], np.float32)
    b = np.concatenate([base + 20 * k for k in range(100)], 0)
    s = np.tile(np.array([0.9, 0.8, 0.7], np.float32), 100)
    for thr in (0.45, 0.5, 0.6, 0.75):
        _single(b, s, thr)
