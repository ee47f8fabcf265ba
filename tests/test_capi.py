"""CPU tier: the C-ABI library builds/loads and exports every function include/yms.h declares;
host-side helpers (shape checks, workspace sizing, plan construction) work without a GPU."""
import ctypes
import os
import re

import pytest
import torch

from yms import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "yms.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(yms_[a-z_0-9]+)\s*\(", txt, flags=re.M)))


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) >= 30
    lib = ctypes.CDLL(L.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    # every declared function is also bound (with argtypes) by the Python layer
    assert set(names) <= set(L.EXPORTED), set(names) - set(L.EXPORTED)


def test_version_and_status():
    assert b"gfx950" in L.lib().yms_version()
    assert L.lib().yms_status_string(1) == b"invalid argument"


def test_host_shape_validation_and_sizes():
    sh = L.ConvShape(2, 64, 64, 32, 64, 3, 2, 1, 32, 32, L.BF16)
    sp = ctypes.pointer(sh)
    # packed weights: cout padded to 128 rows, K = 9 taps x 32 ch = 288 padded to the
    # 128-byte (64 bf16) K tile of the NT kernel -> 320
    assert L.lib().yms_conv_packed_elems(sp, 0) == 128 * 320
    assert L.lib().yms_conv_stats_ld(sp) == 128
    assert L.lib().yms_conv_stats_rows(sp) > 0
    assert L.lib().yms_conv_wgrad_ws_bytes(sp) > 0
    bad = L.ConvShape(2, 64, 64, 32, 64, 3, 2, 1, 31, 32, L.BF16)
    assert L.lib().yms_conv_packed_elems(ctypes.pointer(bad), 0) == 0
    assert L.lib().yms_conv_fwd(ctypes.pointer(bad), None, 8, 0, None, None, 8, 0, None, None, 0, None, 0, 0,
                                None, None) == 1
    assert L.lib().yms_nms_ws_bytes(32, 8400, 80) > 32 * 8400 * 28
    # without the graph kernels' suppressee lists: ~56 B per anchor instead of ~590
    full, base = L.lib().yms_nms_ws_bytes(32, 8400, 80), L.lib().yms_nms_ws_bytes_min(32, 8400, 80)
    assert 32 * 8400 * 40 < base < 32 * 8400 * 80 and full - base > 32 * 8400 * 512


def test_bn_bwd_rows_is_the_launched_block_count():
    """yms_bn_bwd_rows = the number of partial rows the (two-kernel) reduce writes: with
    ppb = ceil(npix / min(256, ceil(npix/64))) the launch covers ceil(npix / ppb) blocks (the fused
    reduce + finalize additionally caps rows at 32768 // c, never above this)."""
    for c in (8, 64, 80, 256, 512, 2048):
        for npix in (1, 63, 64, 65, 100, 32768, 32769, 40001, 44800, 57600, 63 * 640, 7 * 80 * 80, 64 * 160 * 160):
            rows = L.lib().yms_bn_bwd_rows(npix, c)
            cap = max(1, min(256, (npix + 63) // 64))
            ppb = -(-npix // cap)
            assert rows == -(-npix // ppb), (npix, c)
            assert 1 <= rows <= 256 and (rows - 1) * ppb < npix <= rows * ppb, (npix, c)
    assert L.lib().yms_bn_bwd_rows(44801, 64) == 255      # below the cap: ppb 176


def test_null_pointers_rejected_without_gpu():
    sh = L.ConvShape(1, 8, 8, 8, 8, 3, 1, 1, 8, 8, L.F32)
    assert L.lib().yms_conv_fwd(ctypes.pointer(sh), None, 8, 0, None, None, 8, 0, None, None, 0, None, 0, 0,
                                None, None) == 1
    assert L.lib().yms_affine_act(L.BF16, 10, 8, None, 8, 0, None, None, 0, None, 0, 0, None, 8, 0, None) == 1
    assert L.lib().yms_nms_classwise(1, 10, 1, None, None, None, 0.5, None, None, None, None, 0, None) == 1


def test_plan_construction_s640():
    from yms import runner
    from yolov8.yolov8 import YOLOv8
    m = YOLOv8("s", 80)
    x = torch.empty(4, 3, 640, 640, device="meta")
    for tr in (False, True):
        m.train(tr)
        p = runner.get_plan(m, [x], torch.bfloat16, tr)
        assert abs(p.flops / 4 / 1e9 - 25.79) < 0.01
        # 66 modules' ops, the head's three box[i][0] / cls[i][0] pairs as one SiblingConvOp each
        assert len(p.ops) == 63
    with pytest.raises(RuntimeError, match="multiple of 32"):
        runner.get_plan(m, [torch.empty(1, 3, 100, 100, device="meta")], torch.float32, False)


def test_sibling_head_convs_plan(monkeypatch):
    """The head's box[i][0] / cls[i][0] pair (yolov8_head.py:84-85, 99-100) is one SiblingConvOp in a
    16-bit plan: outputs in the slots [0, 64) / [64, 64 + nc) of one buffer, members' parameter
    gradients adjacent in the flat arena (bias, gamma, weight kinds in turn), the same parameter set
    and FLOPs as the unfused plan (YMS_HEAD_FUSE=0 keeps two ConvOps)."""
    from yms import runner
    from yms.plan import SiblingConvOp
    from yolov8.yolov8 import YOLOv8
    m = YOLOv8("s", 20)
    x = torch.empty(2, 3, 256, 256, device="meta")
    m.train(True)
    p = runner.get_plan(m, [x], torch.bfloat16, True)
    sib = [op for op in p.ops if isinstance(op, SiblingConvOp)]
    assert len(sib) == 3
    for i, op in enumerate(sib):
        a, b = op.members
        assert a.mod is m.head.box[i][0] and b.mod is m.head.cls[i][0]
        assert (a.y.off, a.y.c, b.y.off, b.y.c, op.c) == (0, 64, 64, 20, 84) and a.y.buf is b.y.buf
        assert op.shape.cout == 84 and op.shape.cin == a.shape.cin and op.flops == a.flops + b.flops
        order = p.pgrad_order
        for kind in ("pb", "pg", "pw"):
            ia, ib = order.index(getattr(a, kind)), order.index(getattr(b, kind))
            assert ib == ia + 1
    p3 = runner.get_plan(m, [x], torch.float32, True)
    assert sum(isinstance(op, SiblingConvOp) for op in p3.ops) == 3
    monkeypatch.setenv("YMS_HEAD_FUSE", "0")
    m2 = YOLOv8("s", 20)
    m2.train(True)
    p2 = runner.get_plan(m2, [x], torch.bfloat16, True)
    assert not any(isinstance(op, SiblingConvOp) for op in p2.ops) and len(p2.ops) == len(p.ops) + 3
    assert p2.flops == p.flops and len(p2.param_refs) == len(p.param_refs)


def test_stem_input_and_tail_wgrad_order_plan(monkeypatch):
    """16-bit training plan: the input the stem conv reads as NCHW has no arena bytes and no zeroing
    (its 3 -> 8 channel padding was zeroed every step), and only the conv reading the stem's output
    enqueues its weight gradient before its input gradient (YMS_WGRAD_FIRST: 'tail' default, 0 none)."""
    from yms import runner
    from yms.plan import ConvOp
    from yolov8.yolov8 import YOLOv8
    m = YOLOv8("s", 80)
    m.train(True)
    x = torch.empty(4, 3, 128, 128, device="meta")
    p = runner.get_plan(m, [x], torch.bfloat16, True)
    (stem,) = p.stem_inputs.values()
    ib = p.inputs[0].buf
    assert stem is p.ops[0] and not ib.zero and all(off != ib.off or nb == 0 for off, nb in p.zero_ranges)
    tail = [op for op in p.ops if getattr(op, "tail_wgrad_first", False)]
    assert len(tail) == 1 and type(tail[0]) is ConvOp and tail[0].x.buf is stem.y.buf
    p32 = runner.get_plan(m, [x], torch.float32, True)    # fp32: generic input pack, no stem kernel
    assert not p32.stem_inputs and p32.inputs[0].buf.zero
    monkeypatch.setenv("YMS_WGRAD_FIRST", "0")
    m2 = YOLOv8("s", 80)
    m2.train(True)
    p2 = runner.get_plan(m2, [x], torch.bfloat16, True)
    assert not any(getattr(op, "tail_wgrad_first", False) for op in p2.ops)


def test_state_dict_keys_identical_to_reference():
    import json
    from yolov8.yolov8 import YOLOv8
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "state_keys.json")))
    for tag in ("n_80", "s_80", "l_80", "n_1"):
        v, nc = tag.split("_")
        m = YOLOv8(v, int(nc))
        assert [[k, list(t.shape)] for k, t in m.state_dict().items()] == ref[tag], tag
    from yolov8.model.components import yolo_params
    with pytest.raises(ValueError, match="Unknown YOLOv8 version: xs"):
        yolo_params("xs")


def test_cpu_input_raises():
    from yolov8.model.components import Conv
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Conv(3, 8)(torch.zeros(1, 3, 8, 8))


def test_dwconv_host_sizing_follows_the_kernel_selection():
    """Depthwise statistics rows and weight-gradient workspace (host functions, no GPU): the k = 7
    MFMA forward on maps <= 48 wide writes one statistics row per (image, 16-row block); the VALU strip
    forward one per tile (TX 20 / 40 -> TY 12 / 6); the MFMA weight gradient (16-bit, k >= 5, maps <= 64
    wide, k = 5 <= 96) sums whole per-group rows of K*K*C floats, few enough for the one-pass reduce."""
    def sh(n, h, w, c, k, dt):
        return ctypes.pointer(L.DwShape(n, h, w, c, k, dt))
    rows = L.lib().yms_dwconv_stats_rows
    assert rows(sh(64, 40, 40, 288, 7, L.BF16)) == 64 * 3            # MFMA forward: 16-row blocks
    assert rows(sh(3, 18, 28, 48, 7, L.F16)) == 3 * 2
    assert rows(sh(64, 40, 40, 288, 7, L.F32)) == 64 * 1 * 7         # fp32 keeps the strip walker
    assert rows(sh(64, 20, 20, 288, 9, L.BF16)) == 64 * 1 * 2        # k9: strip walker, TX 20 / TY 12
    assert rows(sh(64, 96, 96, 64, 7, L.BF16)) == 64 * 3 * 12        # > 48 wide: TX 32 / TY 8
    ws = L.lib().yms_dwconv_wgrad_ws_bytes
    for (n, h, w, c, k) in ((64, 20, 20, 288, 9), (64, 40, 40, 288, 7), (64, 80, 80, 160, 5), (2, 13, 9, 16, 9)):
        b = ws(sh(n, h, w, c, k, L.BF16))
        row = k * k * c * 4
        assert b > 0 and b % row == 0 and b // row <= 32, (n, h, w, c, k, b // row)
        units = n * ((h + 15) // 16)
        assert b // row <= units
    assert ws(sh(64, 40, 40, 288, 7, L.BF16)) < ws(sh(64, 40, 40, 288, 7, L.F32))   # fp32: tile kernel rows
    assert ws(sh(2, 13, 9, 12, 9, L.BF16)) == 0                                    # C % 8 != 0: rejected
