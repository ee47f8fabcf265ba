"""Dev tool: every weight-gradient launch of one training step of a model, timed isolated under
several kernel selections (env switches read per call), with per-layer and step totals.
   python tools/wgrad_micro.py [version] [batch] [reps]
Configurations: old = register-staged TT kernel only, halo = default 3x3 halo + TT, ring<v> =
ring variant v (+ halo where it is selected), ringall = ring everywhere it applies."""
import collections, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
os.environ.setdefault("YMS_WGRAD_STREAM", "0")
import torch
from yms import _lib as L, set_compute_dtype
from yolov8.yolov8 import YOLOv8
from hiputil import r8

v = sys.argv[1] if len(sys.argv) > 1 else "s"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 10
m = YOLOv8(v, 80).cuda().train()
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(B, 3, 640, 640, device="cuda")
shapes = collections.Counter()
orig = L.call


def call(name, *args):
    if name == "yms_conv_wgrad":
        sh = args[0].contents
        shapes[(sh.n, sh.h, sh.w, sh.cin, sh.cout, sh.k, sh.stride, sh.pad, sh.ho, sh.wo, sh.dtype)] += 1
    return orig(name, *args)


L.call = call
sum((o.float() ** 2).mean() for o in m(x)).backward()
torch.cuda.synchronize()
L.call = orig
del m, x
torch.cuda.empty_cache()

CONFIGS = {
    "old": {"YMS_WG_HALO": "0", "YMS_WG_RING": "0"},
    "halo": {"YMS_WG_HALO": "1", "YMS_WG_RING": "0"},
    "ring": {"YMS_WG_HALO": "1", "YMS_WG_RING": "1"},
    "ringall": {"YMS_WG_HALO": "0", "YMS_WG_RING": "2"},
    "slab10": {"YMS_WG_HALO": "1", "YMS_WG_RING": "1", "YMS_WG_SLAB_RATIO": "0.1"},
    "slab20": {"YMS_WG_HALO": "1", "YMS_WG_RING": "1", "YMS_WG_SLAB_RATIO": "0.2"},
    "slab50": {"YMS_WG_HALO": "1", "YMS_WG_RING": "1", "YMS_WG_SLAB_RATIO": "0.5"},
}
sel = os.environ.get("YMS_WGM_CONFIGS")
if sel:
    CONFIGS = {k: CONFIGS[k] for k in sel.split(",")}
st = L.stream_ptr()
tot = {c: 0.0 for c in CONFIGS}
flops = 0.0
print(f"{'layer':42s} {'x':>3s} " + " ".join(f"{c:>16s}" for c in CONFIGS), flush=True)
for key, cnt in sorted(shapes.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3]):
    n, h, w, ci, co, k, s_, p, ho, wo, dtc = key
    sh = L.ConvShape(n, h, w, ci, co, k, s_, p, ho, wo, dtc)
    sp = ctypes.pointer(sh)
    xb = torch.randn(n, h, w, r8(ci), device="cuda").to(torch.bfloat16)
    dz = torch.randn(n, ho, wo, r8(co), device="cuda").to(torch.bfloat16)
    dw = torch.empty(co, ci, k, k, device="cuda")
    fl = 2.0 * n * ho * wo * co * ci * k * k
    flops += fl * cnt
    row = []
    for c, env in CONFIGS.items():
        os.environ.pop("YMS_WG_SLAB_RATIO", None)
        for a, b in env.items():
            os.environ[a] = b
        wsb = L.lib().yms_conv_wgrad_ws_bytes(sp)
        ws = torch.empty(wsb // 4 + 1, device="cuda")
        fn = lambda: L.call("yms_conv_wgrad", sp, xb.data_ptr(), xb.shape[-1], 0, dz.data_ptr(), dz.shape[-1], 0,
                            ws.data_ptr(), wsb, dw.data_ptr(), 0, st)
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / REPS
        tot[c] += us * cnt
        row.append(f"{us:7.1f}us {fl / us / 1e6:5.0f}TF")
        del ws
    print(f"n{n} {h}x{w} {ci:4d}->{co:4d} k{k} s{s_}".ljust(42) + f" {cnt:3d} " + " ".join(f"{r:>16s}" for r in row),
          flush=True)
print("total per step (isolated sum): " + "  ".join(f"{c} {t / 1e3:.3f} ms ({flops / t / 1e6:.0f} TF/s)"
                                                    for c, t in tot.items()), flush=True)
