"""Dev tool: per-call times of every conv launch of one training step (HIP events on the launch
stream), sorted -- which layers the conv time goes to.
   python tools/layer_prof.py [version] [batch]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import _lib as L, set_compute_dtype
from yolov8.yolov8 import YOLOv8

v = sys.argv[1] if len(sys.argv) > 1 else "s"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = YOLOv8(v, 80).cuda().train()
set_compute_dtype(m, torch.bfloat16)
x = torch.randn(B, 3, 640, 640, device="cuda")
opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
orig = L.call
recs = []
on = [False]


def call(name, *args):
    if not on[0] or not name.startswith(("yms_conv_fwd", "yms_conv_dgrad", "yms_conv_wgrad", "yms_bn_", "yms_affine",
                                         "yms_dwconv")):
        return orig(name, *args)
    st = torch.cuda.ExternalStream(args[-1]) if args[-1] else None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    orig(name, *args)
    e.record(st)
    key = ""
    if name.startswith("yms_conv"):
        sh = args[0].contents
        key = f"{sh.n}x{sh.h}x{sh.w} {sh.cin}->{sh.cout} k{sh.k}s{sh.stride}"
        fl = 2 * sh.n * sh.ho * sh.wo * sh.cout * sh.cin * sh.k * sh.k
    elif name.startswith("yms_dwconv"):
        sh = args[0].contents
        key = f"{sh.n}x{sh.h}x{sh.w} c{sh.c} k{sh.k}"
        fl = 2 * sh.n * sh.h * sh.w * sh.c * sh.k * sh.k
    elif name == "yms_bn_act_bwd_finalize":       # (c, ws, rows, npix, ...)
        key = f"npix {args[3]} c {args[0]}"
        fl = 0
    elif name.startswith(("yms_bn_act", "yms_affine")):   # (dtype, npix, c, ...)
        key = f"npix {args[1]} c {args[2]}"
        fl = 0
    else:
        fl = 0
    recs.append((name, key, s, e, fl))


L.call = call
for i in range(4):
    on[0] = i == 3
    opt.zero_grad(set_to_none=True)
    sum((o.float() ** 2).mean() for o in m(x)).backward()
    opt.step()
torch.cuda.synchronize()
rows = [(n, k, s.elapsed_time(e), fl) for n, k, s, e, fl in recs]
tot = {}
for n, k, t, fl in rows:
    a = tot.setdefault(n, [0, 0.0])
    a[0] += 1
    a[1] += t
print("totals (ms):", {n: (c, round(t, 3)) for n, (c, t) in sorted(tot.items(), key=lambda z: -z[1][1])})
print("top calls:")
for n, k, t, fl in sorted(rows, key=lambda r: -r[2])[:40]:
    print(f"{n:28s} {k:34s} {t * 1e3:8.1f} us {fl / (t * 1e-3) / 1e12 if fl else 0:7.1f} TF/s")
agg = {}
for n, k, t, fl in rows:
    a = agg.setdefault((n, k), [0, 0.0, 0.0])
    a[0] += 1
    a[1] += t
    a[2] += fl
print("per layer shape (count, total us, TF/s):")
for (n, k), (c, t, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{n:28s} {k:34s} x{c:2d} {t * 1e3:9.1f} us {fl / (t * 1e-3) / 1e12 if fl else 0:7.1f} TF/s")
# every fwd / dgrad layer shape with its own roofline: max(FLOPs / 2.5 PF, bytes / 8 TB/s), bytes =
# input + output (16-bit) + weights once
if os.environ.get("YMS_LAYER_ALL"):
    print("fwd / dgrad per layer shape: calls, us per call, roofline us, frac")
    tot_t = tot_r = 0.0
    for (n, k), (c, t, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if n not in ("yms_conv_fwd", "yms_conv_dgrad"):
            continue
        nn, io, ks = k.split()
        bb, hh, ww = (int(v) for v in nn.split("x"))
        ci, co = (int(v) for v in io.split("->"))
        kk, ss = int(ks[1]), int(ks[3])
        ho, wo = (hh + 2 * (kk // 2) - kk) // ss + 1, (ww + 2 * (kk // 2) - kk) // ss + 1
        byt = 2 * (bb * hh * ww * ci + bb * ho * wo * co + ci * co * kk * kk)
        roof = max(fl / c / 2.5e15, byt / 8e12) * 1e6
        tot_t += t * 1e3
        tot_r += roof * c
        print(f"{n:16s} {k:34s} x{c:2d} {t * 1e3 / c:8.1f} us  roof {roof:6.1f} us  frac {roof * c / (t * 1e3):.2f}")
    print(f"total {tot_t:.1f} us, roofline {tot_r:.1f} us, frac {tot_r / tot_t:.3f}")
