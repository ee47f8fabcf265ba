"""Dev tool: the fused BN-reduce input gradients (Plan._find_bnred) vs the separate reduce, per
parameter, on one model (bf16 training step, surrogate loss).
   python tools/diag_bnred.py [version] [batch] [size]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from yms import plan as P
from yolov8.yolov8 import YOLOv8

v = sys.argv[1] if len(sys.argv) > 1 else "s"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H = int(sys.argv[3]) if len(sys.argv) > 3 else 640
torch.manual_seed(0)
sd = YOLOv8(v, 80).state_dict()
x = torch.randn(B, 3, H, H, generator=torch.Generator().manual_seed(1)).cuda()


def run(fused):
    os.environ["YMS_BNRED"] = "1" if fused else "0"
    m = YOLOv8(v, 80).cuda()
    m.load_state_dict(sd)
    m.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        outs = m(x)
    sum((o.float() ** 2).mean() for o in outs).backward()
    torch.cuda.synchronize()
    pl = [p for p in m.__dict__.get("_yms_plans", {}).values()] if hasattr(m, "__dict__") else []
    return {k: p.grad.double().cpu() for k, p in m.named_parameters() if p.grad is not None}, m


ga, ma = run(True)
gb, mb = run(False)
for cache in (getattr(ma, "__dict__", {}),):
    for k, val in cache.items():
        if isinstance(val, dict):
            for pl in val.values():
                if isinstance(pl, P.Plan):
                    for op in pl.ops:
                        if getattr(op, "bnred_for", None) is not None:
                            q = op.bnred_for
                            print(f"fused: consumer k{op.shape.k}s{op.shape.stride} {op.shape.cin}->{op.shape.cout} "
                                  f"@{op.shape.h}x{op.shape.w} acc_x={getattr(op, 'acc_x', '?')} producer c={q.c} "
                                  f"{q.mod.__class__.__name__}")
rows = []
for k in ga:
    a, b = ga[k], gb[k]
    rows.append(((a - b).norm().item() / (b.norm().item() + 1e-30), k))
rows.sort(reverse=True)
for r, k in rows[:25]:
    print(f"{r:10.3e}  {k}")
print("median", sorted(r for r, _ in rows)[len(rows) // 2])

# in-situ check: after every fused input gradient, the separate reduce over the same (z, dx) vs the
# fused partial rows, both through the finalize
from yms import _lib as L
import ctypes
orig = L.call
chk = []


saved = {}


def call(name, *a):
    if name == "yms_bn_act_bwd_finalize" and a[1] in saved:
        ref, nb = saved.pop(a[1])
        cur = torch.empty_like(ref)
        torch.cuda.synchronize()
        orig("yms_copy", ctypes.c_void_p(cur.data_ptr()), ctypes.c_void_p(a[1]), nb, None)
        torch.cuda.synchronize()
        print("DXCHK rows unchanged at the producer's finalize:", torch.equal(cur, ref), "rows arg", a[2])
    if name != "yms_conv_dgrad_bnred":
        orig(name, *a)
        return
    sh = a[0].contents
    nbytes = sh.n * sh.h * sh.w * a[6] * 2
    snap = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    orig("yms_copy", ctypes.c_void_p(snap.data_ptr()), ctypes.c_void_p(a[5]), nbytes, a[17])
    orig(name, *a)
    plain = snap.clone()
    orig("yms_conv_dgrad", a[0], a[1], a[2], a[3], a[4], plain.data_ptr(), a[6], a[7], a[8], a[17])
    cur = torch.empty_like(snap)
    orig("yms_copy", ctypes.c_void_p(cur.data_ptr()), ctypes.c_void_p(a[5]), nbytes, a[17])
    torch.cuda.synchronize()
    print("DXCHK dx bitwise equal to the plain dgrad:", torch.equal(cur, plain))
    nb = L.lib().yms_conv_dgrad_bnred_rows(a[0]) * 2 * sh.cin * 4
    wsc = torch.empty(nb, dtype=torch.uint8, device="cuda")
    orig("yms_copy", ctypes.c_void_p(wsc.data_ptr()), ctypes.c_void_p(a[16]), nb, a[17])
    torch.cuda.synchronize()
    saved[a[16]] = (wsc, nb)
    dx, dxl, dxo = a[5], a[6], a[7]
    z, zl, zo, sc, shf, mi, act, ws, st = a[9], a[10], a[11], a[12], a[13], a[14], a[15], a[16], a[17]
    npix = sh.n * sh.h * sh.w
    c = sh.cin
    rows = L.lib().yms_conv_dgrad_bnred_rows(a[0])
    rows0 = L.lib().yms_bn_bwd_rows(npix, c)
    w0 = torch.empty(rows0 * 2 * c, device="cuda")
    orig("yms_bn_act_bwd_reduce", sh.dtype, npix, c, z, zl, zo, dx, dxl, dxo, sc, shf, mi, act, w0.data_ptr(), st)
    o0 = torch.empty(4 * c, device="cuda")
    o1 = torch.empty(4 * c, device="cuda")
    orig("yms_bn_act_bwd_finalize", c, w0.data_ptr(), rows0, npix, o0.data_ptr(), o0[c:].data_ptr(), o0[2 * c:].data_ptr(), st)
    orig("yms_bn_act_bwd_finalize", c, ws, rows, npix, o1.data_ptr(), o1[c:].data_ptr(), o1[2 * c:].data_ptr(), st)
    torch.cuda.synchronize()
    e = ((o1 - o0).abs().max() / (o0.abs().max() + 1e-30)).item()
    chk.append(e)
    print(f"in-situ k{sh.k}s{sh.stride} {sh.cin}<-{sh.cout} @{sh.h}x{sh.w} acc {a[8]} rows {rows}: rel err {e:.2e}")


L.call = call
os.environ["YMS_BNRED"] = "1"
m = YOLOv8(v, 80).cuda()
m.load_state_dict(sd)
m.train()
with torch.autocast("cuda", dtype=torch.bfloat16):
    outs = m(x)
sum((o.float() ** 2).mean() for o in outs).backward()
torch.cuda.synchronize()
gc = {k: p.grad.double().cpu() for k, p in m.named_parameters() if p.grad is not None}
worst = max(((gc[k] - gb[k]).norm().item() / (gb[k].norm().item() + 1e-30), k) for k in gc)
print("hooked (synchronised) fused model vs separate: worst", worst)
