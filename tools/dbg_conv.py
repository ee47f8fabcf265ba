"""Debug: locate mismatches of one conv fwd shape (dev tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import torch
from hiputil import conv_fwd, nchw, nhwc, ref_conv, shape
from yms import _lib as L
n, cin, h, w, cout, k, s = [int(v) for v in sys.argv[1:8]]
mode = sys.argv[8] if len(sys.argv) > 8 else "affine"
dt = torch.bfloat16
g = torch.Generator().manual_seed(0)
x = torch.randn(n, cin, h, w, generator=g)
wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
sh = shape(n, h, w, cin, cout, k, s, dt)
if mode == "affine":
    y, _ = conv_fwd(nhwc(x, dt), wt, sh, dt, torch.ones(cout).cuda(), torch.zeros(cout).cuda(), 0)
else:
    y, _ = conv_fwd(nhwc(x, dt), wt, sh, dt, stats=True)
z = ref_conv(x, wt, s, dt)
got = nchw(y, cout).cpu()
bad = ((got - z).abs() > 0.05 * z.abs().max()) | got.isnan()
print("bad", bad.sum().item(), "of", bad.numel(), "nan", got.isnan().sum().item())
if bad.any():
    idx = bad.nonzero()
    pix = idx[:, 0] * sh.ho * sh.wo + idx[:, 2] * sh.wo + idx[:, 3]
    print("rows", pix.unique()[:40].tolist(), "...", pix.unique().numel())
    print("cols", idx[:, 1].unique().tolist()[:80])
