"""Dev diagnostic: precision of the conv BN-statistics rows (sum, centred M2) vs fp64."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd"), os.path.join(ROOT, "tests")]
import torch
from hiputil import conv_fwd, merge_moments, nhwc, ref_conv, shape

for (n, cin, h, w, cout, k, s) in [(2, 64, 40, 40, 64, 3, 1), (2, 64, 40, 40, 128, 3, 1), (4, 128, 20, 20, 256, 3, 1),
                                   (2, 256, 20, 20, 32, 1, 1), (3, 32, 33, 17, 48, 3, 2), (8, 64, 80, 80, 64, 1, 1)]:
    for dt in (torch.float32, torch.bfloat16):
        g = torch.Generator().manual_seed(1)
        x = torch.randn(n, cin, h, w, generator=g) + 0.5
        wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
        sp = shape(n, h, w, cin, cout, k, s, dt)
        y, st = conv_fwd(nhwc(x, dt), wt, sp, dt, stats=True)
        z = ref_conv(x, wt, s, dt).double()
        s1, m2 = merge_moments(st, cout, z.numel() // cout)
        r1 = z.sum((0, 2, 3))
        r2 = ((z - z.mean((0, 2, 3), keepdim=True)) ** 2).sum((0, 2, 3))
        print((n, cin, h, w, cout, k, s), str(dt)[6:], "sum err %.2e  M2 err %.2e" % (
            ((s1 - r1).abs() / r2.sqrt()).max().item(), ((m2 - r2).abs() / r2).max().item()))
