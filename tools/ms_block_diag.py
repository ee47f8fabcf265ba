"""Dev diagnostic: one MSBlock (fp32) vs oracle msblock, per-parameter grad error."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from oracle import ms_ref as MS
from oracle import model_ref as M
from yolov8.model.yolo_ms import MSBlock

for (cin, cout, k, L, h, w) in [(384, 128, 3, 1, 4, 6), (64, 64, 3, 1, 4, 6), (64, 64, 3, 1, 16, 24), (192, 64, 3, 1, 8, 12), (384, 128, 3, 1, 16, 16)]:
    blk = MSBlock(cin, cout, k, L)
    sd = {}
    for kk, t in blk.state_dict().items():
        if kk.endswith("num_batches_tracked"):
            sd[kk] = t.clone()
        elif kk.endswith("conv.weight"):
            sd[kk] = M._closed_form(kk, tuple(t.shape), (3.0 / (t.shape[1] * t.shape[2] * t.shape[3])) ** 0.5 * 1.2)
        elif kk.endswith("bn.weight") or kk.endswith("running_var"):
            sd[kk] = M._closed_form(kk, tuple(t.shape), 0.25, base=1.0)
        else:
            sd[kk] = M._closed_form(kk, tuple(t.shape), 0.1)
    blk.load_state_dict(sd)
    blk = blk.cuda().train()
    x = torch.randn(2, cin, h, w, generator=torch.Generator().manual_seed(1))
    cot = torch.randn(2, cout, h, w, generator=torch.Generator().manual_seed(2))
    pr = {"b." + kk: (t.clone().double().requires_grad_(True) if t.is_floating_point() and "running" not in kk else t.clone().double() if t.is_floating_point() else t.clone()) for kk, t in sd.items()}
    xr = x.double().requires_grad_(True)
    yr = MS.msblock(pr, "b", xr, k, L, True)
    (yr * cot.double()).sum().backward()
    xg = x.cuda().requires_grad_(True)
    y = blk(xg)
    (y * cot.cuda()).sum().backward()
    rel = lambda a, b: ((a.double().cpu() - b).norm() / (b.norm() + 1e-30)).item()
    pd = dict(blk.named_parameters())
    errs = sorted((rel(pd[kk[2:]].grad, t.grad), kk) for kk, t in pr.items() if t.grad is not None)
    print((cin, cout, k, L, h, w), "y", rel(y.detach(), yr.detach()), "dx", rel(xg.grad, xr.grad), "worst", errs[-3:])

# depthwise kernels alone at the neck's shapes
import ctypes
import torch.nn.functional as F
from yms import _lib as L
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hiputil import nhwc, nchw, r8
for (n, h, w, c, k) in [(2, 4, 6, 384, 3), (2, 8, 12, 192, 3), (2, 2, 3, 384, 3)]:
    x = torch.randn(n, c, h, w); wt = torch.randn(c, 1, k, k) / k; dz = torch.randn(n, c, h, w)
    sh = L.DwShape(n, h, w, c, k, L.F32); sp = ctypes.pointer(sh)
    xb, dzb, wd = nhwc(x, torch.float32), nhwc(dz, torch.float32), wt.cuda()
    xg = x.clone().requires_grad_(True); wg = wt.clone().requires_grad_(True)
    F.conv2d(xg, wg, None, 1, k // 2, 1, c).backward(dz)
    dx = torch.zeros_like(xb)
    L.call("yms_dwconv_dgrad", sp, dzb.data_ptr(), c, 0, wd.data_ptr(), dx.data_ptr(), c, 0, 0, L.stream_ptr())
    wsb = L.lib().yms_dwconv_wgrad_ws_bytes(sp); ws = torch.empty(wsb // 4, device="cuda"); dw = torch.zeros(c, 1, k, k, device="cuda")
    L.call("yms_dwconv_wgrad", sp, xb.data_ptr(), c, 0, dzb.data_ptr(), c, 0, ws.data_ptr(), wsb, dw.data_ptr(), 0, L.stream_ptr())
    torch.cuda.synchronize()
    print("dw", (n, h, w, c, k), "dx", ((nchw(dx, c).cpu() - xg.grad).norm() / xg.grad.norm()).item(),
          "dw", ((dw.cpu() - wg.grad).norm() / wg.grad.norm()).item())
