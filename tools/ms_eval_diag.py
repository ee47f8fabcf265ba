"""Dev diagnostic: YOLO-MS eval-mode output of the GPU fp32 path and of the CPU fp32 oracle, both
against the fp64 oracle, with running statistics calibrated on another input of the same size."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]
import torch
from oracle import ms_ref as MS
from yolov8.yolov8 import YOLOv8

v, s = sys.argv[1], int(sys.argv[2])
sd = MS.init_params(v, 80)
sd = MS.calibrate(sd, v, 80, torch.randn(1, 3, s, s, generator=torch.Generator().manual_seed(5)))
x = torch.randn(1, 3, s, s, generator=torch.Generator().manual_seed(9))
m = YOLOv8(v, 80).cuda()
m.load_state_dict(sd)
m.head.stride = torch.tensor([8.0, 16.0, 32.0])
m.eval()
y = m(x.cuda()).cpu().double()
with torch.no_grad():
    f = MS.backbone(dict(sd), v, x, False)
    print("backbone out absmax", [round(t.abs().max().item(), 3) for t in f])
    r32 = MS.forward(dict(sd), v, 80, x, False).double()
    r64 = MS.forward({k: (t.double() if t.is_floating_point() else t) for k, t in sd.items()}, v, 80, x.double(), False)
for name, o in (("GPU fp32", y), ("CPU fp32", r32)):
    d = (o[..., 4:] - r64[..., 4:]).abs().flatten()
    print(f"{v} {s}: {name} vs fp64 cls err q50 {d.quantile(0.5).item():.2e} q99 {torch.quantile(d[:16000000], 0.99).item():.2e} "
          f"max {d.max().item():.2e} box rel {((o[..., :4] - r64[..., :4]).norm() / r64[..., :4].norm()).item():.2e}")
