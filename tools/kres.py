"""Summarise hipcc -Rpass-analysis=kernel-resource-usage for a .hip file (dev tool).
usage: python tools/kres.py yolo-ms_amd/csrc/conv_igemm.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src,
                      "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.rsplit(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    n = n.replace("yms::", "").replace("(yms::NTParams)", "").replace("(yms::TTParams)", "")
    if flt and flt not in n:
        continue
    print(f"{n[:88]:88s} v={r.get('VGPRs')} a={r.get('AGPRs')} scr={r.get('ScratchSize [bytes/lane]')} "
          f"occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")
