#!/bin/bash
# round-6 GPU call ad: kernel trace of a few YOLOv8-s training steps: where the per-step buffer copies sit
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06ad; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 4 --warmup 3 --no-cpu-baseline --no-profile --ms-version none > $O/bench.log 2>&1
python3 - $O/trace/run_kernel_trace.csv > $O/copies.txt <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "pack_weight_batched" in r["Kernel_Name"]]
lo, hi = marks[-2], marks[-1]
step = rows[lo:hi]
ctx = collections.Counter()
for i, r in enumerate(step):
    if "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]:
        prev = step[i - 1]["Kernel_Name"][:50] if i else "-"
        nxt = step[i + 1]["Kernel_Name"][:50] if i + 1 < len(step) else "-"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"q{r['Queue_Id']} {r['Kernel_Name'][:30]} {d:.1f} us  after [{prev}]  before [{nxt}]  grid {r.get('Grid_Size','?')}")
PY
gzip -f $O/trace/run_kernel_trace.csv; find $O -name "*.db" -delete
echo done
