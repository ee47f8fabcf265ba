#!/bin/bash
# round-6 GPU call j: kernel trace of the current YOLOv8-s / YOLO-MS-S training step -> per-queue timeline
set -e
O=gpurun_out/r06j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in s ms-s; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 4 --warmup 3 --no-cpu-baseline --no-profile --ms-version none --version $v > $GRAFT_REPO_ROOT/$O/bench_$v.log 2>&1
  python3 $GRAFT_REPO_ROOT/tools/step_timeline.py $GRAFT_REPO_ROOT/$O/trace_$v/run_kernel_trace.csv > $GRAFT_REPO_ROOT/$O/timeline_$v.txt
  python3 $GRAFT_REPO_ROOT/tools/step_tail.py $GRAFT_REPO_ROOT/$O/trace_$v/run_kernel_trace.csv 2 > $GRAFT_REPO_ROOT/$O/tail_$v.txt
  gzip -f $GRAFT_REPO_ROOT/$O/trace_$v/run_kernel_trace.csv; find $GRAFT_REPO_ROOT/$O -name "*.db" -delete
done
echo done
