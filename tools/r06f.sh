#!/bin/bash
# round-6 GPU call f: weight gradient enqueued before the input gradient (A/B), step-tail traces
set -e
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "train or b64" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_train.sh $O/ab 3 "YMS_WGRAD_FIRST=0|" "YMS_WGRAD_FIRST=1|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_WGRAD_FIRST=0|--version ms-s --steps 40" "YMS_WGRAD_FIRST=1|--version ms-s --steps 40"
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
  YMS_WGRAD_FIRST=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace$f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 4 --warmup 2 --no-cpu-baseline --no-profile --ms-version none > /dev/null 2>&1
  python3 $GRAFT_REPO_ROOT/tools/step_tail.py $GRAFT_REPO_ROOT/$O/trace$f/run_kernel_trace.csv 2 > $GRAFT_REPO_ROOT/$O/tail$f.txt
  rm -f $GRAFT_REPO_ROOT/$O/trace$f/run_kernel_trace.csv; find $GRAFT_REPO_ROOT/$O -name "*.db" -delete
done
echo traces done
