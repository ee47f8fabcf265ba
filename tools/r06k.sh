#!/bin/bash
# round-6 GPU call k: loss-backward scale kernel + stem-input arena + tail wgrad-first: tests, A/B, trace
set -e
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_loss_gpu.py tests/test_model_gpu.py tests/test_sibling_gpu.py tests/test_train_conditioned_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_train.sh $O/ab 3 "YMS_WGRAD_FIRST=0|" "YMS_WGRAD_FIRST=tail|" "YMS_WGRAD_FIRST=1|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_WGRAD_FIRST=0|--version ms-s --steps 40" "YMS_WGRAD_FIRST=tail|--version ms-s --steps 40"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 4 --warmup 3 --no-cpu-baseline --no-profile --ms-version none > $GRAFT_REPO_ROOT/$O/bench_s.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/step_timeline.py $GRAFT_REPO_ROOT/$O/trace_s/run_kernel_trace.csv > $GRAFT_REPO_ROOT/$O/timeline_s.txt
gzip -f $GRAFT_REPO_ROOT/$O/trace_s/run_kernel_trace.csv; find $GRAFT_REPO_ROOT/$O -name "*.db" -delete
echo done
