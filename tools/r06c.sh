#!/bin/bash
# round-6 GPU call c: sibling / model tests, in-place output-gradient A/B, per-dispatch PMC of one S step
set -e
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sibling_gpu.py tests/test_model_gpu.py tests/test_loss_gpu.py tests/test_dist_gpu.py tests/test_train_conditioned_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_train.sh $O/ab 3 "YMS_GRAD_INPLACE=0|" "YMS_GRAD_INPLACE=1|"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/step_calls.py $GRAFT_REPO_ROOT/$O/calls_s.json s 3 > $GRAFT_REPO_ROOT/$O/pmc_$c.log 2>&1
  echo "pmc $c done"
done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/layer_prof.py s 64 > $O/layer_prof_s.txt 2>&1
echo layer_prof done
find $O -name "*.db" -delete
