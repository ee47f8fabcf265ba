#!/bin/bash
# round-6 GPU call h: 64-input-channel halo wgrad -- tests, step A/B, per-layer PMC of the wgrads
set -e
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "halo or slab or smaller" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_model_gpu.py -k "b64" > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
bash tools/ab_train.sh $O/ab 3 "YMS_WG_HALO_NB2=0|" "YMS_WG_HALO_NB2=1|"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/step_calls.py $GRAFT_REPO_ROOT/$O/calls_s.json s 3 > $GRAFT_REPO_ROOT/$O/pmc_$c.log 2>&1
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_layers.py $O > $O/wgrad_layers.txt && find $O -name "*.db" -delete
head -6 $O/wgrad_layers.txt
