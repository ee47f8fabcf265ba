#!/bin/bash
# round-6 GPU call l: s_setprio for the main stream's waves (BN / conv) vs the side stream's wgrads, interleaved A/B
set -e
O=gpurun_out/r06l; mkdir -p $O
B=$GRAFT_REPO_ROOT/tools/bin
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=$B/libyms_prio_bn.so|" "YMS_LIB=$B/libyms_prio_all.so|" "YMS_LIB=$B/libyms_prio_all2.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=$B/libyms_prio_bn.so|--version ms-s --steps 40" "YMS_LIB=$B/libyms_prio_all.so|--version ms-s --steps 40"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/step_calls.py $GRAFT_REPO_ROOT/$O/calls_s.json s 3 > $GRAFT_REPO_ROOT/$O/pmc_$c.log 2>&1
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_layers.py $O > $O/wgrad_layers.txt && find $O -name "*.db" -delete
head -40 $O/wgrad_layers.txt
