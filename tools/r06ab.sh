#!/bin/bash
# round-6 GPU call ab: non-temporal stores of the weight gradients' fp32 split-K slabs, interleaved A/B
set -e
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 300 env YMS_LIB=tools/bin/libyms_sn.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k wgrad > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_sn.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_sn.so|--version ms-s --steps 40"
echo done
