#!/bin/bash
# round-6 GPU call ac: forward BN finalize with a shuffle tree (one barrier) vs the all-LDS tree: tests + interleaved A/B
set -e
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_train_conditioned_gpu.py tests/test_model_gpu.py -k "bn or finalize or bf16 or train or fp32" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_train.sh $O/ab 3 "YMS_LIB=tools/bin/libyms_base.so|" "YMS_X=0|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_LIB=tools/bin/libyms_base.so|--version ms-s --steps 40" "YMS_X=0|--version ms-s --steps 40"
echo done
