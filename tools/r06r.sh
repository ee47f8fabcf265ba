#!/bin/bash
# round-6 GPU call p: NT input gradient with the producer's BN-reduce epilogue: tests + interleaved A/B
set -e
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dgrad_bnred_gpu.py > $O/tests_bnred.log 2>&1 || { tail -40 $O/tests_bnred.log; exit 1; }
tail -1 $O/tests_bnred.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_conditioned_gpu.py tests/test_sibling_gpu.py tests/test_model_gpu.py -k "bf16 or lowp or sibling or train" > $O/tests_model.log 2>&1 || { tail -40 $O/tests_model.log; exit 1; }
tail -1 $O/tests_model.log
bash tools/ab_train.sh $O/ab 2 "YMS_BNRED_NT=0|" "YMS_BNRED_NT=1|" "YMS_BNRED_NT=1 YMS_BNRED_MULT=2|" "YMS_BNRED_NT=1 YMS_BNRED_MULT=4|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_BNRED_NT=0|--version ms-s --steps 40" "YMS_BNRED_NT=1|--version ms-s --steps 40"
YMS_BNRED_NT=1 YMS_LAYER_ALL=1 timeout -k 10 200 python -u tools/layer_prof.py s 64 > $O/layers_s.txt 2>&1
echo done
