#!/bin/bash
# round-6 GPU call d: fused BN-reduce direct dgrad -- parity tests, model tests, step A/B, layer times
set -e
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dgrad_bnred_gpu.py tests/test_conv_direct_gpu.py > $O/tests1.log 2>&1 || { tail -40 $O/tests1.log; exit 1; }
tail -1 $O/tests1.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_train_conditioned_gpu.py tests/test_sibling_gpu.py tests/test_stem_gpu.py tests/test_dist_gpu.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
bash tools/ab_train.sh $O/ab 3 "YMS_BNRED=0|" "YMS_BNRED=1|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_BNRED=0|--version ms-s --steps 40" "YMS_BNRED=1|--version ms-s --steps 40"
timeout -k 10 200 python tools/layer_prof.py s 64 > $O/layer_prof_s.txt 2>&1
echo layer_prof done
