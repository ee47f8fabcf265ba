#!/bin/bash
# wgrad register-stage A/B: parity tests, isolated wgrad per layer (variant 1 = one stage, 0 = two), step A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_conv.log 2>&1 || { tail -30 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
for v in 1 0; do
  echo "== YMS_WG_VARIANT=$v"
  YMS_WG_VARIANT=$v timeout -k 10 120 python tools/conv_micro.py 2>&1 | grep wgrad
  YMS_WG_VARIANT=$v YMS_MICRO_SHAPES=ms timeout -k 10 120 python tools/conv_micro.py 2>&1 | grep wgrad
done
bash tools/ab_train.sh gpurun_out/ab_wg 2 "YMS_WG_VARIANT=1|" "YMS_WG_VARIANT=0|" "YMS_WG_VARIANT=1|--version ms-s --steps 30" "YMS_WG_VARIANT=0|--version ms-s --steps 30"
