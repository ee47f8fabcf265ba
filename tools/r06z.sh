#!/bin/bash
# round-6 GPU call z: non-temporal reduce loads for layers whose gy + z exceed the Infinity Cache share (>= 256 / 128 MB), interleaved A/B
set -e
O=gpurun_out/r06z; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_rn256.so|" "YMS_LIB=tools/bin/libyms_rn128.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_rn256.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_rn128.so|--version ms-s --steps 40"
echo done
