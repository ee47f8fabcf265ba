#!/bin/bash
# round-6 GPU call v: non-temporal reads of the weight gradients' split-K slabs in the fixed-order reduce, interleaved A/B
set -e
O=gpurun_out/r06v; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_wr.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_wr.so|--version ms-s --steps 40"
echo done
