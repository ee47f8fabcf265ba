#!/bin/bash
# round-6 GPU call t: non-temporal LDS-DMA operand loads in the ring / halo weight gradients (dz = A, x = B), interleaved A/B
set -e
O=gpurun_out/r06t; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_wa.so|" "YMS_LIB=tools/bin/libyms_wb.so|" "YMS_LIB=tools/bin/libyms_wab.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_wa.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_wb.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_wab.so|--version ms-s --steps 40"
echo done
