#!/bin/bash
# round-6 GPU call y: implicit-GEMM input-gradient grids persistent at 1x / 2x the resident blocks vs one block per tile, interleaved A/B
set -e
O=gpurun_out/r06y; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_dg1.so|" "YMS_LIB=tools/bin/libyms_dg2.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_dg1.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_dg2.so|--version ms-s --steps 40"
echo done
