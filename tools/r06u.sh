#!/bin/bash
# round-6 GPU call u: forward statistics grids at 2x / 4x the resident blocks (dynamic tiles, more statistics rows), interleaved A/B
set -e
O=gpurun_out/r06u; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_fm2.so|" "YMS_LIB=tools/bin/libyms_fm4.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_fm2.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_fm4.so|--version ms-s --steps 40"
echo done
