#!/bin/bash
# round-6 GPU call w: non-temporal last reads in the MS-Block branch sum / its backward (add_views a, b; add_grad2 g), interleaved A/B on YOLO-MS-S
set -e
O=gpurun_out/r06w; mkdir -p $O
bash tools/ab_train.sh $O/ab_ms 3 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_ag.so|--version ms-s --steps 40"
echo done
