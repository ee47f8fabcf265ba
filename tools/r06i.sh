#!/bin/bash
# round-6 GPU call i (re-entry): GPU suite on the current tree, then interleaved A/B of the
# round-6 changes all-off vs all-on (YOLOv8-s and YOLO-MS-S), then each change alone.
set -e
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
OFF="YMS_HEAD_FUSE=0 YMS_BNRED=0 YMS_WG_HALO_NB2=0 YMS_GRAD_INPLACE=0"
bash tools/ab_train.sh $O/ab_s 3 "$OFF|" "YMS_X=1|"
bash tools/ab_train.sh $O/ab_ms 2 "$OFF|--version ms-s --steps 40" "YMS_X=1|--version ms-s --steps 40"
bash tools/ab_train.sh $O/ab_each 2 "YMS_HEAD_FUSE=0|" "YMS_BNRED=0|" "YMS_WG_HALO_NB2=0|" "YMS_GRAD_INPLACE=0|" "YMS_X=1|"
