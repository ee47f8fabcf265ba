#!/bin/bash
# round-6 GPU call x: non-temporal last reads (x, dz) in the depthwise weight gradients, interleaved A/B on YOLO-MS-S / MS-L
set -e
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 300 env YMS_LIB=tools/bin/libyms_dww.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dwconv_gpu.py -k wgrad > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_train.sh $O/ab_ms 3 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_dww.so|--version ms-s --steps 40"
bash tools/ab_train.sh $O/ab_l 2 "YMS_X=0|--version ms-l --steps 16 --warmup 4" "YMS_LIB=tools/bin/libyms_dww.so|--version ms-l --steps 16 --warmup 4"
echo done
