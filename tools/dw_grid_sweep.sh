#!/bin/bash
# depthwise forward/dgrad strip-grid target sweep (YMS_DW_BLOCKS) on the YOLO-MS-S shapes
set -e
mkdir -p gpurun_out
for b in 1024 2048 3072 4096 8192; do
  echo "== YMS_DW_BLOCKS=$b"
  YMS_DW_BLOCKS=$b YMS_MICRO_SHAPES=mss timeout -k 10 120 python tools/dw_micro.py 2>&1 | grep -E "fwd |dgrad "
done
