#!/bin/bash
# wgrad variant / split sweep: total wgrad us of one training step at B=64 (dev tool)
for v in 0 1 2 3; do for w in 4 8; do
  YMS_WG_VARIANT=$v YMS_WG_WPC=$w timeout -k 10 200 python tools/conv_layers.py 64 train > gpurun_out/wg_${v}_${w}.txt 2>&1 || exit 1
  echo "var $v wpc $w: $(grep '^wgrad' gpurun_out/wg_${v}_${w}.txt | awk '{s+=$7} END {print s}') us"
done; done
