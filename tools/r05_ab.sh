#!/bin/bash
# Round 5: tests for the changed kernels, then interleaved A/B of YMS_DIRECT on the training and
# inference benches (YOLOv8-s configs[2] / configs[1]).
T=${1:-r05h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_conv_direct_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit $?
for rep in 1 2 3; do
  for v in 1 0; do
    YMS_DIRECT=$v timeout -k 10 150 python bench.py --mode train --steps 30 --warmup 8 --no-cpu-baseline --no-profile --ms-version none > gpurun_out/$T/tr_${v}_$rep.json 2> gpurun_out/$T/tr_${v}_$rep.err || exit 5
    python -c "import json; d=json.load(open('gpurun_out/$T/tr_${v}_$rep.json')); print('train YMS_DIRECT=$v', $rep, d['value'], d['ms_per_step'])" | tee -a gpurun_out/$T/summary.txt
  done
done
for rep in 1 2; do
  for v in 1 0; do
    YMS_DIRECT=$v timeout -k 10 150 python bench.py --mode infer --steps 40 --warmup 8 --no-cpu-baseline --no-profile --ms-version none > gpurun_out/$T/in_${v}_$rep.json 2> gpurun_out/$T/in_${v}_$rep.err || exit 6
    python -c "import json; d=json.load(open('gpurun_out/$T/in_${v}_$rep.json')); print('infer YMS_DIRECT=$v', $rep, d['value'], d['ms_per_step'])" | tee -a gpurun_out/$T/summary.txt
  done
done
