#!/bin/bash
# stem conv: parity tests, then interleaved A/B (YMS_STEM=0 generic pack + implicit GEMM, 1 = stem kernel)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_stem.log 2>&1 || { tail -40 gpurun_out/t_stem.log; exit 1; }
tail -1 gpurun_out/t_stem.log
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_ms_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { tail -40 gpurun_out/t_model.log; exit 1; }
tail -1 gpurun_out/t_model.log
for r in 1 2; do
  for v in 0 1; do
    YMS_STEM=$v timeout -k 10 200 python bench.py --mode infer --steps 100 --warmup 20 --no-cpu-baseline --no-profile --ms-version none > gpurun_out/stem_inf_$v.json 2>/dev/null
    echo "infer YMS_STEM=$v rep $r: $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/stem_inf_$v.json') if l.startswith('{')][-1]);print(d['infer']['value'], d['infer']['ms_per_batch_median'])")"
  done
done
bash tools/ab_train.sh gpurun_out/ab_stem 2 "YMS_STEM=0|" "YMS_STEM=1|"
