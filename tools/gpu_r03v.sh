mkdir -p gpurun_out/r03v
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bn_gpu.py tests/test_model_gpu.py > gpurun_out/r03v/t.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s; do
  for n in 1 0 1 0; do
    YMS_SPPF_FUSED=$n timeout -k 10 300 $B --version $v > gpurun_out/r03v/b_${v}_$n.json 2>> gpurun_out/r03v/err.txt || exit 1
    echo "$v sppf_fused=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03v/b_${v}_$n.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['ms_per_step_median'])")" | tee -a gpurun_out/r03v/summary.txt
  done
done
