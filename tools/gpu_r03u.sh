# forward BN finalize: 256-thread latency-shaped kernel (default) vs the 1024-thread tree kernel
mkdir -p gpurun_out/r03u
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bn_gpu.py tests/test_train_conditioned_gpu.py tests/test_conv_gpu.py -k "stats or bn or conditioned" > gpurun_out/r03u/t.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 1 0 1 0; do
    YMS_BN_FIN_SMALL=$n timeout -k 10 300 $B --version $v > gpurun_out/r03u/b_${v}_$n.json 2>> gpurun_out/r03u/err.txt || exit 1
    echo "$v fin_small=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03u/b_${v}_$n.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['ms_per_step_median'])")" | tee -a gpurun_out/r03u/summary.txt
  done
done
