mkdir -p gpurun_out/r03q
export PYTHONUNBUFFERED=1
YMS_BN_FIN_V2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bn_gpu.py > gpurun_out/r03q/t.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for f in 0 1 0 1; do
    YMS_BN_FIN_V2=$f timeout -k 10 300 $B --version $v > gpurun_out/r03q/b_${v}_$f.json 2>> gpurun_out/r03q/err.txt || exit 1
    echo "$v fin2=$f $(python -c "import json;d=json.loads(open('gpurun_out/r03q/b_${v}_$f.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['ms_per_step_median'])")" | tee -a gpurun_out/r03q/summary.txt
  done
done
