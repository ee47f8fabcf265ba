# software-pipelined forward affine x items per thread: tests, then interleaved step A/B
set -e
mkdir -p gpurun_out/r03zg
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03zg/tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/r03zg/tests.log)"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for cfg in 0:2 1:2 1:4 1:8 0:2 1:2 1:4 1:8; do
    pp=${cfg%%:*}; it=${cfg##*:}
    YMS_BN_AFFINE_PIPE=$pp YMS_BN_AFFINE_ITERS=$it timeout -k 10 300 $B --version $v > gpurun_out/r03zg/b_${v}_${pp}_$it.json 2>> gpurun_out/r03zg/err.txt
    echo "$v affine_pipe=$pp iters=$it $(python -c "import json;d=json.loads(open('gpurun_out/r03zg/b_${v}_${pp}_$it.json').read().strip().splitlines()[-1]);r=d['roofline'];e=r['bn_elementwise']['by_entry_point'];print(d['ms_per_step'],d['ms_per_step_median'],round(e['affine_act']['ms'],3))")" | tee -a gpurun_out/r03zg/summary.txt
  done
done
