# software-pipelined BN backward reduce: tests, then interleaved step A/B (YMS_BN_RED_PIPE 1 vs 0)
set -e
mkdir -p gpurun_out/r03zb
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03zb/tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/r03zb/tests.log)"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 1 0 1 0; do
    YMS_BN_RED_PIPE=$n timeout -k 10 300 $B --version $v > gpurun_out/r03zb/b_${v}_$n.json 2>> gpurun_out/r03zb/err.txt
    echo "$v pipe=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03zb/b_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];e=r['bn_elementwise']['by_entry_point'];print(d['ms_per_step'],d['ms_per_step_median'],round(e['bn_act_bwd_reduce']['ms'],3),round(e['bn_act_bwd_apply']['ms'],3))")" | tee -a gpurun_out/r03zb/summary.txt
  done
done
