# BN backward apply: U-pixel iterations per thread (fewer, longer blocks), interleaved A/B
mkdir -p gpurun_out/r03t
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 4 8 16 4 8 16; do
    YMS_BN_APPLY_ITERS=$n timeout -k 10 300 $B --version $v > gpurun_out/r03t/b_${v}_$n.json 2>> gpurun_out/r03t/err.txt || exit 1
    echo "$v iters=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03t/b_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],json.dumps({k:round(v['ms'],2) for k,v in r['bn_elementwise']['by_entry_point'].items()}))")" | tee -a gpurun_out/r03t/summary.txt
  done
done
