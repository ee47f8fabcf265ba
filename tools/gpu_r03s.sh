# minimum block count of the BN elementwise passes (affine / apply), interleaved A/B
mkdir -p gpurun_out/r03s
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 0 1024 2048 0 1024 2048; do
    YMS_BN_MINB=$n timeout -k 10 300 $B --version $v > gpurun_out/r03s/b_${v}_$n.json 2>> gpurun_out/r03s/err.txt || exit 1
    echo "$v minb=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03s/b_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],json.dumps({k:round(v['ms'],2) for k,v in r['bn_elementwise']['by_entry_point'].items()}))")" | tee -a gpurun_out/r03s/summary.txt
  done
done
