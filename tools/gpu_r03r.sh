# side stream restricted to a CU subset (spread), interleaved A/B
mkdir -p gpurun_out/r03r
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 0 224 192 160 0 224 192; do
    YMS_SIDE_CUS=$n YMS_SIDE_CU_MODE=1 timeout -k 10 300 $B --version $v > gpurun_out/r03r/b_${v}_$n.json 2>> gpurun_out/r03r/err.txt || exit 1
    echo "$v side_cus=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03r/b_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],round(r['bn_elementwise']['ms_per_step'],2),round(r['by_entry_point']['wgrad']['ms'],2))")" | tee -a gpurun_out/r03r/summary.txt
  done
done
