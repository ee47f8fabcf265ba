# split-K slab round trip cap of the weight gradients (YMS_WG_SLAB_RATIO x the layer's x + dz bytes)
mkdir -p gpurun_out/r03x
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for r in 1.0 0.5 0.25 1.0 0.5 0.25; do
    YMS_WG_SLAB_RATIO=$r timeout -k 10 300 $B --version $v > gpurun_out/r03x/b_${v}_$r.json 2>> gpurun_out/r03x/err.txt || exit 1
    echo "$v ratio=$r $(python -c "import json;d=json.loads(open('gpurun_out/r03x/b_${v}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],round(r['by_entry_point']['dgrad']['ms'],2),round(r['by_entry_point']['wgrad']['ms'],2),round(r['bn_elementwise']['ms_per_step'],2))")" | tee -a gpurun_out/r03x/summary.txt
  done
done
