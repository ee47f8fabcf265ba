# forward affine_act U-pixel iterations per thread (YMS_BN_AFFINE_ITERS; the forward has no side-stream work)
mkdir -p gpurun_out/r03y
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for n in 4 2 1 8 4 2 1 8; do
    YMS_BN_AFFINE_ITERS=$n timeout -k 10 300 $B --version $v > gpurun_out/r03y/b_${v}_$n.json 2>> gpurun_out/r03y/err.txt || exit 1
    echo "$v iters=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03y/b_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],round(r['bn_elementwise']['by_entry_point']['affine_act']['ms'],3))")" | tee -a gpurun_out/r03y/summary.txt
  done
done
