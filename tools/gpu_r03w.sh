# side-stream weight-gradient LDS footprint: default (ring 64 KB + halo <= 64 KB) vs TT only (40 KB)
mkdir -p gpurun_out/r03w
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for cfg in "1 1" "0 0" "1 0" "1 1" "0 0" "1 0"; do
    set -- $cfg
    YMS_WG_RING=$1 YMS_WG_HALO=$2 timeout -k 10 300 $B --version $v > gpurun_out/r03w/b_${v}_$1$2.json 2>> gpurun_out/r03w/err.txt || exit 1
    echo "$v ring=$1 halo=$2 $(python -c "import json;d=json.loads(open('gpurun_out/r03w/b_${v}_$1$2.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],round(r['by_entry_point']['fwd']['ms'],2),round(r['by_entry_point']['dgrad']['ms'],2),round(r['by_entry_point']['wgrad']['ms'],2),round(r['bn_elementwise']['ms_per_step'],2))")" | tee -a gpurun_out/r03w/summary.txt
  done
done
