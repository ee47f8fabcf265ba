# side-stream concurrency A/B: weight-gradient blocks per CU (ring / halo split counts)
mkdir -p gpurun_out/r03o
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for cfg in "4 2" "1 1" "2 1" "8 4" "4 2"; do
    set -- $cfg
    YMS_WG_RING_BPC=$1 YMS_WG_HALO_BPC=$2 timeout -k 10 300 $B --version $v > gpurun_out/r03o/b_${v}_$1_$2.json 2>> gpurun_out/r03o/err.txt || exit 1
    echo "$v $cfg $(python -c "import json;d=json.loads(open('gpurun_out/r03o/b_${v}_$1_$2.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['ms_per_step_median'],round(d['roofline']['bn_elementwise']['ms_per_step'],2),round(d['roofline']['by_entry_point']['wgrad']['ms'],2))")" | tee -a gpurun_out/r03o/summary.txt
  done
done
