# BN-backward reduce: pipelined loop x partial-row cap (fewer, longer reduce blocks), interleaved A/B
set -e
mkdir -p gpurun_out/r03zd
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for v in s ms-s; do
  for cfg in 0:512 1:512 1:256 0:256 0:512 1:512 1:256 0:256; do
    pp=${cfg%%:*}; cap=${cfg##*:}
    YMS_BN_RED_PIPE=$pp YMS_BN_BWD_ROWS_CAP=$cap timeout -k 10 300 $B --version $v > gpurun_out/r03zd/b_${v}_${pp}_$cap.json 2>> gpurun_out/r03zd/err.txt
    echo "$v pipe=$pp cap=$cap $(python -c "import json;d=json.loads(open('gpurun_out/r03zd/b_${v}_${pp}_$cap.json').read().strip().splitlines()[-1]);r=d['roofline'];e=r['bn_elementwise']['by_entry_point'];print(d['ms_per_step'],d['ms_per_step_median'],round(e['bn_act_bwd_reduce']['ms'],3),round(e['bn_act_bwd_apply']['ms'],3))")" | tee -a gpurun_out/r03zd/summary.txt
  done
done
