# branch-sum kernels: items per thread (YMS_ADD_ITERS) on YOLO-MS-S; BN backward apply iters 4/2/1; interleaved
set -e
mkdir -p gpurun_out/r03za
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dwconv_gpu.py -k "add_" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03za/tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/r03za/tests.log)"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
for n in 0 1 2 4 0 1 2 4; do
  YMS_ADD_ITERS=$n timeout -k 10 300 $B --version ms-s > gpurun_out/r03za/add_$n.json 2>> gpurun_out/r03za/err.txt
  echo "ms-s add_iters=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03za/add_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];e=r['bn_elementwise']['by_entry_point'];print(d['ms_per_step'],d['ms_per_step_median'],round(e['add_views']['ms'],3),round(e['add_grad2']['ms'],3))")" | tee -a gpurun_out/r03za/summary.txt
done
for v in s ms-s; do
  for n in 4 2 1 4 2 1; do
    YMS_BN_APPLY_ITERS=$n timeout -k 10 300 $B --version $v > gpurun_out/r03za/ap_${v}_$n.json 2>> gpurun_out/r03za/err.txt
    echo "$v apply_iters=$n $(python -c "import json;d=json.loads(open('gpurun_out/r03za/ap_${v}_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],d['ms_per_step_median'],round(r['bn_elementwise']['by_entry_point']['bn_act_bwd_apply']['ms'],3))")" | tee -a gpurun_out/r03za/summary.txt
  done
done
