#!/bin/bash
# round-6 GPU call n: deeper k-tile rings for the NT implicit-GEMM conv (forward ST 3/4 at one block
# per CU; input gradient ST 3), parity tests on the deep build, then interleaved train / infer A/B
set -e
O=gpurun_out/r06n; mkdir -p $O
B=$GRAFT_REPO_ROOT/tools/bin
YMS_LIB=$B/libyms_nt_f4d3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_model_gpu.py tests/test_sibling_gpu.py > $O/tests_f4d3.log 2>&1 || { tail -30 $O/tests_f4d3.log; exit 1; }
tail -1 $O/tests_f4d3.log
bash tools/ab_train.sh $O/ab 2 "YMS_X=0|" "YMS_LIB=$B/libyms_nt_f3.so|" "YMS_LIB=$B/libyms_nt_f4.so|" "YMS_LIB=$B/libyms_nt_d3.so|" "YMS_LIB=$B/libyms_nt_f4d3.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=$B/libyms_nt_f4d3.so|--version ms-s --steps 40"
for r in 1 2; do for v in base nt_f3 nt_f4; do
  if [ $v = base ]; then L=""; else L="YMS_LIB=$B/libyms_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --mode infer --no-cpu-baseline --no-profile --ms-version none --steps 60 --warmup 10 > $O/inf_${v}_$r.json 2> $O/inf_${v}_$r.err
  echo "infer rep $r $v: $(python3 -c "import json;d=json.loads([l for l in open('$O/inf_${v}_$r.json') if l.startswith('{')][-1]);print(d['infer']['value'] if 'infer' in d else d['value'], d.get('infer',{}).get('ms_per_batch'))")"
done; done
