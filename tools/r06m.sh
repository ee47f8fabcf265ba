#!/bin/bash
# round-6 GPU call m: window-grid NMS with 128-member windows (YMS_NMS_WIN=128) -- bit-exact tests, kernel times
set -e
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nms_gpu.py tests/test_bench_workload_gpu.py > $O/tests64.log 2>&1 || { tail -30 $O/tests64.log; exit 1; }
tail -1 $O/tests64.log
YMS_NMS_WIN=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nms_gpu.py tests/test_bench_workload_gpu.py > $O/tests128.log 2>&1 || { tail -30 $O/tests128.log; exit 1; }
tail -1 $O/tests128.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for w in 64 128; do
  YMS_NMS_WIN=$w timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t${w}_$r -o run -- python bench.py --mode infer --nms-overlap 0 --no-cpu-baseline --no-profile --steps 20 --warmup 5 --ms-version none > $O/t${w}_$r.json 2> $O/t${w}_$r.err
  echo "== win $w rep $r"; python tools/nms_kstats.py $O/t${w}_$r/run_results.db | grep -E "wgrid_kernel|per call"
  find $O/t${w}_$r -name "*.db" -delete
done; done
