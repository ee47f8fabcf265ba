# r04c: prologue conv (yms_conv_fwd_pro) parity + step A/B, NMS kernel breakdown
set -e
O=gpurun_out/r04c; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_pro_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests.log)"
bash tools/train_ab.sh r04c/ab_pro_s YMS_PRO 0 1
AB_ARGS="--version ms-s" bash tools/train_ab.sh r04c/ab_pro_mss YMS_PRO 0 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/nmsprof -o run -- python tools/nms_bench.py > $O/nms_bench_prof.txt 2>&1
echo done
