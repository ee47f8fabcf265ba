# r04e: full GPU suite on the round-4 tree (aliased MSBlock concat, 1x1 prologue convs), prologue A/B,
# default bench line
set -e
O=gpurun_out/r04e; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests.log)"
bash tools/train_ab.sh r04e/ab_pro_s YMS_PRO 0 1
AB_ARGS="--version ms-s" bash tools/train_ab.sh r04e/ab_pro_mss YMS_PRO 0 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo "bench: $(tail -c 300 $O/bench.json)"
