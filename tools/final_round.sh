#!/bin/bash
# End-of-round measurement on one GPU box (run through gpurun from the repo root):
# full GPU test suite, default bench line, configs[3]/[4] and YOLO-MS lines, rocprof stats + PMC
# traffic of the default train/infer commands.  Outputs under gpurun_out/<tag>/.
set -e
TAG=${1:-r02c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
timeout -k 10 300 python bench.py --version l --no-infer --steps 30 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs3_l_train.json" 2> "$OUT/bench_l.err"
timeout -k 10 300 python bench.py --mode infer --size 1280 --dtype f16 --infer-batch 8 --steps 50 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs4_s1280_f16_infer.json" 2> "$OUT/bench_1280.err"
timeout -k 10 300 python bench.py --version ms-l --no-infer --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_ms_l_train.json" 2> "$OUT/bench_ms_l.err"
echo "config lines done"
bash tools/profile_round.sh $TAG
echo "profile done"
