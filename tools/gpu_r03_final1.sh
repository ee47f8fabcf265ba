# round-3 final measurement, part 1: GPU suite, smoke, default bench line, configs[3]/[4], YOLO-MS-L
set -e
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
timeout -k 10 300 python bench.py --version l --no-infer --steps 30 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs3_l_train.json" 2> "$OUT/bench_l.err"
timeout -k 10 300 python bench.py --mode infer --size 1280 --dtype f16 --infer-batch 8 --steps 50 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs4_s1280_f16_infer.json" 2> "$OUT/bench_1280.err"
timeout -k 10 300 python bench.py --version ms-l --no-infer --steps 10 --warmup 3 --no-cpu-baseline --ms-version none > "$OUT/bench_ms_l_train.json" 2> "$OUT/bench_ms_l.err"
echo "config lines done"
