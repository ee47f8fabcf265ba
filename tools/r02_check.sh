#!/bin/bash
# Round-2 re-measure on a GPU box (run through gpurun from the repo root):
# GPU tests, default bench line, YOLO-MS-S bench line and its rocprof kernel stats.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  echo "tests done"; tail -2 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
echo "bench done"; cat "$OUT/bench_default.json"
timeout -k 10 300 python bench.py --version ms-s --steps 30 --warmup 10 --no-cpu-baseline > "$OUT/bench_ms_s.json" 2> "$OUT/bench_ms_s.err"
echo "ms-s bench done"; cat "$OUT/bench_ms_s.json"
timeout -k 10 300 python tools/layer_prof.py ms-s 64 > "$OUT/layer_prof_ms_s.txt" 2>&1
echo "layer prof done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ms_s_stats" -o run -- \
  python3 "$ROOT/bench.py" --version ms-s --mode train --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/ms_s_prof.json" 2>&1
cd "$ROOT"
python3 tools/rocprof_summary.py stats "$OUT/ms_s_stats/run_kernel_stats.csv" > "$OUT/ms_s_stats_summary.txt"
find "$OUT" -name "*.db" -delete
for f in $(find "$OUT" -name "*.csv" -size +4M); do head -c 200000 "$f" > "$f.head"; rm -f "$f"; done
echo "all done"
