#!/bin/bash
# Round-6 end-of-round measurement, in parts that each fit one gpurun call (run from the repo root):
#   tools/final_r06.sh tests   -- full GPU suite + default bench line + configs[3] / [4] / YOLO-MS-L lines
#   tools/final_r06.sh prof    -- rocprofv3 stats + PMC traffic of configs[2] / [1] (YOLOv8-s) and YOLO-MS-S
#   tools/final_r06.sh prof_l  -- the same for the YOLO-MS-L training step
set -e
TAG=${TAG:-r06final}
PART=${1:-tests}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
sha256sum yolo-ms_amd/yms/libyms.so > "$OUT/libyms_sha256_$PART.txt"
if [ "$PART" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  echo "bench done"
  timeout -k 10 300 python bench.py --version l --no-infer --steps 30 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs3_l_train.json" 2> "$OUT/bench_l.err"
  timeout -k 10 300 python bench.py --mode infer --size 1280 --dtype f16 --infer-batch 8 --steps 50 --warmup 10 --no-cpu-baseline --ms-version none > "$OUT/bench_configs4_s1280_f16_infer.json" 2> "$OUT/bench_1280.err"
  timeout -k 10 300 python bench.py --version ms-l --no-infer --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_ms_l_train.json" 2> "$OUT/bench_ms_l.err"
  echo "config lines done"
elif [ "$PART" = prof ]; then
  bash tools/profile_round.sh $TAG
  MODES="train infer" EXTRA="--version ms-s" bash tools/profile_round.sh ${TAG}_ms_s
elif [ "$PART" = prof_l ]; then
  MODES="train" EXTRA="--version ms-l" bash tools/profile_round.sh ${TAG}_ms_l
fi
echo "part $PART done"
