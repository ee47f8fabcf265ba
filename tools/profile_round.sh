#!/bin/bash
# Profile the bench command on a GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh r02                       # configs[2] train + configs[1] infer
#   MODES=train EXTRA="--version l" tools/profile_round.sh r02_l            # configs[3]
#   MODES=infer EXTRA="--size 1280 --dtype f16 --infer-batch 8" tools/profile_round.sh r02_s1280   # configs[4]
# 1) rocprofv3 --kernel-trace --stats of bench.py --mode train and --mode infer -> per-kernel times
# 2-4) separate PMC passes (FETCH_SIZE | WRITE_SIZE | MFMA busy) of a short bench run
# Outputs under gpurun_out/<tag>/; copy the summaries into profiles/ afterwards.
set -e
TAG=${1:-r01}
MODES=${MODES:-train infer}
EXTRA=${EXTRA:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for mode in $MODES; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$mode" -o run -- \
    python3 "$ROOT/bench.py" --mode $mode --steps 10 --warmup 3 --no-cpu-baseline --ms-version none $EXTRA > "$OUT/bench_$mode.json" 2> "$OUT/bench_$mode.err"
done
echo "stats done"
# PMC passes per mode (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950)
for mode in $MODES; do
  for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    d=pmc_${mode}_$(echo "$c" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/$d" -o run -- \
      python3 "$ROOT/bench.py" --mode $mode --steps 2 --warmup 1 --no-cpu-baseline --no-profile --ms-version none $EXTRA \
      > "$OUT/$d.json" 2> "$OUT/$d.err"
    echo "pmc $mode $c done"
  done
done
# condense on the box (raw csvs can exceed gpurun's 64 MiB pull limit)
set +e
cd "$ROOT"
for e in "$OUT"/*.err; do echo "== $e"; grep -v "^[EWI]2026\|^[EWI][0-9]\{8\}" "$e" | tail -5; done
ls -la "$OUT"/*/ | head -40
du -sh "$OUT"/* > "$OUT/sizes.txt" || true
for mode in $MODES; do
  python3 tools/rocprof_summary.py stats "$OUT/stats_$mode/run_kernel_stats.csv" > "$OUT/stats_${mode}_summary.txt"
done
python3 tools/rocprof_summary.py traffic "$OUT" > "$OUT/pmc_traffic.json"
find "$OUT" -name "*.db" -delete
for f in $(find "$OUT" -name "*.csv" -size +4M); do head -c 200000 "$f" > "$f.head"; rm -f "$f"; done
echo "summaries done"
