#!/bin/bash
# Interleaved A/B of bench.py training variants on one box: tools/ab_train.sh OUTDIR REPS "ENV1|ARGS1" "ENV2|ARGS2" ...
OUT=$1; REPS=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    envs=${v%%|*}; args=${v#*|}
    env $envs timeout -k 10 200 python bench.py --mode train --no-cpu-baseline --no-profile --ms-version none --steps 60 --warmup 10 $args \
      > "$OUT/v${i}_r$r.json" 2> "$OUT/v${i}_r$r.err" || { echo "variant $i failed"; exit 1; }
    echo "rep $r v$i [$v]: $(python3 -c "import json;d=json.loads([l for l in open('$OUT/v${i}_r$r.json') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['ms_per_step_median'])")"
    i=$((i+1))
  done
done
