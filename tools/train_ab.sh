#!/bin/bash
# interleaved A/B/.. of one env knob on the training bench: tools/train_ab.sh TAG VAR VALUE...
# (extra bench.py arguments in $AB_ARGS, e.g. AB_ARGS="--version ms-s")
set -e
O=gpurun_out/$1; VAR=$2; shift 2; mkdir -p $O
for rep in 1 2 3; do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 120 python bench.py --mode train --steps 20 --warmup 5 --no-cpu-baseline --no-profile --ms-version none $AB_ARGS \
      > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$VAR=$v', $rep, d['value'], d['ms_per_step'])"
  done
done
