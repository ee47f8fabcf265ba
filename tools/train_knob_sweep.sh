#!/bin/bash
# A/B of the wgrad knobs on the training bench (run through gpurun from the repo root):
#   tools/train_knob_sweep.sh TAG
# one bench process per setting, each under its own time limit; stops at the first failure
set -e
O=gpurun_out/$1; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --mode train --steps 20 --warmup 5 --no-cpu-baseline --no-profile \
    > $O/$name.json 2> $O/$name.err
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run base YMS_WG_WPC=4
run wpc2 YMS_WG_WPC=2
run wpc3 YMS_WG_WPC=3
run wpc6 YMS_WG_WPC=6
run var1 YMS_WG_VARIANT=1
run var2 YMS_WG_VARIANT=2
run var3 YMS_WG_VARIANT=3
run base2 YMS_WG_WPC=4
