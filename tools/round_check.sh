#!/bin/bash
# End-of-round check on a GPU box (run through gpurun from the repo root): tools/round_check.sh TAG
# full GPU suite, smoke(), the default bench line and the configs[3] / configs[4] / MS-L lines.
set -e
TAG=${1:-check}
O=gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || true
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || true
tail -1 $O/smoke.log
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 240 python bench.py --mode train --version l --steps 30 --warmup 5 --no-cpu-baseline --ms-version none > $O/bench_configs3_l_train.json 2> $O/l.err
timeout -k 10 300 python bench.py --mode train --version ms-l --steps 20 --warmup 5 --no-cpu-baseline --ms-version none > $O/bench_ms_l_train.json 2> $O/msl.err
timeout -k 10 240 python bench.py --mode infer --size 1280 --dtype f16 --infer-batch 8 --no-cpu-baseline --ms-version none > $O/bench_configs4_s1280_f16_infer.json 2> $O/c4.err
for f in $O/bench*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
