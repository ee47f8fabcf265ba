#!/bin/bash
# round-6 GPU call o: current-tree per-layer profile (S, MS-S) + default bench line
set -e
O=gpurun_out/r06o; mkdir -p $O
YMS_LAYER_ALL=1 timeout -k 10 200 python -u tools/layer_prof.py s 64 > $O/layers_s.txt 2>&1
YMS_LAYER_ALL=1 timeout -k 10 200 python -u tools/layer_prof.py ms-s 64 > $O/layers_ms_s.txt 2>&1
timeout -k 10 300 python -u bench.py --ms-version none > $O/bench.json 2> $O/bench.err
echo done
