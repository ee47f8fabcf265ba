#!/bin/bash
# Round 5: kernel traces of the training step replayed from a HIP graph vs eager
O=gpurun_out/r05l; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python3 $R/bench.py --mode train --steps 10 --warmup 4 --no-cpu-baseline --no-profile --ms-version none --graph 0 > $R/$O/eager.json 2> $R/$O/eager.err || exit 3
timeout -k 10 240 python3 $R/bench.py --mode train --steps 10 --warmup 4 --no-cpu-baseline --no-profile --ms-version none --graph 1 > $R/$O/graph.json 2> $R/$O/graph.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tr_eager -o run -- python3 $R/bench.py --mode train --steps 4 --warmup 3 --no-cpu-baseline --no-profile --ms-version none --graph 0 > /dev/null 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tr_graph -o run -- python3 $R/bench.py --mode train --steps 4 --warmup 3 --no-cpu-baseline --no-profile --ms-version none --graph 1 > /dev/null 2>&1 || exit 6
