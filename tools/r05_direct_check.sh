#!/bin/bash
# Round 5 dev check: the direct small-channel 3x3 kernel's GPU tests, then the conv microbenchmark
# of its layers for the tree's library and any A/B libraries named after the tag
# (tools/bin/libyms_<name>.so), only after a clean or assertion-only test exit.
T=${1:-r05b}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_direct_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_direct_tests.log 2>&1
rc=$?
if [ $rc -le 1 ]; then
  for lib in tree "$@"; do
    if [ $lib = tree ]; then L=; else L=tools/bin/libyms_$lib.so; fi
    echo "== $lib" >> gpurun_out/${T}_conv_micro.txt
    YMS_LIB=$L YMS_MICRO_SHAPES=direct timeout -k 10 300 python tools/conv_micro.py 30 >> gpurun_out/${T}_conv_micro.txt 2>&1 || exit 3
  done
fi
exit $rc
