# Dev: depthwise MFMA weight-gradient check (GPU tests + micro + kernel trace); run through gpurun
set -e
mkdir -p gpurun_out/dwm
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dwconv_gpu.py > gpurun_out/dwm/test.log 2>&1
YMS_MICRO_SHAPES=k79 YMS_DWM_OPS=wgrad timeout -k 10 120 python tools/dw_micro.py > gpurun_out/dwm/micro_on.log 2>&1
export TMPDIR=/tmp
YMS_MICRO_SHAPES=k79 YMS_DWM_OPS=wgrad timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dwm/p_v3 -o run -- python tools/dw_micro.py > gpurun_out/dwm/p_v3.log 2>&1
