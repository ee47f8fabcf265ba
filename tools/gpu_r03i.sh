mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dwconv_gpu.py > gpurun_out/r03i_t1.log 2>&1 && \
YMS_MICRO_SHAPES=mss YMS_DWM_OPS=fwd_stats,dgrad,fwd YMS_DWM_VARIANTS="old=YMS_DW_TX:32,YMS_DW_BLOCKS:2048,YMS_DW_WAITALL:1;nowait=YMS_DW_TX:32,YMS_DW_BLOCKS:2048;tx=YMS_DW_BLOCKS:2048,YMS_DW_WAITALL:1;grid=YMS_DW_TX:32,YMS_DW_WAITALL:1;new=" timeout -k 10 300 python tools/dw_micro.py > gpurun_out/r03i_dwm.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py -k "b64 and ms" > gpurun_out/r03i_t2.log 2>&1
