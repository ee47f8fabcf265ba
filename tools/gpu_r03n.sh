mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dwconv_gpu.py > gpurun_out/r03n_t1.log 2>&1 && \
YMS_MICRO_SHAPES=mss YMS_DWM_OPS=wgrad YMS_DWM_VARIANTS="old=YMS_DW_WG3:0,YMS_DW_WGK:0;new=" timeout -k 10 300 python tools/dw_micro.py > gpurun_out/r03n_dwm.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py -k "b64 and ms" tests/test_ms_gpu.py tests/test_train_conditioned_gpu.py > gpurun_out/r03n_t2.log 2>&1
