mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dwconv_gpu.py > gpurun_out/r03k_t1.log 2>&1 && \
YMS_MICRO_SHAPES=mss YMS_DWM_OPS=wgrad YMS_DWM_VARIANTS="old=YMS_DW_WG3:0;g4=YMS_DW_WG3_G:4;g8=YMS_DW_WG3_G:8" timeout -k 10 300 python tools/dw_micro.py > gpurun_out/r03k_dwm.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py -k "b64 and ms" tests/test_ms_gpu.py tests/test_train_conditioned_gpu.py > gpurun_out/r03k_t2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train --version ms-s > gpurun_out/r03k_bm_new.json 2> gpurun_out/r03k_bm_new.err && \
YMS_DW_WG3=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train --version ms-s > gpurun_out/r03k_bm_old.json 2> gpurun_out/r03k_bm_old.err
