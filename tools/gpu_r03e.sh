mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export YMS_MICRO_SHAPES=wg
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "wgrad or large" > gpurun_out/r03_t6.log 2>&1 && \
timeout -k 10 200 python tools/conv_micro.py 20 wgrad > gpurun_out/r03_wg_small.txt 2>&1 && \
YMS_WG_HALO_BIG=1 timeout -k 10 200 python tools/conv_micro.py 20 wgrad > gpurun_out/r03_wg_big.txt 2>&1 && \
YMS_WG_HALO=0 timeout -k 10 200 python tools/conv_micro.py 20 wgrad > gpurun_out/r03_wg_old.txt 2>&1 && \
unset YMS_MICRO_SHAPES && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03_b4_small.json 2> gpurun_out/r03_b4_small.err && \
YMS_WG_HALO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03_b4_old.json 2> gpurun_out/r03_b4_old.err && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03_b4_small2.json 2> gpurun_out/r03_b4_small2.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_data_gpu.py > gpurun_out/r03_t7.log 2>&1
