mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "wgrad or large" > gpurun_out/r03_t5.log 2>&1 && \
timeout -k 10 300 python tools/conv_micro.py 20 > gpurun_out/r03_conv_micro_halo2.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03_b3.json 2> gpurun_out/r03_b3.err && \
YMS_WG_HALO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03_b3_nohalo.json 2> gpurun_out/r03_b3_nohalo.err && \
timeout -k 10 200 python tools/layer_prof.py s 64 > gpurun_out/r03_layer_prof_s_halo.txt 2>&1
