mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "wgrad" > gpurun_out/r03f_t1.log 2>&1 && \
timeout -k 10 300 python tools/wgrad_micro.py s 64 10 > gpurun_out/r03f_wgm_s.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03f_b_ring.json 2> gpurun_out/r03f_b_ring.err && \
YMS_WG_RING=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03f_b_old.json 2> gpurun_out/r03f_b_old.err && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none > gpurun_out/r03f_b_ring2.json 2> gpurun_out/r03f_b_ring2.err
