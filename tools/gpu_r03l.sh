mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train --version ms-s"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03l_gpu_tests.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r03l_bm_on1.json 2> gpurun_out/r03l_bm_on1.err && \
YMS_DW_BNRED=0 timeout -k 10 300 $B > gpurun_out/r03l_bm_off1.json 2> gpurun_out/r03l_bm_off1.err && \
timeout -k 10 300 $B > gpurun_out/r03l_bm_on2.json 2> gpurun_out/r03l_bm_on2.err && \
YMS_DW_BNRED=0 timeout -k 10 300 $B > gpurun_out/r03l_bm_off2.json 2> gpurun_out/r03l_bm_off2.err && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --ms-version none > gpurun_out/r03l_b.json 2> gpurun_out/r03l_b.err
