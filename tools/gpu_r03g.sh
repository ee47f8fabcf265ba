mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "wgrad_ring" > gpurun_out/r03g_t1.log 2>&1 && \
YMS_WGM_CONFIGS=halo,ring0,ring3 timeout -k 10 300 python tools/wgrad_micro.py ms-s 64 10 > gpurun_out/r03g_wgm_mss.txt 2>&1 && \
YMS_WG_RING=0 timeout -k 10 300 $B > gpurun_out/r03g_b_old.json 2> gpurun_out/r03g_b_old.err && \
YMS_WG_RING_VAR=3 timeout -k 10 300 $B > gpurun_out/r03g_b_r3.json 2> gpurun_out/r03g_b_r3.err && \
timeout -k 10 300 $B > gpurun_out/r03g_b_r0.json 2> gpurun_out/r03g_b_r0.err && \
YMS_WG_RING=0 timeout -k 10 300 $B --version ms-s > gpurun_out/r03g_bm_old.json 2> gpurun_out/r03g_bm_old.err && \
YMS_WG_RING_VAR=3 timeout -k 10 300 $B --version ms-s > gpurun_out/r03g_bm_r3.json 2> gpurun_out/r03g_bm_r3.err && \
timeout -k 10 300 $B --version ms-s > gpurun_out/r03g_bm_r0.json 2> gpurun_out/r03g_bm_r0.err && \
YMS_WG_RING=0 timeout -k 10 300 $B > gpurun_out/r03g_b_old2.json 2> gpurun_out/r03g_b_old2.err
