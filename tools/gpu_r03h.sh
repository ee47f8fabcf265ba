mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train"
YMS_WGRAD_STREAM=0 timeout -k 10 300 $B > gpurun_out/r03h_b_ser.json 2> gpurun_out/r03h_b_ser.err && \
timeout -k 10 300 $B > gpurun_out/r03h_b_ovl.json 2> gpurun_out/r03h_b_ovl.err && \
YMS_WGRAD_STREAM=0 timeout -k 10 300 $B --version ms-s > gpurun_out/r03h_bm_ser.json 2> gpurun_out/r03h_bm_ser.err && \
timeout -k 10 300 $B --version ms-s > gpurun_out/r03h_bm_ovl.json 2> gpurun_out/r03h_bm_ovl.err
