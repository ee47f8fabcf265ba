mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_gpu.py > gpurun_out/r03_t3.log 2>&1
rc=$?
echo "conv tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_micro.py 20 > gpurun_out/r03_conv_micro_halo.txt 2>&1 && \
YMS_WG_HALO=0 timeout -k 10 300 python tools/conv_micro.py 20 > gpurun_out/r03_conv_micro_nohalo.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_model_gpu.py::test_configs_b64_bf16_layers_vs_fp32" > gpurun_out/r03_t4.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/r03_b2.json 2> gpurun_out/r03_b2.err && \
YMS_WG_HALO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/r03_b2_nohalo.json 2> gpurun_out/r03_b2_nohalo.err
