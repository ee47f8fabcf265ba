mkdir -p gpurun_out
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_loss_gpu.py tests/test_stem_gpu.py "tests/test_model_gpu.py::test_configs_b64_bf16_layers_vs_fp32" > gpurun_out/r03_t1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_b1.json 2> gpurun_out/r03_b1.err
