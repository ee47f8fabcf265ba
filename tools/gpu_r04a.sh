# r04a: MS family recalibrated to model_zoos.md, SimplifiedYOLOLoss drop-in, dw fusion plan test
set -e
O=gpurun_out/r04a; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_ms_gpu.py tests/test_loss_gpu.py tests/test_dwconv_gpu.py \
  "tests/test_model_gpu.py::test_configs_b64_bf16_layers_vs_fp32" tests/test_train_conditioned_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 300 python bench.py --version ms-s --ms-version none --steps 30 --warmup 10 --no-cpu-baseline > $O/bench_ms_s.json 2> $O/bench_ms_s.err
timeout -k 10 300 python bench.py --version ms-l --ms-version none --steps 10 --warmup 5 --no-cpu-baseline --no-infer > $O/bench_ms_l.json 2> $O/bench_ms_l.err
echo "bench done"
