# r04b: window NMS (tests + latency), recalibrated XS/S (tests, bench), depthwise wgrad2 micro,
# conv tile A/B (NT variants 7, 8) and the small-GEMM ring weight gradient
set -e
O=gpurun_out/r04b; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_nms_gpu.py tests/test_ms_gpu.py \
  "tests/test_model_gpu.py::test_configs_b64_bf16_layers_vs_fp32[ms-s]" \
  -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 120 python tools/nms_bench.py > $O/nms_bench.txt 2>&1
timeout -k 10 300 python bench.py --version ms-s --ms-version none --steps 30 --warmup 10 --no-cpu-baseline > $O/bench_ms_s.json 2> $O/bench_ms_s.err
YMS_MICRO_SHAPES=mss4 YMS_DWM_OPS=wgrad YMS_DWM_VARIANTS="wg2=YMS_DW_WG2:1;tile=YMS_DW_WG2:0" timeout -k 10 120 python tools/dw_micro.py > $O/dw_micro.txt 2>&1
for v in 0 7 8; do
  YMS_NT_VARIANT=$v timeout -k 10 240 python tools/conv_micro.py 20 > $O/conv_micro_v$v.txt 2>&1
  echo "conv_micro v$v done"
done
YMS_WGM_CONFIGS=halo,ring0,ringsmall timeout -k 10 300 python tools/wgrad_micro.py s 64 10 > $O/wgrad_micro_s.txt 2>&1
YMS_WGM_CONFIGS=halo,ring0,ringsmall timeout -k 10 300 python tools/wgrad_micro.py ms-s 64 10 > $O/wgrad_micro_ms_s.txt 2>&1
echo done
