mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-infer --ms-version none --mode train --version ms-s"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dwconv_gpu.py tests/test_ms_gpu.py tests/test_train_conditioned_gpu.py > gpurun_out/r03m_t1.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py -k "b64 and ms" > gpurun_out/r03m_t2.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r03m_bm_on1.json 2> gpurun_out/r03m_bm_on1.err && \
YMS_DW_BNIN=0 timeout -k 10 300 $B > gpurun_out/r03m_bm_off1.json 2> gpurun_out/r03m_bm_off1.err && \
timeout -k 10 300 $B > gpurun_out/r03m_bm_on2.json 2> gpurun_out/r03m_bm_on2.err && \
YMS_DW_BNIN=0 timeout -k 10 300 $B > gpurun_out/r03m_bm_off2.json 2> gpurun_out/r03m_bm_off2.err
