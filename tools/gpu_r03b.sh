mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/conv_micro.py 20 > gpurun_out/r03_conv_micro.txt 2>&1 && \
timeout -k 10 200 python tools/layer_prof.py s 64 > gpurun_out/r03_layer_prof_s.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_train_conditioned_gpu.py -s > gpurun_out/r03_t2.log 2>&1
