mkdir -p gpurun_out
timeout -k 10 300 python tools/layer_prof.py s 64 > gpurun_out/r03p_layers_s.txt 2>&1
