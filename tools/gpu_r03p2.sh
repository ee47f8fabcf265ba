mkdir -p gpurun_out
timeout -k 10 300 python tools/layer_prof.py ms-s 64 > gpurun_out/r03p_layers_ms_s.txt 2>&1
