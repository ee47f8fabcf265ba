bash tools/gpu_r03_final2.sh r03e
