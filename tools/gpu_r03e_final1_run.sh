bash tools/gpu_r03_final1.sh r03e
