# r04d: prologue restricted to 1x1 consumers: step A/B
set -e
O=gpurun_out/r04d; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/train_ab.sh r04d/ab_pro_s YMS_PRO 0 1
AB_ARGS="--version ms-s" bash tools/train_ab.sh r04d/ab_pro_mss YMS_PRO 0 1
echo done
