# Dev: depthwise MFMA weight-gradient A/B over tools/bin/libyms_*.so variants (run through gpurun)
set -e
mkdir -p gpurun_out/dwm
for v in default "$@"; do
  if [ $v = default ]; then L=; else L=tools/bin/libyms_$v.so; fi
  echo "== $v" >> gpurun_out/dwm/ab.log
  YMS_LIB=$L YMS_MICRO_SHAPES=k79 YMS_DWM_OPS=wgrad timeout -k 10 120 python tools/dw_micro.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/dwm/ab.log
done
