# Dev A/B: build libyms.so variants with extra compiler defines into tools/bin/ (run on the CPU host):
#   bash tools/ab_lib.sh NAME "-DFOO=0 ..."   -> tools/bin/libyms_NAME.so  (select with YMS_LIB=...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=$2
B=$R/tools/bin/build_$NAME
mkdir -p $B
cd $R/yolo-ms_amd/csrc
for f in conv_igemm conv_direct wgrad_halo wgrad_ring stem dwconv map_eval bn_pool head_nms det_loss preprocess; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics $DEFS -c $f.hip -o $B/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/bin/libyms_$NAME.so $B/*.o -L/opt/rocm/lib -lamdhip64
rm -rf $B
echo built tools/bin/libyms_$NAME.so
