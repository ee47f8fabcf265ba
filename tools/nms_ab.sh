# Dev A/B of NMS library variants (sync inference, rocprof kernel trace per variant):
#   bash tools/nms_ab.sh TAG LIB1 LIB2 ...   (LIB = path or "tree")
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in "$@"; do
  N=$(basename $L .so)
  if [ "$L" = tree ]; then unset YMS_LIB; else export YMS_LIB=$GRAFT_REPO_ROOT/$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_$N -o run -- python bench.py --mode infer --nms-overlap 0 --no-cpu-baseline --no-profile --steps 20 --warmup 5 > gpurun_out/${TAG}_$N.json 2> gpurun_out/${TAG}_$N.err
  echo "== $N"; python tools/nms_kstats.py gpurun_out/${TAG}_$N/run_results.db | grep -E "wgrid_kernel|per call"
done
