set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s640 -o run -- python3 $R/bench.py --mode infer --no-cpu-baseline > $O/b640.json 2> $O/b640.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s1280 -o run -- python3 $R/bench.py --size 1280 --dtype f16 --mode infer --infer-batch 8 --no-cpu-baseline > $O/b1280.json 2> $O/b1280.err
cd $R
for s in s640 s1280; do python3 tools/rocprof_summary.py stats $O/$s/run_kernel_stats.csv > $O/${s}_summary.txt; done
find $O -name "*.db" -delete; find $O -name "*trace*.csv" -delete
