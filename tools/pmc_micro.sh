# PMC passes over tools/conv_micro.py (dev tool; run through gpurun from the repo root):
#   bash tools/pmc_micro.sh [op]      op in fwd|dgrad|wgrad|fwd_stats (default fwd)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OP=${1:-fwd}
O=$R/gpurun_out/micro_$OP
mkdir -p $O
timeout -k 10 300 python3 $R/tools/conv_micro.py 20 $OP > $O/times.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/conv_micro.py 2 $OP > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -o run -- python3 $R/tools/conv_micro.py 2 $OP > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/tools/conv_micro.py 2 $OP > /dev/null 2>&1
cd $R && python3 tools/pmc_table.py $O > $O/table.txt
find $O -name "*.db" -delete
echo done
