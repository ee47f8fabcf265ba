# Dev: PMC passes over tools/dw_micro.py (k7/k9 weight gradient), run through gpurun from the repo root
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/dwpmc
mkdir -p $O
export YMS_MICRO_SHAPES=k79 YMS_DWM_OPS=wgrad
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d $O/p4 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1 || true
cd $R && python3 tools/pmc_table.py $O > $O/table.txt
find $O -name "*.db" -delete
echo done
