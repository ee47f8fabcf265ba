# Dev (r05z record): PMC passes over tools/dw_micro.py forward (k3@160 c64) for an all-k MFMA forward build
# (tools/bin/libyms_fmall.so from a DW_FM_ALL define that was removed after the measurement)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export YMS_MICRO_SHAPES=k3big YMS_DWM_OPS=fwd
cd /tmp && export TMPDIR=/tmp
for v in fmall; do
  O=$R/gpurun_out/dwpmc_$v; mkdir -p $O
  export YMS_LIB=$R/tools/bin/libyms_$v.so
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/tools/dw_micro.py > /dev/null 2>&1
  cd $R && python3 tools/pmc_table.py $O > $O/table.txt && cd /tmp
  find $O -name "*.db" -delete
done
echo done
