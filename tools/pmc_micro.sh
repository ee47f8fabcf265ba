set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/micro
timeout -k 10 300 python3 $R/tools/conv_micro.py 20 > $R/gpurun_out/micro/times.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/micro/p1 -o run -- python3 $R/tools/conv_micro.py 2 fwd > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/micro/p2 -o run -- python3 $R/tools/conv_micro.py 2 fwd > /dev/null 2>&1
echo done
