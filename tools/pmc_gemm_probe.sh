cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/tools/gemm_bench.py --prec 1 --cfgs=1 --sk 0 --reps 10 --pool 100000 --sets 8 --sorted --bias-act --shapes 10541,512,512,1,1,1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcA -o run -- $B > $R/gpurun_out/pmcA.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcB -o run -- $B > $R/gpurun_out/pmcB.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcC -o run -- $B > $R/gpurun_out/pmcC.log 2>&1
