set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
cd $R
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc1 -o p1 --output-format csv -- python3 tools/lab_gemm_pmc.py cfg3 0 > gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA -d gpurun_out/pmc2 -o p2 --output-format csv -- python3 tools/lab_gemm_pmc.py cfg3 0 > gpurun_out/pmc2.log 2>&1
echo ok
