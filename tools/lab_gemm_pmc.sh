# Kernel lab (not product code): PMC passes over the compress GEMMs and the library GEMM of the same
# product at two config shapes (tools/lab_gemm_pmc.py).  Output under gpurun_out/pmc_<shape>_<pass>.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
for shape in ${SHAPES:-cfg1 cfg3}; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_${shape}_1 -o p --output-format csv -- python3 tools/lab_gemm_pmc.py $shape ${VARIANT:-1} > gpurun_out/pmc_${shape}_1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM -d gpurun_out/pmc_${shape}_2 -o p --output-format csv -- python3 tools/lab_gemm_pmc.py $shape ${VARIANT:-1} > gpurun_out/pmc_${shape}_2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_${shape}_3 -o p --output-format csv -- python3 tools/lab_gemm_pmc.py $shape ${VARIANT:-1} > gpurun_out/pmc_${shape}_3.log 2>&1
done
echo ok
