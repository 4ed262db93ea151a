set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_cf; mkdir -p $O
for m in 0 2; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex compress_film -d $O/m${m}_a -o run --output-format csv -- python3 tools/prof_compress_fused.py $m 5 > $O/m${m}_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --kernel-include-regex compress_film -d $O/m${m}_b -o run --output-format csv -- python3 tools/prof_compress_fused.py $m 5 > $O/m${m}_b.log 2>&1
done
echo done
