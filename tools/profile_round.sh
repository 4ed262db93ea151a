#!/bin/bash
# Profile the aggregation kernels at every BASELINE config shape (tools/prof_kernels.py), a training
# step of every config (tools/prof_train_step.py), the headline layer's training step
# (tools/exp_headline_train.py) and the headline bench command on the GPU box:
# kernel trace + stats, then one PMC pass per counter group (aggregation kernels; the matrix-core
# compress GEMMs and the encoder)
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; <= 8 SQ counters per pass).
# Usage: tools/profile_round.sh <round> ; output under gpurun_out/prof_<round>/, summarised into
# profiles/ by tools/pmc_summary.py.
set -euo pipefail
R=${1:-r03}
ITERS=${ITERS:-20}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
BENCH_ARGS="--steps 20 --warmup 5 --kernel-iters 20 --no-cpu-baseline --configs="
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/bench" -o run --output-format csv \
  -- python3 bench.py $BENCH_ARGS > "$OUT/bench_trace.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 tools/prof_kernels.py "$ITERS" > "$OUT/trace.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/train" -o run --output-format csv \
  -- python3 tools/prof_train_step.py 5 1 2 3 4 --no-fwd > "$OUT/train.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/headline_train" -o run --output-format csv \
  -- python3 tools/exp_headline_train.py 20 > "$OUT/headline_train.log" 2>&1
pass() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "film_" -d "$OUT/pmc_$name" -o run \
    --output-format csv -- python3 tools/prof_kernels.py 5 > "$OUT/pmc_$name.log" 2>&1
}
pass FETCH FETCH_SIZE
pass WRITE WRITE_SIZE
pass SQ1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass SQ2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
pass GRBM GRBM_GUI_ACTIVE GRBM_COUNT
# matrix-core kernels: the split-bf16 compress GEMMs (configs[3] layer shape) and the edge encoder
for op in fwd dgrad wgrad wgrad3; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-include-regex "gemm_n" -d "$OUT/pmc_gemm_$op" -o run --output-format csv -- python3 tools/prof_compress.py 5 $op > "$OUT/pmc_gemm_$op.log" 2>&1
done
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex "encoder" -d "$OUT/pmc_encoder" -o run --output-format csv -- python3 tools/prof_encoder.py 5 > "$OUT/pmc_encoder.log" 2>&1
echo "profile $R done"
