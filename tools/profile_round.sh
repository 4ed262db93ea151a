#!/bin/bash
# Profile the benchmark on the GPU box: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Usage: tools/profile_round.sh r01
# Output under gpurun_out/prof_<round>/; tools/pmc_traffic.py turns it into profiles/*.json.
set -euo pipefail
R=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
BENCH_ARGS="--steps 20 --warmup 5 --kernel-iters 20 --no-cpu-baseline --no-block"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $BENCH_ARGS > "$OUT/bench_trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "film_" -d "$OUT/pmc_$C" -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --kernel-iters 3 --no-cpu-baseline --no-block > "$OUT/pmc_$C.log" 2>&1
done
echo "profile $R done"
