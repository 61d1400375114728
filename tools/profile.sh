#!/bin/bash
# Collect the rocprofv3 evidence for bench.py on one MI355X (run under gpurun):
#   pass 0: --kernel-trace --stats            (kernel durations; compare with bench.py's HIP events)
#   pass 1/1b: SQ counters (instructions, waits, LDS, memory)  pass 2: FETCH_SIZE   pass 3: WRITE_SIZE
# Counters are collected in their own runs with --kernel-trace only (never with
# --sys-trace / runtime traces).  Output: gpurun_out/prof_<tag>/...
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
STEPS=${STEPS:-200}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/trace.json" 2> "$OUT/trace.err"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sq" -o run \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    -- $B > "$OUT/sq.json" 2> "$OUT/sq.err"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sq2" -o run \
    --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH \
    -- $B > "$OUT/sq2.json" 2> "$OUT/sq2.err" || echo "sq2 pass failed (see $OUT/sq2.err)"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fetch" -o run --pmc FETCH_SIZE \
    -- $B > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/write" -o run --pmc WRITE_SIZE \
    -- $B > "$OUT/write.json" 2> "$OUT/write.err"
echo "profile passes done: $OUT"
