#!/bin/bash
# Instruction-cache counters for the step and reset kernels (one --pmc pass per workload,
# kernel trace only).  usage (under gpurun): bash tools/pmc_icache.sh <tag>
set -u
TAG=${1:-ic}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ic_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c3" -o run --pmc $C \
    -- python3 $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo "c3 pass rc=$?"; tail -3 "$OUT/c3.err"; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/bb" -o run --pmc $C \
    -- python3 $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline --done-on-bounds > "$OUT/bb.json" 2> "$OUT/bb.err" || { echo "bb pass rc=$?"; tail -3 "$OUT/bb.err"; exit 1; }
echo done
