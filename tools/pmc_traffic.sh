#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes only (HBM traffic per launch) for a library variant.
# usage (under gpurun): bash tools/pmc_traffic.sh <tag> [lib tag]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LIBT=${2:-}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
[ -n "$LIBT" ] && export CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$LIBT.so
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 200 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/trace.json" 2> "$OUT/trace.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fetch" -o run --pmc FETCH_SIZE -- $B > "$OUT/fetch.json" 2> "$OUT/fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/write" -o run --pmc WRITE_SIZE -- $B > "$OUT/write.json" 2> "$OUT/write.err" || exit $?
echo "traffic passes done: $OUT"
