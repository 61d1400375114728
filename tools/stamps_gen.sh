#!/bin/bash
# Stamp runs (a diagnostic build given as CP_LIB_PATH) of the latency-shaped regimes: B = 1, 256, 4,096 envs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-stamps_gen}
mkdir -p "$OUT"
st() { local n=$1; shift; env "$@" timeout -k 10 180 python tools/stamps.py > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }; echo "$n done"; }
st b1_wide B=1 STEPS=200 WARM=20
st b256_wide B=256 STEPS=100 WARM=20
st c2_wide B=4096 STEPS=60 WARM=20
exit 0
