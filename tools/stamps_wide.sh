#!/bin/bash
# Stamp runs of the WIDE narrowphase split (box selection + broadphase + cache, box_box, gather + rows)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-stamps_wide}
mkdir -p "$OUT"
export CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_stamps.so
st() { local n=$1; shift; env "$@" timeout -k 10 180 python tools/stamps.py > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }; echo "$n done"; }
st b1_lat B=1 STEPS=200 WARM=20 SHAPE=latency,latency
st b1_wide B=1 STEPS=200 WARM=20 SHAPE=wide,wide
st c2_lat B=4096 STEPS=60 WARM=20 SHAPE=latency,latency
st c2_wide B=4096 STEPS=60 WARM=20 SHAPE=wide,wide
st bounds_lat B=65536 STEPS=40 WARM=20 BOUNDS=1 SHAPE=throughput,latency
st bounds_wide B=65536 STEPS=40 WARM=20 BOUNDS=1 SHAPE=throughput,wide
