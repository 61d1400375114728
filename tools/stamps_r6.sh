#!/bin/bash
# Round-6 stamp runs (stamp build: python -m cartpoleplusplus_amd.build --stamps): the driver's C3 window
# (steps 6-25 after a burst reset) by slow-path set, and the latency regimes on the two-lane and WIDE layouts.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-stamps_r6}
mkdir -p "$OUT"
export CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_stamps.so
st() { local n=$1; shift; env "$@" timeout -k 10 180 python tools/stamps.py > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }; echo "$n done"; }
st c3_window B=65536 STEPS=20 WARM=5
st c3_late B=65536 STEPS=20 WARM=150
st b1_lat B=1 STEPS=200 WARM=20 SHAPE=latency,latency
st b1_wide B=1 STEPS=200 WARM=20 SHAPE=wide,wide
st c2_lat B=4096 STEPS=60 WARM=20 SHAPE=latency,latency
st c2_wide B=4096 STEPS=60 WARM=20 SHAPE=wide,wide
st bounds_lat B=65536 STEPS=40 WARM=20 BOUNDS=1 SHAPE=throughput,latency
st bounds_wide B=65536 STEPS=40 WARM=20 BOUNDS=1 SHAPE=throughput,wide
