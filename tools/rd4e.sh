#!/bin/bash
# Round-4 render session (under gpurun): the reciprocal checker, the raster tests on each variant
# library, the C5 A/B of base against the variants (twice), then the rocprofv3 passes of the C5 bench.
# usage: bash tools/rd4e.sh "rcp pairs" [profile-tag]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${1:-rcp}
mkdir -p $R/gpurun_out
timeout -k 10 60 tools/micro/rcp_exact > gpurun_out/rcp_exact.json || exit 1
cut -c1-1500 gpurun_out/rcp_exact.json
for v in $V; do
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
      --timeout-method thread tests/test_gpu_raster.py > gpurun_out/raster_$v.log 2>&1 || { echo "$v raster tests failed"; tail -20 gpurun_out/raster_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/raster_$v.log)"
done
bash tools/variant_c5.sh base $V base $V || exit 1
[ -n "${2:-}" ] && STEPS=50 BENCH_ARGS="--raster --no-median --no-steady-state" bash tools/profile.sh $2
exit 0
