#!/bin/bash
# Round-4 final evidence on one MI355X (under gpurun), every step under its own time limit, stops at the
# first failure:  bash tools/round4_final.sh <tag> [suite|bench]
#   suite: the GPU test suite (as the driver runs it) and smoke()
#   bench: the default bench line (the driver's command) and the C5 raster line
set -u
TAG=${1:-rd4z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
case ${2:-suite} in
suite)
  bash tools/gpu_tests.sh $TAG || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log ;;
bench)
  timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
  tail -c 400 gpurun_out/bench_$TAG.json; echo
  timeout -k 10 300 python -u bench.py --raster --no-cpu-baseline > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo "c5 rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));print('C5', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" ;;
esac
