#!/bin/bash
# Round-5 GPU sessions (under gpurun): every step under its own time limit, stops at the first failure.
#   bash tools/round5.sh <tag> <steps...>   steps: suite | smoke | bench | bench20 | prof | pmc | c5
set -u
TAG=${1:-rd5}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for step in "$@"; do
  case $step in
  suite)
    bash tools/gpu_tests.sh $TAG || exit 1 ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
    tail -1 gpurun_out/smoke_$TAG.log ;;
  bench)
    timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
    tail -c 600 gpurun_out/bench_$TAG.json; echo ;;
  bench20)
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.json 2> gpurun_out/bench20_$TAG.err || { echo "bench20 rc=$?"; tail -5 gpurun_out/bench20_$TAG.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench20_$TAG.json'));print('k20', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('nonfinite_envs'))" ;;
  prof)
    bash tools/prof_quick.sh $TAG > gpurun_out/prof_$TAG.txt 2>&1 || { echo "prof rc=$?"; tail -5 gpurun_out/prof_$TAG.txt; exit 1; }
    head -12 gpurun_out/prof_$TAG.txt ;;
  pmc)
    STEPS=200 timeout -k 10 1200 bash tools/profile.sh $TAG > gpurun_out/pmc_$TAG.txt 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc_$TAG.txt; exit 1; } ;;
  c5)
    timeout -k 10 300 python -u bench.py --raster --no-cpu-baseline > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo "c5 rc=$?"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));print('C5', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
