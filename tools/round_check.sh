#!/bin/bash
# Round evidence on one MI355X (run under gpurun): GPU parity suite, the default bench line
# (with cpu_baseline + parity legs), then the rocprofv3 passes of tools/profile.sh.
# usage: bash tools/round_check.sh <tag>
set -u
TAG=${1:-rxx}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
bash tools/profile.sh $TAG || exit $?
