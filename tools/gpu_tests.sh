#!/bin/bash
# The GPU suite as the driver runs it (one process, per-test timeout), log under gpurun_out/.
# usage (under gpurun): bash tools/gpu_tests.sh <tag> [pytest args...]
set -u
TAG=${1:-dev}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
exit $rc
