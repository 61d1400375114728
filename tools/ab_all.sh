#!/bin/bash
# A/B of library variants (under gpurun): the GPU suite on the build (skip with SUITE=0), then per variant
# C3 (300 steps), C3 + bounds (SAME_STEP) and C2 (--continuous), each through tools/variant_bench.sh.
set -u
if [ "${SUITE:-1}" = 1 ]; then bash tools/gpu_tests.sh ${TAG:-ab} || exit 1; fi
echo "== C3"; bash tools/variant_bench.sh "$@" || exit 1
echo "== bounds"; BENCH_ARGS="--done-on-bounds" bash tools/variant_bench.sh "$@" || exit 1
echo "== C2"; BENCH_ARGS="--continuous" bash tools/variant_bench.sh "$@" || exit 1
