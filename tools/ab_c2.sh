#!/bin/bash
# A/B of latency-step-kernel variants (under gpurun): GPU suite on the build, then C2 (--continuous, 4,096
# envs), C2 discrete and the B = 1 gym mirror per variant library.
set -u
bash tools/gpu_tests.sh ${TAG:-rd5i} || exit 1
BENCH_ARGS="--continuous" bash tools/variant_bench.sh "$@" || exit 1
BENCH_ARGS="--batch 4096" bash tools/variant_bench.sh "$@" || exit 1
for t in "$@"; do
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'tools'); import host_boundary as h, json; print('B1 $t', json.dumps(h.gym_mirror(steps=1500)))" || exit 1
done
