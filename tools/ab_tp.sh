#!/bin/bash
# Round-5 A/B of the lean structure loops in the throughput step kernel (under gpurun): the GPU suite on the
# build, then C3 (300 steps) and the driver's 20-step window for each variant library.
set -u
bash tools/gpu_tests.sh ${TAG:-rd5h} || exit 1
bash tools/variant_bench.sh "$@" || exit 1
for t in "$@"; do
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline > gpurun_out/k20_$t.json 2> gpurun_out/k20_$t.err || { echo "k20 $t failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/k20_$t.json'));print('k20 $t', d['value'], 'kernel ms', d['roofline']['avg_launch_ms'])"
done
