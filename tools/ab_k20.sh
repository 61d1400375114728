#!/bin/bash
# The driver's 20-step window (--steps 20 --warmup 5) for each variant library, twice in alternation.
set -u
for rep in 1 2; do for t in "$@"; do
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline > gpurun_out/k20_$t.json 2> gpurun_out/k20_$t.err || { echo "k20 $t failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/k20_$t.json'));print('k20 $t', d['value'], 'kernel ms', d['roofline']['avg_launch_ms'])"
done; done
