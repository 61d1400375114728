#!/bin/bash
# Bench several prebuilt library variants (cartpoleplusplus_amd/libcartpole_hip_<tag>.so) back to back.
# usage (under gpurun): [BENCH_ARGS="--continuous"] bash tools/variant_bench.sh tag1 tag2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for t in "$@"; do
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 300 python bench.py --steps 300 --warmup 10 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$t.json 2> gpurun_out/var_$t.err || { echo "$t failed rc=$?"; tail -3 gpurun_out/var_$t.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var_$t.json'));print('$t', d['value'], 'kernel ms', d['roofline']['avg_launch_ms'], 'reset ms', d['roofline']['reset_kernel_avg_ms'])"
done
