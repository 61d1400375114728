#!/bin/bash
# C5 (raster) bench of prebuilt library variants: render kernel ms and env-steps/s.
# usage (under gpurun): bash tools/variant_c5.sh tag1 tag2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for t in "$@"; do
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 300 python bench.py --raster --steps 200 --warmup 10 --no-median --no-steady-state \
      --no-cpu-baseline > gpurun_out/c5_$t.json 2> gpurun_out/c5_$t.err || { echo "$t failed rc=$?"; tail -3 gpurun_out/c5_$t.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_$t.json'));r=d['roofline'];print('$t', d['value'], 'render ms', r['avg_launch_ms'], 'frac', r['frac'], 'step ms', r['step_kernel_avg_ms'])"
done
