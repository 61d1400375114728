#!/bin/bash
# bench.py --raster with several prebuilt library variants (diagnostic)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for t in "$@"; do
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 300 python bench.py --raster --steps 100 --warmup 5 \
      --no-cpu-baseline > gpurun_out/rvar_$t.json 2> gpurun_out/rvar_$t.err || { echo "$t failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rvar_$t.json'));print('$t', d['value'], 'render ms', d['roofline']['avg_launch_ms'])"
done
