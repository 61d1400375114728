#!/bin/bash
# C5: the round-3 small-frame render kernel (CP_RENDER_V1=1) against the current one, same library.
# usage (under gpurun): bash tools/ab_render.sh [reps]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for i in $(seq 1 ${1:-2}); do
  for v in 1 0; do
    CP_RENDER_V1=$v timeout -k 10 300 python bench.py --raster --steps 200 --warmup 10 --no-median --no-steady-state \
        --no-cpu-baseline > gpurun_out/c5v$v.json 2> gpurun_out/c5v$v.err || { echo "v1=$v failed"; tail -3 gpurun_out/c5v$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/c5v$v.json'));r=d['roofline'];print('render_v1=$v', d['value'], 'render ms', r['avg_launch_ms'], 'frac', r['frac'], 'step ms', r['step_kernel_avg_ms'])"
  done
done
