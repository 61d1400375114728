#!/bin/bash
# SAME_STEP bounds regime over a window holding the max_episode_len boundary (steps 61-260), per reset layout
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-bounds_window_ab}
mkdir -p "$OUT"
for rep in ${REPS:-1}; do for s in ${SHAPES:-latency wide wide64}; do
  n=ss_${s}_$rep
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --done-on-bounds \
      --steps ${STEPS:-200} --warmup ${WARM:-60} --reset-shape $s > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,2), 'step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'), d['config'].get('kernel_shape'))"
done; done
exit 0
