#!/bin/bash
# CP_SHAPE_LIST against the single-layout reset shapes in the bounds regime: SAME_STEP over the bench's secondary
# window (steps 61-110) and over one holding the max_episode_len boundary (61-260), NEXT_STEP over 21-120 and
# 61-260.  usage (under gpurun): bash tools/list_ab.sh OUTTAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-list_ab}
mkdir -p "$OUT"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --done-on-bounds "$@" \
      > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,2), 'step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'), d['config'].get('kernel_shape'))"
}
for rep in ${REPS:-1 2}; do
  for s in ${SHAPES:-wide64 list latency}; do
    run ss50_${s}_$rep --steps 50 --warmup 60 --reset-shape $s
    run ss200_${s}_$rep --steps 200 --warmup 60 --reset-shape $s
    run ns100_${s}_$rep --autoreset next_step --steps 100 --warmup 20 --reset-shape $s
    run ns200_${s}_$rep --autoreset next_step --steps 200 --warmup 60 --reset-shape $s
  done
done
exit 0
