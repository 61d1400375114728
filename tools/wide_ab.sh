#!/bin/bash
# A/B of the WIDE layouts (round 6: 16 or 8 lanes per env) against the two-lane latency layout: C2, the bounds
# regime's reset list, a larger latency batch, and the B = 1 gym mirror with its kernel times
# (tools/mirror_rate.py).  Usage: bash tools/wide_ab.sh TAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-wide_ab}
mkdir -p "$OUT"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', d['value'], 'step', r['avg_launch_ms'], 'reset', r['reset_kernel_avg_ms'], d['config']['kernel_shape'])"
}
for rep in ${REPS:-1 2}; do
  for s in ${SHAPES:-latency wide wide8}; do
    run c2_${s}_$rep --continuous --steps 400 --warmup 20 --shape $s
    run bounds_${s}_$rep --done-on-bounds --steps 100 --warmup 20 --shape throughput --reset-shape $s
    run b8192_${s}_$rep --continuous --batch 8192 --steps 300 --warmup 20 --shape $s
    timeout -k 10 120 python tools/mirror_rate.py --shape $s > "$OUT/b1_${s}_$rep.json" 2> "$OUT/b1_${s}_$rep.err" || { echo "b1 $s failed"; exit 1; }
    echo "b1 $s $(cat $OUT/b1_${s}_$rep.json)"
  done
done
