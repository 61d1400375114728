#!/bin/bash
# The bounds regime's reset list (B = 65,536, SAME_STEP) on the reset-kernel layouts: two-lane latency, WIDE
# (16 lanes per env, 4 envs per wave) and WIDE64 (one env per wave).  Usage: bash tools/reset_ab.sh TAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-reset_ab}
mkdir -p "$OUT"
for rep in 1 2; do
  for s in latency wide wide64; do
    timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --done-on-bounds --steps 100 \
        --warmup 20 --shape throughput --reset-shape $s > "$OUT/bounds_${s}_$rep.json" 2> "$OUT/bounds_${s}_$rep.err" \
        || { echo "$s failed"; tail -3 "$OUT/bounds_${s}_$rep.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bounds_${s}_$rep.json'));r=d['roofline'];print('bounds $s', round(d['value']), 'reset ms', r['reset_kernel_avg_ms'])"
  done
done
