#!/bin/bash
# Small batches: the latency step kernel on the two-lane and the WIDE layout (continuous actions, 300 steps),
# and the B = 1 mirror with the step on the two-lane layout and the reset on WIDE.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-small_b}
mkdir -p "$OUT"
for b in 1 4 16 64 256; do
  for s in latency wide; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-steady-state --no-median --continuous --batch $b --steps 300 \
        --warmup 20 --shape $s > "$OUT/b${b}_$s.json" 2> "$OUT/b${b}_$s.err" || { echo "b$b $s failed"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b${b}_$s.json'));print('B=$b $s', round(d['value']), 'step ms', d['roofline']['avg_launch_ms'])"
  done
done
for rs in "latency wide" "wide wide" "latency latency"; do
  set -- $rs
  echo "mirror step=$1 reset=$2 $(timeout -k 10 120 python tools/mirror_rate.py --shape $1 --reset-shape $2)"
done
