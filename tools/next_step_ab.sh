#!/bin/bash
# NEXT_STEP autoreset in the bounds regime with each latency reset layout (the reset list runs on the second
# stream beside the next call's step kernel).  usage (under gpurun): bash tools/next_step_ab.sh OUTTAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-next_step_ab}
mkdir -p "$OUT"
for rep in ${REPS:-1 2}; do for s in ${SHAPES:-latency wide8 wide wide64}; do
  n=ns_${s}_$rep
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --done-on-bounds --autoreset next_step \
      --steps ${STEPS:-100} --warmup ${WARM:-20} --reset-shape $s > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,2), 'step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'), d['config'].get('kernel_shape'))"
done; done
exit 0
