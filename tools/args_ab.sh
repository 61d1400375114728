#!/bin/bash
# A/B of prebuilt library variants (cartpoleplusplus_amd/libcartpole_hip_<tag>.so) on one bench.py command line,
# alternating the variants.  usage (under gpurun): ARGS="--dtype f64 --steps 300" bash tools/args_ab.sh OUTTAG tag1 tag2 ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in ${REPS:-1 2}; do
  for t in "$@"; do
    n=${t}_$rep
    CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 200 python bench.py --no-cpu-baseline \
        --no-steady-state --no-median ${ARGS:-} > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3), 'M step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'), d['config'].get('kernel_shape'))"
  done
done
exit 0
