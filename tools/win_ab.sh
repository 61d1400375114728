#!/bin/bash
# A/B of prebuilt library variants (cartpoleplusplus_amd/libcartpole_hip_<tag>.so) on the driver's window
# (--steps 20 --warmup 5: steps 6-25 of the first episode) and a 300-step line, alternating the variants.
# usage (under gpurun): bash tools/win_ab.sh OUTTAG tag1 tag2 ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
run() {  # name tag args...
  local n=$1 t=$2; shift 2
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-steady-state --no-median "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,2), 'M step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'))"
}
for rep in ${REPS:-1 2}; do
  for t in "$@"; do
    run win_${t}_$rep $t --steps 20 --warmup 5
    run c300_${t}_$rep $t --steps 300 --warmup 10
    [ -n "${BOUNDS:-}" ] && run bnd_${t}_$rep $t --done-on-bounds --steps 100 --warmup 20
  done
done
exit 0
