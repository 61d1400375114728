#!/bin/bash
# A/B of prebuilt library variants (cartpoleplusplus_amd/libcartpole_hip_<tag>.so) on the latency-shaped regimes:
# C2 (4,096 envs, WIDE step kernel), the bounds regime's reset lists (WIDE64 reset kernel), 256 envs and the
# B = 1 gym mirror, alternating the variants.  usage (under gpurun): bash tools/lib_ab.sh OUTTAG tag1 tag2 ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
run() {  # name tag args...
  local n=$1 t=$2; shift 2
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-steady-state --no-median "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3), 'M step', r['avg_launch_ms'], 'reset', r.get('reset_kernel_avg_ms'), d['config'].get('kernel_shape'))"
}
for rep in ${REPS:-1 2}; do
  for t in "$@"; do
    run c2_${t}_$rep $t --continuous --steps 400 --warmup 20
    run bnd_${t}_$rep $t --done-on-bounds --steps 100 --warmup 20
    run b256_${t}_$rep $t --continuous --batch 256 --steps 300 --warmup 20
    CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 120 python tools/mirror_rate.py \
        > "$OUT/b1_${t}_$rep.json" 2> "$OUT/b1_${t}_$rep.err" || { echo "b1 $t failed"; exit 1; }
    echo "b1_${t}_$rep $(cat $OUT/b1_${t}_$rep.json)"
  done
done
exit 0
