#!/bin/bash
# A/B of prebuilt library variants on the driver's window (--steps 20 --warmup 5) and a 300-step window,
# alternating the variants so box drift hits both alike.
# usage (under gpurun): bash tools/ab_window.sh tag1 tag2 ...   ("base" = the default libcartpole_hip.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for t in "$@"; do
    lib=$R/cartpoleplusplus_amd/libcartpole_hip_$t.so; [ "$t" = base ] && lib=$R/cartpoleplusplus_amd/libcartpole_hip.so
    for a in "--steps 20 --warmup 5" "--steps 300 --warmup 10"; do
      CP_LIB_PATH=$lib timeout -k 10 300 python bench.py $a --no-cpu-baseline > gpurun_out/abw_$t.json 2> gpurun_out/abw_$t.err \
          || { echo "$t failed rc=$?"; tail -3 gpurun_out/abw_$t.err; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/abw_$t.json').read().strip().splitlines()[-1]);print('$t', '$a', d['value'], 'kernel ms', d['roofline']['avg_launch_ms'], 'cycle', d['steady_state']['value'])"
    done
  done
done
