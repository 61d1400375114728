#!/bin/bash
# One perf iteration on the GPU box: GPU suite, C3 / C2 / bounds bench lines, stamps (bounds).
# usage (under gpurun): bash tools/perf_check.sh <tag>
set -u
TAG=${1:-dev}
mkdir -p gpurun_out
bash tools/gpu_tests.sh $TAG || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b3_$TAG.json 2> gpurun_out/b3_$TAG.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --continuous > gpurun_out/b2_$TAG.json 2> gpurun_out/b2_$TAG.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --done-on-bounds --steps 200 > gpurun_out/bb_$TAG.json 2> gpurun_out/bb_$TAG.err || exit $?
if [ -f cartpoleplusplus_amd/libcartpole_hip_stamps.so ]; then
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_stamps.so BOUNDS=1 STEPS=60 timeout -k 10 300 python tools/stamps.py > gpurun_out/stb_$TAG.json 2>/dev/null || exit $?
fi
python - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for k in ("b3", "b2", "bb"):
    d = json.load(open(f"gpurun_out/{k}_{t}.json"))
    print(k, "value", d["value"], "ms/step", d["ms_per_step"], "kernel", d["roofline"]["avg_launch_ms"],
          "reset", d["roofline"]["reset_kernel_avg_ms"], "steady", d["steady_state"]["value"])
try:
    s = json.load(open(f"gpurun_out/stb_{t}.json"))["reset_kernel"]
    print("reset stamps", {k: round(v) for k, v in s["cycles_per_wave_substep"].items()}, "sweeps",
          round(s["sweeps_per_wave_substep"], 1), "cyc/sweep", round(s["cycles_per_sweep"]))
except Exception as e:
    print("no stamps", e)
PY
