#!/bin/bash
# One GPU iteration: parity tests, a short bench, and the stamp breakdown.
# usage (under gpurun): bash tools/gpu_check.sh <tag> [bench args...]
set -u
TAG=${1:-dev}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value', d['value'], 'kernel ms', d['roofline']['avg_launch_ms'], 'ms/step', d['ms_per_step'])"
if [ -f cartpoleplusplus_amd/libcartpole_hip_stamps.so ]; then
  CP_LIB_PATH=$R/cartpoleplusplus_amd/libcartpole_hip_stamps.so timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps_$TAG.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/stamps_$TAG.json'))['step_kernel'];print(json.dumps(d['cycles_per_wave_substep']), 'sweeps', round(d['sweeps_per_wave_substep'],1), 'cyc/sweep', round(d['cycles_per_sweep']))"
fi
