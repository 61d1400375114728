#!/bin/bash
# Round-3 evidence on one MI355X (under gpurun): the default bench line (cpu_baseline + parity legs),
# the fused K = 1 rollout experiment, then the rocprofv3 passes (tools/profile.sh) of the per-step and
# the rollout benches.  Every step under its own time limit; stops at the first failure.
set -u
TAG=${1:-rd3f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json; echo
timeout -k 10 300 python -u bench.py --rollout 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_roll1.json 2> gpurun_out/bench_${TAG}_roll1.err || exit 1
bash tools/profile.sh $TAG || exit 1
python tools/summarize_profile.py $TAG || exit 1
BENCH_ARGS="--rollout 200" bash tools/profile.sh ${TAG}_roll || exit 1
python tools/summarize_profile.py ${TAG}_roll || exit 1
echo "round3 check done"
