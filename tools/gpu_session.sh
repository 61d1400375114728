#!/bin/bash
# One GPU session (under gpurun): the GPU suite, smoke, then bench lines given as arguments
# (each "tag|bench args"), every step under its own time limit; stops at the first failure.
# usage: [PYTEST_K="expr"] [SKIP_TESTS=1] bash tools/gpu_session.sh <tag> ["name|--bench --args" ...]
set -u
TAG=${1:-dev}; shift || true
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; cat gpurun_out/smoke_$TAG.log | tail -2; [ $rc -ne 0 ] && exit $rc
fi
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  echo "bench $name: $args"
  timeout -k 10 600 python -u bench.py $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $name rc=$rc"; tail -5 gpurun_out/bench_${TAG}_$name.err; exit $rc; }
  python - "$name" gpurun_out/bench_${TAG}_$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], d["value"], d["unit"], "ms/step", d["ms_per_step"], "kernel", r.get("avg_launch_ms"),
      "reset", r.get("reset_kernel_avg_ms"), "shape", d["config"].get("kernel_shape"),
      "ss", (d.get("steady_state") or {}).get("value"))
PY
done
