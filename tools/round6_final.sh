#!/bin/bash
# Round-6 evidence on the final build (under gpurun): PART=1 the GPU suite, smoke() and the rocprofv3 passes
# (tools/profile.sh); PART=2 the default bench line and the driver's 20-step window.  Usage: PART=n bash
# tools/round6_final.sh TAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rd7z}
O=$R/gpurun_out
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$O/${TAG}_pytest.log" 2>&1
  rc=$?; tail -3 "$O/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1 || { cat "$O/${TAG}_smoke.log"; exit 1; }
  tail -1 "$O/${TAG}_smoke.log"
  bash tools/profile.sh "$TAG" || exit 1
else
  timeout -k 10 900 python bench.py > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || { tail -5 "$O/${TAG}_bench.err"; exit 1; }
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$O/${TAG}_bench20.json" 2> "$O/${TAG}_bench20.err" \
      || { tail -5 "$O/${TAG}_bench20.err"; exit 1; }
  echo "benches done"
fi
