#!/bin/bash
# Quick per-kernel durations of bench.py under rocprofv3 (kernel trace + stats only).
# usage (under gpurun): bash tools/prof_quick.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q}; shift || true
OUT=$R/gpurun_out/pq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]; n = n[:n.find("(")] if "(" in n else n
    print(f"{n[:60]:60s} calls {int(r['Calls']):6d} avg_us {float(r['AverageNs'])/1e3:9.2f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
