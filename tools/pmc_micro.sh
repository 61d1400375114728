#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the step kernel's access shapes (tools/micro/soa_traffic.hip):
# two counter passes, each its own run with --kernel-trace only, then a per-kernel summary
# (counter per launch / algorithmic bytes).  usage (under gpurun): bash tools/pmc_micro.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-micro}
OUT=$R/gpurun_out/pmc_micro_$TAG
mkdir -p $OUT
BIN=$R/tools/micro/soa_traffic
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $BIN 20 > $OUT/plain.jsonl || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- $BIN 20 > $OUT/fetch.out 2> $OUT/fetch.err || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- $BIN 20 > $OUT/write.out 2> $OUT/write.err || exit $?
python3 - $OUT <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
alg = {json.loads(l)["kernel"]: json.loads(l) for l in open(out + "/plain.jsonl")}
res = {}
for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
    fs = glob.glob(f"{out}/{cnt.split('_')[0].lower()}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != cnt:
                continue
            n = r["Kernel_Name"]; n = n[:n.find("(")] if "(" in n else n
            acc[(n, r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (n, d), v in acc.items():
        per[n].append(sum(v))
    for n, v in per.items():
        res.setdefault(n, {})[cnt + "_KiB_per_launch"] = sum(v) / len(v)
for n, d in res.items():
    a = alg.get(n)
    if a:
        d.update(a)
        if a["alg_read_bytes"]:
            d["fetch_over_alg_read"] = round(d.get("FETCH_SIZE_KiB_per_launch", 0) * 1024 / a["alg_read_bytes"], 4)
        if a["alg_write_bytes"]:
            d["write_over_alg_write"] = round(d.get("WRITE_SIZE_KiB_per_launch", 0) * 1024 / a["alg_write_bytes"], 4)
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
