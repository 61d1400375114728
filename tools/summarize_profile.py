#!/usr/bin/env python3
"""Summarize a tools/profile.sh run into profiles/<tag>_pmc.json.

Per kernel: launches, average duration (kernel-trace), SQ counters per launch, and
HBM traffic per launch from FETCH_SIZE / WRITE_SIZE (KiB units).  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B request, i.e. half the
bytes of wide coalesced reads, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is
exact for 16-B streaming stores.  Round 4 calibrated both on the step kernel's own access shape
(4-B per-lane buffer loads / stores over the state SoA, two lanes per env; tools/micro/soa_traffic.hip,
profiles/rd4a_pmc_micro.json): FETCH_SIZE = 0.50 x the bytes read, WRITE_SIZE = 1.00 x the bytes
written, so the same correction holds.  The JSON carries the raw counters too.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def kernel_key(name):
    ns = "cp64::" if "cp64::" in name else ""
    if "cp_step_kernel" in name:
        kind = "discrete" if ("<1>" in name or "<1," in name) else "continuous"
        lqr = ",lqr" if ("<1, true" in name or "<0, true" in name) else ""
        return f"{ns}cp_step_kernel<{kind}{lqr}>"
    if "cp_rollout_kernel" in name:
        kind = "discrete" if ("<1>" in name or "<1," in name) else "continuous"
        return f"{ns}cp_rollout_kernel<{kind}>"
    if "cp_reset_kernel" in name:
        return f"{ns}cp_reset_kernel"
    if "cp_render_small2_kernel" in name:
        return "cp_render_small2_kernel"
    for k in ("cp_init_kernel", "cp_mask_to_list_kernel", "cp_render_small_kernel",
              "cp_render_kernel", "cp_raster_table_kernel", "cp_event_kernel"):
        if k in name:
            return k
    for k in ("count_kernel", "free_count_kernel", "plan_kernel", "write_kernel", "sample_kernel"):
        if "cprm::" + k in name:
            return "cp_replay_" + k
    return None


def counters(path):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kernel_key(r["Kernel_Name"])
            if k:
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in tot.items()}, \
        {k: len(v) for k, v in disp.items()}


def durations(path):
    d = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kernel_key(r["Kernel_Name"])
            if k:
                d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return d


def bench_line(path):
    """The JSON line bench.py printed under the profiler (the pass's stdout), or None."""
    if not os.path.exists(path):
        return None
    line = None
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                line = ln
    return json.loads(line) if line else None


def workload_keys(prof_dir):
    """bench.py's PMC_KEYS for the profiled run, from the bench lines every pass printed: the
    counters count only for this workload and this library (bench.py _pmc_match).  Passes that
    disagree (a rebuilt library between passes) leave the summary without keys, so it never matches."""
    keys = []
    for sub in ("trace", "sq", "sq2", "fetch", "write"):
        b = bench_line(os.path.join(prof_dir, sub + ".json"))
        if b is None:
            continue
        c = b.get("config", {})
        keys.append({"batch": c.get("envs_per_gpu"), "repeats": c.get("action_repeats"),
                     "action_kind": c.get("action_kind"), "dtype": b.get("dtype"),
                     "step_shape": c.get("kernel_shape", {}).get("step"),
                     "lib_sha256": b.get("build", {}).get("lib_sha256")})
    if not keys or any(k != keys[0] for k in keys) or any(v is None for v in keys[0].values()):
        return None
    return keys[0]


def main(prof_dir, tag, out_dir):
    res = {"tag": tag, "source": os.path.relpath(prof_dir), "kernels": {}}
    w = workload_keys(prof_dir)
    if w is not None:
        res["workload"] = w
    dur = durations(os.path.join(prof_dir, "trace", "run_kernel_trace.csv"))
    p1 = os.path.join(prof_dir, "sq", "run_counter_collection.csv")   # absent in traffic-only runs
    sq, n_sq = counters(p1) if os.path.exists(p1) else ({}, {})
    p2 = os.path.join(prof_dir, "sq2", "run_counter_collection.csv")
    if os.path.exists(p2):
        sq2, _ = counters(p2)
        for k, cs in sq2.items():
            sq.setdefault(k, {}).update(cs)
    fe, _ = counters(os.path.join(prof_dir, "fetch", "run_counter_collection.csv"))
    wr, _ = counters(os.path.join(prof_dir, "write", "run_counter_collection.csv"))
    for k in dur:
        ent = {"launches": len(dur[k]), "avg_ms": sum(dur[k]) / len(dur[k]),
               "min_ms": min(dur[k]), "max_ms": max(dur[k])}
        if k in sq:
            ent["sq_per_launch"] = sq[k]
            ent["sq_launches"] = n_sq[k]
        if k in fe and k in wr:
            f_kib, w_kib = fe[k].get("FETCH_SIZE", 0.0), wr[k].get("WRITE_SIZE", 0.0)
            ent["FETCH_SIZE_KiB_per_launch"] = f_kib
            ent["WRITE_SIZE_KiB_per_launch"] = w_kib
            ent["hbm_bytes_per_launch"] = int((2 * f_kib + w_kib) * 1024)
        res["kernels"][k] = ent
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{tag}_pmc.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(path)
    return res


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    main(os.path.join(root, "gpurun_out", f"prof_{tag}"), tag, os.path.join(root, "profiles"))
