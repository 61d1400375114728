"""Diagnostic: how the step kernel's work changes with the step index inside an episode (oracle
side of DESIGN.md §5 "Episode phase").  Runs the bench workload (C3's config and bench.py's own
hashed action stream) on the ORC_STATS oracle build from a burst reset, and reports per bucket
of steps what decides a wave's cost in the GPU kernel:
  - sweeps: per env solve, and the 64-lane wave's max (32 consecutive envs, per substep);
  - the share of solves at the sweep cap;
  - merged envs (a cross-island contact: the wave runs the cross rows, cp_physics.h sweeps());
  - waves whose ground-cart rows are not all +z (the wave runs the generic rows, not isl_row_ez).
Pair to tools/step_profile.py (GPU time per step index).

usage: python tools/episode_phase.py [--envs 1024] [--steps 199] [--bucket 5] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=199, help="< the 200-step episode (no autoreset inside)")
    ap.add_argument("--bucket", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    from row_classes import build_stats_oracle
    os.environ["ORC_LIB_OVERRIDE"] = build_stats_oracle()
    import ctypes as C
    import bench
    from cartpoleplusplus_amd import abi, native
    from oracle import oracle as O

    B, R, T = a.envs, 3, a.steps
    assert B % 32 == 0 and T < bench.WINDOW
    cfg = native.default_config(num_envs=B, action_repeats=R, steps_per_repeat=1, max_episode_len=bench.WINDOW,
                                initial_force=55.0, autoreset=1, seed=bench.SEED)
    env = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    lib = env.lib
    lib.orc_stats_open.argtypes = [C.c_char_p]
    acts = bench.make_actions(False, B, 0, T, bench.SEED, torch.device("cpu")).numpy()
    env.reset()
    path = "/tmp/orc_episode_phase.txt"
    lib.orc_stats_open(path.encode())
    for t in range(T):
        env.step(np.ascontiguousarray(acts[t]))
    lib.orc_stats_open(None)
    # one record per island solve: per step call, env-major, then substep, then island
    r = np.loadtxt(path, dtype=np.int64).reshape(T, B, R, 2, -1)
    cnt, merged, sw, ez = r[..., 0:5], r[:, :, :, 0, 10], r[:, :, :, 0, 11], r[..., 12:17]
    W = B // 32
    wave = lambda x: x.reshape(T, W, 32, *x.shape[2:])  # noqa: E731
    cap = cfg.phys.solver_iterations
    wsw = wave(sw).max(2)                                   # (T, W, R)
    wmerged = wave(merged).max(2)
    gc_notz = ((cnt[..., 0] > 0) & (ez[..., 0] == 0))       # ground-cart rows not +z (per island)
    wnotz = wave(gc_notz).any(axis=(2, 4))                  # (T, W, R)
    out = {"envs": B, "steps": T, "bucket": a.bucket, "workload": "C3 config, bench.py actions, from a burst reset",
           "buckets": []}
    for t0 in range(0, T, a.bucket):
        s = slice(t0, min(T, t0 + a.bucket))
        out["buckets"].append({
            "steps": f"{t0 + 1}-{min(T, t0 + a.bucket)}",
            "env_sweeps": round(float(sw[s].mean()), 2),
            "capped_solves": round(float((sw[s] >= cap).mean()), 4),
            "wave_sweeps": round(float(wsw[s].mean()), 2),
            "merged_envs": round(float(merged[s].mean()), 4),
            "waves_with_merged_env": round(float(wmerged[s].mean()), 3),
            "waves_ground_cart_not_z": round(float(wnotz[s].mean()), 3),
        })
    txt = json.dumps(out)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
