"""Diagnostic: what would binning envs into waves by cost buy the step kernel?  

The step kernel runs 32 envs per 64-lane wave, and a wave pays, in every substep, its slowest env's
PGS sweeps and the wave-uniform slow paths of any of its envs (a merged env: the cross rows; a
ground-cart manifold that is not +z: the generic ground rows).  This replays the bench workload
(C3's config, bench.py's hashed actions, from a burst reset) on the ORC_STATS oracle build and prices
the waves of every step under several env->wave maps:

  natural     env i in wave i // 32 (the kernel as built)
  prev-K      envs sorted by a key taken from the step k steps earlier (re-binned every k steps),
              then cut into waves of 32: the key is (merged, non-+z ground rows, max sweeps)
  perfect     sorted by the step's own max sweeps: an upper bound no predictor reaches

Cost of a wave-substep (cycles, from the stamp builds of DESIGN.md §5): NARROW for the narrowphase
and row setup, plus max-sweeps x SWEEP x (1 + MERGED_X if any env merged) x (1 + NOTZ_X if any
non-+z ground rows).  Reports wave-sweeps and the modelled cost relative to natural, per step bucket.

usage: python tools/binning_sim.py [--envs 2048] [--steps 199] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

NARROW, SWEEP, MERGED_X, NOTZ_X = 40e3, 3.6e3, 0.6, 0.25


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=199)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import ctypes as C

    import torch
    from row_classes import build_stats_oracle
    os.environ["ORC_LIB_OVERRIDE"] = build_stats_oracle()
    import bench
    from cartpoleplusplus_amd import abi, native
    from oracle import oracle as O

    B, R, T = a.envs, 3, a.steps
    cfg = native.default_config(num_envs=B, action_repeats=R, steps_per_repeat=1, max_episode_len=bench.WINDOW,
                                initial_force=55.0, autoreset=1, seed=bench.SEED)
    env = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    env.lib.orc_stats_open.argtypes = [C.c_char_p]
    acts = bench.make_actions(False, B, 0, T, bench.SEED, torch.device("cpu")).numpy()
    env.reset()
    path = "/tmp/orc_binning.txt"
    env.lib.orc_stats_open(path.encode())
    for t in range(T):
        env.step(np.ascontiguousarray(acts[t]))
    env.lib.orc_stats_open(None)
    r = np.loadtxt(path, dtype=np.int64).reshape(T, B, R, 2, -1)
    cnt, merged, sw, ez = r[..., 0:5], r[:, :, :, 0, 10] > 0, r[..., 11].max(-1), r[..., 12:17]
    notz = ((cnt[..., 0] > 0) & (ez[..., 0] == 0)).any(-1)          # (T, B, R)
    # per env and step: the key a binning pass would see
    msw = sw.max(-1)                                                 # (T, B) max sweeps over substeps
    mer = merged.any(-1)
    nz = notz.any(-1)

    def cost(order, t):
        """cycles of step t's waves when envs run in `order` (a permutation of 0..B-1)."""
        s, m, z = sw[t][order], merged[t][order], notz[t][order]       # (B, R)
        W = B // 32
        ws = s.reshape(W, 32, R).max(1)
        wm = m.reshape(W, 32, R).any(1)
        wz = z.reshape(W, 32, R).any(1)
        c = NARROW + ws * SWEEP * (1 + MERGED_X * wm) * (1 + NOTZ_X * wz)
        return float(c.sum()), float(ws.sum()), float(wm.mean()), float(wz.mean())

    def key_order(t):
        k = mer[t].astype(np.int64) * 4096 + nz[t].astype(np.int64) * 1024 + msw[t]
        return np.argsort(-k, kind="stable")

    natural = np.arange(B)
    policies = {"natural": lambda t, st: natural}
    for k in (1, 5, 20):
        def pol(t, st, k=k):
            if t == 0:
                return natural
            if (t - 1) % k == 0 or "o" not in st:
                st["o"] = key_order(t - 1)
            return st["o"]
        policies[f"prev-{k}"] = pol
    policies["perfect"] = lambda t, st: np.argsort(-(mer[t] * 4096 + nz[t] * 1024 + msw[t]), kind="stable")
    res = {}
    for name, pol in policies.items():
        st = {}
        res[name] = np.array([cost(pol(t, st), t) for t in range(T)])   # (T, 4)
    buckets = [(0, 10), (10, 25), (25, 75), (75, 100), (100, T)]
    out = {"envs": B, "steps": T, "model": {"narrow": NARROW, "sweep": SWEEP, "merged_x": MERGED_X, "notz_x": NOTZ_X},
           "buckets": []}
    for lo, hi in buckets:
        row = {"steps": f"{lo + 1}-{hi}"}
        base = res["natural"][lo:hi, 0].sum()
        for name, v in res.items():
            row[name] = {"cost_rel": round(float(v[lo:hi, 0].sum() / base), 3),
                         "wave_sweeps": round(float(v[lo:hi, 1].mean() / (B // 32) / R), 1),
                         "waves_merged": round(float(v[lo:hi, 2].mean()), 3),
                         "waves_notz": round(float(v[lo:hi, 3].mean()), 3)}
        out["buckets"].append(row)
    out["episode"] = {name: round(float(v[:, 0].sum() / res["natural"][:, 0].sum()), 3) for name, v in res.items()}
    out["env_sweeps_mean"] = round(float(sw.mean()), 2)
    txt = json.dumps(out, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(json.dumps(out) + "\n")
    print(txt)


if __name__ == "__main__":
    main()
