#!/usr/bin/env python3
"""The README's random-agent deciles (README.md:76-92) under every [ext] alternative of the physics
model.

    python tools/deciles_alternatives.py [--episodes 100] [--precisions f32,f64] [--out FILE]

For the default model and each alternative of tools/sensitivity.py (oracle switches: split islands,
ERP 1.0 / 0.8, relative margin, no / full warm start, velocity friction direction, persistent
manifold (+ no warm start), no early exit, 10 iterations), in fp32 and fp64, the four README
configurations run as tools/deciles.py runs them (R = 2, bounds termination on, <= 200 steps, one
uniform action per cart and step from the list, 100 envs = 100 episodes, Philox bumps seed 0).
Per case: the deciles, the mean, and the log-distance to the README's deciles
(mean |ln(ours / README)| over the 11 deciles).  For the F_init 55 cases the pole's state where each
episode ends (the step where it terminates, or step 200) is classified to test DESIGN.md §3's
hypothesis "the cart slides out, the pole lands upright on its 1 cm base":
  on_cart_upright   pole centre within 2 cm of its on-cart height (0.35 m), tilt < 0.35 rad
  on_ground_upright pole centre within 2 cm of its on-ground height (0.30 m), tilt < 0.35 rad
  toppled           tilt >= 0.35 rad (the bounds check's angle)
  off_plate         pole centre below 0.25 m with tilt < 0.35 (fell off the 3 m ground box)
Oracle only (test infrastructure).  A loose check: the README measured the upstream single-pair env.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from cartpoleplusplus_amd import abi  # noqa: E402
from oracle import oracle as O  # noqa: E402

from deciles import CASES, MAX_LEN, README  # noqa: E402
from sensitivity import ALTERNATIVES  # noqa: E402


def tilt(q):
    """angle between the pole's body z axis and world z, from quaternions (..., 4) xyzw"""
    x, y = q[..., 0], q[..., 1]
    cz = 1.0 - 2.0 * (x * x + y * y)
    return np.arccos(np.clip(cz, -1.0, 1.0))


def classify(pose):
    """pose (n, 7) of pole 1 (xyz, quat) -> counts per class"""
    z, th = pose[:, 2], tilt(pose[:, 3:7])
    up = th < 0.35
    out = {"on_cart_upright": int((up & (np.abs(z - 0.35) < 0.02)).sum()),
           "on_ground_upright": int((up & (np.abs(z - 0.30) < 0.02)).sum()),
           "toppled": int((~up).sum()),
           "off_plate": int((up & (z < 0.25)).sum())}
    out["other"] = len(z) - sum(out.values())
    return out


def run_case(precision, phys, F, actions, n, seed=0, R=2):
    cfg = O.default_config(num_envs=n, action_repeats=R, initial_force=F, seed=seed, done_on_bounds=1,
                           max_episode_len=MAX_LEN, autoreset=0)
    for k, v in phys.items():
        if isinstance(v, dict):          # array field: {index: value}
            for i, x in v.items():
                getattr(cfg.phys, k)[i] = x
        else:
            setattr(cfg.phys, k, v)
    env = O.Envs(cfg, precision=precision)
    env.reset()
    rng = np.random.default_rng(seed)
    length = np.zeros(n, np.int64)
    final = np.zeros((n, 7), np.float32)
    choice = np.asarray(actions, np.int8)
    for t in range(MAX_LEN):
        a = choice[rng.integers(0, len(choice), (n, 2))]
        obs, _, done = env.step(np.ascontiguousarray(a))
        newly = done.astype(bool) & (length == 0)
        length[newly] = t + 1
        final[newly] = obs[newly, -1, 1]            # pole pose at the last repeat of the ending step
        if (length > 0).all():
            break
    rest = length == 0
    length[rest] = MAX_LEN
    final[rest] = obs[rest, -1, 1]
    return length, final


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--precisions", default="f32,f64")
    ap.add_argument("--only", default=None, help="comma list of alternative names (default: all + default)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    alts = {"default": ("the model as built (DESIGN.md §3)", {})}
    alts.update({k: v for k, v in ALTERNATIVES.items()})
    # diagnostic, not a model alternative: the carts with the ground's default friction instead of the
    # URDF's <lateral_friction value="0.0"/> (models/cart.urdf): does a cart that grips its pole tip it over?
    alts["diag_cart_friction_0.5"] = ("DIAGNOSTIC (not a reading of the fork): cart lateral friction 0.5 instead "
                                      "of cart.urdf's 0.0, so the pole's base grips its cart",
                                      {"friction": {abi.CP_BODY_CART: 0.5, abi.CP_BODY_CART2: 0.5}})
    if a.only:
        keep = set(a.only.split(","))
        alts = {k: v for k, v in alts.items() if k in keep}
    out = {"note": "README.md:76-92 measured the upstream single-pair env (loose check); oracle runs of this model "
                   "with bounds termination on, R = 2, 100 envs = 100 episodes",
           "episodes": a.episodes, "readme": README, "alternatives": {}}
    for name, (desc, phys) in alts.items():
        for prec in a.precisions.split(","):
            key = f"{name}/{prec}"
            row = {"description": desc, "precision": prec, "cases": {}}
            dist = []
            for F, acts in CASES:
                case = f"F{int(F)}/actions={','.join(map(str, acts))}"
                L, final = run_case(prec, phys, F, acts, a.episodes)
                d = np.percentile(L, np.linspace(0, 100, 11))
                ld = float(np.mean(np.abs(np.log(d / np.asarray(README[case], np.float64)))))
                dist.append(ld)
                c = {"deciles": [round(float(x), 2) for x in d], "mean": round(float(L.mean()), 2),
                     "log_dist_to_readme": round(ld, 3)}
                if F > 0:
                    c["pole_at_episode_end"] = classify(final)
                row["cases"][case] = c
            row["mean_log_dist"] = round(float(np.mean(dist)), 3)
            out["alternatives"][key] = row
            print(key, row["mean_log_dist"], {k: (v["deciles"][5], v.get("pole_at_episode_end"))
                                              for k, v in row["cases"].items()}, flush=True)
    rank = sorted(out["alternatives"].items(), key=lambda kv: kv[1]["mean_log_dist"])
    out["ranking"] = [(k, v["mean_log_dist"]) for k, v in rank]
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
