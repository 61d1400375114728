#!/usr/bin/env python3
"""Sensitivity of the pose to every [ext] choice of the physics model.

    python tools/sensitivity.py [--envs 128] [--steps 200] [--precision f64] [--out FILE]

pybullet is not in this container, so "pose drift < 1e-4 vs pybullet" cannot be
measured.  What can be measured is how far each plausible alternative for a Bullet mechanism
that the model restates from memory moves the pose: each alternative runs SURVEY.md §8d's
parity matrix (seed 0, F_init 0 / 55 x action streams zero / constant (0.5, -0.25) / random
U[-1,1], R = 3, 200 steps from reset) on the CPU oracle, against the default model in the same
precision, and the report gives max |dpos| / |dquat| over the envs at steps 20 / 100 / 200 and
the first step where |dpos| exceeds 1e-4.  The fp32-vs-fp64 rows give the scale of rounding
alone.  Oracle only (test infrastructure): the alternatives are cp_physics fields or
CP_MODEL_* flags the oracle implements.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cartpoleplusplus_amd import abi  # noqa: E402
from oracle import oracle as O  # noqa: E402

# name -> (description and provenance, overrides of cp_physics fields)
ALTERNATIVES = {
    "split_islands": ("each cart-pole island its own solver group and stopping decision "
                      "(btContactSolverInfo::m_minimumSolverBatchSize <= 1; the default model batches both "
                      "islands, m_minimumSolverBatchSize = 128)", {"model_flags": abi.CP_MODEL_SPLIT_ISLANDS}),
    "urdf_contact_erp_1": ("penetration corrected with erp = 1.0 (the URDFs' <contact_erp value=\"1.0\"/>, "
                           "if pybullet applied it) instead of btContactSolverInfo::m_erp = 0.2", {"erp": 1.0}),
    "erp2_0.8": ("penetration corrected with btContactSolverInfo::m_erp2 = 0.8 (the multibody contact rows' "
                 "ERP in the Bullet versions that select m_erp2 when split impulse is off) instead of m_erp = 0.2",
                 {"erp": 0.8}),
    "relative_margin": ("speculative contacts only up to 2.9 mm (the relative breaking threshold of the cart pairs, "
                        "0.02 x the cart's bounding radius) instead of 0.02 m, in the default model",
                        {"contact_margin": 0.0029}),
    "no_warmstart": ("contact impulses start at 0 every substep (btMultiBodyConstraintSolver without "
                     "SOLVER_USE_ARTICULATED_WARMSTARTING / the `if (0)` of Bullet 2.87-2.88) instead of "
                     "0.85 x the cached impulse", {"warmstart": 0.0}),
    "full_warmstart": ("warm start with factor 1.0 instead of m_warmstartingFactor = 0.85", {"warmstart": 1.0}),
    "velocity_friction_dir": ("first friction direction along the lateral relative velocity (rigid-body "
                              "convertContact default) instead of btPlaneSpace1 only (multibody solver)",
                              {"model_flags": abi.CP_MODEL_VEL_FRICTION}),
    "persistent_manifold": ("Bullet's persistent manifold: new points only from overlapping boxes, matched to "
                            "the cached point nearest in A's frame within the pair's relative breaking threshold "
                            "(0.02 x the smaller bounding radius: 2.9 mm cart pairs, 5.0 mm pole-ground / pole-pole; "
                            "getCacheEntry / replaceContactPoint / sortCachedPoints), dropped by "
                            "refreshContactPoints; instead of a fresh <= 4-point set with speculative points up to "
                            "0.02 m and feature-id warm start",
                            {"model_flags": abi.CP_MODEL_PERSISTENT}),
    "persistent_no_warmstart": ("persistent manifold and no warm start (the multibody solver of the Bullet "
                                "versions whose pybullet ran this fork)",
                                {"model_flags": abi.CP_MODEL_PERSISTENT, "warmstart": 0.0}),
    "no_early_exit": ("all 50 sweeps every substep (leastSquaresResidualThreshold 0, btContactSolverInfo's "
                      "default) instead of pybullet's 1e-7", {"residual_threshold": 0.0}),
    "iterations_10": ("10 PGS sweeps (btContactSolverInfo::m_numIterations default) instead of pybullet's 50",
                      {"solver_iterations": 10}),
    "no_velocity_clamp": ("no clamp of the base velocity coordinates (the round-4 model) instead of "
                          "btMultiBody::applyDeltaVeeMultiDof's +-m_maxCoordinateVelocity = 100",
                          {"max_coord_velocity": 0.0}),
    "sleeping": ("Bullet's deactivation (URDF_ENABLE_SLEEPING, or the pybullet builds before the flag existed): "
                 "a body whose |w|^2 + |v|^2 stays below 0.05 for 2 s stops being awake, and an island with no "
                 "awake body sleeps (neither integrated nor solved) until an active body's AABB touches it",
                 {"model_flags": abi.CP_MODEL_SLEEPING}),
}
CASES = [(F, s) for F in (0.0, 55.0) for s in ("zero", "constant", "random")]


def rollout(precision, F, stream, envs, steps, phys=None, seed=0):
    """(steps + 1, envs, R, 2, 7) float32 obs from reset; phys overrides cp_physics fields."""
    cfg = O.default_config(num_envs=envs, action_repeats=3, initial_force=float(F), seed=seed)
    for k, v in (phys or {}).items():
        setattr(cfg.phys, k, v)
    env = O.Envs(cfg, precision=precision)
    out = [env.reset()]
    rng = np.random.default_rng(seed)
    obs = np.zeros((envs, 3, 2, 7), np.float32)
    rew = np.zeros(envs, np.float32)
    done = np.zeros(envs, np.uint8)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    for _ in range(steps):
        if stream == "zero":
            a = np.zeros((envs, 2, 2), np.float32)
        elif stream == "constant":
            a = np.broadcast_to(np.array([0.5, -0.25], np.float32), (envs, 2, 2)).copy()
        else:
            a = rng.uniform(-1, 1, (envs, 2, 2)).astype(np.float32)
        env.step_omp(a, abi.CP_ACTION_CONTINUOUS, obs, rew, done, threads)
        out.append(obs.copy())
    return np.stack(out)


def diffs(a, b, steps):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    dp = d[..., 0:3].reshape(d.shape[0], -1).max(axis=1)
    dq = d[..., 3:7].reshape(d.shape[0], -1).max(axis=1)
    first = np.nonzero(dp > 1e-4)[0]
    at = [k for k in (20, 100, steps) if k <= steps]
    return {"max_dpos": float(dp.max()), "max_dquat": float(dq.max()),
            "dpos_at_step": {str(k): float(dp[k]) for k in at}, "dquat_at_step": {str(k): float(dq[k]) for k in at},
            "first_step_dpos_over_1e-4": int(first[0]) if len(first) else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--precision", choices=("f32", "f64"), default="f64")
    ap.add_argument("--only", default=None, help="comma-separated alternative names")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    names = args.only.split(",") if args.only else list(ALTERNATIVES)
    base = {}
    out = {"envs": args.envs, "steps": args.steps, "precision": args.precision, "repeats": 3,
           "reference": "the default model (DESIGN.md §3) in the same precision",
           "note": "oracle only; pybullet absent (SURVEY.md §8c), so these are model-to-model distances between "
                   "plausible restatements of Bullet, not distances to pybullet", "alternatives": {}}
    for F, s in CASES:
        base[(F, s)] = rollout(args.precision, F, s, args.envs, args.steps)
    rnd = {}
    for F, s in CASES:   # rounding alone: the default model in fp32 against fp64
        other = "f32" if args.precision == "f64" else "f64"
        rnd[f"F{int(F)}/{s}"] = diffs(rollout(other, F, s, args.envs, args.steps), base[(F, s)], args.steps)
    out["rounding_fp32_vs_fp64"] = rnd
    for name in names:
        desc, phys = ALTERNATIVES[name]
        cases = {}
        for F, s in CASES:
            r = rollout(args.precision, F, s, args.envs, args.steps, phys)
            nonfinite = int((~np.isfinite(r)).reshape(r.shape[0], r.shape[1], -1).any(axis=(0, 2)).sum())
            cases[f"F{int(F)}/{s}"] = diffs(np.where(np.isfinite(r), r, base[(F, s)]), base[(F, s)], args.steps)
            cases[f"F{int(F)}/{s}"]["nonfinite_envs"] = nonfinite
        worst = max(c["max_dpos"] for c in cases.values())
        firsts = [c["first_step_dpos_over_1e-4"] for c in cases.values() if c["first_step_dpos_over_1e-4"] is not None]
        out["alternatives"][name] = {"description": desc, "overrides": phys, "cases": cases,
                                     "max_dpos_any_case": worst,
                                     "moves_pose_over_1e-4_within_steps": bool(firsts),
                                     "earliest_step_over_1e-4": min(firsts) if firsts else None}
        print(f"{name:26s} max|dpos| {worst:9.3e}  earliest >1e-4 step {min(firsts) if firsts else None}", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
