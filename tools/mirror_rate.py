#!/usr/bin/env python3
"""bench.py's gym_mirror_rate (B = 1 drop-in surface, resets inside the loop) with the step / reset kernel
shape forced (--shape latency | wide | auto); prints one JSON object."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd import bullet_cartpole  # noqa: E402


def kernel_times(shape, steps=300, reset=None):
    """B = 1 step and reset kernel times (HIP events around each launch, cp_timing) for one shape."""
    import torch
    from cartpoleplusplus_amd.batched import BatchedCartpole
    env = BatchedCartpole(1, 0, action_repeats=2, initial_force=55.0, seed=3, autoreset=True)
    env.set_kernel_shape(shape, reset or shape)
    env.reset()
    a = torch.zeros((1, 2), dtype=torch.int8, device="cuda")
    for _ in range(20):
        env.step(a)
    torch.cuda.synchronize()
    env.timing_begin(steps + 8)
    t0 = time.perf_counter()
    for _ in range(steps):
        env.step(a)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tm = env.timing_end()
    env.close()
    return {"step_kernel_us": round(tm["step_ms"] / max(1, tm["step_launches"]) * 1e3, 2),
            "reset_kernel_ms": round(tm["reset_ms"] / max(1, tm["reset_launches"]), 3) if tm["reset_launches"] else None,
            "eager_call_us": round(wall / steps * 1e6, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="auto")
    ap.add_argument("--reset-shape", default=None)
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    kt = kernel_times(a.shape, reset=a.reset_shape or a.shape)
    p = argparse.ArgumentParser()
    bullet_cartpole.add_opts(p)
    opts = p.parse_args(["--initial-force", "55"])
    env = bullet_cartpole.BulletCartpole(opts, discrete_actions=True)
    env._env.set_kernel_shape(a.shape, a.reset_shape or a.shape)
    rng = np.random.default_rng(0)
    np.random.seed(0)
    env.reset()
    for _ in range(20):            # warm-up (graph capture)
        env.step(rng.integers(0, 5, 2))
    env.reset()
    t0 = time.perf_counter()
    env.reset()
    t_reset = time.perf_counter() - t0
    n, resets, t0 = 0, 0, time.perf_counter()
    while n < a.steps:
        _, _, done, _ = env.step(rng.integers(0, 5, 2))
        n += 1
        if done:
            env.reset()
            resets += 1
    dt = time.perf_counter() - t0
    shape = env._env.kernel_shape()
    env.close()
    print(json.dumps({"value": round(n / dt, 1), "ms_per_step": round(dt / n * 1e3, 4), "reset_ms": round(t_reset * 1e3, 3),
                      "resets": resets, "shape": shape, **kt}))


if __name__ == "__main__":
    main()
