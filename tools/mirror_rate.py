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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="auto")
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    p = argparse.ArgumentParser()
    bullet_cartpole.add_opts(p)
    opts = p.parse_args(["--initial-force", "55"])
    env = bullet_cartpole.BulletCartpole(opts, discrete_actions=True)
    env._env.set_kernel_shape(a.shape, a.shape)
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
                      "resets": resets, "shape": shape}))


if __name__ == "__main__":
    main()
