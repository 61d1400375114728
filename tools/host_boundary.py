#!/usr/bin/env python3
"""Host-boundary rates: what a caller that hands host buffers across the boundary gets.

(a) the gym mirror (`cartpoleplusplus_amd.bullet_cartpole.BulletCartpole`, B = 1, the reference's
    surface: numpy action in, numpy obs copy out every step), random discrete actions;
(b) the batched env at C3 (B = 65,536, R = 3, autoreset) with host actions uploaded and obs copied
    back to host memory every step (PCIe in both directions, pinned host buffers).
Prints one JSON object."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd import bullet_cartpole  # noqa: E402
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402


def gym_mirror(steps=300, graph=True):
    p = argparse.ArgumentParser()
    bullet_cartpole.add_opts(p)
    opts = p.parse_args([])
    env = bullet_cartpole.BulletCartpole(opts, discrete_actions=True)
    env.use_graph = graph
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    env.reset()
    t_reset = time.perf_counter() - t0
    n = 0
    t0 = time.perf_counter()
    while n < steps:
        _, _, done, _ = env.step(rng.integers(0, 5, 2))
        n += 1
        if done:
            env.reset()
    dt = time.perf_counter() - t0
    return {"env_steps_per_s": round(n / dt, 1), "ms_per_step": round(dt / n * 1e3, 4),
            "reset_ms": round(t_reset * 1e3, 2), "action_repeats": opts.action_repeats,
            "step_as_hipgraph": graph,
            "note": "B = 1, numpy action in, numpy obs copy out per step (resets inside the loop included)"}


def batched_pcie(B=65536, steps=400, warmup=20):
    env = BatchedCartpole(B, 0, action_repeats=3, steps_per_repeat=1, max_episode_len=200, initial_force=55.0,
                          autoreset=True, seed=1234)
    rng = np.random.default_rng(1234)
    host_act = torch.from_numpy(rng.integers(0, 5, (warmup + steps, B, 2)).astype(np.int8)).pin_memory()
    dev_act = torch.empty((B, 2), dtype=torch.int8, device="cuda")
    host_obs = torch.empty((B, 3, 2, 7), dtype=torch.float32).pin_memory()
    env.reset()
    for t in range(warmup):
        dev_act.copy_(host_act[t], non_blocking=True)
        obs, _, _ = env.step(dev_act)
        host_obs.copy_(obs, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        dev_act.copy_(host_act[warmup + t], non_blocking=True)
        obs, _, _ = env.step(dev_act)
        host_obs.copy_(obs, non_blocking=True)
        torch.cuda.current_stream().synchronize()   # the caller reads the obs before its next action
    dt = time.perf_counter() - t0
    return {"env_steps_per_s": round(B * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4),
            "bytes_per_step": {"h2d_actions": B * 2, "d2h_obs": B * 3 * 2 * 7 * 4},
            "note": "C3 config; per step: actions H2D, step, obs D2H into pinned memory, host sync"}


if __name__ == "__main__":
    print(json.dumps({"gym_mirror_B1": gym_mirror(), "gym_mirror_B1_eager": gym_mirror(graph=False),
                      "batched_pcie_C3": batched_pcie()}), flush=True)
