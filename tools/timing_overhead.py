#!/usr/bin/env python3
"""Diagnostic: does recording HIP events around every launch (bench.py's live kernel timing)
cost wall time?  Runs the bench workload (C3) K steps with and without cp_timing_begin and
prints ms per step for each (event strides (1, 1), (4, 1), (4, 4), none), 3 rounds."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402

B, R, K, W = 65536, 3, 600, 20
env = BatchedCartpole(B, 0, action_repeats=R, steps_per_repeat=1, max_episode_len=200, initial_force=55.0,
                      autoreset=True, seed=1234)
gen = torch.Generator(device="cuda").manual_seed(1234)
actions = torch.randint(0, 5, (W + K, B, 2), dtype=torch.int8, device="cuda", generator=gen)
env.reset()
for t in range(W):
    env.step(actions[t])
torch.cuda.synchronize()
for rnd in range(3):
    for timed in ((1, 1), (4, 1), (4, 4), None):
        if timed:
            env.timing_begin(K)
            env.timing_stride(*timed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(K):
            env.step(actions[W + t])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if timed:
            env.timing_end()
        print(f"round {rnd} event strides (step, reset) {timed} ms/step {dt / K * 1e3:.4f}", flush=True)
