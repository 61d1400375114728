"""Diagnostic: wall time of each cp_step after a burst reset, per step index (HIP events on the
library's launch stream, every call), for the C3 workload.  Answers "is an early-episode step
(the driver's `--steps 20 --warmup 5` window: steps 6-25 after the reset) slower than a late one,
and is that the physics or a cold GPU?".

Runs the same 300 steps three times in one process: right after handle creation (cold), again
after a fresh reset, and a third time after a fresh reset.  Prints one JSON line: per-phase means
over step ranges, and the first 40 per-step values.

usage (GPU): python tools/step_profile.py [--steps 300] [--batch 65536]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (action generator and workload constants)
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402


def run(env, actions, n):
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    env.reset()
    torch.cuda.synchronize()
    ev[0].record(st)
    for t in range(n):
        env.step(actions[t])
        ev[t + 1].record(st)
    torch.cuda.synchronize()
    return [ev[t].elapsed_time(ev[t + 1]) for t in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--phases", type=int, default=3)
    ap.add_argument("--full", action="store_true", help="also print every step's time")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, R = a.batch, 3
    env = BatchedCartpole(B, 0, action_repeats=R, steps_per_repeat=1, max_episode_len=bench.WINDOW,
                          initial_force=55.0, autoreset="same_step", seed=bench.SEED)
    actions = bench.make_actions(False, B, 0, a.steps, bench.SEED, dev)
    out = {"batch": B, "steps": a.steps}
    for phase in ("cold", "second", "third")[:a.phases]:
        ms = run(env, actions, a.steps)
        rng = {f"{lo}-{hi}": round(sum(ms[lo - 1:hi]) / (hi - lo + 1), 4)
               for lo, hi in ((1, 5), (6, 25), (26, 100), (101, 199), (200, 200), (201, min(a.steps, 399)), (26, 225), (206, 405))
               if hi <= a.steps}
        out[phase] = {"mean_ms_by_steps": rng, "first40": [round(x, 4) for x in ms[:40]]}
        if a.full:
            out[phase]["all"] = [round(x, 4) for x in ms]
    env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
