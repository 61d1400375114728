#!/usr/bin/env python3
"""Episode-length deciles of a random agent, next to the reference README's (README.md:76-92).

    python tools/deciles.py [--backend oracle|gpu|both] [--episodes 100] [--out FILE]

The README's numbers come from the *upstream* env (one cart-pole pair, angle termination,
other URDFs) driven by `random_action_agent.py --initial-force=F --actions=A --num-eval=100
| deciles.py`, and deciles.py prints np.percentile(lengths, linspace(0, 100, 11)).  Here the
same four configurations run on this model with the reference fork's commented-out bounds
termination switched on (bullet_cartpole.py:243-253: |x|, |y| of the pole > 3 m or its roll /
pitch > 0.35 rad), R = 2 (the reference default, :23), episodes of at most 200 steps, one
random action per cart and step drawn uniformly from the `--actions` list (the discrete
table, abi.DISCRETE_TABLE), 100 episodes = 100 envs of one batch (Philox bumps, seed 0).
A loose statistical check only ("upstream env, loose check"): the scene differs from the one
the README measured.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cartpoleplusplus_amd import abi  # noqa: E402

README = {  # README.md:80, :84, :88, :92
    "F0/actions=0": [200, 200, 200, 200, 200, 200, 200, 200, 200, 200, 200],
    "F0/actions=0,1,2,3,4": [16, 22.9, 26, 28, 31.6, 35, 37.4, 42.3, 48.4, 56.1, 79],
    "F55/actions=0": [6, 7, 7, 8, 8.6, 9, 11, 12.3, 15, 21, 39],
    "F55/actions=0,1,2,3,4": [3, 5.9, 7, 7.7, 8, 9, 10, 11, 13, 15, 32],
}
CASES = [(0.0, (0,)), (0.0, (0, 1, 2, 3, 4)), (55.0, (0,)), (55.0, (0, 1, 2, 3, 4))]
MAX_LEN = 200


def episode_lengths(backend, F, actions, n, seed=0, R=2):
    """Length (steps, the terminating one included) of one episode per env, n envs."""
    rng = np.random.default_rng(seed)
    kw = dict(num_envs=n, action_repeats=R, initial_force=F, seed=seed, done_on_bounds=1,
              max_episode_len=MAX_LEN, autoreset=0)
    if backend == "oracle":
        from oracle import oracle as O
        env = O.Envs(O.default_config(**kw))
        env.reset()
        step = lambda a: env.step(a)[2]  # noqa: E731
    else:
        import torch

        from cartpoleplusplus_amd import native
        from cartpoleplusplus_amd.batched import BatchedCartpole
        cfg = native.default_config(**kw)
        env = BatchedCartpole(n, 0, config=abi.cp_config.from_buffer_copy(cfg))
        env.reset()
        step = lambda a: env.step(torch.from_numpy(a).to(env.device))[2].cpu().numpy()  # noqa: E731
    length = np.zeros(n, np.int64)
    choice = np.asarray(actions, np.int8)
    for t in range(MAX_LEN):
        a = choice[rng.integers(0, len(choice), (n, 2))]
        done = step(np.ascontiguousarray(a)).astype(bool)
        newly = done & (length == 0)
        length[newly] = t + 1
        if (length > 0).all():
            break
    length[length == 0] = MAX_LEN
    return length


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=("oracle", "gpu", "both"), default="both")
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    backends = ("oracle", "gpu") if args.backend == "both" else (args.backend,)
    out = {"note": "upstream env, loose check: README.md:76-92 measured the upstream single-pair env; this model "
                   "has two pairs, the fork's URDFs and its commented-out bounds termination switched on",
           "episodes": args.episodes, "repeats": 2, "max_episode_len": MAX_LEN, "cases": {}}
    for F, acts in CASES:
        key = f"F{int(F)}/actions={','.join(map(str, acts))}"
        row = {"readme_upstream": README[key]}
        for b in backends:
            L = episode_lengths(b, F, acts, args.episodes)
            row[b] = [round(float(x), 2) for x in np.percentile(L, np.linspace(0, 100, 11))]
            row[b + "_mean"] = round(float(L.mean()), 2)
        if len(backends) == 2:
            row["gpu_equals_oracle"] = row["gpu"] == row["oracle"]
        out["cases"][key] = row
        print(key, json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
