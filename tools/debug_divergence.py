"""Locate the first substep where the HIP kernel and the oracle diverge.

Runs the GPU library and the oracle in lockstep with R = 1, S = 1 (one substep
per step) from the same reset, random continuous actions, and prints the
differing state fields of the first diverging envs.  GPU box only; diagnostic.

    python tools/debug_divergence.py [--B 96] [--steps 600] [--iters 50] [--warmstart 0.85]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd import abi, native  # noqa: E402
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402
from oracle import oracle as O  # noqa: E402

FIELD_NAMES = {}
for d, nm in enumerate(["cart", "pole", "cart2", "pole2"]):
    for c, cn in enumerate(["x", "y", "z", "qx", "qy", "qz", "qw", "vx", "vy", "vz", "wx", "wy", "wz"]):
        FIELD_NAMES[abi.CP_SF_BODY(d, c)] = f"{nm}.{cn}"
for i in range(abi.CP_NUM_ISLANDS):
    for j in range(abi.CP_ISLAND_PAIRS):
        FIELD_NAMES[abi.CP_SF_WS_ID(i, j)] = f"ws_id[{i}][{j}]"
        for k in range(4):
            FIELD_NAMES[abi.CP_SF_WS_LAM(i, j, k)] = f"ws_lam[{i}][{j}][{k}]"


def ws_ids(st, e):
    return [hex(st[abi.CP_SF_WS_ID(i, j):abi.CP_SF_WS_ID(i, j) + 1, e].view(np.uint32)[0])
            for i in range(abi.CP_NUM_ISLANDS) for j in range(abi.CP_ISLAND_PAIRS)]


ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=96)
ap.add_argument("--seed", type=int, default=7)
ap.add_argument("--steps", type=int, default=600)
ap.add_argument("--iters", type=int, default=None)
ap.add_argument("--warmstart", type=float, default=None)
args = ap.parse_args()
B = args.B
O.build()
cfg = native.default_config(num_envs=B, action_repeats=1, steps_per_repeat=1, initial_force=55.0, seed=args.seed,
                            max_episode_len=100000)
if args.iters is not None:
    cfg.phys.solver_iterations = args.iters
if args.warmstart is not None:
    cfg.phys.warmstart = args.warmstart
g = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
o = O.Envs(abi.cp_config.from_buffer_copy(cfg))
g.reset()
o.reset()
rng = np.random.default_rng(123)
prev = o.get_state().copy()
for t in range(args.steps):
    a = rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
    g.step(torch.from_numpy(a).cuda())
    o.step(a)
    gs = g.get_state().cpu().numpy()
    os_ = o.get_state()
    diff = gs.view(np.uint32) != os_.view(np.uint32)
    envs = np.nonzero(diff.any(axis=0))[0]
    if len(envs) == 0:
        prev = os_.copy()
        continue
    print(f"substep {t}: {len(envs)} envs differ: {envs[:10].tolist()}")
    for e in envs[:2]:
        print("  prev ws ids:", ws_ids(prev, e))
        print("  gpu  ws ids:", ws_ids(gs, e))
        print("  orc  ws ids:", ws_ids(os_, e))
        for f in np.nonzero(diff[:, e])[0][:40]:
            print("  env", e, FIELD_NAMES.get(f, f), float(gs[f, e]), float(os_[f, e]))
    break
else:
    print(f"no divergence in {args.steps} substeps")
