#!/usr/bin/env python3
"""Diagnostic: how often is a 64-lane wave uniform in one of the lean structure classes?

Builds the ORC_STATS oracle (test infrastructure, tools/row_classes.py) and records every island solve of
  reset  -- one burst reset of B envs after 30 steps (130 substeps: 100 settle + 30 bump), or
  steps  -- one 199-step episode of the bench workload from a burst reset,
then groups islands into waves as the kernels do (32 envs = 64 lanes) and reports, per phase, the share of
wave-substeps (and of wave-sweeps) in which every active lane is c4k_ok (cart on the ground with +z rows,
0-4 cart-pole rows, nothing else) or p1_ok (pole on the ground, 4 + 4 friction points, cart off or +z).

usage: python tools/wave_classes.py reset|steps [--envs 2048]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def classes(a):
    cnt, fcnt, merged, sw, ez = a[..., 0:5], a[..., 5:10], a[..., 10], a[..., 11], a[..., 12:17]
    c4k = ((cnt[..., 0] == 4) & (cnt[..., 1] == 0) & (merged == 0) & (ez[..., 0] == 1) & (fcnt[..., 0] == 0)
           & (fcnt[..., 2] == 0))
    p1 = ((cnt[..., 1] == 4) & (fcnt[..., 1] == 4) & (ez[..., 1] == 1) & (cnt[..., 2] == 0) & (fcnt[..., 0] == 0)
          & (fcnt[..., 2] == 0) & (merged == 0) & ((cnt[..., 0] == 0) | ((cnt[..., 0] == 4) & (ez[..., 0] == 1))))
    return c4k, p1, sw, merged


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("reset", "steps"))
    ap.add_argument("--envs", type=int, default=2048)
    args = ap.parse_args()
    import row_classes as rc
    os.environ["ORC_LIB_OVERRIDE"] = rc.build_stats_oracle()
    from cartpoleplusplus_amd import abi
    from oracle import oracle as O
    B, T = args.envs, 200
    cfg = O.default_config(num_envs=B, action_repeats=3, initial_force=55.0, seed=1234, autoreset=1)
    env = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    lib = env.lib
    lib.orc_stats_open.argtypes = [C.c_char_p]
    env.reset()
    rng = np.random.default_rng(1)
    path = b"/tmp/orc_wave_classes.txt"
    if args.mode == "reset":
        for _ in range(30):
            env.step(rng.integers(0, 5, (B, 2)).astype(np.int8))
        lib.orc_stats_open(path)
        env.reset()
        lib.orc_stats_open(None)
        a = np.loadtxt(path.decode(), dtype=np.int64).reshape(B, 130, 2, -1)   # env, substep, island
        c4k, p1, sw, _ = classes(a)
        W = B // 32
        for name, ph in (("settle", slice(0, 100)), ("bump", slice(100, 130))):
            k, s = c4k[:, ph], sw[:, ph]
            kw = k.reshape(W, 32, -1, 2).transpose(0, 2, 1, 3).reshape(W, k.shape[1], 64)
            sww = s.reshape(W, 32, -1, 2).transpose(0, 2, 1, 3).reshape(W, s.shape[1], 64)
            allk = np.all(kw | (sww == 0), axis=2)
            print(f"{name}: island sweeps mean {s.mean():.2f}, capped {np.mean(s >= 50):.3f}, islands c4k {k.mean():.3f}, "
                  f"wave-substeps all-c4k {allk.mean():.3f}")
    else:
        lib.orc_stats_open(path)
        for _ in range(T - 1):
            env.step(rng.integers(0, 5, (B, 2)).astype(np.int8))
        lib.orc_stats_open(None)
        a = np.loadtxt(path.decode(), dtype=np.int64).reshape(T - 1, B, 3, 2, -1)   # step, env, substep, island
        c4k, p1, sw, merged = classes(a)
        W = B // 32

        def wave(x):
            return x.reshape(T - 1, W, 32, 3, 2).transpose(0, 1, 3, 2, 4).reshape(T - 1, W, 3, 64)
        act = wave(sw > 0)
        a4 = np.all(wave(c4k) | ~act, 3)
        ap_ = np.all(wave(p1) | ~act, 3)
        nm = ~np.any(wave(merged > 0) & act, 3)
        wsw = wave(sw).max(3)
        for lo, hi in ((1, 5), (6, 10), (11, 25), (26, 100), (101, 199)):
            s = slice(lo - 1, hi)
            tot = wsw[s].sum()
            print(f"steps {lo}-{hi}: wave-substeps all-c4k {a4[s].mean():.3f} all-p1 {ap_[s].mean():.3f}; wave-sweep "
                  f"share all-c4k {wsw[s][a4[s]].sum() / tot:.3f} all-p1 {wsw[s][ap_[s]].sum() / tot:.3f} "
                  f"no-merged {wsw[s][nm[s]].sum() / tot:.3f}; islands c4k {c4k[s].mean():.3f} p1 {p1[s].mean():.3f}")


if __name__ == "__main__":
    main()
