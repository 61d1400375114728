"""Diagnostic: how much of a PGS sweep does a 64-lane wave pay for row-structure divergence?

Builds an ORC_STATS variant of the CPU oracle (test infrastructure) into /tmp, runs the bench
workload (random discrete actions, R = 3) on B envs, and records for every island solve its
row structure (normal points of local pairs 0..4, friction points of 0..4) and its sweep count.
Then it prices the sweeps of each wave (32 envs = 64 lanes, the kernel's env->lane map) with
per-row-loop instruction counts read off the step kernel's ISA (`ROW_COST`), in three layouts:

  current    the kernel as built: per sweep, every row loop runs max(count over active lanes) trips
  sorted     envs regrouped into waves by their row-structure signature (an upper bound on what
             a class sort of the env order could buy: signatures of the same substep)
  generic    one row loop for every kind of row: max(rows over active lanes) trips of one body

usage: python tools/row_classes.py [--envs 4096] [--warmup 60] [--steps 40]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# VALU+LDS instructions per loop trip (step kernel ISA, tools/isa loops): normal rows of local pairs
# 0, 1 (ground-dynamic, 49) and 2 (cart-pole, 81); friction point (2 rows) of pairs 0/1 (92) and 2 (155)
ROW_COST = {"n": [49, 49, 81], "f": [92, 92, 155]}
GENERIC_NORMAL, GENERIC_FRICTION = 85, 170


def build_stats_oracle():
    out = "/tmp/libcp_oracle_stats.so"
    src = os.path.join(ROOT, "oracle", "cp_oracle.c")
    cmd = ["gcc", "-O2", "-fPIC", "-std=c11", "-march=x86-64-v3", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
           "-DORC_STATS", "-shared", "-o", out, src, "-lm"]
    subprocess.check_call(cmd)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    os.environ["ORC_LIB_OVERRIDE"] = build_stats_oracle()
    from cartpoleplusplus_amd import abi
    from oracle import oracle as O

    B, R = args.envs, 3
    cfg = O.default_config(num_envs=B, action_repeats=R, initial_force=55.0, seed=1234, autoreset=1)
    env = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    lib = env.lib
    lib.orc_stats_open.argtypes = [C.c_char_p]
    env.reset()
    rng = np.random.default_rng(1234)
    for _ in range(args.warmup):
        env.step(rng.integers(0, 5, (B, 2)).astype(np.int8))
    path = "/tmp/orc_stats.txt"
    lib.orc_stats_open(path.encode())
    for _ in range(args.steps):
        env.step(rng.integers(0, 5, (B, 2)).astype(np.int8))
    lib.orc_stats_open(None)
    a = np.loadtxt(path, dtype=np.int64)
    # rows: per step, per env, per substep, 2 islands (merged envs also emit 2 lines)
    a = a.reshape(args.steps, B, R, 2, -1)
    cnt, fcnt, merged, sw, ez = a[..., 0:5], a[..., 5:10], a[..., 10], a[..., 11], a[..., 12:17]
    print(f"island solves: {sw.size}, merged env-substeps {merged[..., 0].mean():.4f}")
    print(f"sweeps: mean {sw.mean():.2f}, median {np.median(sw):.0f}, capped(50) {np.mean(sw >= 50):.3f}")
    sig = [tuple(x) for x in np.concatenate([cnt[..., :3], fcnt[..., :3]], -1).reshape(-1, 6)]
    from collections import Counter
    c = Counter(sig)
    print("top island signatures (cnt0 cnt1 cnt2 | fcnt0 fcnt1 fcnt2): share, capped share")
    swf = sw.reshape(-1)
    sigs = np.array(sig)
    for s, n in c.most_common(8):
        m = np.all(sigs == np.array(s), axis=1)
        print(f"  {s[:3]} | {s[3:]}: {n / len(sig):.3f}  capped {np.mean(swf[m] >= 50):.3f}  mean sweeps {swf[m].mean():.1f}")

    def wave_cost(c3, f3, s, generic=False):
        """c3, f3: (lanes, 3); s: (lanes,) sweeps -> instruction trips for the wave's sweeps"""
        tot = 0
        for it in range(int(s.max()) if s.size else 0):
            act = s > it
            if generic:
                tot += c3[act].sum(1).max() * GENERIC_NORMAL + f3[act].sum(1).max() * GENERIC_FRICTION
            else:
                tot += sum(c3[act, j].max() * ROW_COST["n"][j] for j in range(3))
                tot += sum(f3[act, j].max() * ROW_COST["f"][j] for j in range(3))
        return tot

    nw = B // 32

    def layout_cost(t, r, order=None, generic=False):
        c3 = cnt[t, :, r, :, :3]
        f3 = fcnt[t, :, r, :, :3]
        s = sw[t, :, r, :]
        if order is not None:
            c3, f3, s = c3[order], f3[order], s[order]
        c3, f3, s = c3.reshape(B * 2, 3), f3.reshape(B * 2, 3), s.reshape(B * 2)
        return sum(wave_cost(c3[w * 64:(w + 1) * 64], f3[w * 64:(w + 1) * 64], s[w * 64:(w + 1) * 64], generic)
                   for w in range(nw))

    def sig_key(t, r):
        return np.concatenate([cnt[t, :, r, :, :3].reshape(B, 6), fcnt[t, :, r, :, :3].reshape(B, 6)], 1)

    modes = {"current": [], "generic rows": [], "sorted by own signature": [],
             "sorted by own signature + sweeps (oracle bound)": [], "sorted by previous step's sweeps": [],
             "sorted by previous step's signature + sweeps": []}
    for t in range(1, args.steps):
        prev_sw = sw[t - 1].max(axis=(1, 2))
        prev_key = np.concatenate([sig_key(t - 1, R - 1), prev_sw[:, None]], 1)
        o_prev_sw = np.argsort(prev_sw, kind="stable")
        o_prev = np.lexsort(prev_key.T[::-1])
        for r in range(R):
            own = sig_key(t, r)
            o_sig = np.lexsort(own.T[::-1])
            o_sig_sw = np.lexsort(np.concatenate([own, sw[t, :, r, :].max(1, keepdims=True)], 1).T[::-1])
            modes["current"].append(layout_cost(t, r))
            modes["generic rows"].append(layout_cost(t, r, generic=True))
            modes["sorted by own signature"].append(layout_cost(t, r, o_sig))
            modes["sorted by own signature + sweeps (oracle bound)"].append(layout_cost(t, r, o_sig_sw))
            modes["sorted by previous step's sweeps"].append(layout_cost(t, r, o_prev_sw))
            modes["sorted by previous step's signature + sweeps"].append(layout_cost(t, r, o_prev))
    base = np.mean(modes["current"])
    print("sweep instructions per wave-substep:")
    for k, v in modes.items():
        print(f"  {k:50s} {np.mean(v) / nw:8.0f}  ({np.mean(v) / base:.2f}x)")

if __name__ == "__main__":
    main()
