"""Cost of the §8f rows on top of the C3 step at full size (one MI355X):
    base    env.step (C3: B=65,536, R=3, discrete, autoreset)
    lqr     env.step with the in-kernel LQR policy + 8-state readback (f4)
    ingest  env.step + ReplayMemory.after_step (f3; 2^22-event ring, 42-float states)
    sample  ReplayMemory.sample(n) alone (device gather)
Timed with HIP events on torch's current stream (all launches go there).  Prints one
JSON line; per-event / per-sample algorithmic bytes as in DESIGN.md §Replay memory."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402
from cartpoleplusplus_amd.lqr import exact_gains  # noqa: E402
from cartpoleplusplus_amd.replay_memory import ReplayMemory  # noqa: E402


def timed(fn, steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for t in range(steps):
        fn(t)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--ring", type=int, default=1 << 22)
    ap.add_argument("--sample", type=int, default=65536)
    args = ap.parse_args()
    B, K, R = args.batch, args.steps, 3
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    acts = torch.randint(0, 5, (K, B, 2), dtype=torch.int8, device=dev, generator=g)
    out = {"batch": B, "steps": K}

    env = BatchedCartpole(B, 0, action_repeats=R, initial_force=55.0, autoreset=True, seed=1234)
    env.reset()
    for t in range(20):
        env.step(acts[t])
    out["base_ms"] = timed(lambda t: env.step(acts[t]), K)

    env.enable_lqr(torch.from_numpy(exact_gains()), state8=True)
    for t in range(20):
        env.step(acts[t])
    out["lqr_ms"] = timed(lambda t: env.step(acts[t]), K)
    env.enable_lqr(None)

    rm = ReplayMemory(args.ring, (R, 2, 7), 2, 1.5, num_envs=B)
    env.reset()
    rm.after_reset(env)

    def ingest(t):
        env.step(acts[t])
        rm.after_step(env, acts[t])
    for t in range(20):
        ingest(t)
    out["ingest_ms"] = timed(ingest, K)
    out["ingest_extra_ms"] = out["ingest_ms"] - out["base_ms"]
    rm.check()
    n = args.sample
    out["sample_n"] = n
    out["sample_ms"] = timed(lambda t: rm.sample(n), K)
    D = R * 2 * 7
    # per sample: 2 slot reads (8) + 2 f16 state rows read + written + action/reward/mask + idx
    sample_bytes = n * (8 + 4 * D * 2 + 2 * (2 * 4 + 4 + 4) + 4)
    out["sample_GBps"] = sample_bytes / (out["sample_ms"] * 1e-3) / 1e9
    out["replay_size"] = rm.size()
    out["env_steps_per_s"] = {k: B / (out[k + "_ms"] * 1e-3) for k in ("base", "lqr", "ingest")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
