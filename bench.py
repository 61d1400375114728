#!/usr/bin/env python3
"""bench.py — batched cartpole++ env-steps/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2] / SURVEY.md §8d C3, per GPU): 65,536 envs, discrete
5-action random policy (int8 actions pre-generated in HBM), action_repeats R = 3,
steps_per_repeat 1, initial_force 55, max_episode_len 200 with in-kernel autoreset,
fp32.  A "step" is one env-step of every env: one cp_step call = one fused R-substep
kernel launch + one compacted reset launch.  Envs shard across ranks (seed 1234+rank,
global env ids offset rank*B); the only collective is an RCCL all-gather of the
episode returns once per 200-step window (C4).  value = N*B*K / max-over-ranks wall.

roofline: the step kernel's algorithmic HBM bytes per launch over
its average duration from HIP events recorded on its launch stream in the timed region
(every 4th launch sampled: the events themselves cost wall time).
cpu_baseline: the CPU oracle (a port: same algorithm, gcc -O2, OpenMP) on a bounded
sample of the same workload, rank 0 at N = 1 only.
parity: max |pose diff| over 200 steps of 512 C3 envs against the oracle's fp32 build
(bit-exact bar) and its fp64 build (drift), rank 0 at N = 1 only, after the timed region.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402
from cartpoleplusplus_amd.dist import gather_returns, return_histogram, shard_spec  # noqa: E402

METRIC = "env-steps/sec at batch=65,536, 1→8 MI355X; max |pose−pybullet| over 200 steps"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured)
WINDOW = 200            # episode-return reporting window (steps)
# HIP events around every 4th step-kernel launch (every reset launch): each recorded event
# costs the stream a few microseconds (tools/timing_overhead.py: 0.761 ms/step with events on
# every launch, 0.755 with this sampling, 0.748 without events)
STEP_EVENT_STRIDE = 4


def step_kernel_bytes(R, action_bytes):
    """Algorithmic HBM bytes one env moves in one step-kernel launch."""
    state_read = 52 + 6 + 2            # 4 bodies x 13, 2 pending forces x 3, steps, done
    state_write = 52 + 6 + 1           # bodies, pending forces, steps
    warm_cache = 2 * (10 + 40)         # warm-start ids + impulses, read + write once per step
    return 4 * (state_read + state_write + warm_cache) + action_bytes + 4 * 14 * R + 4 + 1 + 8


def render_kernel_bytes(H, W, C, R):
    """Algorithmic HBM bytes of one env's raster obs (render kernel): the float16 image
    (H, W, 3, C, R) written once, the R x 4 repeat-end poses read, one list entry."""
    return 2 * H * W * 3 * C * R + 4 * R * 4 * 7 + 4


def pmc_traffic(kernel, batch, repeats):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_pmc.json, tools/profile.sh + tools/summarize_profile.py), if it was
    collected on this workload; else None."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for p in reversed(paths):
        with open(p) as f:
            d = json.load(f)
        k = d.get("kernels", {}).get(kernel)
        if k and "hbm_bytes_per_launch" in k and d.get("batch", batch) == batch and d.get("repeats", repeats) == repeats:
            return k["hbm_bytes_per_launch"], os.path.relpath(p, ROOT)
    return None, None


def pmc_valu(kernel, batch, repeats):
    """VALU wave-instructions per launch of `kernel` (SQ_INSTS_VALU) from the newest
    committed PMC summary of this workload, else None."""
    import glob
    for p in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))):
        with open(p) as f:
            d = json.load(f)
        k = d.get("kernels", {}).get(kernel)
        if k and "SQ_INSTS_VALU" in k.get("sq_per_launch", {}) and d.get("batch", batch) == batch \
                and d.get("repeats", repeats) == repeats:
            return k["sq_per_launch"]["SQ_INSTS_VALU"], os.path.relpath(p, ROOT)
    return None, None


# MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, a wave64 VALU instruction takes 2 issue
# cycles of its SIMD (one wave alone sustains one per 4), 2.4 GHz max clock
VALU_PEAK_WINST_PER_S = 256 * 4 * 2.4e9 / 2


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(R, budget_s):
    """Oracle (port) on the host: same workload on a bounded env sample."""
    import numpy as np

    from cartpoleplusplus_amd import abi
    from oracle import oracle as O
    O.build()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def run(B, steps):
        cfg = O.default_config(num_envs=B, action_repeats=R, initial_force=55.0, seed=1234, autoreset=1)
        e = O.Envs(cfg)
        e.reset()
        rng = np.random.default_rng(1234)
        acts = rng.integers(0, 5, (steps, B, 2)).astype(np.int8)
        obs = np.zeros((B, R, 2, 7), np.float32)
        rew = np.zeros(B, np.float32)
        done = np.zeros(B, np.uint8)
        t0 = time.perf_counter()
        used = 1
        for t in range(steps):
            used = e.step_omp(acts[t], abi.CP_ACTION_DISCRETE, obs, rew, done, threads)
        return time.perf_counter() - t0, used

    probe_b = 256
    dt, _ = run(probe_b, 20)
    rate = probe_b * 20 / dt
    steps = WINDOW + 1                  # one full episode incl. an in-step autoreset
    B = int(min(65536, max(256, rate * budget_s / steps)))
    B -= B % 64
    dt, used = run(B, steps)
    return {"value": round(B * steps / dt, 1), "unit": "env-steps/s", "cores": used, "kind": "port",
            "sample": f"oracle/cp_oracle.c fp32 (same algorithm, gcc -O2 -march=x86-64-v3, OpenMP) on {B} envs x "
                      f"{steps} steps of the same workload (R={R}, discrete random actions, autoreset incl.); "
                      f"{dt:.1f} s wall on {used} threads"}


def parity_check(device, R, B=512, steps=WINDOW):
    """Checker leg (rank 0, N = 1, next to cpu_baseline): the second half of the metric,
    max |pose - ref| over 200 steps.  pybullet is absent, so the refs are
    the oracle's fp32 build (the kernel's bar: bit-exact) and its fp64 build (the
    precision pybullet's double btScalar would compute the same algorithm in).  Same C3
    config as the timed run (seed 1234, random discrete actions, autoreset), B envs,
    `steps` steps from reset; obs = (R, 2, 7) cart + pole poses per repeat."""
    import numpy as np

    from cartpoleplusplus_amd import abi
    from oracle import oracle as O
    O.build()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    cfg = O.default_config(num_envs=B, action_repeats=R, initial_force=55.0, seed=1234, autoreset=1)
    gpu = BatchedCartpole(B, device.index, config=abi.cp_config.from_buffer_copy(cfg))
    orc = {p: O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=p) for p in ("f32", "f64")}
    g = gpu.reset().cpu().numpy()
    o = {p: e.reset() for p, e in orc.items()}
    rng = np.random.default_rng(1234)
    d64 = np.zeros((steps + 1, B))
    d32 = np.abs(g - o["f32"]).reshape(B, -1).max(1)
    d64[0] = np.abs(g.astype(np.float64) - o["f64"]).reshape(B, -1).max(1)
    rew = np.zeros(B, np.float32)
    done = np.zeros(B, np.uint8)
    for t in range(steps):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        g = gpu.step(torch.from_numpy(a).to(device))[0].cpu().numpy()
        for p, e in orc.items():
            o[p] = np.zeros((B, R, 2, 7), np.float32)
            e.step_omp(a, abi.CP_ACTION_DISCRETE, o[p], rew, done, threads)
        d32 = np.maximum(d32, np.abs(g - o["f32"]).reshape(B, -1).max(1))
        d64[t + 1] = np.abs(g.astype(np.float64) - o["f64"]).reshape(B, -1).max(1)
    gpu.close()
    per_env = d64.max(0)
    return {"envs": B, "steps": steps, "workload": "C3 config (seed 1234, random discrete actions, autoreset)",
            "max_abs_pose_diff_vs_oracle_f32": float(d32.max()), "bit_exact_vs_oracle_f32": bool(d32.max() == 0.0),
            "max_abs_pose_drift_vs_oracle_f64": float(per_env.max()),
            "median_env_max_drift_vs_oracle_f64": float(np.median(per_env)),
            "max_drift_vs_oracle_f64_after_step": {str(k): float(d64[k].max()) for k in (1, 20, 100, steps)},
            "vs_pybullet": None,
            "note": "pybullet is not installed (parity with it unpinned); the fp64 column is the same algorithm in "
                    "double precision: fp32 rounding differences grow through contact events (DESIGN.md §7)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--raster", action="store_true",
                    help="BASELINE.json configs[4] (C5): + in-kernel 50x50x3 fp16 raster obs per repeat")
    ap.add_argument("--cameras", type=int, default=1)
    ap.add_argument("--done-on-bounds", action="store_true",
                    help="the reference's commented-out bounds termination (bullet_cartpole.py:243-253): "
                         "episodes end early, so the C4 return histogram is not degenerate (diagnostic config)")
    ap.add_argument("--solver-iterations", type=int, default=None,
                    help="override the PGS sweep cap (default: the model's 50; non-default runs are diagnostics)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    B, R, K, W = args.batch, args.repeats, args.steps, args.warmup
    spec = shard_spec(B, rank, world, seed=1234 + rank)
    env = BatchedCartpole(B, local, action_repeats=R, steps_per_repeat=1, max_episode_len=200,
                          initial_force=55.0, autoreset=True, seed=spec["seed"], done_on_bounds=args.done_on_bounds,
                          env_id_offset=spec["env_id_offset"],
                          **({} if args.solver_iterations is None else {"solver_iterations": args.solver_iterations}))
    if args.raster:
        env.enable_raster(True, num_cameras=args.cameras)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    actions = torch.randint(0, 5, (W + K, B, 2), dtype=torch.int8, device=dev, generator=gen)
    env.reset()
    for t in range(W):
        env.step(actions[t])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    log(f"rank {rank}: B={B} R={R} warmup {W} done; timing {K} steps")

    env.timing_begin(K)
    env.timing_stride(STEP_EVENT_STRIDE, 1)
    hist = None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(K):
        env.step(actions[W + t])
        if (t + 1) % WINDOW == 0:
            r, _ = env.episode_returns()
            hist = return_histogram(gather_returns(r), 200)   # RCCL all-gather when world > 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tm = env.timing_end()
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    value = world * B * K / elapsed
    per_launch_s = tm["step_ms"] / max(1, tm["step_launches"]) / 1e3
    bytes_launch = B * step_kernel_bytes(R, 2)
    achieved = bytes_launch / per_launch_s / 1e9
    kernel = "cp_step_kernel<discrete>"
    traffic, traffic_src = pmc_traffic(kernel, B, R)
    if args.raster:
        # C5: the render kernel writes 2.9 GB per step and is the dominant HBM consumer
        rc = env.raster_cfg
        per_launch_s = tm["render_ms"] / max(1, tm["render_launches"]) / 1e3  # one launch per step
        bytes_launch = B * render_kernel_bytes(rc.height, rc.width, rc.num_cameras, R)
        achieved = bytes_launch / per_launch_s / 1e9
        kernel = "cp_render_small_kernel"
        traffic, traffic_src = pmc_traffic(kernel, B, R)
    valu = None
    if not args.raster:
        vi, vsrc = pmc_valu(kernel, B, R)
        if vi is not None:
            ach = vi / per_launch_s
            valu = {"bound": "valu-issue (secondary; the kernel is latency-bound, DESIGN.md §5)",
                    "wave_instructions_per_launch": vi, "achieved": round(ach / 1e12, 4),
                    "peak": round(VALU_PEAK_WINST_PER_S / 1e12, 4), "unit": "T wave-instr/s",
                    "frac": round(ach / VALU_PEAK_WINST_PER_S, 4), "source": vsrc + " SQ_INSTS_VALU"}
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (random discrete actions, Philox bump pushes; no pybullet, see DESIGN.md)",
        "config": {"workload": ("C5: batch=65,536 envs/GPU, discrete 5-action, R=3, S=1, autoreset at 200, "
                                "initial_force=55, fp32 physics + in-kernel raster obs 50x50x3xR fp16 to HBM "
                                f"({args.cameras} camera(s); BASELINE.json configs[4])") if args.raster else
                               ("C3: batch=65,536 envs/GPU, discrete 5-action, R=3, S=1, autoreset at 200, "
                                "initial_force=55, fp32 (BASELINE.json configs[2]; N>1 = C4 with RCCL all-gather "
                                "of episode returns per 200-step window)"),
                   "global_batch": world * B, "envs_per_gpu": B, "action_repeats": R, "steps_per_repeat": 1,
                   "parallelism": f"dp{world} (independent env shards, no per-step collective)",
                   "solver_iterations": env.cfg.phys.solver_iterations},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": traffic_src and (traffic_src + " (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 "
                                                        "per launch, rocprofv3 --pmc, separate passes"),
                     "kernel": kernel,
                     "bytes_per_launch": bytes_launch,
                     "avg_launch_ms": round(per_launch_s * 1e3, 4),
                     "launches": tm["step_launches"],
                     "launch_sample_stride": STEP_EVENT_STRIDE,
                     "reset_kernel_avg_ms": round(tm["reset_ms"] / max(1, tm["reset_launches"]), 4),
                     **({"step_kernel_avg_ms": round(tm["step_ms"] / max(1, tm["step_launches"]), 4),
                         "render_launches": tm["render_launches"]} if args.raster else {})},
        "valu": valu,
        "episode_return_hist_nonzero": None if hist is None else int((hist > 0).sum().item()),
        "done_on_bounds": bool(args.done_on_bounds),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        out["cpu_baseline"] = cpu_baseline(R, args.cpu_seconds)
        log("parity vs oracle ...")
        out["parity"] = parity_check(dev, R)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
