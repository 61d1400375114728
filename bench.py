#!/usr/bin/env python3
"""bench.py — batched cartpole++ env-steps/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]                       # C3 (default)
    python bench.py --continuous --batch 4096                             # C2
    python bench.py --raster                                              # C5
    python bench.py --gpus N                                              # C4: launches N ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W            # C4, externally launched

Multi-GPU launch: with --gpus N > 1 and no WORLD_SIZE in the environment, this process counts the
visible devices (dist.visible_gpu_count(): KFD sysfs topology + accessible render nodes, never the HIP
runtime), refuses with a
clear error when fewer than N are visible, and otherwise starts torch.distributed.run with N
ranks on 127.0.0.1 as a CHILD process (no exec, no GPU call in this parent) and exits with its
code; the ranks run this same file.  Under an external launcher WORLD_SIZE must equal --gpus.
Every rank checks the process group's size (rccl_world_size in the line) against --gpus.

Workloads (the line's config.workload is derived from the arguments):
  C2  4,096 envs, continuous (B,2,2) U[-1,1] actions, R = 3
  C3  65,536 envs per GPU, discrete 5-action U{0..4}, R = 3 (the headline, configs[2])
  C4  C3 on N GPUs: envs shard (global env id = rank*B + i keys the bump Philox stream and
      the action stream, one seed on every rank), RCCL all-gather of the episode returns
  C5  C3 + in-kernel 50x50x3 fp16 raster obs
All: steps_per_repeat 1, initial_force 55, max_episode_len 200, in-kernel autoreset, fp32.
A "step" is one env-step of every env: one cp_step call = one fused R-substep kernel
launch + one compacted reset launch.  Actions are pre-generated in HBM (a hash of
(seed, global env id, step, cart)), so sharded runs see the unsharded job's actions.

Timing: W untimed steps, then EXACTLY K steps between barrier + synchronize; value =
N*B*K / max-over-ranks wall.  A K-step window need not contain an autoreset burst (every
episode is 200 steps) or, at N > 1, a return gather; so the line also reports
resets_in_window, collectives_in_window, and a steady_state sub-object: one more full
200-step cycle (its reset burst and one gather included) timed the same way.
SURVEY.md §8d's "median of 5 runs": `median5` holds the headline window and 4 more K-step
windows right after it (same definition as value, each its own barrier + synchronize), and
steady_state.median5 five consecutive 200-step cycles; value itself stays the first window.

roofline: the step kernel's algorithmic HBM bytes per launch over its
average duration from HIP events recorded on its launch stream in the timed region
(every 4th launch sampled: the events themselves cost wall time).
cpu_baseline (rank 0, N = 1): the oracle (a port: same algorithm, gcc -O3 -march=native,
the kernel's results) on bounded samples: C3 on every CPU of the process's affinity mask
(OpenMP; `value`), on 16 threads and on one core, and C1.
parity (rank 0, N = 1): SURVEY.md §8d's matrix, GPU vs the oracle's fp32 build (bit-exact
bar) and fp64 build (drift), with and without the PGS early exit; every GPU handle of the
parity leg runs the kernel shapes the timed region ran (cp_set_kernel_shape).
secondary (rank 0, N = 1, the default C3 run only): the other configurations DESIGN.md §5
reports (cp_rollout K = 200, bounds termination in both autoreset modes, fp64, C2), each on a
fresh handle and timed the same way, so the driver's own run observes them.
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

from cartpoleplusplus_amd import abi  # noqa: E402
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402
from cartpoleplusplus_amd.dist import gather_returns, return_histogram, shard_spec, visible_gpu_count  # noqa: E402

METRIC = "env-steps/sec at batch=65,536, 1→8 MI355X; max |pose−pybullet| over 200 steps"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured)
WINDOW = 200            # episode length = return-gather window (steps)
SEED = 1234             # one seed for bumps and actions, on every rank
# HIP events around every 4th step-kernel launch (every reset launch): each recorded event
# costs the stream a few microseconds (tools/timing_overhead.py: 0.761 ms/step with events on
# every launch, 0.755 with this sampling, 0.748 without events)
STEP_EVENT_STRIDE = 4
# MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, a wave64 VALU instruction takes 2 issue
# cycles of its SIMD (one wave alone sustains one per 4), 2.4 GHz max clock
VALU_PEAK_WINST_PER_S = 256 * 4 * 2.4e9 / 2


def native_lib_path():
    from cartpoleplusplus_amd import native
    return native.LIB_PATH


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------- actions
_M32 = 0xFFFFFFFF


def _mix32(x):
    """lowbias32 integer hash (Wellons), on int64 tensors holding 32-bit values."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def action_block(continuous, gid, t0, n, seed):
    """Actions of steps [t0, t0+n) for global env ids `gid` (int64, device): a pure function
    of (seed, global env id, step, cart), so a shard computes exactly the rows the unsharded
    job would give its envs.  continuous: float32 (n, B, 2, 2) U[-1, 1) (the declared Box,
    bullet_cartpole.py:94); discrete: int8 (n, B, 2) U{0..4}."""
    dev = gid.device
    t = torch.arange(t0, t0 + n, device=dev, dtype=torch.int64).view(n, 1, 1)
    c = torch.arange(4 if continuous else 2, device=dev, dtype=torch.int64).view(1, 1, -1)
    g = gid.view(1, -1, 1)
    x = _mix32((seed * 0x9E3779B1 + t * 0x85EBCA77 + c * 0xC2B2AE3D) & _M32)
    x = _mix32((x ^ (g & _M32)) & _M32)
    x = _mix32((x + ((g >> 32) * 0x27D4EB2F)) & _M32)
    if continuous:
        u = (x >> 8).to(torch.float32) * (1.0 / (1 << 24))
        return (2.0 * u - 1.0).view(n, -1, 2, 2)
    return ((x * 5) >> 32).to(torch.int8)


def make_actions(continuous, B, env_id_offset, steps, seed, dev):
    gid = torch.arange(env_id_offset, env_id_offset + B, device=dev, dtype=torch.int64)
    blocks, t, chunk = [], 0, max(1, (1 << 24) // (B * 4))
    while t < steps:
        n = min(chunk, steps - t)
        blocks.append(action_block(continuous, gid, t, n, seed))
        t += n
    return torch.cat(blocks)


# ------------------------------------------------------------------- roofline
def step_kernel_bytes(R, action_bytes, real_bytes=4):
    """Algorithmic HBM bytes one env moves in one step-kernel launch; the
    state SoA holds the handle's real type (4 B, or 8 B for the fp64 variant)."""
    state_read = 52 + 6 + 2            # 4 bodies x 13, 2 pending forces x 3, steps, done
    state_write = 52 + 6 + 1           # bodies, pending forces, steps
    warm_cache = 2 * (10 + 40)         # warm-start ids + impulses, read + write once per step
    return real_bytes * (state_read + state_write + warm_cache) + action_bytes + 4 * 14 * R + 4 + 1 + 8


def render_kernel_bytes(H, W, C, R):
    """Algorithmic HBM bytes of one env's raster obs (render kernel): the float16 image
    (H, W, 3, C, R) written once, the R x 4 repeat-end poses read, one list entry."""
    return 2 * H * W * 3 * C * R + 4 * R * 4 * 7 + 4


def _pmc_files():
    import glob
    return list(reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))))


def lib_sha256(path=None):
    """sha256 of the HIP library this process runs (CP_LIB_PATH or the in-tree build): a PMC summary
    counts only for the binary it was collected on."""
    import hashlib
    from cartpoleplusplus_amd import native
    with open(path or native.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# the keys a PMC summary's "workload" must carry, equal to the timed run's, for its counters to be
# attached to the bench line (tools/summarize_profile.py writes them from the profiled bench line)
PMC_KEYS = ("batch", "repeats", "action_kind", "dtype", "step_shape", "lib_sha256")


def _pmc_match(d, want):
    """None when summary d was collected on the workload `want` (every PMC_KEYS entry present and
    equal), else the reason it does not count.  A missing key is a mismatch, never a match."""
    w = d.get("workload")
    if not isinstance(w, dict):
        return "no workload keys"
    for k in PMC_KEYS:
        if k not in w:
            return f"no {k!r} key"
        if w[k] != want.get(k):
            return f"{k} {w[k]!r} != {want.get(k)!r}"
    return None


def _pmc_lookup(kernel, want, get, files=None):
    """(value, source, None) from the newest summary of `kernel` that matches `want`, else
    (None, None, reason)."""
    reasons = []
    for p in (_pmc_files() if files is None else files):
        with open(p) as f:
            d = json.load(f)
        k = d.get("kernels", {}).get(kernel)
        v = get(k) if k else None
        if v is None:
            continue
        why = _pmc_match(d, want)
        if why is None:
            return v, os.path.relpath(p, ROOT), None
        reasons.append(f"{os.path.basename(p)}: {why}")
    if not reasons:
        return None, None, f"no PMC summary holds {kernel}"
    more = f" (+{len(reasons) - 3} more)" if len(reasons) > 3 else ""
    return None, None, "no PMC summary matches the timed workload and library: " + "; ".join(reasons[:3]) + more


def pmc_traffic(kernel, want, files=None):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_pmc.json, tools/profile.sh + tools/summarize_profile.py) collected on this
    workload with this library -> (bytes, source, reason-if-None)."""
    return _pmc_lookup(kernel, want, lambda k: k.get("hbm_bytes_per_launch"), files)


def pmc_valu(kernel, want, files=None):
    """VALU wave-instructions per launch of `kernel` (SQ_INSTS_VALU), same matching."""
    return _pmc_lookup(kernel, want, lambda k: k.get("sq_per_launch", {}).get("SQ_INSTS_VALU"), files)


# ------------------------------------------------------------------- workload
def workload(args, world):
    B, R = args.batch, args.repeats
    act = "continuous 2D action U[-1,1] (B,2,2) fp32" if args.continuous else "discrete 5-action U{0..4} int8"
    name = "custom"
    if args.raster:
        name = "C5" if (B == 65536 and not args.continuous) else "custom"
    elif args.continuous:
        name = "C2" if B == 4096 else "custom"
    elif B == 65536:
        name = "C4" if world > 1 else "C3"
    idx = {"C2": 1, "C3": 2, "C4": 3, "C5": 4}.get(name)
    s = (f"{name}: batch={B:,} envs/GPU x {world} GPU(s) = {B * world:,} envs, {act}, R={R}, S=1, "
         f"autoreset at {WINDOW}, initial_force=55, {args.dtype}")
    if args.raster:
        s += f", + in-kernel raster obs 50x50x3xR fp16 to HBM ({args.cameras} camera(s))"
    if world > 1:
        s += ", RCCL all-gather of episode returns per 200-step window"
    if args.done_on_bounds:
        s += ", bounds termination on (bullet_cartpole.py:243-253)"
    if args.solver_iterations is not None:
        s += f", solver_iterations={args.solver_iterations} (diagnostic)"
    if getattr(args, "streams", 1) > 1:
        s += f", as {args.streams} shard handles of {B // args.streams:,} envs on {args.streams} HIP streams"
    if getattr(args, "shape", "auto") != "auto":
        s += f", kernel shape {args.shape}"
    if getattr(args, "reset_shape", None) not in (None, "auto"):
        s += f", reset kernel shape {args.reset_shape}"
    if getattr(args, "persistent", False):
        s += ", CP_MODEL_PERSISTENT contact model (Bullet's persistent manifold; model-fidelity variant)"
    if getattr(args, "sleeping", False):
        s += ", CP_MODEL_SLEEPING (Bullet's deactivation of resting islands; model-fidelity variant)"
    if getattr(args, "rollout", 0):
        s += f", cp_rollout launches of up to {args.rollout} steps (not the per-step cp_step headline)"
    if getattr(args, "autoreset", "same_step") == "next_step":
        s += (", NEXT_STEP autoreset (gymnasium >= 1.0 / envpool semantics: a finishing env's reset is handed "
              "out by the next call and runs on a library stream in between; value counts simulated env-steps "
              "only, not those reset-only calls)")
    if idx is not None:
        s += f" (BASELINE.json configs[{idx}])"
    return name, s


class StreamShards:
    """`--streams S`: the GPU's batch as S shard handles of B/S envs (the C4 shard rule inside one
    GPU: one seed, env_id_offset = global id of the shard's first env, actions keyed by global env
    id, so every env computes exactly what it computes in one B-env handle), each stepped on its
    own HIP stream.  One cp_step per shard per step; a shard's next step starts as soon as ITS
    previous step is done, so the tail of one shard's launch overlaps the other shards' waves.
    Exposes the subset of BatchedCartpole that main() uses."""

    def __init__(self, S, B, device, env_id_offset, **kw):
        assert B % S == 0, "--streams must divide the batch"
        self.S, self.b = S, B // S
        self.envs = [BatchedCartpole(self.b, device, env_id_offset=env_id_offset + k * self.b, **kw) for k in range(S)]
        self.streams = [torch.cuda.Stream(self.envs[0].device) for _ in range(S)]
        self.cfg = self.envs[0].cfg
        self.device = self.envs[0].device

    def _each(self, fn):
        cur = torch.cuda.current_stream(self.device)
        out = []
        for e, st in zip(self.envs, self.streams):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                out.append(fn(e))
        for st in self.streams:
            cur.wait_stream(st)
        return out

    def set_kernel_shape(self, step, reset):
        for e in self.envs:
            e.set_kernel_shape(step, reset)

    def kernel_shape(self):
        return self.envs[0].kernel_shape()

    def reset(self):
        self._each(lambda e: e.reset())

    def step(self, actions):
        # no cross-stream waits between steps: each shard's stream orders its own steps
        for k, (e, st) in enumerate(zip(self.envs, self.streams)):
            with torch.cuda.stream(st):
                e.step(actions[k * self.b:(k + 1) * self.b])

    def rollout(self, actions):
        for k, (e, st) in enumerate(zip(self.envs, self.streams)):
            with torch.cuda.stream(st):
                e.rollout(actions[:, k * self.b:(k + 1) * self.b])

    def episode_returns(self):
        rs = self._each(lambda e: e.episode_returns())
        return torch.cat([r for r, _ in rs]), torch.cat([n for _, n in rs])

    def get_state(self):
        return torch.cat(self._each(lambda e: e.get_state()), dim=1)

    def timing_begin(self, n):
        for e in self.envs:
            e.timing_begin(n)

    def timing_stride(self, a, b):
        for e in self.envs:
            e.timing_stride(a, b)

    def timing_end(self):
        ts = [e.timing_end() for e in self.envs]
        out = {k: sum(t[k] for t in ts) / len(ts) for k in ("step_ms", "reset_ms", "render_ms")}
        out.update({k: ts[0][k] for k in ("step_launches", "reset_launches", "render_launches")})
        return out

    def nonfinite_counts(self):
        return torch.cat(self._each(lambda e: e.nonfinite_counts()))

    def close(self):
        for e in self.envs:
            e.close()


def episodes(env):
    """Per-env episode counters (resets so far), int64 on the device."""
    st = env.get_state()[abi.CP_SF_EPISODE]
    if st.dtype == torch.float64:
        return st.view(torch.int32)[0::2].to(torch.int64)
    return st.view(torch.int32).to(torch.int64)


def pending(env):
    """CP_AUTORESET_NEXT_STEP: envs whose reset ran (or is in flight) and is handed out by the next step."""
    st = env.get_state()[abi.CP_SF_DONE]
    d = st.view(torch.int32)[0::2] if st.dtype == torch.float64 else st.view(torch.int32)
    return int((d >= 2).sum().item())


def simulated_steps(env, B, K, ep0, p0, next_step):
    """Env-steps simulated by K calls: B*K, less the calls that only hand out a NEXT_STEP reset (the
    resets launched before the window's end, minus the ones still pending after it, plus the ones
    pending at its start).  -> (env-steps, resets run in the window)."""
    ran = int((episodes(env) - ep0).sum().item())
    if not next_step:
        return B * K, ran
    return B * K - (ran + p0 - pending(env)), ran


LAST_ENQUEUE_S = 0.0


def timed(env, actions, t0, K, world, dev, gather_at_end, rollout=0):
    """K steps between barrier + synchronize; -> (max-over-ranks seconds, histogram, gathers).
    rollout > 0: the steps run as cp_rollout launches of up to `rollout` steps, split at the
    200-step window boundaries (where the return gather runs)."""
    hist, gathers = None, 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    start = time.perf_counter()
    t = 0
    while t < K:
        if rollout:
            n = min(rollout, K - t, WINDOW - (t0 + t) % WINDOW)
            env.rollout(actions[t0 + t:t0 + t + n])
        else:
            n = 1
            env.step(actions[t0 + t])
        t += n
        if (t0 + t) % WINDOW == 0:
            r, _ = env.episode_returns()
            hist = return_histogram(gather_returns(r), WINDOW)   # RCCL all-gather when world > 1
            gathers += 1
    if gather_at_end and gathers == 0:
        r, _ = env.episode_returns()
        hist = return_histogram(gather_returns(r), WINDOW)
        gathers += 1
    global LAST_ENQUEUE_S
    LAST_ENQUEUE_S = time.perf_counter() - start   # host time to enqueue the K steps (diagnostic)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - start], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item()), hist, gathers


# ----------------------------------------------------------------- CPU legs
def host_cpus():
    """The CPUs this process may actually use: the affinity mask, capped by the cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs_quota_us) and by OMP_NUM_THREADS when the launcher sets it to the
    process's CPU share.  On the GPU box the mask lists the whole machine (256) while the share is
    16: 256 OpenMP threads on 16 CPUs time-slice through every per-step barrier (16 k env-steps/s
    measured, rd3f) instead of using the 16 CPUs."""
    import math
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                info["cgroup_quota_cpus"] = math.ceil(int(q) / int(per))
        except (OSError, ValueError):
            pass
    if info["cgroup_quota_cpus"] is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                info["cgroup_quota_cpus"] = math.ceil(q / per)
        except (OSError, ValueError):
            pass
    n = info["affinity_cpus"]
    if info["cgroup_quota_cpus"]:
        n = min(n, info["cgroup_quota_cpus"])
    try:
        if info["omp_num_threads"]:
            n = min(n, int(info["omp_num_threads"]))
    except ValueError:
        pass
    info["usable_cpus"] = max(1, n)
    return info


def cpu_baseline(R, budget_s):
    """The oracle (port) on the host, -O3 -march=native: C3 on all cores, C3 on one core,
    C1 (B = 1, R = 2) on one core; each a bounded sample of about budget_s seconds."""
    import numpy as np

    from oracle import oracle as O
    cpus = host_cpus()
    all_cpus = cpus["usable_cpus"]
    lib = O.load("native")

    def run(B, steps, threads_, R_, seed):
        cfg = O.default_config(num_envs=B, action_repeats=R_, initial_force=55.0, seed=seed, autoreset=1)
        e = O.Envs(cfg, precision="native")
        e.reset()
        rng = np.random.default_rng(seed)
        acts = rng.integers(0, 5, (steps, B, 2)).astype(np.int8)
        obs = np.zeros((B, R_, 2, 7), np.float32)
        rew = np.zeros(B, np.float32)
        done = np.zeros(B, np.uint8)
        t0 = time.perf_counter()
        used = 1
        for t in range(steps):
            used = e.step_omp(acts[t], abi.CP_ACTION_DISCRETE, obs, rew, done, threads_)
        return time.perf_counter() - t0, used, obs

    # the native build computes the parity build's numbers (no fast-math, no contraction)
    B0 = 64
    _, _, o_nat = run(B0, 3, 1, R, 7)
    cfg = O.default_config(num_envs=B0, action_repeats=R, initial_force=55.0, seed=7, autoreset=1)
    e32 = O.Envs(cfg)
    e32.reset()
    rng = np.random.default_rng(7)
    for _ in range(3):
        o32 = e32.step(rng.integers(0, 5, (B0, 2)).astype(np.int8))[0]
    same = bool(np.array_equal(o_nat, o32))

    def sized(threads_, budget):
        probe_b = 64 * threads_
        dt, _, _ = run(probe_b, 10, threads_, R, SEED)
        rate = probe_b * 10 / dt
        steps = WINDOW + 1                  # one full episode incl. an in-step autoreset
        B = int(min(65536, max(64, rate * budget / steps)))
        B -= B % 64
        dt, used, _ = run(max(B, 64), steps, threads_, R, SEED)
        return {"value": round(max(B, 64) * steps / dt, 1), "cores": used,
                "sample": f"{max(B, 64)} envs x {steps} steps ({dt:.1f} s)"}

    omp = sized(all_cpus, budget_s)
    t16 = sized(16, budget_s / 2) if all_cpus > 16 else omp
    one = sized(1, budget_s / 2)
    # C1: B = 1, R = 2 (reference default), discrete random actions, seeds 0..9, autoreset
    c1_steps, c1_t = 0, 0.0
    for seed in range(10):
        dt, _, _ = run(1, 2 * WINDOW, 1, 2, seed)
        c1_steps += 2 * WINDOW
        c1_t += dt
        if c1_t > budget_s / 2:
            break
    return {"value": omp["value"], "unit": "env-steps/s", "cores": omp["cores"], "kind": "port",
            "sample": (f"oracle/cp_oracle.c fp32 built gcc -O3 -march=native (same algorithm; bit-identical "
                       f"to the parity build: {same}), C3 workload (R={R}, discrete random actions, autoreset "
                       f"incl.), OpenMP on {omp['cores']} threads (every CPU the process may use: the "
                       f"affinity mask capped by the cgroup quota and the launcher's OMP_NUM_THREADS share): "
                       f"{omp['sample']}"),
            "threads_16": {"value": t16["value"], "unit": "env-steps/s", "cores": t16["cores"],
                           "sample": "C3 workload, " + t16["sample"]},
            "single_thread": {"value": one["value"], "unit": "env-steps/s", "cores": 1,
                              "sample": "C3 workload, " + one["sample"]},
            "c1_single_thread": {"value": round(c1_steps / c1_t, 1), "unit": "env-steps/s", "cores": 1,
                                 "sample": f"C1: B=1, R=2, discrete random actions, seeds 0..{seed}, "
                                           f"{c1_steps} steps incl. {c1_steps // WINDOW} resets ({c1_t:.1f} s)"},
            **cpus,
            "pybullet": "not importable (SURVEY.md §8c): the reference's own CPU path cannot be timed here"}


def gym_mirror_rate(steps=400):
    """The reference's own surface (BulletCartpole, B = 1, R = 2, discrete, numpy in / numpy copy
    out per step; the step one launch over pinned host buffers, step_io "zero_copy") on this GPU,
    for comparison with the CPU path's C1 rate: a B = 1 step is latency-bound (2 substeps of one wave)."""
    import argparse

    import numpy as np

    from cartpoleplusplus_amd import bullet_cartpole
    p = argparse.ArgumentParser()
    bullet_cartpole.add_opts(p)
    opts = p.parse_args(["--initial-force", "55"])
    env = bullet_cartpole.BulletCartpole(opts, discrete_actions=True)
    rng = np.random.default_rng(0)
    np_state = np.random.get_state()   # the mirror draws its bumps from np.random, as the reference does
    np.random.seed(0)
    try:
        env.reset()
        for _ in range(20):   # warm-up: the step graph's capture and the first launches stay out of the window
            env.step(rng.integers(0, 5, 2))
        t0 = time.perf_counter()
        env.reset()
        t_reset = time.perf_counter() - t0
        n, resets, t0 = 0, 0, time.perf_counter()
        while n < steps:
            _, _, done, _ = env.step(rng.integers(0, 5, 2))
            n += 1
            if done:
                env.reset()
                resets += 1
        dt = time.perf_counter() - t0
        step_io = env.step_io
        shape = "/".join(env._env.kernel_shape())
    finally:
        env.close()
        np.random.set_state(np_state)
    return {"value": round(n / dt, 1), "unit": "env-steps/s", "ms_per_step": round(dt / n * 1e3, 4),
            "reset_ms": round(t_reset * 1e3, 2), "step_io": step_io,
            "kernel_shape": shape,
            "sample": f"C1 config on the GPU: B=1, R=2, F_init 55, discrete random actions, {n} steps incl. "
                      f"{resets} resets ({dt:.2f} s), after 20 warm-up steps"}


def _pose_diffs(g, o):
    """per-step max over envs/repeats of |dpos| (xyz of cart + pole) and |dquat|."""
    import numpy as np
    d = np.abs(g.astype(np.float64) - o.astype(np.float64))
    return float(d[..., 0:3].max()), float(d[..., 3:7].max())


def _oracle_threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def parity_case(device, R, B, F, stream, steps, thr=None, seed=0, precision="f32", shape=None):
    """One SURVEY §8d parity run: B envs from reset (seed, F_init = F), 200 steps of one
    continuous action stream, GPU vs oracle; per step the max |dpos| and |dquat|.
    precision "f32": the fp32 kernels vs the oracle's f32 and f64 builds; "f64": the fp64
    kernel variant vs the oracle's f64 build."""
    import numpy as np

    from oracle import oracle as O
    threads = _oracle_threads()
    over = {} if thr is None else {"residual_threshold": thr}
    cfg = O.default_config(num_envs=B, action_repeats=R, initial_force=float(F), seed=seed, autoreset=0)
    for k, v in over.items():
        setattr(cfg.phys, k, v)
    if precision == "f64":
        cfg.precision = abi.CP_PRECISION_F64
    gpu = BatchedCartpole(B, device.index, config=abi.cp_config.from_buffer_copy(cfg))
    if shape is not None and precision == "f32":
        gpu.set_kernel_shape(*shape)
    orc = {p: O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=p)
           for p in (("f32", "f64") if precision == "f32" else ("f64",))}
    g = gpu.reset().cpu().numpy()
    o = {p: e.reset() for p, e in orc.items()}
    rng = np.random.default_rng(seed)
    rows = {p: [_pose_diffs(g, o[p])] for p in orc}
    # per env: the first step whose |dpos| (any repeat, cart or pole) exceeds 1e-4 (steps + 1: never)
    first_env = {p: np.full(B, steps + 1, np.int64) for p in orc}

    def track(p, t, gg, oo):
        d = np.abs(gg[..., 0:3].astype(np.float64) - oo[..., 0:3].astype(np.float64)).reshape(B, -1).max(1)
        f = first_env[p]
        f[(d > 1e-4) & (f > steps)] = t
    rew = np.zeros(B, np.float32)
    done = np.zeros(B, np.uint8)
    for t in range(steps):
        if stream == "zero":
            a = np.zeros((B, 2, 2), np.float32)
        elif stream == "constant":
            a = np.broadcast_to(np.array([0.5, -0.25], np.float32), (B, 2, 2)).copy()
        else:
            a = rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
        g = gpu.step(torch.from_numpy(a).to(device))[0].cpu().numpy()
        for p, e in orc.items():
            o[p] = np.zeros((B, R, 2, 7), np.float32)
            e.step_omp(a, abi.CP_ACTION_CONTINUOUS, o[p], rew, done, threads)
            rows[p].append(_pose_diffs(g, o[p]))
            track(p, t + 1, g, o[p])
    gpu.close()
    out = {}
    for p, r in rows.items():
        r = np.array(r)   # (steps + 1, 2): step 0 = after reset
        first = np.nonzero(r[:, 0] > 1e-4)[0]
        out[p] = {"max_dpos": float(r[:, 0].max()), "max_dquat": float(r[:, 1].max()),
                  "dpos_at_step": {str(k): float(r[k, 0]) for k in (0, 1, 20, 100, steps)},
                  "dquat_at_step": {str(k): float(r[k, 1]) for k in (0, 1, 20, 100, steps)},
                  "first_step_dpos_over_1e-4": int(first[0]) if len(first) else None,
                  # the tolerance held, per env: steps from reset with |dpos| <= 1e-4 (min / median over envs)
                  "steps_within_1e-4_min_env": int(first_env[p].min() - 1),
                  "steps_within_1e-4_median_env": float(np.median(first_env[p] - 1))}
    return out


def parity_c3(device, R, shape, B=2048, steps=WINDOW + 20):
    """The bench workload itself (C3: bench.py's hashed discrete actions, autoreset, seed 1234)
    on the kernel shapes the timed region ran: GPU vs the fp32 oracle over 220 steps (one
    autoreset burst inside), the bit-exact bar."""
    import numpy as np

    from oracle import oracle as O
    threads = _oracle_threads()
    cfg = O.default_config(num_envs=B, action_repeats=R, initial_force=55.0, seed=SEED, autoreset=1)
    gpu = BatchedCartpole(B, device.index, config=abi.cp_config.from_buffer_copy(cfg))
    gpu.set_kernel_shape(*shape)
    ran = gpu.kernel_shape()
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    g, o = gpu.reset().cpu().numpy(), orc.reset()
    d, nbits = float(np.abs(g - o).max()), int(np.count_nonzero(g.view(np.uint32) != o.view(np.uint32)))
    acts = make_actions(False, B, 0, steps, SEED, device)
    rew = np.zeros(B, np.float32)
    done = np.zeros(B, np.uint8)
    for t in range(steps):
        g = gpu.step(acts[t])[0].cpu().numpy()
        o = np.zeros((B, R, 2, 7), np.float32)
        orc.step_omp(np.ascontiguousarray(acts[t].cpu().numpy()), abi.CP_ACTION_DISCRETE, o, rew, done, threads)
        d = max(d, float(np.abs(g - o).max()))
        nbits += int(np.count_nonzero(g.view(np.uint32) != o.view(np.uint32)))   # also catches -0.0 vs +0.0
    gpu.close()
    return {"envs": B, "steps": steps, "kernel_shape": {"step": ran[0], "reset": ran[1]},
            "max_abs_pose_diff": d, "elements_with_different_bits": nbits, "bit_exact": nbits == 0}


def parity_check(device, R, shape, B=128, steps=WINDOW):
    """SURVEY.md §8d's parity matrix: seed 0, F_init in {0, 55} x action streams {zero,
    constant (0.5, -0.25), random U[-1,1]}, 200 steps from reset, |dpos| and |dquat|
    separately, against the oracle's fp32 build (the kernel's bar: 0) and its fp64 build
    (the same algorithm in double precision: what pybullet's double btScalar would compute
    IF its algorithm is this one).  "early_exit": Bullet's stopping rule (max squared row
    residual <= 1e-7); "fixed_sweeps": threshold 0, every substep runs all 50 sweeps, so
    drift there is rounding alone, without the early exit's sweep-count jumps."""
    matrix = {}
    for variant, thr in (("early_exit", None), ("fixed_sweeps", 0.0)):
        for F in (0, 55):
            for stream in ("zero", "constant", "random"):
                log(f"  parity {variant} F={F} {stream}")
                matrix[f"{variant}/F{F}/{stream}"] = parity_case(device, R, B, F, stream, steps, thr, shape=shape)
    worst32 = max(max(v["f32"]["max_dpos"], v["f32"]["max_dquat"]) for v in matrix.values())
    # the fp32 tolerance the product holds (north_star's "stated fp32 tolerance on pose"): against the
    # same algorithm in fp64 (pybullet's btScalar is double), |dpos| <= 1e-4 m for the first N steps of
    # each case, N per the worst env and the median env (the early-exit rows are the product config)
    tol = {k.split("/", 1)[1]: {"worst_env_steps": v["f64"]["steps_within_1e-4_min_env"],
                                "median_env_steps": v["f64"]["steps_within_1e-4_median_env"]}
           for k, v in matrix.items() if k.startswith("early_exit/")}
    # the fp64 kernel variant (cp_config.precision = F64) on the early-exit cases: the GPU
    # computing the double-precision algorithm, against the oracle's fp64 build
    f64 = {}
    for F in (0, 55):
        for stream in ("zero", "constant", "random"):
            log(f"  parity fp64 kernel F={F} {stream}")
            r = parity_case(device, R, B, F, stream, steps, None, precision="f64")["f64"]
            f64[f"early_exit/F{F}/{stream}"] = {"max_dpos": r["max_dpos"], "max_dquat": r["max_dquat"]}
    worst64 = max(max(v["max_dpos"], v["max_dquat"]) for v in f64.values())
    return {"envs_per_case": B, "steps": steps, "repeats": R, "actions": "continuous (B,2,2)",
            "kernel_shape": {"step": shape[0], "reset": shape[1]},
            "bit_exact_vs_oracle_f32": worst32 == 0.0, "max_abs_diff_vs_oracle_f32": worst32,
            "fp32_tolerance": {"bound_m": 1e-4, "vs": "oracle fp64 build (same algorithm, double precision)",
                               "steps_within_bound": tol},
            "fp64_kernel_vs_oracle_f64": {"bit_exact": worst64 == 0.0, "max_abs_diff": worst64, "cases": f64},
            "c3_workload_vs_oracle_f32": parity_c3(device, R, shape),
            "matrix": matrix, "vs_pybullet": None,
            "note": "pybullet is not installed (parity with it unpinned, SURVEY.md §8c); f64 = the oracle's "
                    "algorithm in double precision, state kept in double (DESIGN.md §7)"}


# ------------------------------------------------------------ secondary lines
# Configurations other than the headline, measured inside the default run (rank 0, N = 1) so the
# driver's own run observes them: each on a fresh handle, reset + W untimed steps, then K steps
# timed like the headline (synchronize on both sides).  (name, envs, steps, kwargs, continuous,
# rollout K): the BASELINE.json configs and the modes DESIGN.md §5 reports.
SECONDARY = (
    ("C3_rollout_k200", 65536, 200, {}, False, 200),
    ("C3_bounds_next_step", 65536, 200, {"done_on_bounds": True, "autoreset": "next_step"}, False, 0),
    ("C3_bounds_same_step", 65536, 50, {"done_on_bounds": True}, False, 0),
    ("C3_f64", 65536, 200, {"precision": "f64"}, False, 0),
    ("C2_continuous_4096", 4096, 200, {}, True, 0),
    # the model switch of DESIGN.md §3 (latency-shaped kernels) and C5 (BASELINE configs[4]) in the driver's run
    ("C3_sleeping", 65536, 200, {"model_flags": abi.CP_MODEL_SLEEPING}, False, 0),
    ("C5_raster", 65536, 100, {"raster": True}, False, 0),
)


def secondary_lines(dev, R, W=20):
    """Each SECONDARY config: {value env-steps/s, ms_per_step, steps, warmup, resets}.  Bounds
    termination needs its episodes desynchronised before the window: W + 40 untimed steps."""
    out = {}
    for name, B, K, kw, continuous, rollout in SECONDARY:
        kw = dict(kw)
        autoreset = kw.pop("autoreset", "same_step")
        raster = kw.pop("raster", False)
        next_step = autoreset == "next_step"
        w = W + (40 if kw.get("done_on_bounds") else 0)
        if rollout:   # warm-up = one full-window launch, so the timed launch (from the window boundary) has
            w = WINDOW  # the same K: kernel, output buffers and the rollout's temporaries all warm
        env = BatchedCartpole(B, dev.index, action_repeats=R, steps_per_repeat=1, max_episode_len=WINDOW,
                              initial_force=55.0, autoreset=autoreset, seed=SEED, **kw)
        actions = make_actions(continuous, B, 0, w + K, SEED, dev)
        if raster:
            env.enable_raster(True)
        env.reset()
        if rollout:   # warm-up through the kernel itself, its output buffers allocated up front (~2 GB)
            env.reserve_rollout(rollout)
            env.rollout(actions[:w])
        else:
            for t in range(w):
                env.step(actions[t])
        r_, _ = env.episode_returns()   # the return-gather path warm (a window boundary falls in every leg)
        return_histogram(gather_returns(r_), WINDOW)
        del r_
        torch.cuda.synchronize()
        ep0 = episodes(env)
        p0 = pending(env) if next_step else 0
        if raster:   # the render kernel's own time (HIP events around each launch): its HBM roofline
            env.timing_begin(K)
            env.timing_stride(STEP_EVENT_STRIDE, 1)
        el, _, _ = timed(env, actions, w, K, 1, dev, gather_at_end=False, rollout=rollout)
        sim, ran = simulated_steps(env, B, K, ep0, p0, next_step)
        rend = {}
        if raster:
            tm = env.timing_end()
            rc = env.raster_cfg
            ms = tm["render_ms"] / max(1, tm["render_launches"])
            gbs = B * render_kernel_bytes(rc.height, rc.width, rc.num_cameras, R) / (ms / 1e3) / 1e9
            rend = {"render_avg_launch_ms": round(ms, 4), "render_achieved_GBps": round(gbs, 1),
                    "render_hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
        out[name] = {"value": round(sim / el, 1), "unit": "env-steps/s", "ms_per_step": round(el / K * 1e3, 4),
                     "envs": B, "steps": K, "warmup": w, "resets_in_window": ran,
                     "kernel_shape": dict(zip(("step", "reset"), env.kernel_shape())),
                     **({"rollout_k": rollout} if rollout else {}), **kw,
                     **({"autoreset": autoreset} if next_step else {}),
                     **({"raster": "50x50x3 fp16, 1 camera", "render_kernel": env.render_kernel_name(), **rend}
                        if raster else {})}
        env.close()
        del actions
        torch.cuda.synchronize()
    return out


# ----------------------------------------------------------------------- launch
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv, dry_run=False):
    """`--gpus N` without an external launcher: run this file as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) in a CHILD process and
    return its exit code.  Nothing here touches the GPU: dist.visible_gpu_count() counts the
    devices from the KFD topology in sysfs and the render nodes this process may open (amdsmi
    when sysfs has none), never through the HIP runtime, so the ranks own the GPUs from the start
    and no process that initialised the GPU ever execs.  The parent checks that HIP is still
    uninitialised right before the spawn and says so on a status line.  Fewer visible devices
    than N is an error (exit 2)."""
    import subprocess
    if not dry_run:
        visible, source = visible_gpu_count()
        hip_init = bool(torch.cuda.is_initialized())
        log(f"bench.py launcher: visible_gpus={visible} source={source} hip_initialized={hip_init}")
        if visible < n:
            log(f"bench.py: --gpus {n} needs {n} visible GPUs, {visible} visible "
                f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')!r}); not launching")
            return 2
        assert not torch.cuda.is_initialized(), "the launcher parent must not initialise HIP before the spawn"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    log("bench.py: launching " + " ".join(cmd))
    return subprocess.call(cmd, env=env)


def dry_run_rank(args, world, rank):
    """`--cpu-dry-run` (tests/test_bench_launch.py): the launch and collective path of a rank with no
    GPU work: the gloo process group, the shard rule and the return gather + histogram of bench's
    C4 window on synthetic returns (each env's return = its global id mod 201)."""
    dist.init_process_group("gloo")
    try:
        got = dist.get_world_size()
        if got != args.gpus:
            raise SystemExit(f"bench.py: process group has {got} ranks, --gpus {args.gpus}")
        B = args.batch or 65536
        spec = shard_spec(B, rank, world, seed=SEED)
        ids = torch.arange(spec["env_id_offset"], spec["env_id_offset"] + B, dtype=torch.int64)
        allret = gather_returns((ids % (WINDOW + 1)).to(torch.float32))
        hist = return_histogram(allret, WINDOW)
        expect = return_histogram((torch.arange(world * B) % (WINDOW + 1)).to(torch.float32), WINDOW)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "rccl_world_size": got, "backend": "gloo",
                              "global_batch": spec["global_batch"], "gathered": int(allret.numel()),
                              "hist_equal_unsharded": bool(torch.equal(hist, expect))}), flush=True)
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None, help="envs per GPU (default 65,536; 4,096 with --continuous)")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--continuous", action="store_true", help="C2: continuous (B,2,2) U[-1,1] actions")
    ap.add_argument("--dtype", choices=("f32", "f64"), default="f32",
                    help="f64: the fp64 kernel variant (cp_config.precision; the parity mode, DESIGN.md §7)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the cpu_baseline, parity and secondary legs (profiling runs: only the headline's kernels)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-steady-state", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary configurations (rollout, bounds, fp64, C2) measured after the headline")
    ap.add_argument("--raster", action="store_true",
                    help="BASELINE.json configs[4] (C5): + in-kernel 50x50x3 fp16 raster obs per repeat")
    ap.add_argument("--cameras", type=int, default=1)
    ap.add_argument("--done-on-bounds", action="store_true",
                    help="the reference's commented-out bounds termination (bullet_cartpole.py:243-253): "
                         "episodes end early, so the C4 return histogram is not degenerate (diagnostic config)")
    ap.add_argument("--rollout", type=int, default=0, metavar="K",
                    help="run the steps as cp_rollout launches of up to K steps (one launch advances every env "
                         "through K steps; a separately labelled line, not the per-step headline)")
    ap.add_argument("--streams", type=int, default=1, metavar="S",
                    help="run the GPU's batch as S shard handles on S HIP streams (the C4 shard rule inside one "
                         "GPU; each env computes what it computes in one handle)")
    ap.add_argument("--shape", choices=("auto", "throughput", "latency", "wide", "wide8"), default="auto",
                    help="kernel shapes (cp_set_kernel_shape) of the step and autoreset kernels")
    ap.add_argument("--reset-shape", choices=("auto", "throughput", "latency", "wide", "wide8", "wide64", "list"), default=None,
                    help="the autoreset kernel's shape when it differs from --shape")
    ap.add_argument("--sleeping", action="store_true",
                    help="the CP_MODEL_SLEEPING model (Bullet's deactivation: resting islands sleep after 2 s; "
                         "latency-shaped kernels; a model-fidelity variant, not the headline)")
    ap.add_argument("--persistent", action="store_true",
                    help="the CP_MODEL_PERSISTENT contact model (Bullet's persistent manifold; latency-shaped "
                         "kernels; a model-fidelity variant, not the headline)")
    ap.add_argument("--autoreset", choices=("same_step", "next_step"), default="same_step",
                    help="same_step: a finishing env is reset in its step (the headline); next_step: the reset is "
                         "handed out by the next step (gymnasium >= 1.0 / envpool), overlapped with the steps")
    ap.add_argument("--solver-iterations", type=int, default=None,
                    help="override the PGS sweep cap (default: the model's 50; non-default runs are diagnostics)")
    ap.add_argument("--no-median", action="store_true",
                    help="skip the 4 extra K-step windows and 4 extra cycles of the median-of-5 (median5)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="launch / collective path only, on CPU with gloo (no GPU work; tests the --gpus N launcher)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 4096 if args.continuous else 65536
    next_step = args.autoreset == "next_step"
    if next_step and (args.rollout or args.raster or args.streams > 1):
        ap.error("--autoreset next_step steps through cp_step only (no --rollout / --raster / --streams)")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], dry_run=args.cpu_dry_run))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but the launcher's WORLD_SIZE is {world}: they must agree")
    if args.cpu_dry_run:
        if world == 1:
            ap.error("--cpu-dry-run is for --gpus N > 1 (the launch path)")
        dry_run_rank(args, world, rank)
        return
    ndev = torch.cuda.device_count()
    if local >= ndev:
        raise SystemExit(f"bench.py: rank {rank} has LOCAL_RANK {local} but {ndev} GPU(s) are visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    rccl_world = dist.get_world_size() if world > 1 else 1
    if rccl_world != args.gpus:
        raise SystemExit(f"bench.py: process group has {rccl_world} ranks, --gpus {args.gpus}")

    B, R, K, W = args.batch, args.repeats, args.steps, args.warmup
    spec = shard_spec(B, rank, world, seed=SEED)
    env_kw = dict(action_repeats=R, steps_per_repeat=1, max_episode_len=WINDOW, initial_force=55.0,
                  autoreset=args.autoreset, seed=spec["seed"], done_on_bounds=args.done_on_bounds, precision=args.dtype,
                  **({} if args.solver_iterations is None else {"solver_iterations": args.solver_iterations}),
                  **({"model_flags": (abi.CP_MODEL_PERSISTENT if args.persistent else 0)
                      | (abi.CP_MODEL_SLEEPING if args.sleeping else 0)} if (args.persistent or args.sleeping) else {}))
    if args.streams > 1:
        env = StreamShards(args.streams, B, local, spec["env_id_offset"], **env_kw)
    else:
        env = BatchedCartpole(B, local, env_id_offset=spec["env_id_offset"], **env_kw)
    if args.shape != "auto" or args.reset_shape not in (None, "auto"):
        env.set_kernel_shape(args.shape, args.reset_shape or args.shape)
    if args.raster:
        env.enable_raster(True, num_cameras=args.cameras)
    ss_steps = 0 if args.no_steady_state else WINDOW
    n_med = 1 if args.no_median else 5
    actions = make_actions(args.continuous, B, spec["env_id_offset"], W + n_med * (K + ss_steps), SEED, dev)
    env.reset()
    if args.rollout and args.streams == 1:   # the rollout kernel loaded, its output buffers allocated (~2 GB)
        env.reserve_rollout(args.rollout)
        if W:
            env.rollout(actions[:W])
    else:
        for t in range(W):
            env.step(actions[t])
    # warm the return-gather path too (cp_episode_returns, the RCCL all-gather, torch's bincount):
    # their first call in a process loads code objects and sets up buffers, ~17 ms once, which would
    # otherwise land in whichever timed window holds the first 200-step boundary
    r_, _ = env.episode_returns()
    return_histogram(gather_returns(r_), WINDOW)
    del r_
    torch.cuda.synchronize()
    log(f"rank {rank}: B={B} R={R} warmup {W} done; timing {K} steps")

    ep0 = episodes(env)
    p0 = pending(env) if next_step else 0
    env.timing_begin(K)
    env.timing_stride(1 if args.rollout else STEP_EVENT_STRIDE, 1)
    elapsed, hist, gathers = timed(env, actions, W, K, world, dev, gather_at_end=world > 1, rollout=args.rollout)
    enqueue_ms = LAST_ENQUEUE_S / K * 1e3
    tm = env.timing_end()
    simulated, resets = simulated_steps(env, B, K, ep0, p0, next_step)

    def window(t0, n):
        """One more n-step window from step t0, timed like the headline: (value over ranks, seconds,
        resets, gathers, histogram, host enqueue s)."""
        epj = episodes(env)
        pj = pending(env) if next_step else 0
        el_, hist_, g_ = timed(env, actions, t0, n, world, dev, gather_at_end=world > 1, rollout=args.rollout)
        enq_ = LAST_ENQUEUE_S
        sim_, ran_ = simulated_steps(env, B, n, epj, pj, next_step)
        r_ = torch.tensor([ran_, sim_], device=dev, dtype=torch.int64)
        if world > 1:
            dist.all_reduce(r_)
        return int(r_[1].item()) / el_, el_, int(r_[0].item()), g_, hist_, enq_

    def med5(vals):
        s = sorted(vals)
        return {"median": round(s[len(s) // 2], 1), "min": round(s[0], 1), "max": round(s[-1], 1),
                "spread": round((s[-1] - s[0]) / s[len(s) // 2], 4), "values": [round(v, 1) for v in vals]}

    rt = torch.tensor([resets, simulated], device=dev, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(rt)
    value = int(rt[1].item()) / elapsed   # = world * B * K / elapsed except for NEXT_STEP's reset-only calls
    win_values = [value]
    for j in range(1, n_med):
        win_values.append(window(W + j * K, K)[0])
    median5 = None if n_med == 1 else {
        **med5(win_values), "windows": n_med, "steps_per_window": K,
        "note": "SURVEY.md §8d median of 5: the headline window (values[0] = value) and 4 more K-step windows "
                "right after it, each between barrier + synchronize"}

    steady = None
    if ss_steps:
        t_ss = W + n_med * K
        cyc = [window(t_ss + j * ss_steps, ss_steps) for j in range(n_med)]
        v2, el2, ran2, g2, hist2, enq2 = cyc[0]
        steady = {"steps": ss_steps, "ms_per_step": round(el2 / ss_steps * 1e3, 4),
                  "host_enqueue_ms_per_step": round(enq2 / ss_steps * 1e3, 4),
                  "value": round(v2, 1), "resets": ran2, "collectives": g2,
                  **({"median5": med5([c[0] for c in cyc])} if n_med > 1 else {}),
                  "note": "one full 200-step episode cycle (its autoreset burst included) after the timed "
                          "windows, timed the same way; median5 over 5 consecutive cycles (value = the first)"}
        hist = cyc[-1][4] if cyc[-1][4] is not None else hist

    # envs whose state went non-finite at any point of the run (every window above included)
    nf = torch.tensor([int((env.nonfinite_counts() > 0).sum().item())], device=dev, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(nf)
    kind = "continuous" if args.continuous else "discrete"
    per_launch_s = tm["step_ms"] / max(1, tm["step_launches"]) / 1e3
    bytes_launch = B * step_kernel_bytes(R, 16 if args.continuous else 2, 8 if args.dtype == "f64" else 4)
    kernel = f"cp_step_kernel<{kind}>" if args.dtype == "f32" else f"cp64::cp_step_kernel<{kind}>"
    if args.rollout:   # one launch = many env-steps: per-step kernel time = launch time / steps per launch
        per_launch_s = tm["step_ms"] / 1e3 / K
        kernel = kernel.replace("cp_step_kernel", "cp_rollout_kernel") + " (time per env-step of the launch)"
    achieved = bytes_launch / per_launch_s / 1e9
    shape = env.kernel_shape()
    lib_hash = lib_sha256()
    want = {"batch": B, "repeats": R, "action_kind": kind, "dtype": args.dtype, "step_shape": shape[0],
            "lib_sha256": lib_hash}
    traffic, traffic_src, traffic_why = pmc_traffic(kernel, want)
    if args.raster:
        # C5: the render kernel writes 2.9 GB per step and is the dominant HBM consumer
        rc = env.raster_cfg
        per_launch_s = tm["render_ms"] / max(1, tm["render_launches"]) / 1e3  # one launch per step
        bytes_launch = B * render_kernel_bytes(rc.height, rc.width, rc.num_cameras, R)
        achieved = bytes_launch / per_launch_s / 1e9
        kernel = env.render_kernel_name()   # the library's own choice (cp_render_kernel_name)
        traffic, traffic_src, traffic_why = pmc_traffic(kernel, want)
    valu = None
    if not args.raster:
        vi, vsrc, valu_why = pmc_valu(kernel, want)
        if vi is None:
            valu = {"null_reason": valu_why}
        else:
            ach = vi / per_launch_s
            valu = {"bound": "valu-issue (secondary; the kernel is latency-bound, DESIGN.md §5)",
                    "wave_instructions_per_launch": vi, "achieved": round(ach / 1e12, 4),
                    "peak": round(VALU_PEAK_WINST_PER_S / 1e12, 4), "unit": "T wave-instr/s",
                    "frac": round(ach / VALU_PEAK_WINST_PER_S, 4), "source": vsrc + " SQ_INSTS_VALU"}
    name, wl = workload(args, world)
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "host_enqueue_ms_per_step": round(enqueue_ms, 4),
        "median5": median5,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (hashed random actions keyed by global env id, Philox bump pushes; no pybullet, "
                "see DESIGN.md)",
        "config": {"workload": wl, "name": name, "global_batch": world * B, "envs_per_gpu": B, "action_repeats": R,
                   "steps_per_repeat": 1, "action_kind": kind, "kernel_shape": {"step": shape[0], "reset": shape[1]},
                   "parallelism": f"dp{world} (independent env shards, no per-step collective)",
                   "solver_iterations": env.cfg.phys.solver_iterations,
                   "residual_threshold": env.cfg.phys.residual_threshold},
        "resets_in_window": int(rt[0].item()),
        "autoreset": args.autoreset,
        **({"simulated_env_steps": int(rt[1].item()), "calls_x_envs": world * B * K} if next_step else {}),
        "collectives_in_window": gathers if world > 1 else 0,
        "rccl_world_size": rccl_world,
        "steady_state": steady,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": traffic_src and (traffic_src + " (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 "
                                                        "per launch, rocprofv3 --pmc, separate passes; "
                                                        "same workload and library sha256"),
                     **({"traffic_null_reason": traffic_why} if traffic is None else {}),
                     "kernel": kernel,
                     "bytes_per_launch": bytes_launch,
                     "avg_launch_ms": round(per_launch_s * 1e3, 4),
                     "launches": tm["step_launches"],
                     "launch_sample_stride": 1 if args.rollout else STEP_EVENT_STRIDE,
                     "reset_kernel_avg_ms": round(tm["reset_ms"] / max(1, tm["reset_launches"]), 4),
                     **({"step_kernel_avg_ms": round(tm["step_ms"] / max(1, tm["step_launches"]), 4),
                         "render_launches": tm["render_launches"]} if args.raster else {})},
        "valu": valu,
        "build": {"lib": os.path.relpath(native_lib_path(), ROOT), "lib_sha256": lib_hash},
        "episode_return_hist_nonzero": None if hist is None else int((hist > 0).sum().item()),
        "done_on_bounds": bool(args.done_on_bounds),
        "nonfinite_envs": int(nf.item()),
        "nonfinite_note": "envs (over all ranks) whose state went non-finite during the run (cp_nonfinite_counts); 0 "
                          "since the coordinate-velocity clamp (btMultiBody m_maxCoordinateVelocity, DESIGN.md §3) "
                          "bounds the loose-pole yaw spin that used to diverge",
    }
    env.close()
    del actions
    headline = not (args.rollout or args.continuous or args.dtype != "f32" or args.done_on_bounds or args.persistent
                    or args.sleeping
                    or args.streams > 1 or args.raster or next_step or args.shape != "auto"
                    or args.reset_shape not in (None, "auto")
                    or args.solver_iterations is not None or args.batch != 65536 or args.repeats != 3)
    if rank == 0 and world == 1 and headline and not (args.no_secondary or args.no_cpu_baseline):
        log("secondary configurations ...")
        out["secondary"] = secondary_lines(dev, R)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        out["cpu_baseline"] = cpu_baseline(R, args.cpu_seconds)
        out["gym_mirror_b1_gpu"] = gym_mirror_rate()   # a GPU B = 1 measurement, beside (not in) cpu_baseline
        if not args.no_parity:
            log("parity vs oracle ...")
            out["parity"] = parity_check(dev, R, shape)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
