#!/usr/bin/env python3
"""Phase breakdown of the step and reset kernels from a stamp build (diagnostic, not a benchmark):
    python -m cartpoleplusplus_amd.build --stamps
    CP_LIB_PATH=.../libcartpole_hip_stamps.so python tools/stamps.py
Runs the bench workload (B envs, discrete, R=3, autoreset; BOUNDS=1 adds the reference's bounds
termination, whose desynchronised resets run the latency-shaped reset kernel) and prints
s_memtime cycles per wave per substep for each phase of each kernel.  Stamp fences perturb the
schedule: read the shares, not the absolute time (cdna_hip_programming.md §7)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402

B = int(os.environ.get("B", "65536"))
steps = int(os.environ.get("STEPS", "150"))
warm = int(os.environ.get("WARM", "20"))
bounds = os.environ.get("BOUNDS", "0") == "1"
env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True, seed=1234, done_on_bounds=bounds)
if os.environ.get("SHAPE"):   # e.g. SHAPE=latency,wide (step, reset); default: the library's choice
    env.set_kernel_shape(*os.environ["SHAPE"].split(","))
gen = torch.Generator(device="cuda").manual_seed(1234)
acts = torch.randint(0, 5, (steps + warm, B, 2), dtype=torch.int8, device="cuda", generator=gen)
env.reset()
for t in range(warm):
    env.step(acts[t])
out = (C.c_uint64 * 64)()
rc = env.lib.cp_debug_stamps(env.h, out, 1)
assert rc == 1, "not a stamp build (set CP_LIB_PATH to libcartpole_hip_stamps.so)"
for t in range(steps):
    env.step(acts[warm + t])
env.lib.cp_debug_stamps(env.h, out, 0)
res = {"B": B, "steps": steps, "done_on_bounds": bounds, "kernel_shape": env.kernel_shape()}
for name, base in (("step_kernel", 0), ("reset_kernel", 16)):
    narrow, vel, solve, integ, sweeps, substeps, total, waves = list(out)[base:base + 8]
    sel, bb, rows = list(out)[base + 8:base + 11]
    per = lambda x: x / max(1, substeps)  # noqa: E731
    res[name] = {"waves": waves, "substeps_per_wave": substeps / max(1, waves),
                 "cycles_per_wave_substep": {"narrowphase+setup": per(narrow), "velocity+warmstart": per(vel),
                                             "pgs_sweeps": per(solve), "integrate+cache": per(integ),
                                             "kernel_total_per_substep": total / max(1, substeps)},
                 "narrowphase_split_per_wave_substep": {"box_selection": per(sel), "box_box": per(bb),
                                                        "row_setup": per(rows)},
                 "sweeps_per_wave_substep": sweeps / max(1, substeps),
                 "cycles_per_sweep": solve / max(1, sweeps),
                 "kernel_cycles_per_wave": total / max(1, waves)}
    wmax, rt_end, rt_start_c, rt_sum, rt_max = list(out)[base + 11:base + 16]
    if waves and rt_sum:
        # s_memrealtime is a 100 MHz clock; the spans below are summed over every launch of the run
        mean_rt = rt_sum / waves
        res[name]["wave_duration"] = {"longest_wave_cycles": wmax, "mean_wave_us": mean_rt / 100.0,
                                      "longest_wave_us": rt_max / 100.0,
                                      "shader_clock_ghz": (total / waves) / mean_rt / 10.0,
                                      "first_start_to_last_end_us_all_launches":
                                          (rt_end - ((~rt_start_c) & (2 ** 64 - 1))) / 100.0}
o = list(out)
res["step_kernel"]["waves_by_slow_paths"] = {
    ("+".join(n for bit, n in ((1, "merged"), (2, "ground_cart_not_z"), (4, "ground_pole_not_z")) if f & bit) or "none"):
        {"waves": o[32 + 2 * f], "mean_us": o[33 + 2 * f] / max(1, o[32 + 2 * f]) / 100.0}
    for f in range(8) if o[32 + 2 * f]}
res["step_kernel"]["wave_duration_hist_50us"] = o[48:64]
print(json.dumps(res, indent=1))
