#!/usr/bin/env python3
"""Phase breakdown of the step kernel from a stamp build (diagnostic, not a benchmark):
    hipcc ... -DCP_STAMPS -o cartpoleplusplus_amd/libcartpole_hip_stamps.so
    CP_LIB_PATH=.../libcartpole_hip_stamps.so python tools/stamps.py
Runs the bench workload (B=65536, discrete, R=3, autoreset) and prints s_memtime
cycles per wave per substep for each phase.  Stamp fences perturb the schedule:
read the shares, not the absolute time (cdna_hip_programming.md §7)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402

B = int(os.environ.get("B", "65536"))
steps = int(os.environ.get("STEPS", "150"))
env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True, seed=1234)
gen = torch.Generator(device="cuda").manual_seed(1234)
acts = torch.randint(0, 5, (steps + 20, B, 2), dtype=torch.int8, device="cuda", generator=gen)
env.reset()
for t in range(20):
    env.step(acts[t])
out = (C.c_uint64 * 16)()
rc = env.lib.cp_debug_stamps(env.h, out, 1)
assert rc == 1, "not a stamp build (set CP_LIB_PATH to libcartpole_hip_stamps.so)"
for t in range(steps):
    env.step(acts[20 + t])
env.lib.cp_debug_stamps(env.h, out, 0)
res = {"B": B, "steps": steps}
for name, vals in (("head", list(out)[:8]), ("tail", list(out)[8:])):
    narrow, vel, solve, integ, sweeps, substeps, total, waves = vals
    per = lambda x: x / max(1, substeps)
    res[name] = {"waves": waves, "substeps_per_wave": substeps / max(1, waves),
                 "cycles_per_wave_substep": {"narrowphase+setup": per(narrow), "velocity+warmstart": per(vel),
                                             "pgs_sweeps": per(solve), "integrate+cache": per(integ),
                                             "kernel_total_per_substep": total / max(1, substeps)},
                 "sweeps_per_wave_substep": sweeps / max(1, substeps),
                 "cycles_per_sweep": solve / max(1, sweeps),
                 "kernel_cycles_per_wave": total / max(1, waves)}
print(json.dumps(res, indent=1))
