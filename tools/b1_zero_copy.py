#!/usr/bin/env python3
"""B = 1 step latency: the gym mirror's graph path (H2D action copy, cp_step, D2H obs and readback copies,
stream sync) against cp_step reading its action from and writing its outputs to pinned host memory directly
(zero-copy: no copy operations around the kernel).  Both compared for equal outputs.  Prints JSON."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cartpoleplusplus_amd import abi  # noqa: E402
from cartpoleplusplus_amd.batched import BatchedCartpole  # noqa: E402


def make(shape):
    env = BatchedCartpole(1, 0, action_repeats=2, initial_force=55.0, seed=5, max_episode_len=100000)
    env.set_kernel_shape(shape, shape)
    env.reset()
    return env


def run_graph(env, acts):
    dev_act = torch.zeros((1, 2, 2), device="cuda")
    h_act = torch.zeros((1, 2, 2)).pin_memory()
    h_obs = torch.zeros((1, env.R, 2, 7)).pin_memory()
    env.enable_readback(True)
    h_rb = torch.zeros(env.readback.shape).pin_memory()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            dev_act.copy_(h_act, non_blocking=True)
            obs, _, _ = env.step(dev_act)
            h_obs.copy_(obs, non_blocking=True)
            h_rb.copy_(env.readback, non_blocking=True)
    torch.cuda.current_stream().wait_stream(s)
    out = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts:
        h_act.numpy()[...] = a
        g.replay()
        torch.cuda.current_stream().synchronize()
        out.append(h_obs.numpy().copy())
    return time.perf_counter() - t0, np.stack(out)


def dev_ptr(t):
    """The device address of pinned host tensor t (hipHostGetDevicePointer), or an error: the kernel must only
    touch host memory the runtime has mapped for the GPU."""
    hip = C.CDLL("libamdhip64.so")
    p = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not p.value:
        raise RuntimeError(f"hipHostGetDevicePointer failed ({rc}): pinned memory not mapped for the GPU")
    return C.c_void_p(p.value)


def run_zero_copy(env, acts):
    lib = env.lib
    h_act = torch.zeros((1, 2, 2)).pin_memory()
    h_obs = torch.zeros((1, env.R, 2, 7)).pin_memory()
    h_rew = torch.zeros(1).pin_memory()
    h_done = torch.zeros(1, dtype=torch.uint8).pin_memory()
    h_rb = torch.zeros(abi.readback_shape(1, env.R, env.S)).pin_memory()
    d_act, d_obs, d_rew, d_done, d_rb = (dev_ptr(t) for t in (h_act, h_obs, h_rew, h_done, h_rb))
    assert lib.cp_set_readback(env.h, d_rb, 1) == 0
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    out = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts:
        h_act.numpy()[...] = a
        rc = lib.cp_step(env.h, d_act, abi.CP_ACTION_CONTINUOUS, d_obs, d_rew, d_done, None, sp)
        assert rc == 0
        st.synchronize()
        out.append(h_obs.numpy().copy())
    return time.perf_counter() - t0, np.stack(out)


def main():
    n = 400
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (n + 20, 1, 2, 2)).astype(np.float32)
    res = {"device_ptr_equals_host_ptr": None}
    t = torch.zeros(4).pin_memory()
    res["device_ptr_equals_host_ptr"] = dev_ptr(t).value == t.data_ptr()
    for shape in ("latency", "wide"):
        e1, e2 = make(shape), make(shape)
        run_graph(e1, acts[:20])
        run_zero_copy(e2, acts[:20])
        tg, og = run_graph(e1, acts[20:])
        tz, oz = run_zero_copy(e2, acts[20:])
        res[shape] = {"graph_us_per_step": round(tg / n * 1e6, 2), "zero_copy_us_per_step": round(tz / n * 1e6, 2),
                      "same_obs": bool(np.array_equal(og.view(np.uint32), oz.view(np.uint32)))}
        e1.close()
        e2.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
