"""The opt-in head/tail substep pipeline (CP_PIPELINE=1) against the CPU
oracle: the same bit-exact bar as the fused step kernel.

The handle reads CP_PIPELINE / CP_HEAD_SWEEPS at cp_create, so each case sets them
around the constructor only.  head = 0 sends every env through the tail kernel,
head = 4 splits envs between the kernels, head = 50 finishes every env in the head.
"""
import os

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.lqr import exact_gains

pytestmark = pytest.mark.gpu


def _pair(O, head, **kw):
    cfg = native.default_config(**kw)
    old = {k: os.environ.get(k) for k in ("CP_PIPELINE", "CP_HEAD_SWEEPS")}
    os.environ["CP_PIPELINE"] = "1"
    os.environ["CP_HEAD_SWEEPS"] = str(head)
    try:
        gpu = BatchedCartpole(cfg.num_envs, 0, config=abi.cp_config.from_buffer_copy(cfg))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    return gpu, orc


def _np(t):
    return t.detach().cpu().numpy()


def _same(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, what
    bits = (lambda x: x.view(np.uint32)) if a.dtype == np.float32 else (lambda x: x)
    if not np.array_equal(bits(a), bits(b)):
        d = np.abs(a.astype(np.float64) - b.astype(np.float64))
        raise AssertionError(f"{what}: {np.count_nonzero(d)} elements differ, max |diff| {np.nanmax(d):.3e}")


@pytest.mark.parametrize("head", [0, 4, 50])
def test_pipeline_discrete_autoreset_bounds(oracle_mod, head):
    B = 256
    gpu, orc = _pair(oracle_mod, head, num_envs=B, action_repeats=3, initial_force=55.0, seed=31, autoreset=1,
                     done_on_bounds=1, max_episode_len=60)
    _same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(3)
    for t in range(130):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od = orc.step(a)
        _same(_np(go), oo, f"obs t={t}")
        _same(_np(gr), orw, f"reward t={t}")
        _same(_np(gd), od, f"done t={t}")
    _same(_np(gpu.get_state()), orc.get_state(), "final state")


def test_pipeline_continuous_repeats_substeps(oracle_mod):
    B = 96
    gpu, orc = _pair(oracle_mod, 4, num_envs=B, action_repeats=3, steps_per_repeat=4, initial_force=55.0, seed=7)
    _same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(11)
    for t in range(60):
        a = rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od = orc.step(a)
        _same(_np(go), oo, f"obs t={t}")
        _same(_np(gd), od, f"done t={t}")
    _same(_np(gpu.get_state()), orc.get_state(), "final state")


def test_pipeline_lqr_per_env_gains(oracle_mod):
    B = 128
    gpu, orc = _pair(oracle_mod, 4, num_envs=B, action_repeats=3, initial_force=55.0, seed=21, autoreset=1)
    rng = np.random.default_rng(5)
    K = (exact_gains()[None] * rng.uniform(0.0, 1.5, (B, 1, 1, 8))).astype(np.float32)
    gpu.enable_lqr(torch.from_numpy(K), per_env=True, done_pos=0.02, done_angle=0.02)
    orc.set_lqr(K, per_env=True, state8=True, done_pos=0.02, done_angle=0.02)
    _same(_np(gpu.reset()), orc.reset(), "reset obs")
    for t in range(80):
        a = rng.uniform(-0.3, 0.3, (B, 2, 2)).astype(np.float32)
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od = orc.step(a)
        _same(_np(go), oo, f"obs t={t}")
        _same(_np(gd), od, f"done t={t}")
        _same(_np(gpu.state8), orc.state8, f"state8 t={t}")
    _same(_np(gpu.get_state()), orc.get_state(), "final state")
