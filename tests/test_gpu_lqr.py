"""LQR closed-loop policy + 8-state readback on the MI355X, bit-exact
against the oracle: obs / reward / done / 8-states / full state, per-env gains (the
reference's A/B gain search, random_action_agent.py:300-330, batched across envs) and
the shared exact gains (:812-829)."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi
from cartpoleplusplus_amd.lqr import exact_gains
from tests.test_gpu_parity import _assert_same, _np, _pair, shapes

pytestmark = pytest.mark.gpu


def _same_state(gpu, orc, what):
    _assert_same(_np(gpu.get_state()).view(np.uint32), orc.get_state().view(np.uint32), what)


@shapes
def test_per_env_gains_autoreset_bounds(oracle_mod, shape):
    B = 128
    gpu, orc = _pair(oracle_mod, shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=21, autoreset=1)
    rng = np.random.default_rng(5)
    K = (exact_gains()[None] * rng.uniform(0.0, 1.5, (B, 1, 1, 8))).astype(np.float32)
    gpu.enable_lqr(torch.from_numpy(K), per_env=True, done_pos=0.02, done_angle=0.02)
    assert gpu.kernel_shape() == tuple(shape)   # the requested shapes survive cp_set_lqr
    orc.set_lqr(K, per_env=True, state8=True, done_pos=0.02, done_angle=0.02)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    n_done = 0
    for t in range(120):
        a = rng.uniform(-0.3, 0.3, (B, 2, 2)).astype(np.float32)
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs t={t}")
        _assert_same(_np(gr), orw, f"reward t={t}")
        _assert_same(_np(gd), od, f"done t={t}")
        _assert_same(_np(gpu.state8), orc.state8, f"state8 t={t}")
        n_done += int(od.sum())
    _same_state(gpu, orc, "final")
    assert n_done > 0      # the bounds termination fired somewhere


@shapes
@pytest.mark.parametrize("R,S", [(2, 2), (1, 1)])
def test_exact_gains_discrete(oracle_mod, R, S, shape):
    B = 64
    gpu, orc = _pair(oracle_mod, shape, num_envs=B, action_repeats=R, steps_per_repeat=S, initial_force=55.0, seed=8)
    gpu.enable_lqr(torch.from_numpy(exact_gains()))
    orc.set_lqr(exact_gains(), state8=True)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(9)
    for t in range(60):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs t={t}")
        _assert_same(_np(gpu.state8), orc.state8, f"state8 t={t}")
    _same_state(gpu, orc, "final")
    # switching the policy off returns to the open-loop kernel
    gpu.enable_lqr(None)
    orc.set_lqr(None)
    a = rng.integers(0, 5, (B, 2)).astype(np.int8)
    _assert_same(_np(gpu.step(torch.from_numpy(a).cuda())[0]), orc.step(a)[0], "obs after off")


def test_lqr_rejects_state8_without_gains():
    from cartpoleplusplus_amd.batched import BatchedCartpole
    env = BatchedCartpole(8, 0)
    buf = torch.zeros((8, 2, 1, 2, 8), device="cuda")
    assert env.lib.cp_set_lqr(env.h, None, 0, buf.data_ptr(), 0.0, 0.0) != 0
    assert abi.CP_ACTION_CONTINUOUS == 0
