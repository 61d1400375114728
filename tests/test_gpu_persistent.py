"""CP_MODEL_PERSISTENT on the MI355X: Bullet's persistent contact manifold (new points from
overlapping boxes only, getCacheEntry matching within the pair's relative breaking threshold,
replaceContactPoint keeping the applied impulse, sortCachedPoints for a 5th point,
refreshContactPoints removal; per-row normals) in the PM kernel variants, bit-exact against the
oracle's persistent_manifold (oracle/cp_oracle.c) in fp32 and fp64: obs, done, terminal obs and
the state SoA.  The manifolds themselves live in a buffer outside the state SoA, so every case runs
GPU and oracle from the same reset."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from tests.test_gpu_parity import _assert_same, _np

pytestmark = pytest.mark.gpu


def _pm_pair(O, precision="f32", **kw):
    cfg = native.default_config(**kw)
    cfg.phys.model_flags = abi.CP_MODEL_PERSISTENT
    if precision == "f64":
        cfg.precision = abi.CP_PRECISION_F64
    gpu = BatchedCartpole(cfg.num_envs, 0, config=abi.cp_config.from_buffer_copy(cfg))
    assert gpu.kernel_shape() == ("latency", "latency")
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=precision)
    return gpu, orc


def _same_state(gpu, orc, what):
    g, o = _np(gpu.get_state()), orc.get_state()
    if g.dtype == np.float64:   # raw bits, a NaN (any payload) only where the other side has one
        nan = np.isnan(g)
        assert np.array_equal(nan, np.isnan(o)), what
        _assert_same(np.where(nan, 0, g.view(np.uint64)), np.where(nan, 0, o.view(np.uint64)), what)
    else:
        _assert_same(g, o, what)


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_persistent_continuous_200_steps(oracle_mod, precision):
    B = 96
    gpu, orc = _pm_pair(oracle_mod, precision, num_envs=B, action_repeats=3, initial_force=55.0, seed=7)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    _same_state(gpu, orc, "reset state")
    rng = np.random.default_rng(123)
    for t in range(200):
        a = rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
    _same_state(gpu, orc, "after 200 steps")


def test_persistent_discrete_bounds_autoreset_and_merged(oracle_mod):
    """Autoreset (the manifolds are emptied by the teleport) with bounds termination, and carts
    pushed into each other (cross-pair points with their own normals, the merged solve)."""
    B = 128
    gpu, orc = _pm_pair(oracle_mod, num_envs=B, action_repeats=3, initial_force=55.0, seed=99, autoreset=1,
                        done_on_bounds=1, max_episode_len=40)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset")
    rng = np.random.default_rng(5)
    merged = 0
    for t in range(120):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        if t % 40 < 15:   # cart right, cart2 left: the pairs collide in the middle
            a[: B // 2] = np.array([2, 1], np.int8)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od, ot = orc.step(a, terminal=True)
        merged += int(orc.merged().sum())
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
        d = od.astype(bool)
        _assert_same(_np(gpu.terminal_obs)[d], ot[d], f"terminal obs step {t}")
    _same_state(gpu, orc, "autoreset")
    assert merged > 0


def test_persistent_rollout_equals_steps(oracle_mod):
    B, K = 64, 50
    cfg = native.default_config(num_envs=B, action_repeats=2, initial_force=55.0, seed=3, autoreset=1,
                                max_episode_len=20)
    cfg.phys.model_flags = abi.CP_MODEL_PERSISTENT
    a_env = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    b_env = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    a_env.reset()
    b_env.reset()
    g = torch.Generator(device="cuda").manual_seed(2)
    acts = torch.randint(0, 5, (K, B, 2), device="cuda", generator=g, dtype=torch.int8)
    ro, _, rd = a_env.rollout(acts)
    for k in range(K):
        so, _, sd = b_env.step(acts[k])
        _assert_same(_np(ro[k]), _np(so), f"obs step {k}")
        _assert_same(_np(rd[k]), _np(sd), f"done step {k}")
    _assert_same(_np(a_env.get_state()), _np(b_env.get_state()), "state")


def test_persistent_rejects_throughput_shape():
    cfg = native.default_config(num_envs=8)
    cfg.phys.model_flags = abi.CP_MODEL_PERSISTENT
    env = BatchedCartpole(8, 0, config=cfg)
    with pytest.raises(native.CartpoleError):
        env.set_kernel_shape("throughput", "throughput")
    with pytest.raises(native.CartpoleError):      # the WIDE layout is built for the default model only
        env.set_kernel_shape("wide", "latency")
    assert env.kernel_shape() == ("latency", "latency")


def test_persistent_set_state_mid_episode_clears_manifolds(oracle_mod):
    """cp_set_state on a persistent-manifold handle clears the manifolds (they are not
    part of the state SoA): a get_state -> set_state round trip mid-episode, on both sides, then
    50 more steps bit-exact; and the steps after it differ from an uninterrupted run only through
    the rebuilt contacts (the cleared cache is observable, not silently stale)."""
    B = 96
    gpu, orc = _pm_pair(oracle_mod, num_envs=B, action_repeats=3, initial_force=55.0, seed=17)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(41)
    acts = rng.uniform(-1, 1, (80, B, 2, 2)).astype(np.float32)
    for t in range(30):
        gpu.step(torch.from_numpy(acts[t]).cuda())
        orc.step(acts[t])
    st = _np(gpu.get_state())
    gpu.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    for t in range(30, 80):
        go, _, gd = gpu.step(torch.from_numpy(acts[t]).cuda())
        oo, _, od = orc.step(acts[t])
        _assert_same(_np(go), oo, f"obs step {t} after set_state")
        _assert_same(_np(gd), od, f"done step {t}")
    _same_state(gpu, orc, "after set_state + 50 steps")
