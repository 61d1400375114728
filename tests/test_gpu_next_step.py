"""CP_AUTORESET_NEXT_STEP on the GPU vs the oracle's NEXT_STEP mode (tests/test_oracle_next_step.py pins
that mode against SAME_STEP on the CPU), bit for bit, through the C-ABI.

The HIP path runs each finishing env's reset on a library stream between two cp_step calls,
overlapped with the next call's step kernel; the oracle resets eagerly in the step
and holds the obs.  Per call the outputs must be equal, and the state after every checkpoint (each
state read first joins the in-flight reset, so both hold the reset envs' new state).  Covered:
desynchronised resets (bounds termination), a burst where every env ends in the same call, envs
that were never reset (done 1: the step-after-done outputs), a cp_reset mask over pending and
running envs, both kernel shapes, fp64, and the entry points that refuse NEXT_STEP handles."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from test_gpu_parity import SHAPE_IDS, SHAPES, _assert_same, _np

pytestmark = pytest.mark.gpu


def _pair(O, shape=None, precision="f32", **kw):
    cfg = native.default_config(autoreset=abi.CP_AUTORESET_NEXT_STEP, **kw)
    if precision == "f64":
        cfg.precision = abi.CP_PRECISION_F64
    gpu = BatchedCartpole(cfg.num_envs, 0, config=abi.cp_config.from_buffer_copy(cfg))
    if shape is not None:
        gpu.set_kernel_shape(*shape)
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=precision)
    return gpu, orc


def _pending(orc):
    return abi.state_ints(orc.get_state()[abi.CP_SF_DONE]) >= 2


def _state(gpu, orc, what):
    _assert_same(_np(gpu.get_state()), orc.get_state(), what + " state")


def _drive(gpu, orc, B, calls, rng, kind, what, check_state_every=10, reset_at=None):
    seen_pending = 0
    for t in range(calls):
        if reset_at is not None and t == reset_at:   # mask: pending and running envs
            pend = _pending(orc)
            mask = np.zeros(B, np.uint8)
            mask[np.nonzero(pend)[0][:3]] = 1
            mask[np.nonzero(~pend)[0][:5]] = 1
            go = _np(gpu.reset(torch.from_numpy(mask).cuda()).clone())
            oo = orc.reset(mask, obs=_np(gpu.obs).copy())
            _assert_same(go, oo, f"{what}: cp_reset obs at call {t}")
            _state(gpu, orc, f"{what}: after cp_reset at call {t}")
        if kind == abi.CP_ACTION_DISCRETE:
            a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        else:
            a = rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
        seen_pending += int(_pending(orc).sum())
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od, ot = orc.step(a, terminal=True, obs=_np(go).copy())
        _assert_same(_np(go), oo, f"{what}: obs call {t}")
        _assert_same(_np(gr), orw, f"{what}: reward call {t}")
        _assert_same(_np(gd), od, f"{what}: done call {t}")
        done = od.astype(bool)
        _assert_same(_np(gpu.terminal_obs)[done], ot[done], f"{what}: terminal obs call {t}")
        if check_state_every and t % check_state_every == check_state_every - 1:
            _state(gpu, orc, f"{what}: call {t}")
    return seen_pending


@pytest.mark.parametrize("shape", SHAPES, ids=SHAPE_IDS)
def test_next_step_bounds_bitexact(oracle_mod, shape):
    B = 130
    gpu, orc = _pair(oracle_mod, shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=99, done_on_bounds=1,
                     max_episode_len=40)
    mask = np.ones(B, np.uint8)
    mask[-4:] = 0     # never reset: done 1, the step-after-done outputs (bullet_cartpole.py:179-181)
    _assert_same(_np(gpu.reset(torch.from_numpy(mask).cuda())), orc.reset(mask), "reset")
    rng = np.random.default_rng(5)
    n = _drive(gpu, orc, B, 120, rng, abi.CP_ACTION_DISCRETE, "bounds", reset_at=60)
    assert n > B, n    # many resets handed out, in different calls
    _state(gpu, orc, "end")
    gr_, gl_ = gpu.episode_returns()
    orr, orl = orc.episode_returns()
    _assert_same(_np(gr_), orr, "episode returns")
    _assert_same(_np(gl_), orl, "episode lengths")


@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency"), ("wide", "wide")],
                         ids=["tp-tp", "lat-lat", "wide-wide"])
def test_next_step_burst_every_env_at_once(oracle_mod, shape):
    """Fixed-length episodes: every env ends in the same call, so the next call's step kernel skips
    every env and the fixup hands out B resets."""
    B = 96
    gpu, orc = _pair(oracle_mod, shape, num_envs=B, action_repeats=2, initial_force=55.0, seed=4, max_episode_len=12)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset")
    rng = np.random.default_rng(8)
    n = _drive(gpu, orc, B, 40, rng, abi.CP_ACTION_CONTINUOUS, "burst", check_state_every=6)
    assert n == 3 * B, n   # calls 12, 25, 38 hand out every env's reset


def test_next_step_f64(oracle_mod):
    B = 64
    gpu, orc = _pair(oracle_mod, None, "f64", num_envs=B, action_repeats=3, initial_force=55.0, seed=13,
                     done_on_bounds=1, max_episode_len=25)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset")
    rng = np.random.default_rng(21)
    assert _drive(gpu, orc, B, 70, rng, abi.CP_ACTION_DISCRETE, "f64", reset_at=30) > B


def test_next_step_refusals():
    env = BatchedCartpole(64, 0, action_repeats=2, autoreset="next_step")
    env.reset()
    with pytest.raises(native.CartpoleError, match="NEXT_STEP"):
        env.rollout(torch.zeros((2, 64, 2), dtype=torch.int8))
    with pytest.raises(native.CartpoleError, match="NEXT_STEP"):
        env.enable_raster()
    env.step(torch.zeros((64, 2), dtype=torch.int8))
    env.close()   # a reset may be in flight: cp_destroy waits for it


@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency"), ("wide", "wide")],
                         ids=["tp-tp", "lat-lat", "wide-wide"])
def test_next_step_lqr_done_thresholds(oracle_mod, shape):
    """The in-kernel LQR policy with the agent's done thresholds (per-env gains) under NEXT_STEP: the
    8-states of the reset-only calls are left as they were, on both sides."""
    from cartpoleplusplus_amd.lqr import exact_gains
    B = 128
    gpu, orc = _pair(oracle_mod, shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=21)
    rng = np.random.default_rng(5)
    K = (exact_gains()[None] * rng.uniform(0.0, 1.5, (B, 1, 1, 8))).astype(np.float32)
    gpu.enable_lqr(torch.from_numpy(K), per_env=True, done_pos=0.02, done_angle=0.02)
    orc.set_lqr(K, per_env=True, state8=True, done_pos=0.02, done_angle=0.02)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset")
    pend = 0
    for t in range(100):
        a = rng.uniform(-0.3, 0.3, (B, 2, 2)).astype(np.float32)
        pend += int(_pending(orc).sum())
        go, gr, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, orw, od = orc.step(a, obs=_np(go).copy())
        _assert_same(_np(go), oo, f"obs call {t}")
        _assert_same(_np(gr), orw, f"reward call {t}")
        _assert_same(_np(gd), od, f"done call {t}")
        _assert_same(_np(gpu.state8), orc.state8, f"state8 call {t}")
    _state(gpu, orc, "final")
    assert pend > 0


def test_next_step_persistent_manifold(oracle_mod):
    """NEXT_STEP with the persistent-manifold contact model (latency-shaped kernels): the in-flight
    reset clears the env's manifolds while the next step kernel runs the other envs."""
    B = 64
    cfg = native.default_config(autoreset=abi.CP_AUTORESET_NEXT_STEP, num_envs=B, action_repeats=2,
                                initial_force=55.0, seed=7, done_on_bounds=1, max_episode_len=20)
    cfg.phys.model_flags = abi.CP_MODEL_PERSISTENT
    gpu = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    orc = oracle_mod.Envs(abi.cp_config.from_buffer_copy(cfg))
    _assert_same(_np(gpu.reset()), orc.reset(), "reset")
    rng = np.random.default_rng(3)
    assert _drive(gpu, orc, B, 50, rng, abi.CP_ACTION_DISCRETE, "pm", check_state_every=10) > 0
