"""The oracle's alternative contact models (cp_physics.model_flags, DESIGN.md §3 sensitivity study),
checked on the CPU: what each must leave unchanged and what it must do.

- CP_MODEL_VEL_FRICTION computes the default model's numbers, bit for bit, when nothing slides (zero
  force, no actions); CP_MODEL_SPLIT_ISLANDS stays within rounding of them (the two islands then stop
  at their own sweeps instead of the slower one's);
- CP_MODEL_PERSISTENT (Bullet's persistent manifold with the relative breaking threshold) settles the
  scene to the resting heights, stays finite under pushes, and is deterministic.  (Under zero force
  its standing poles spin up about their axis and, in fp64, topple within ~150 steps: DESIGN.md §3);
- CP_MODEL_SLEEPING (Bullet's deactivation) puts a resting body to sleep after its 2 s timeout and
  freezes its island, leaves the default model untouched when off, and keeps the README's zero-force
  stability;
- the GPU implements exactly the flags CP_MODEL_GPU_FLAGS names (cp_create rejects the others,
  tests/test_abi_cpu.py)."""
import math

import numpy as np
import pytest

from cartpoleplusplus_amd import abi


def _run(O, flags, F=0.0, steps=60, B=16, actions="zero", precision="f32", seed=0):
    cfg = O.default_config(num_envs=B, action_repeats=3, initial_force=F, seed=seed)
    cfg.phys.model_flags = flags
    env = O.Envs(cfg, precision=precision)
    out = [env.reset()]
    rng = np.random.default_rng(seed)
    for _ in range(steps):
        a = np.zeros((B, 2, 2), np.float32) if actions == "zero" else rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)
        out.append(env.step(a)[0])
    return np.stack(out), env


def test_velocity_friction_equals_default_at_rest(oracle_mod):
    base, _ = _run(oracle_mod, 0)
    alt, _ = _run(oracle_mod, abi.CP_MODEL_VEL_FRICTION)
    assert np.array_equal(base.view(np.uint32), alt.view(np.uint32))


def test_split_islands_within_rounding_at_rest(oracle_mod):
    base, _ = _run(oracle_mod, 0)
    alt, _ = _run(oracle_mod, abi.CP_MODEL_SPLIT_ISLANDS)
    assert np.array_equal(base[:17].view(np.uint32), alt[:17].view(np.uint32))   # the reset and first steps
    assert np.abs(base.astype(np.float64) - alt).max() < 1e-4


@pytest.mark.parametrize("flag", [abi.CP_MODEL_SPLIT_ISLANDS, abi.CP_MODEL_VEL_FRICTION])
def test_alternatives_differ_under_pushes(oracle_mod, flag):
    base, _ = _run(oracle_mod, 0, F=55.0, actions="random")
    alt, _ = _run(oracle_mod, flag, F=55.0, actions="random")
    assert np.isfinite(alt).all() and not np.array_equal(base, alt)


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_persistent_settles_to_rest(oracle_mod, precision):
    obs, _ = _run(oracle_mod, abi.CP_MODEL_PERSISTENT, steps=1, precision=precision)
    cart, pole = obs[0, ..., 0, :], obs[0, ..., 1, :]
    # after the reset's 100 settle + 30 zero-force bump substeps: cart 0.05 + 0.025, pole 0.075 + 0.025 + 0.25
    assert np.abs(cart[..., 2] - 0.075).max() < 2e-4
    assert np.abs(pole[..., 2] - 0.35).max() < 2e-4
    q = pole[..., 3:7].astype(np.float64)
    assert (1.0 - 2.0 * (q[..., 0] ** 2 + q[..., 1] ** 2)).min() > math.cos(math.radians(1.0))   # upright


def test_persistent_pushed_finite_and_deterministic(oracle_mod):
    a, _ = _run(oracle_mod, abi.CP_MODEL_PERSISTENT, F=55.0, actions="random", steps=80, B=32)
    b, _ = _run(oracle_mod, abi.CP_MODEL_PERSISTENT, F=55.0, actions="random", steps=80, B=32)
    assert np.isfinite(a).all()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    base, _ = _run(oracle_mod, 0, F=55.0, actions="random", steps=80, B=32)
    assert not np.array_equal(a, base)   # a different contact model


def test_persistent_reset_forgets_the_manifold(oracle_mod):
    """A reset teleports the bodies (resetBasePositionAndOrientation): no cached point survives, so
    a second reset of the same env from the same pending force repeats the first one."""
    cfg = oracle_mod.default_config(num_envs=4, action_repeats=2, initial_force=0.0)
    cfg.phys.model_flags = abi.CP_MODEL_PERSISTENT
    env = oracle_mod.Envs(cfg)
    first = env.reset().copy()
    env.step(np.zeros((4, 2, 2), np.float32))
    st = env.get_state()
    for c in range(2):   # the pending forces the step left are zero (zero actions)
        assert not st[abi.CP_SF_PENDING(c, 0)].any()
    second = env.reset()
    assert np.array_equal(first.view(np.uint32), second.view(np.uint32))


def test_gpu_flags_are_the_persistent_and_sleeping_models():
    assert abi.CP_MODEL_GPU_FLAGS == abi.CP_MODEL_PERSISTENT | abi.CP_MODEL_SLEEPING


def _sleep_scene(O, B=16, steps=200, precision="f32", flags=abi.CP_MODEL_SLEEPING):
    """pole 1 laid flat on the plate away from its cart (its own island); the cart jiggled awake"""
    cfg = O.default_config(num_envs=B, action_repeats=3, initial_force=0.0, seed=3, max_episode_len=1000)
    cfg.phys.model_flags = flags
    env = O.Envs(cfg, precision=precision)
    env.reset()
    st = env.get_state()
    s45 = math.sqrt(0.5)
    for i in range(B):
        for c, v in enumerate((0.40 + 0.004 * i, 0.0, 0.055, 0.0, s45, 0.0, s45)):
            st[abi.CP_SF_BODY(1, c), i] = v
    env.set_state(st)
    hist = []
    for t in range(steps):
        a = np.zeros((B, 2), np.int8)
        a[:, 0] = 1 + (t % 2)
        env.step(a)
        s = env.get_state()
        hist.append((abi.state_ints(s)[[abi.CP_SF_SLEEP_ACT(k) for k in range(4)]].copy(),
                     s[[abi.CP_SF_SLEEP_TIMER(k) for k in range(4)]].astype(np.float64), s.copy()))
    return hist, env


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_sleeping_timeout_and_frozen_island(oracle_mod, precision):
    """CP_MODEL_SLEEPING (btMultiBody::checkMotionAndSleepIfRequired + the island manager, [ext]): the
    resting pole's timer runs from the teleport (set_state keeps its value, 0 after the reset) in steps
    of dt; once past the 2 s timeout the pole is not awake, the next step's island pass puts its
    island (the pole alone) to sleep, and from then on its pose is frozen bit for bit and its
    velocities are 0.  The jiggled cart stays ACTIVE and awake throughout."""
    hist, _ = _sleep_scene(oracle_mod, precision=precision)
    dt = float(np.float32(1.0 / 240.0))
    acts = np.array([h[0] for h in hist])        # (steps, 4 bodies, B)
    tmr = np.array([h[1] for h in hist])
    slept = np.argmax((acts[:, 1] & 15) == abi.CP_ACT_SLEEPING, axis=0)
    assert (slept > 0).all() and (slept >= 150).all() and (slept <= 170).all(), slept
    for i, k in enumerate(slept):
        assert (acts[k - 1, 1, i] & abi.CP_ACT_AWAKE) == 0          # no longer awake one step before
        assert tmr[k - 1, 1, i] > 2.0
        s0, s1 = hist[k][2], hist[-1][2]
        assert np.array_equal(s0[[abi.CP_SF_BODY(1, c) for c in range(7)], i],
                              s1[[abi.CP_SF_BODY(1, c) for c in range(7)], i])   # frozen pose
        assert (s1[[abi.CP_SF_BODY(1, c) for c in range(7, 13)], i] == 0).all()
    assert ((acts[:, 0] & 15) == abi.CP_ACT_ACTIVE).all() and ((acts[:, 0] & abi.CP_ACT_AWAKE) != 0).all()
    assert np.allclose(tmr[:100, 1, 0], dt * 3 * np.arange(1, 101), rtol=1e-4)   # the timer runs in dt steps


def test_sleeping_off_leaves_the_model_unchanged(oracle_mod):
    """Without the flag the sleep fields keep their initial value (ACTIVE | AWAKE, timer 0) and the
    physics is the default model's, bit for bit."""
    a, env_a = _run(oracle_mod, 0, F=55.0, actions="random", steps=40)
    st = env_a.get_state()
    assert (abi.state_ints(st)[[abi.CP_SF_SLEEP_ACT(k) for k in range(4)]] == abi.CP_ACT_ACTIVE | abi.CP_ACT_AWAKE).all()
    assert (st[[abi.CP_SF_SLEEP_TIMER(k) for k in range(4)]] == 0).all()
    hist, _ = _sleep_scene(oracle_mod, steps=200, flags=0)
    assert all((h[0] == abi.CP_ACT_ACTIVE | abi.CP_ACT_AWAKE).all() for h in hist)


def test_sleeping_zero_force_stability(oracle_mod):
    """README.md:77-80 under the sleeping model: every zero-force episode lasts 200 steps with the pole
    upright (the standing pole's slow yaw spin keeps it awake, so nothing freezes mid-balance)."""
    obs, _ = _run(oracle_mod, abi.CP_MODEL_SLEEPING, steps=200, B=16)
    q = obs[-1][..., 1, 3:7].astype(np.float64)
    assert (1.0 - 2.0 * (q[..., 0] ** 2 + q[..., 1] ** 2)).min() > math.cos(math.radians(2.0))


def test_oracle_rejects_non_finite_model_parameters(oracle_mod):
    """The oracle refuses what cp_create refuses: a NaN velocity clamp, and with the
    sleeping model a non-finite or negative sleep threshold."""
    cfg = oracle_mod.default_config(num_envs=2)
    cfg.phys.max_coord_velocity = float("nan")
    with pytest.raises(ValueError):
        oracle_mod.Envs(cfg)
    cfg = oracle_mod.default_config(num_envs=2)
    cfg.phys.model_flags = abi.CP_MODEL_SLEEPING
    cfg.phys.sleep_epsilon = -0.5
    with pytest.raises(ValueError):
        oracle_mod.Envs(cfg)
    cfg.phys.sleep_epsilon = 0.05
    cfg.phys.max_coord_velocity = 0.0          # <= 0: the documented off switch, accepted
    oracle_mod.Envs(cfg)
