"""The oracle's alternative contact models (cp_physics.model_flags, DESIGN.md §3 sensitivity study),
checked on the CPU: what each must leave unchanged and what it must do.

- CP_MODEL_VEL_FRICTION computes the default model's numbers, bit for bit, when nothing slides (zero
  force, no actions); CP_MODEL_SPLIT_ISLANDS stays within rounding of them (the two islands then stop
  at their own sweeps instead of the slower one's);
- CP_MODEL_PERSISTENT (Bullet's persistent manifold with the relative breaking threshold) settles the
  scene to the resting heights, stays finite under pushes, and is deterministic.  (Under zero force
  its standing poles spin up about their axis and, in fp64, topple within ~150 steps: DESIGN.md §3);
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


def test_gpu_flags_are_the_persistent_model_only():
    assert abi.CP_MODEL_GPU_FLAGS == abi.CP_MODEL_PERSISTENT
