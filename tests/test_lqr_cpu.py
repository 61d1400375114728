"""LQR policy + 8-state readback, oracle side: the 8-state is the
reference's pole state (random_action_agent.py:121-135), the force is
disturbance + (-K s) from the pre-step state (:92-104, :897-901), termination needs
both pairs out of bounds (:108-119, :908)."""
import numpy as np
import pytest

from cartpoleplusplus_amd import abi
from cartpoleplusplus_amd.lqr import ANGLE_THRESHOLD, POSITION_THRESHOLD, exact_gains, lqr_control_forces


def _envs(O, B=6, R=2, S=1, **kw):
    cfg = O.default_config(num_envs=B, action_repeats=R, steps_per_repeat=S, initial_force=55.0, seed=3, **kw)
    e = O.Envs(cfg)
    e.reset()
    return e


def test_exact_gains_constants():
    g = exact_gains()
    assert g.shape == (2, 2, 8)
    assert g[0, 0, 0] == np.float32(-2.82843) and g[1, 1, 7] == np.float32(-15.3304)
    assert POSITION_THRESHOLD == 3.0 and ANGLE_THRESHOLD == pytest.approx(0.785398, abs=1e-6)
    assert np.allclose(lqr_control_forces(g[0], np.ones(8)), -g[0].astype(np.float64).sum(axis=1))


def test_zero_gains_change_nothing(oracle_mod):
    a_env, b_env = _envs(oracle_mod), _envs(oracle_mod)
    b_env.set_lqr(np.zeros((2, 2, 8), np.float32), state8=True)
    rng = np.random.default_rng(0)
    for _ in range(30):
        a = rng.uniform(-1, 1, (6, 2, 2)).astype(np.float32)
        oa = a_env.step(a)
        ob = b_env.step(a)
        for x, y in zip(oa, ob):
            assert np.array_equal(x, y)
    assert np.array_equal(a_env.get_state().view(np.uint32), b_env.get_state().view(np.uint32))


def test_state8_is_the_pole_readback(oracle_mod):
    """8-state = (x - x0, vx, y, vy, roll, wx, pitch, wy) of each pole, after every substep."""
    e = _envs(oracle_mod, R=3, S=2)
    e.set_lqr(np.zeros((2, 2, 8), np.float32), state8=True)
    rng = np.random.default_rng(1)
    cfg = e.cfg
    x0 = [cfg.phys.spawn_pos[abi.CP_BODY_POLE][0], cfg.phys.spawn_pos[abi.CP_BODY_POLE2][0]]
    for _ in range(5):
        *_, rb = e.step(rng.uniform(-1, 1, (6, 2, 2)).astype(np.float32), readback=True, readback_bug=False)
        rb = rb.reshape(6, 2, 3, 2, 4, 3)                 # (B, pair, R, S, xyz/rpy/v/w, 3)
        s8 = e.state8                                     # (B, R, S, pair, 8)
        for p in range(2):
            r = rb[:, p]
            exp = np.stack([r[..., 0, 0] - np.float32(x0[p]), r[..., 2, 0], r[..., 0, 1], r[..., 2, 1],
                            r[..., 1, 0], r[..., 3, 0], r[..., 1, 1], r[..., 3, 1]], axis=-1)
            assert np.array_equal(s8[:, :, :, p], exp)


def test_force_is_disturbance_plus_lagged_control(oracle_mod):
    """R = S = 1: the pending force after the step is R(q_cart) (F a + u), u = -K s8 of
    the state BEFORE the substep (the reference computes control, then steps)."""
    e = _envs(oracle_mod, B=4, R=1, S=1)
    rng = np.random.default_rng(2)
    K = rng.uniform(-20, 20, (4, 2, 2, 8)).astype(np.float32)
    e.set_lqr(K, per_env=True, state8=True)
    a = rng.uniform(-1, 1, (4, 2, 2)).astype(np.float32)
    e.step(a)
    s_prev = e.state8[:, 0, 0].astype(np.float64)         # after substep 1 -> control of substep 2
    e.step(a)
    st = e.get_state()
    F = e.cfg.action_force
    for i in range(4):
        for p, dyn in ((0, 0), (1, 2)):
            q = st[[abi.CP_SF_BODY(dyn, 3 + k) for k in range(4)], i].astype(np.float64)
            x, y, z, w = q
            Rm = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                           [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                           [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
            fw = st[[abi.CP_SF_PENDING(p, k) for k in range(3)], i].astype(np.float64)
            local = Rm.T @ fw
            u = -K[i, p].astype(np.float64) @ s_prev[i, p]
            assert np.allclose(local[:2], F * a[i, p].astype(np.float64) + u, rtol=1e-4, atol=1e-3)
            assert abs(local[2]) < 1e-3


def test_termination_needs_both_pairs(oracle_mod):
    e = _envs(oracle_mod, B=3, R=1)
    e.set_lqr(np.zeros((2, 2, 8), np.float32), done_pos=1e-9, done_angle=1e-9)
    _, _, d = e.step(np.zeros((3, 2, 2), np.float32))
    assert d.all()
    e = _envs(oracle_mod, B=3, R=1)
    e.set_lqr(np.zeros((2, 2, 8), np.float32), done_pos=100.0, done_angle=3.0)
    _, _, d = e.step(np.zeros((3, 2, 2), np.float32))
    assert not d.any()
    # only pair 0 out of the position bound: not done; both out: done
    for shift, expect in (((0.5, 0.0), False), ((0.5, 0.5), True)):
        e = _envs(oracle_mod, B=3, R=1)
        e.set_lqr(np.zeros((2, 2, 8), np.float32), done_pos=0.2, done_angle=3.0)
        st = e.get_state()
        for p in range(2):
            for dyn in (2 * p, 2 * p + 1):
                st[abi.CP_SF_BODY(dyn, 0)] += np.float32(shift[p])
        e.set_state(st)
        _, _, d = e.step(np.zeros((3, 2, 2), np.float32))
        assert d.all() == expect and d.any() == expect
