"""Analytic known-answer and property tests of the CPU oracle's physics
(pybullet is unavailable, so these — not pybullet outputs — are
what pin the arithmetic).  Each test states the closed form it checks."""
import math

import numpy as np
import pytest

from cartpoleplusplus_amd import abi

DT = 1.0 / 240.0


def _world(O, prec="f32", **kw):
    return O.World(O.default_config(**kw), precision=prec)


def test_philox_known_answers(oracle_mod):
    # Random123 kat_vectors, philox4x32_10
    assert oracle_mod.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle_mod.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E,
                                                                             0xA20BC7C6, 0x6D5451FD]
    assert oracle_mod.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                                    [0xA4093822, 0x299F31D0]) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_sincos_turns_accuracy(oracle_mod):
    import ctypes as C
    lib = oracle_mod.load()
    us = np.concatenate([np.linspace(0, 1, 4001, endpoint=False), np.random.default_rng(0).random(2000)])
    err = 0.0
    for u in us.astype(np.float32):
        s, c = C.c_float(), C.c_float()
        lib.orc_sincos_turns(float(u), C.byref(s), C.byref(c))
        th = 2 * math.pi * float(u)
        err = max(err, abs(s.value - math.sin(th)), abs(c.value - math.cos(th)))
    assert err < 3e-7


def test_box_inertia_formula():
    """URDF inertias equal the solid-box formula I = m/3 (h_j^2 + h_k^2) (models/*.urdf,
    MomentsOfInertia.nb)."""
    from cartpoleplusplus_amd import native
    p = native.default_config().phys
    for b, m in ((1, 1.0), (2, 5.0), (3, 1.0), (4, 5.0)):
        h = np.array(p.half_extents[b][:], np.float64)
        exp = m / 3.0 * np.array([h[1] ** 2 + h[2] ** 2, h[0] ** 2 + h[2] ** 2, h[0] ** 2 + h[1] ** 2])
        np.testing.assert_allclose(np.array(p.inertia[b][:], np.float64), exp, rtol=1e-6)
        assert p.inv_mass[b] == pytest.approx(1.0 / m)


@pytest.mark.parametrize("prec,tol", [("f64", 1e-12), ("f32", 2e-5)])
def test_free_fall_with_damping(oracle_mod, prec, tol):
    """A body far from any contact follows v' = v + dt (g - v (k + k|v|)), z' = z + dt v'."""
    w = _world(oracle_mod, prec)
    w.reset_pose(1, (0.0, 0.0, 5.0), (0, 0, 0, 1))        # cart lifted 5 m
    w.reset_pose(2, (0.0, 0.0, 9.0), (0, 0, 0, 1))        # pole above it, never touching in 24 steps
    # the model's constants are fp32 values (cp_physics); evaluate the recursion in fp64
    dt, g, k = (float(np.float32(x)) for x in (1.0 / 240.0, -9.81, 0.04))
    z0 = 5.0
    z, v = z0, 0.0
    for _ in range(24):
        w.step()
        v = v + dt * (g - v * (k + k * abs(v)))
        z = z + dt * v
    assert abs(w.pose(1)[2] - z) < tol
    assert abs(w.velocity(1)[2] - v) < tol
    # and close to the undamped closed form 1/2 g t^2 (damping is ~1e-3 relative here)
    t = 24 * DT
    assert abs((z0 - w.pose(1)[2]) - 0.5 * 9.81 * t * t) < 2e-3


def test_resting_heights_after_settle(oracle_mod):
    """After the reset's 100 settle steps the cart rests on the ground top (z = 0.05 + 0.025)
    and the pole on the cart top (0.075 + 0.025 + 0.25)."""
    w = _world(oracle_mod)
    for _ in range(100):
        w.step()
    for cart, pole in ((1, 2), (3, 4)):
        assert abs(w.pose(cart)[2] - 0.075) < 2e-4
        assert abs(w.pose(pole)[2] - 0.35) < 5e-4
        assert np.abs(w.velocity(cart)[:3]).max() < 5e-3
    assert w.overflow == 0


def test_impulse_on_frictionless_cart(oracle_mod):
    """Cart-ground and cart-pole friction are 0 (product combine with mu_cart = 0), so a
    horizontal force F on a resting cart gives dv = F dt / m in one substep."""
    w = _world(oracle_mod, "f64")
    for _ in range(100):
        w.step()
    v0 = w.velocity(1)[0]
    pole_v0 = w.velocity(2)[0]
    w.apply_force_link(1, (12.0, 0.0, 0.0))
    w.step()
    dv = w.velocity(1)[0] - v0
    assert dv == pytest.approx(12.0 * DT / 1.0, rel=2e-3)
    assert abs(w.velocity(2)[0] - pole_v0) < 1e-4      # frictionless: the pole is not dragged


def test_force_is_consumed_by_one_step(oracle_mod):
    """pybullet clears external forces after stepSimulation: a force applied once acts for
    exactly one substep (bullet_cartpole.py applies it AFTER each step, :199-207)."""
    w = _world(oracle_mod, "f64")
    for _ in range(100):
        w.step()
    w.apply_force_link(1, (12.0, 0.0, 0.0))
    w.step()
    v1 = w.velocity(1)[0]
    w.step()
    assert abs(w.velocity(1)[0] - v1) < 1e-3 * abs(v1)   # only damping acts afterwards


def test_link_frame_force_is_rotated(oracle_mod):
    """LINK_FRAME: the world force is R(q) f.  A cart yawed by 90 deg pushed along local x moves along +y."""
    w = _world(oracle_mod, "f64")
    s = math.sqrt(0.5)
    w.reset_pose(1, (0.0, 0.0, 3.0), (0.0, 0.0, s, s))   # in the air: no contact
    w.reset_pose(2, (0.0, 0.0, 6.0), (0, 0, 0, 1))
    w.apply_force_link(1, (10.0, 0.0, 0.0))
    w.step()
    v = w.velocity(1)
    assert v[1] == pytest.approx(10.0 * DT, rel=1e-3) and abs(v[0]) < 1e-6


def test_zero_force_pole_stays_up_200_steps(oracle_mod):
    """README.md:77-80 analogue: with --initial-force=0 and no action every episode
    reaches 200 steps (bounds termination on: |x|,|y| < 3 and |roll|,|pitch| < 0.35)."""
    for R in (2, 3):
        cfg = oracle_mod.default_config(num_envs=4, action_repeats=R, initial_force=0.0, done_on_bounds=1)
        e = oracle_mod.Envs(cfg)
        e.reset()
        a = np.zeros((4, 2, 2), np.float32)
        for t in range(200):
            _, _, d = e.step(a)
            if t < 199:
                assert not d.any(), f"R={R}: fell at step {t}"
        assert d.all()
        _, n = e.episode_returns()
        assert (n == 200).all()


def test_cart_slides_out_pole_drops_to_ground(oracle_mod):
    """Frictionless cart-pole contact (mu_cart = 0): a cart kicked to 1 m/s slides out
    from under the pole without dragging it; the pole drops the cart's 5 cm onto the
    ground and rests at z = 0.05 + 0.25 (ground top + half length), x unchanged."""
    w = _world(oracle_mod, "f64")
    for _ in range(100):
        w.step()
    w.apply_force_link(1, (240.0, 0.0, 0.0))    # dv = F dt / m = 1 m/s
    for _ in range(240):
        w.step()
    assert w.pose(1)[0] == pytest.approx(0.88, abs=0.02)   # ~1 m/s with quadratic damping
    p = w.pose(2)
    assert p[2] == pytest.approx(0.30, abs=1e-3)
    assert abs(p[0]) < 0.01 and abs(p[1]) < 0.01


def test_unit_quaternions_and_no_overflow_random_rollout(oracle_mod):
    cfg = oracle_mod.default_config(num_envs=48, action_repeats=3, initial_force=200.0, seed=3)
    e = oracle_mod.Envs(cfg)
    e.reset()
    rng = np.random.default_rng(1)
    for _ in range(200):
        obs, _, _ = e.step(rng.uniform(-1, 1, (48, 2, 2)).astype(np.float32))
        q = obs[..., 3:7].astype(np.float64)
        assert np.abs(np.linalg.norm(q, axis=-1) - 1).max() < 2e-6
        assert np.isfinite(obs).all()
    s = e.get_state()
    for d in range(4):
        q = s[abi.CP_SF_BODY(d, 3):abi.CP_SF_BODY(d, 7)].astype(np.float64)
        assert np.abs(np.linalg.norm(q, axis=0) - 1).max() < 2e-6


def test_fp32_vs_fp64_drift_zero_force(oracle_mod):
    """Precision drift of the fp32 model against the same algorithm in fp64, on the
    well-conditioned zero-force trajectory: 100 settle + 600 substeps (= 200 env-steps at R=3)."""
    w32, w64 = _world(oracle_mod, "f32"), _world(oracle_mod, "f64")
    worst = 0.0
    for _ in range(700):
        w32.step()
        w64.step()
        for b in range(1, 5):
            worst = max(worst, float(np.abs(w32.pose(b)[:3] - w64.pose(b)[:3]).max()))
    assert worst < 1e-3


def test_bump_stream_depends_on_env_and_episode(oracle_mod):
    cfg = oracle_mod.default_config(num_envs=4, action_repeats=2, initial_force=55.0, seed=9)
    e = oracle_mod.Envs(cfg)
    o1 = e.reset().copy()
    o2 = e.reset().copy()                       # episode counter advanced -> new pushes
    assert not np.array_equal(o1, o2)
    assert not np.array_equal(o1[0], o1[1])     # different env ids
    cfg2 = oracle_mod.default_config(num_envs=4, action_repeats=2, initial_force=55.0, seed=9, env_id_offset=1)
    e2 = oracle_mod.Envs(cfg2)
    assert np.array_equal(e2.reset()[0], o1[1])  # global env id = offset + i


def _settle(O, prec="f32", n=10, lift2=False, pre=60, **phys):
    """Sweeps per substep of n substeps after `pre` settle substeps at the default rule (the
    spawn poses start 5 mm apart: the first substeps' rows are speculative, with lambda 0)."""
    w = O.World(O.default_config(), precision=prec)
    if lift2:   # second assembly far above the first: island 1 without rows
        w.reset_pose(3, (1.0, 0.0, 50.0), (0, 0, 0, 1))
        w.reset_pose(4, (1.0, 0.0, 60.0), (0, 0, 0, 1))
    for _ in range(pre):
        w.step()
    for k, v in phys.items():
        setattr(w.cfg.phys, k, v)
    its = []
    for _ in range(n):
        w.step()
        its.append(w.last_iterations)
    return its


def test_stopping_rule_threshold_zero_runs_every_sweep(oracle_mod):
    """Bullet's loop stops after the first sweep whose max squared row residual is <=
    leastSquaresResidualThreshold, else after solver_iterations sweeps: with threshold 0,
    resting contacts (nonzero corrections in every sweep) run all sweeps."""
    assert _settle(oracle_mod, residual_threshold=0.0, solver_iterations=17) == [17] * 10


def test_stopping_rule_huge_threshold_runs_one_sweep(oracle_mod):
    """Any sweep passes a huge threshold: exactly one sweep per substep with rows (Bullet
    checks after the sweep, so at least one always runs)."""
    assert _settle(oracle_mod, residual_threshold=1e6) == [1] * 10


def test_stopping_rule_default_between(oracle_mod):
    its = _settle(oracle_mod, n=40)
    assert all(1 <= i <= 50 for i in its) and max(its) > 1


def test_one_stop_decision_per_env(oracle_mod):
    """Both islands are one solver group: the env's sweep count is at
    least what either assembly needs alone (here: the second assembly lifted out of contact)."""
    for prec in ("f32", "f64"):
        joint = _settle(oracle_mod, prec, n=30)
        alone = _settle(oracle_mod, prec, n=30, lift2=True)
        assert all(j >= a for j, a in zip(joint, alone))


def _spin(O, prec, lim, omega, steps):
    cfg = O.default_config()
    cfg.phys.max_coord_velocity = lim
    w = O.World(cfg, precision=prec)
    w.reset_pose(1, (0.0, 0.0, 50.0), (0, 0, 0, 1))        # cart and pole far above the plate: free flight
    w.reset_pose(2, (0.0, 0.0, 60.0), (0, 0, 0, 1))
    for k in range(3):
        w.w.omega[1][k] = omega[k]
    out = []
    for _ in range(steps):
        w.step()
        out.append(w.velocity(2)[3:].copy())
    return np.array(out)


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_coordinate_velocity_clamp(oracle_mod, prec):
    """btMultiBody::applyDeltaVeeMultiDof clamps each base velocity coordinate to +-100
    (m_maxCoordinateVelocity [ext]).  A pole spinning at 150 rad/s about its own axis
    in free flight: quadratic damping alone gives 150 - dt 150 k (1 + 150) after one step; the clamp
    caps it at exactly 100 (the clamp comes after the damping, in the same velocity update).  With a
    transverse rate added, every coordinate stays within +-100 for 400 steps of free flight."""
    w1 = _spin(oracle_mod, prec, 100.0, (0.0, 0.0, 150.0), 1)[0]
    w0 = _spin(oracle_mod, prec, 0.0, (0.0, 0.0, 150.0), 1)[0]
    dt, k = float(np.float32(DT)), float(np.float32(0.04))
    assert w1[2] == 100.0 and w1[0] == 0.0 and w1[1] == 0.0
    assert w0[2] == pytest.approx(150.0 - dt * 150.0 * k * (1.0 + 150.0), rel=1e-5)
    clamped = _spin(oracle_mod, prec, 100.0, (30.0, 0.0, 150.0), 400)
    assert np.isfinite(clamped).all() and np.abs(clamped).max() <= 100.0


def test_f64_double_pushes_differ_from_rounded(oracle_mod):
    """The fp64 oracle keeps the reference's float64 pushes (orc_envs_set_bump_forces64): the same
    forces rounded to float32 first reset to another state, while the fp32
    oracle gives one state for both (it rounds the doubles itself)."""
    import numpy as np
    from cartpoleplusplus_amd import abi
    B = 8
    rng = np.random.default_rng(5)
    th = rng.random((B, 30, 2)) * 2 * np.pi
    f = np.stack([55.0 * np.cos(th), 55.0 * np.sin(th)], -1)
    assert f.dtype == np.float64
    states = {}
    for prec in ("f64", "f32"):
        for kind, forces in (("double", f), ("rounded", f.astype(np.float32))):
            cfg = oracle_mod.default_config(num_envs=B, action_repeats=3, initial_force=55.0,
                                            bump_mode=abi.CP_BUMP_HOST)
            env = oracle_mod.Envs(cfg, precision=prec)
            env.set_bump_forces(forces)
            env.reset()
            states[prec, kind] = env.get_state()
    assert not np.array_equal(states["f64", "double"], states["f64", "rounded"])
    assert np.array_equal(states["f32", "double"].view(np.uint32), states["f32", "rounded"].view(np.uint32))
