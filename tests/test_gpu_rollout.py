"""cp_rollout (K env-steps in one launch, per-lane step/reset state machine, cp_env.h) against
K cp_step calls on a second handle and against the oracle: obs, reward, done, terminal obs of
every step, episode returns and the final state SoA, bit for bit, on both kernel shapes.
Episodes end at different steps (bounds termination, short max_episode_len), so lanes of one
wave are in different phases (step / reset) in the same substep trip."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.lqr import exact_gains
from tests.test_gpu_parity import _assert_same, _np, shapes

pytestmark = pytest.mark.gpu


def _handles(shape, **kw):
    cfg = native.default_config(**kw)
    hs = []
    for _ in range(2):
        h = BatchedCartpole(cfg.num_envs, 0, config=abi.cp_config.from_buffer_copy(cfg))
        h.set_kernel_shape(*shape)
        hs.append(h)
    return cfg, hs


def _stepwise(env, actions):
    obs, rew, done, term = [], [], [], []
    for k in range(actions.shape[0]):
        o, r, d = env.step(actions[k])
        obs.append(o.clone())
        rew.append(r.clone())
        done.append(d.clone())
        term.append(env.terminal_obs.clone() if env.terminal_obs is not None else None)
    return torch.stack(obs), torch.stack(rew), torch.stack(done), term


def _compare(roll, step_env, actions, what):
    ro, rr, rd = roll.rollout(actions)
    so, sr, sd, st = _stepwise(step_env, actions)
    _assert_same(_np(rd), _np(sd), what + " done")
    _assert_same(_np(rr), _np(sr), what + " reward")
    _assert_same(_np(ro), _np(so), what + " obs")
    if roll.rollout_terminal_obs is not None:
        d = _np(sd).astype(bool)
        for k in range(actions.shape[0]):
            _assert_same(_np(roll.rollout_terminal_obs[k])[d[k]], _np(st[k])[d[k]], f"{what} terminal obs step {k}")
    _assert_same(_np(roll.get_state()), _np(step_env.get_state()), what + " state")
    # the step()-level attributes follow the handle after a rollout
    _assert_same(_np(roll.obs), _np(step_env.obs), what + " .obs")
    _assert_same(_np(roll.reward), _np(step_env.reward), what + " .reward")
    _assert_same(_np(roll.done), _np(step_env.done), what + " .done")
    if roll.terminal_obs is not None:
        _assert_same(_np(roll.terminal_obs), _np(step_env.terminal_obs), what + " .terminal_obs")
    _assert_same(_np(roll.episode_returns()[0]), _np(step_env.episode_returns()[0]), what + " returns")
    _assert_same(_np(roll.episode_returns()[1]), _np(step_env.episode_returns()[1]), what + " lengths")
    # the rollout kernel's own copies of the non-finite counter
    _assert_same(_np(roll.nonfinite_counts()), _np(step_env.nonfinite_counts()), what + " nonfinite counts")
    return _np(rd)


@shapes
def test_rollout_equals_steps_discrete_bounds_autoreset(shape):
    B, K = 192, 90
    _, (roll, step_env) = _handles(shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=31, autoreset=1,
                                   done_on_bounds=1, max_episode_len=35)
    roll.reset()
    step_env.reset()
    # desynchronised episodes: every env starts at its own step counter, so resets fall on many
    # different steps and the lanes of a wave are in different phases in the same substep trip
    st = _np(roll.get_state())
    st.view(np.int32)[abi.CP_SF_STEPS] = np.random.default_rng(8).integers(0, 35, B)
    for env in (roll, step_env):
        env.set_state(torch.from_numpy(st).cuda())
    g = torch.Generator(device="cuda").manual_seed(5)
    acts = torch.randint(0, 5, (K, B, 2), device="cuda", generator=g, dtype=torch.int8)
    d = _compare(roll, step_env, acts, "discrete")
    assert d.sum() > B and len({int(k) for k in np.nonzero(d)[0]}) > 25   # resets spread over many steps
    # a second rollout continues where the first ended
    acts2 = torch.randint(0, 5, (17, B, 2), device="cuda", generator=g, dtype=torch.int8)
    _compare(roll, step_env, acts2, "discrete, second rollout")


@shapes
def test_rollout_continuous_vs_oracle(oracle_mod, shape):
    B, K = 96, 60
    cfg, (roll, _) = _handles(shape, num_envs=B, action_repeats=2, steps_per_repeat=2, initial_force=55.0, seed=4,
                              autoreset=1, max_episode_len=25)
    orc = oracle_mod.Envs(abi.cp_config.from_buffer_copy(cfg))
    _assert_same(_np(roll.reset()), orc.reset(), "reset")
    rng = np.random.default_rng(3)
    a = rng.uniform(-1, 1, (K, B, 2, 2)).astype(np.float32)
    go, gr, gd = roll.rollout(torch.from_numpy(a).cuda())
    for k in range(K):
        oo, orw, od, ot = orc.step(a[k], terminal=True)
        _assert_same(_np(go[k]), oo, f"obs step {k}")
        _assert_same(_np(gd[k]), od, f"done step {k}")
        dk = od.astype(bool)
        _assert_same(_np(roll.rollout_terminal_obs[k])[dk], ot[dk], f"terminal obs step {k}")
    _assert_same(_np(roll.get_state()), orc.get_state(), "final state")


@shapes
def test_rollout_lqr_policy_and_step_after_done(shape):
    B, K = 64, 30
    _, (roll, step_env) = _handles(shape, num_envs=B, action_repeats=2, initial_force=55.0, seed=12,
                                   max_episode_len=12)
    for env in (roll, step_env):
        env.enable_lqr(torch.from_numpy(exact_gains()), state8=False)
        env.reset()
    a = torch.zeros((K, B, 2, 2), device="cuda")
    d = _compare(roll, step_env, a, "lqr, no autoreset")
    assert d[12:].all() and not d[:11].any()     # steps after done return the last obs, done 1


def test_rollout_rejects_side_outputs():
    env = BatchedCartpole(16, 0, action_repeats=2)
    env.reset()
    env.enable_readback(True)
    with pytest.raises(native.CartpoleError):
        env.rollout(torch.zeros((3, 16, 2), dtype=torch.int8, device="cuda"))
    env.enable_readback(False)
    o, r, d = env.rollout(torch.zeros((3, 16, 2), dtype=torch.int8, device="cuda"))
    assert o.shape == (3, 16, 2, 2, 7) and torch.isfinite(o).all()
    assert env.lib.cp_rollout(env.h, 0, o.data_ptr(), 1, o.data_ptr(), r.data_ptr(), d.data_ptr(), None, None) != 0


@shapes
def test_rollout_discrete_bounds_desynchronised_vs_oracle(oracle_mod, shape):
    """The discrete, bounds-termination, desynchronised-reset rollout straight against the oracle
    (not only against cp_step): every step's obs, reward, done and terminal obs, then the state."""
    B, K = 128, 80
    cfg, (roll, _) = _handles(shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=77, autoreset=1,
                              done_on_bounds=1, max_episode_len=30)
    orc = oracle_mod.Envs(abi.cp_config.from_buffer_copy(cfg))
    _assert_same(_np(roll.reset()), orc.reset(), "reset")
    st = _np(roll.get_state())
    st.view(np.int32)[abi.CP_SF_STEPS] = np.random.default_rng(21).integers(0, 30, B)
    roll.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    a = np.random.default_rng(22).integers(0, 5, (K, B, 2)).astype(np.int8)
    go, gr, gd = roll.rollout(torch.from_numpy(a).cuda())
    go, gr, gd, gt = _np(go), _np(gr), _np(gd), _np(roll.rollout_terminal_obs)
    ks = set()
    for k in range(K):
        oo, orw, od, ot = orc.step(np.ascontiguousarray(a[k]), terminal=True)
        _assert_same(go[k], oo, f"obs step {k}")
        _assert_same(gr[k], orw, f"reward step {k}")
        _assert_same(gd[k], od, f"done step {k}")
        dk = od.astype(bool)
        _assert_same(gt[k][dk], ot[dk], f"terminal obs step {k}")
        ks |= {k} if dk.any() else set()
    assert gd.sum() > B and len(ks) > 20          # resets on many different steps
    _assert_same(_np(roll.get_state()), orc.get_state(), "final state")
    _assert_same(_np(roll.episode_returns()[0]), orc.episode_returns()[0], "returns")


@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency")], ids=["tp", "lat"])
def test_rollout_full_size_c3_k200_across_the_burst(oracle_mod, shape):
    """cp_rollout at the size bench.py times it (C3_rollout_k200): 65,536 envs, bench's hashed
    discrete actions, K = 200 in one launch; every step counter starts at 190, so the 65,536-env
    autoreset burst happens at k = 9 inside the launch.  All envs: finite obs, unit quaternions,
    done exactly at k = 9.  Four 128-env blocks (incl. the last) re-simulated on the oracle from the
    same state: every step's obs, done and terminal obs bit for bit, then the block's final state."""
    import bench
    B, K = 65536, 200
    cfg, (roll, _) = _handles(shape, num_envs=B, action_repeats=3, initial_force=55.0, seed=bench.SEED,
                              autoreset=1, max_episode_len=200)
    roll.reset()
    st = _np(roll.get_state())
    st.view(np.int32)[abi.CP_SF_STEPS] = 190
    roll.set_state(torch.from_numpy(st).cuda())
    acts = bench.make_actions(False, B, 0, K, bench.SEED, roll.device)
    go, gr, gd = roll.rollout(acts)
    # finite obs and unit quaternions on every env: the coordinate-velocity clamp (btMultiBody's
    # m_maxCoordinateVelocity) bounds the loose pole's yaw spin that used to diverge
    fin = torch.isfinite(go).flatten(2).all(2).all(0)
    bad = set(torch.nonzero(~fin).flatten().tolist())
    counted = set(torch.nonzero(roll.nonfinite_counts()).flatten().tolist())
    assert not bad and not counted, (sorted(bad)[:8], sorted(counted)[:8])
    q = go[:, fin][..., 3:7].double()
    assert bool(torch.allclose(q.norm(dim=-1), torch.ones_like(q[..., 0]), atol=1e-5))
    dsum = gd.sum(1).cpu().numpy()
    assert dsum[9] == B and dsum[:9].sum() == 0 and dsum[10:].sum() == 0
    a_np = acts.cpu().numpy()
    gst = _np(roll.get_state())
    for lo in (0, 17000, 40960, B - 128):
        sub = abi.cp_config.from_buffer_copy(cfg)
        sub.num_envs, sub.env_id_offset = 128, lo
        orc = oracle_mod.Envs(sub)
        orc.set_state(np.ascontiguousarray(st[:, lo:lo + 128]))
        bo, bd, bt = _np(go[:, lo:lo + 128]), _np(gd[:, lo:lo + 128]), _np(roll.rollout_terminal_obs[:, lo:lo + 128])
        for k in range(K):
            oo, orw, od, ot = orc.step(np.ascontiguousarray(a_np[k, lo:lo + 128]), terminal=True)
            _assert_same(bo[k], oo, f"block {lo} obs step {k}")
            _assert_same(bd[k], od, f"block {lo} done step {k}")
            if od.any():
                _assert_same(bt[k][od.astype(bool)], ot[od.astype(bool)], f"block {lo} terminal obs step {k}")
        _assert_same(gst[:, lo:lo + 128], orc.get_state(), f"block {lo} final state")
    roll.close()


def test_rollout_buffers_reserved_and_grow_only():
    """reserve_rollout(K) allocates the outputs up front; a shorter rollout returns views of the same
    buffers (no allocation inside a timed region), a longer one grows them."""
    env = BatchedCartpole(16, 0, action_repeats=2, autoreset=True)
    env.reset()
    env.reserve_rollout(8)
    o1, r1, d1 = env.rollout(torch.zeros((5, 16, 2), dtype=torch.int8, device="cuda"))
    p = o1.data_ptr()
    o2, r2, d2 = env.rollout(torch.zeros((3, 16, 2), dtype=torch.int8, device="cuda"))
    assert o2.shape == (3, 16, 2, 2, 7) and r2.shape == (3, 16) and d2.shape == (3, 16)
    assert o2.data_ptr() == p and env.rollout_terminal_obs.shape == (3, 16, 2, 2, 7)
    assert torch.equal(env.obs, o2[-1])
    o3, _, _ = env.rollout(torch.zeros((10, 16, 2), dtype=torch.int8, device="cuda"))
    assert o3.shape[0] == 10 and torch.isfinite(o3).all()
    env.close()


@pytest.mark.parametrize("clear", [False, True], ids=["reference", "clear-force"])
@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency")], ids=["tp", "lat"])
def test_rollout_seeded_nans_vs_oracle(oracle_mod, clear, shape):
    """The rollout kernel's inline reset_force, its step-end and reset-end non-finite counters
     against the oracle: NaNs seeded through cp_set_state (a NaN cart quaternion, whose
    LINK-frame action force is NaN and survives the reset unless CP_RESET_CLEAR_NONFINITE_FORCE, and a
    NaN pole yaw rate), autoreset inside the launch; obs (NaN positions), done, the counters and the
    state, as tests/test_gpu_nonfinite.py does for cp_step."""
    B, K, EP = 64, 40, 15
    cfg = native.default_config(num_envs=B, action_repeats=3, initial_force=55.0, seed=5, autoreset=1,
                                max_episode_len=EP)
    cfg.reset_flags = abi.CP_RESET_CLEAR_NONFINITE_FORCE if clear else 0
    roll = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    roll.set_kernel_shape(*shape)
    orc = oracle_mod.Envs(abi.cp_config.from_buffer_copy(cfg))
    _assert_same(_np(roll.reset()), orc.reset(), "reset obs")
    st = _np(roll.get_state())
    st[abi.CP_SF_BODY(0, 3), 3] = np.nan
    st[abi.CP_SF_BODY(1, 12), 9] = np.nan
    roll.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    a = np.random.default_rng(3).integers(0, 5, (K, B, 2)).astype(np.int8)
    go, _, gd = roll.rollout(torch.from_numpy(a).cuda())
    go, gd = _np(go), _np(gd)
    for k in range(K):
        oo, _, od = orc.step(np.ascontiguousarray(a[k]))
        _assert_same(go[k], oo, f"obs step {k}")
        _assert_same(gd[k], od, f"done step {k}")
    _assert_same(_np(roll.nonfinite_counts()), orc.nonfinite(), "nonfinite counts")
    g, o = _np(roll.get_state()), orc.get_state()
    assert np.array_equal(np.isnan(g), np.isnan(o))
    _assert_same(np.where(np.isnan(g), 0, g), np.where(np.isnan(o), 0, o), "state")
    n = orc.nonfinite()
    assert n[9] >= 1 and n[3] >= EP and ((n[3] == EP) if clear else (n[3] > EP + 1))
    roll.close()


def test_rollout_returns_before_the_kernel_ends():
    """rollout() enqueues and returns: no host wait on the launch (the terminal-obs bookkeeping is a
    device-side select), so rollouts of several handles on their own streams overlap."""
    import time
    B, K = 65536, 100
    env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True)
    env.reset()
    acts = torch.randint(0, 5, (K, B, 2), device="cuda", dtype=torch.int8)
    env.reserve_rollout(K)
    env.rollout(acts[:2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    env.rollout(acts)
    enq = time.perf_counter() - t0
    pending = not torch.cuda.current_stream().query()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    assert pending, f"the stream was idle when rollout() returned (enqueue {enq * 1e3:.2f} ms, total {total * 1e3:.1f} ms)"
    assert enq < 0.5 * total, (enq, total)
    env.close()
