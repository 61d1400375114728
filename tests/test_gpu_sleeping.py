"""CP_MODEL_SLEEPING (Bullet's deactivation) on the GPU against the oracle, fp32 and fp64:
the sleep timers, activation words, poses and velocities bit for bit through sleep and wake transitions.

Scenario: F_init 0, pole 1 laid flat on the plate 0.3 m in front of its cart
(cp_set_state), which its 2 s sleep timeout puts to sleep (its island is the pole alone: the cart is
0.3 m away); the cart is kept awake by alternating pushes, then driven into the sleeping pole, whose
island it joins (their AABBs overlap) -- the pole wakes, is shoved, and many poles fall asleep again.
The second case is the C3-like workload (F_init 55, random discrete pushes, autoreset) with long
episodes, where loose poles come to rest and sleep.  The model runs the latency-shaped kernels."""
import math

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from tests.test_gpu_parity import _assert_same, _np

pytestmark = pytest.mark.gpu


def _handles(O, precision, **kw):
    cfg = native.default_config(**kw)
    cfg.phys.model_flags = abi.CP_MODEL_SLEEPING
    if precision == "f64":
        cfg.precision = abi.CP_PRECISION_F64
    gpu = BatchedCartpole(cfg.num_envs, 0, config=abi.cp_config.from_buffer_copy(cfg))
    assert gpu.kernel_shape() == ("latency", "latency")
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=precision)
    return gpu, orc


def _same_state(gpu, orc, what):
    g, o = _np(gpu.get_state()), orc.get_state()
    if g.dtype == np.float64:
        assert np.array_equal(g.view(np.uint64), o.view(np.uint64)), what
    else:
        _assert_same(g, o, what)
    return o


def _sleeping(st):
    return (abi.state_ints(st)[[abi.CP_SF_SLEEP_ACT(k) for k in range(4)]] & 15) == abi.CP_ACT_SLEEPING


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_sleep_and_wake_vs_oracle(oracle_mod, precision):
    B = 64
    gpu, orc = _handles(oracle_mod, precision, num_envs=B, action_repeats=3, initial_force=0.0, seed=3,
                        max_episode_len=1000)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    st = orc.get_state()
    s45 = math.sqrt(0.5)
    for i in range(B):   # pole 1 lying along +x on the plate, 0.3 m from its cart
        for c, v in enumerate((0.40 + 0.004 * i, 0.02 * (i % 5), 0.055, 0.0, s45, 0.0, s45)):
            st[abi.CP_SF_BODY(1, c), i] = v
    gpu.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    prev = _sleeping(st)
    sleeps = wakes = 0
    for t in range(240):
        a = np.zeros((B, 2), np.int8)
        a[:, 0] = (1 + (t % 2)) if t < 170 else 2      # jiggle the cart (awake), then drive it into the pole
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
        if t % 10 == 9 or 160 <= t <= 200:
            o = _same_state(gpu, orc, f"state step {t}")
            sl = _sleeping(o)
            sleeps += int((~prev & sl).sum())
            wakes += int((prev & ~sl).sum())
            prev = sl
    assert sleeps >= 40 and wakes >= 40, (sleeps, wakes)
    assert (orc.nonfinite() == 0).all()
    gpu.close()


def test_sleeping_c3_workload_long_episodes_vs_oracle(oracle_mod):
    """F_init 55, random discrete pushes, autoreset at 400 steps: loose poles come to rest and sleep
    (none of this model's standing poles does: their slow yaw spin keeps |w|^2 above 0.05)."""
    B = 256
    gpu, orc = _handles(oracle_mod, "f32", num_envs=B, action_repeats=3, initial_force=55.0, seed=1234,
                        autoreset=1, max_episode_len=400)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(1)
    for t in range(260):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
    o = _same_state(gpu, orc, "final state")
    assert int(_sleeping(o).any(0).sum()) >= 20
    gpu.close()


def test_sleeping_rollout_equals_steps():
    """cp_rollout of the sleeping model (its own SLP instantiation) against cp_step, bit for bit: poles
    laid flat with their sleep timers near the timeout fall asleep inside the launch, episodes end and
    reset (waking everything) inside it too."""
    B, K = 128, 60
    kw = dict(num_envs=B, action_repeats=3, initial_force=55.0, seed=9, autoreset=1, max_episode_len=40)
    hs = []
    for _ in range(2):
        cfg = native.default_config(**kw)
        cfg.phys.model_flags = abi.CP_MODEL_SLEEPING
        hs.append(BatchedCartpole(B, 0, config=cfg))
    roll, step_env = hs
    roll.reset()
    step_env.reset()
    st = _np(roll.get_state()).copy()
    s45 = math.sqrt(0.5)
    for i in range(B):
        for c, v in enumerate((0.45 + 0.002 * i, -0.3, 0.055, 0.0, s45, 0.0, s45)):
            st[abi.CP_SF_BODY(1, c), i] = v
        for c in range(7, 13):
            st[abi.CP_SF_BODY(1, c), i] = 0.0
    st[abi.CP_SF_SLEEP_TIMER(1)] = 1.9
    st.view(np.int32)[abi.CP_SF_STEPS] = np.random.default_rng(2).integers(0, 40, B)
    for env in hs:
        env.set_state(torch.from_numpy(st).cuda())
    acts = torch.from_numpy(np.random.default_rng(4).integers(0, 5, (K, B, 2)).astype(np.int8)).cuda()
    ro, rr, rd = roll.rollout(acts)
    slept = False
    for k in range(K):
        so, sr, sd = step_env.step(acts[k])
        _assert_same(_np(ro[k]), _np(so), f"obs step {k}")
        _assert_same(_np(rd[k]), _np(sd), f"done step {k}")
        if k < 30:
            slept |= bool(_sleeping(_np(step_env.get_state())).any())
    _assert_same(_np(roll.get_state()), _np(step_env.get_state()), "state")
    assert slept and int(_np(rd).sum()) > B
    for env in hs:
        env.close()


def test_sleeping_rejects_lqr_and_persistent():
    cfg = native.default_config(num_envs=16)
    cfg.phys.model_flags = abi.CP_MODEL_SLEEPING | abi.CP_MODEL_PERSISTENT
    with pytest.raises(native.CartpoleError):
        BatchedCartpole(16, 0, config=cfg)
    cfg.phys.model_flags = abi.CP_MODEL_SLEEPING
    env = BatchedCartpole(16, 0, config=cfg)
    with pytest.raises(native.CartpoleError):
        env.enable_lqr(torch.zeros((2, 2, 8)))
    with pytest.raises(native.CartpoleError):
        env.set_kernel_shape("throughput", "throughput")
    with pytest.raises(native.CartpoleError):
        env.set_kernel_shape("latency", "wide")
    env.close()
