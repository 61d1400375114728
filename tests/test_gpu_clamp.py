"""The coordinate-velocity clamp (cp_physics.max_coord_velocity = 100: btMultiBody's
m_maxCoordinateVelocity, applied by applyDeltaVeeMultiDof after the unconstrained update and after
the solver's write-back [ext]) on the GPU against the oracle, fp32 on every kernel-shape
pair and fp64: envs seeded through cp_set_state with body velocities past the clamp (a pole spinning
at 180 rad/s about its axis, the state that used to diverge through the explicit gyroscopic term; a
cart thrown at 150 m/s; a pole tumbling at -120 rad/s), then 40 steps with random pushes and
autoreset.  Obs, done and the state SoA bit for bit; every velocity coordinate within +-100
afterwards; the off switch (max_coord_velocity = 0) reproduces the unclamped model."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from tests.test_gpu_parity import SHAPES, SHAPE_IDS, _assert_same, _np

pytestmark = pytest.mark.gpu

B, STEPS = 64, 40


def _seed_fast(st):
    w = lambda d, c: abi.CP_SF_BODY(d, 10 + c)   # noqa: E731  angular velocity
    v = lambda d, c: abi.CP_SF_BODY(d, 7 + c)    # noqa: E731  linear velocity
    st[w(1, 2), 0:8] = 180.0                     # pole: yaw spin past the clamp
    st[w(1, 0), 0:8] = 3.0
    st[w(3, 2), 8:16] = -140.0                   # pole2
    st[w(3, 1), 8:16] = 2.5
    st[v(0, 0), 16:20] = 150.0                   # cart thrown past the clamp
    st[w(1, 0), 20:24] = -120.0                  # pole tumbling
    return st


def _vel_rows():
    return [abi.CP_SF_BODY(d, c) for d in range(4) for c in range(7, 13)]


def _run(O, shape, precision, lim):
    cfg = native.default_config(num_envs=B, action_repeats=3, initial_force=55.0, seed=19, autoreset=1,
                                max_episode_len=25)
    cfg.phys.max_coord_velocity = lim
    if precision == "f64":
        cfg.precision = abi.CP_PRECISION_F64
    gpu = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    if shape is not None:
        gpu.set_kernel_shape(*shape)
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg), precision=precision)
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    st = _seed_fast(_np(gpu.get_state()).copy())
    gpu.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    rng = np.random.default_rng(23)
    peak = 0.0
    for t in range(STEPS):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
        if t < 3:
            peak = max(peak, float(np.nanmax(np.abs(orc.get_state()[_vel_rows()]))))
    g, o = _np(gpu.get_state()), orc.get_state()
    if precision == "f64":
        assert np.array_equal(g.view(np.uint64), o.view(np.uint64)), "state bits"
    else:
        _assert_same(g, o, "state")
    gpu.close()
    return o, peak


@pytest.mark.parametrize("shape", SHAPES, ids=SHAPE_IDS)
def test_clamp_fp32_vs_oracle(oracle_mod, shape):
    o, peak = _run(oracle_mod, shape, "f32", 100.0)
    assert np.isfinite(o[:abi.CP_SF_STEPS]).all()
    assert peak <= 100.0, peak


def test_clamp_fp64_vs_oracle(oracle_mod):
    o, peak = _run(oracle_mod, None, "f64", 100.0)
    assert np.isfinite(o[:abi.CP_SF_STEPS]).all()
    assert peak <= 100.0, peak


def test_clamp_off_is_the_unclamped_model(oracle_mod):
    """max_coord_velocity <= 0 switches the clamp off (the round-4 model): still bit-exact, and the
    seeded velocities survive the first steps past 100."""
    _, peak = _run(oracle_mod, SHAPES[0], "f32", 0.0)
    assert peak > 100.0, peak
