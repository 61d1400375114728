"""Raster obs on the MI355X: the render kernel's float16 pixels vs the
oracle's ray caster on the same poses, bit for bit, through the C-ABI.

The poses come from the GPU env itself (get_state after the call: the last repeat's
frame; after a reset every repeat slot holds the reset frame).  The conversion to
float16 is the reference's (bullet_cartpole.py:289-294), restated in oracle.u8_to_f16."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole

pytestmark = pytest.mark.gpu


def _poses(state, e):
    out = np.zeros((4, 7), np.float32)
    for d in range(4):
        out[d] = state[abi.CP_SF_BODY(d, 0):abi.CP_SF_BODY(d, 0) + 7, e]
    return out


def _expect(O, rc, phys, state, e, cam):
    return O.u8_to_f16(O.render_frame(rc, phys, _poses(state, e), cam)).view(np.uint16)


def _check_env(O, env, pix, state, e, r):
    rc = env.raster_cfg
    for cam in range(rc.num_cameras):
        got = pix[e, :, :, :, cam, r].view(np.uint16)
        exp = _expect(O, rc, env.cfg.phys, state, e, cam)
        if not np.array_equal(got, exp):
            bad = np.argwhere(got != exp)
            raise AssertionError(f"env {e} cam {cam} repeat {r}: {len(bad)} channel values differ, first {bad[:3]}")


def test_reset_frames_bitexact(oracle_mod):
    env = BatchedCartpole(40, 0, action_repeats=3, initial_force=55.0, seed=3)
    env.enable_raster(True, num_cameras=2)
    env.reset()
    pix = env.pixels.cpu().numpy()
    st = env.get_state().cpu().numpy()
    assert pix.shape == (40, 50, 50, 3, 2, 3) and pix.dtype == np.float16
    for e in range(0, 40, 7):
        for r in range(3):
            _check_env(oracle_mod, env, pix, st, e, r)


@pytest.mark.parametrize("R,C", [(3, 1), (1, 2)])
def test_step_frames_bitexact(oracle_mod, R, C):
    B = 48
    env = BatchedCartpole(B, 0, action_repeats=R, initial_force=55.0, seed=11)
    env.enable_raster(True, num_cameras=C)
    env.reset()
    rng = np.random.default_rng(1)
    for t in range(25):
        a = torch.from_numpy(rng.uniform(-1, 1, (B, 2, 2)).astype(np.float32)).cuda()
        env.step(a)
        if t % 8 == 7:
            pix = env.pixels.cpu().numpy()
            st = env.get_state().cpu().numpy()
            for e in range(0, B, 5):
                _check_env(oracle_mod, env, pix, st, e, R - 1)


def test_other_sizes_and_done_envs_keep_pixels(oracle_mod):
    """A 37 x 23 image (odd pixel count: the 2-byte copy path), and an env that is done
    before the step keeps its pixels (bullet_cartpole.py:179-181)."""
    B = 10
    env = BatchedCartpole(B, 0, action_repeats=1, initial_force=55.0, seed=5, max_episode_len=3)
    env.enable_raster(True, width=37, height=23)
    env.reset()
    act = torch.zeros((B, 2, 2), device="cuda")
    for _ in range(3):
        env.step(act)
    assert env.done.all()
    before = env.pixels.clone()
    st = env.get_state().cpu().numpy()
    _check_env(oracle_mod, env, env.pixels.cpu().numpy(), st, 4, 0)
    env.step(act)
    assert torch.equal(before, env.pixels)


@pytest.mark.parametrize("W,H,C,R", [(100, 20, 2, 3), (160, 120, 1, 2), (90, 70, 2, 2)])
def test_large_frames_wave_path(oracle_mod, W, H, C, R):
    """Frames whose depth / id buffers exceed the small-frame kernel's LDS budget go to
    the one-wave-per-env kernel (160 x 120, 90 x 70 x 2 cameras); 100 x 20 stays small."""
    env = BatchedCartpole(6, 0, action_repeats=R, initial_force=55.0, seed=9)
    env.enable_raster(True, width=W, height=H, num_cameras=C)
    env.reset()
    env.step(torch.zeros((6, 2, 2), device="cuda"))
    pix = env.pixels.cpu().numpy()
    st = env.get_state().cpu().numpy()
    for e in range(6):
        _check_env(oracle_mod, env, pix, st, e, R - 1)


def test_autoreset_frames_show_the_new_episode(oracle_mod):
    B = 32
    env = BatchedCartpole(B, 0, action_repeats=2, initial_force=55.0, seed=8, autoreset=True, max_episode_len=4)
    env.enable_raster(True)
    env.reset()
    a = torch.zeros((B, 2), dtype=torch.int8, device="cuda")
    for t in range(4):
        env.step(a)
    assert env.done.all()
    pix = env.pixels.cpu().numpy()
    st = env.get_state().cpu().numpy()
    for e in range(0, B, 6):
        for r in range(2):
            _check_env(oracle_mod, env, pix, st, e, r)


def test_gym_mirror_raw_pixels():
    import argparse
    from cartpoleplusplus_amd import bullet_cartpole as bc
    p = argparse.ArgumentParser()
    bc.add_opts(p)
    opts = p.parse_args(["--use-raw-pixels", "--num-cameras", "2", "--action-repeats", "3"])
    env = bc.BulletCartpole(opts, discrete_actions=True)
    s = env.reset()
    assert s.shape == (50, 50, 3, 2, 3) and s.dtype == np.float32
    assert env.observation_space.shape == (50, 50, 3, 2, 3)
    assert np.array_equal(s[..., 0], s[..., 2])           # every repeat slot: the reset frame
    assert 0.0 <= s.min() and s.max() <= 1.0
    s2, r, d, _ = env.step([1, 2])
    assert s2.shape == s.shape and r == 1.0 and not d


def test_full_size_c5_properties_and_subset(oracle_mod):
    """C5 at its full size (B = 65,536, 50 x 50 x 3, 1 camera, R = 3: 2.95 GB of float16
    frames per step, the throughput-shaped step kernel and the one-block-per-env render
    kernel): every pixel finite and in [0, 1]; the last repeat's frame of 48 envs spread
    over the batch bit-exact against the oracle's ray caster."""
    B = 65536
    env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, seed=1234, autoreset=True)
    env.enable_raster(True)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(3):
        env.step(torch.randint(0, 5, (B, 2), device="cuda", generator=gen, dtype=torch.int8))
    px = env.pixels
    assert px.shape == (B, 50, 50, 3, 1, 3) and px.dtype == torch.float16
    assert bool(torch.isfinite(px).all()) and float(px.min()) >= 0.0 and float(px.max()) <= 1.0
    idx = np.sort(np.random.default_rng(3).choice(B, 48, replace=False))
    pix = px[torch.from_numpy(idx).cuda()].cpu().numpy()
    st = env.get_state().cpu().numpy()[:, idx]
    for k in range(len(idx)):
        _check_env(oracle_mod, env, pix, st, k, 2)


@pytest.mark.parametrize("R,C,W,H", [(3, 1, 50, 50), (2, 1, 50, 50), (1, 1, 37, 23), (4, 1, 41, 29), (6, 1, 30, 20),
                                     (1, 2, 50, 50), (2, 2, 50, 50), (3, 2, 37, 23)])
def test_render_v2_equals_v1_every_pixel(monkeypatch, R, C, W, H):
    """cp_render_small2_kernel<C, R> (round 4: code words of 5-bit fields, 16-bit at C * R <= 3 and
    32-bit up to 6, packed stage writes, reciprocal rectangles, the exact short reciprocal) against the
    round-3 small-frame kernel (CP_RENDER_V1=1 at cp_create), every (C, R) it is instantiated for:
    every pixel of every env, frame and step equal, bit for bit (both are held to the oracle by the
    tests above)."""
    B, T = 64, 12
    out = []
    for v1 in ("1", "0"):
        monkeypatch.setenv("CP_RENDER_V1", v1)
        env = BatchedCartpole(B, 0, action_repeats=R, initial_force=55.0, seed=21)
        env.enable_raster(True, num_cameras=C, width=W, height=H)
        env.reset()
        frames = [env.pixels.clone()]
        g = torch.Generator(device="cuda").manual_seed(4)
        for _ in range(T):
            env.step(torch.rand((B, 2, 2), device="cuda", generator=g) * 2 - 1)
            frames.append(env.pixels.clone())
        out.append(torch.stack(frames).view(torch.int16))
        env.close()
    assert torch.equal(out[0], out[1])


def test_render_kernel_name_is_the_launchers_choice(monkeypatch):
    """cp_render_kernel_name reports launch_render's choice: the compile-time (C, R) small2 instances when
    their LDS fits, the round-3 block kernel otherwise (or with the CP_RENDER_V1 diagnostic), the
    wave kernel for large frames; None with the raster obs off."""
    from cartpoleplusplus_amd.batched import BatchedCartpole
    monkeypatch.delenv("CP_RENDER_V1", raising=False)
    cases = [(1, 3, 50, 50, "cp_render_small2_kernel"), (2, 3, 50, 50, "cp_render_small2_kernel"),
             (1, 5, 50, 50, "cp_render_small_kernel"), (1, 2, 160, 120, "cp_render_kernel")]
    for C_, R, W, H, name in cases:
        env = BatchedCartpole(8, 0, action_repeats=R)
        assert env.render_kernel_name() is None
        env.enable_raster(True, num_cameras=C_, width=W, height=H)
        assert env.render_kernel_name() == name, (C_, R, W, H, env.render_kernel_name())
        env.close()
    monkeypatch.setenv("CP_RENDER_V1", "1")
    env = BatchedCartpole(8, 0, action_repeats=3)
    env.enable_raster(True)
    assert env.render_kernel_name() == "cp_render_small_kernel"
    env.close()
