"""Raster obs (bullet_cartpole.py:277-306) without a GPU: the C
layout of cp_raster_config, its defaults against the reference's constants, and
known answers of the oracle's ray caster (the restatement the kernel is checked
against bit for bit in tests/test_gpu_raster.py).  Pixel parity with pybullet's
TinyRenderer is unpinned: pybullet is not available."""
import ctypes as C
import math
import os
import subprocess

import numpy as np
import pytest

from cartpoleplusplus_amd import abi, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cartpole_amd.h")
SPAWN = np.array([[0, 0, 0.075, 0, 0, 0, 1], [0, 0, 0.35, 0, 0, 0, 1],
                  [1, 0, 0.075, 0, 0, 0, 1], [1, 0, 0.35, 0, 0, 0, 1]], np.float32)


def test_raster_config_layout_matches_c(tmp_path):
    prog = tmp_path / "rl.c"
    prog.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu\\n", sizeof(cp_raster_config), offsetof(cp_raster_config, eye),
         offsetof(cp_raster_config, tan_half_fov), offsetof(cp_raster_config, background),
         offsetof(cp_raster_config, color));
  return 0;
}}""")
    exe = tmp_path / "rl"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    R = abi.cp_raster_config
    assert got == [C.sizeof(R), R.eye.offset, R.tan_half_fov.offset, R.background.offset, R.color.offset]


def test_raster_defaults_are_the_references():
    rc = native.default_raster_config()
    assert (rc.width, rc.height, rc.num_cameras) == (50, 50, 1)          # add_opts :27, :35, :37
    assert [list(e) for e in rc.eye] == [[0, 0.75, 0.75], [0.75, 0, 0.75]]  # :278-279
    assert list(rc.target) == pytest.approx([0, 0, 0.3]) and list(rc.up) == [0, 0, 1]  # :280-281
    assert rc.tan_half_fov == pytest.approx(math.tan(math.radians(15)), rel=1e-6)      # fov 30 :283
    assert rc.far_plane == 20
    colors = [list(c) for c in rc.color]                                  # models/*.urdf
    assert colors[1] == pytest.approx([0.9, 0.2, 0.1]) and colors[2] == pytest.approx([0.2, 0.7, 0.1])
    assert colors[3] == pytest.approx([0.2, 0.9, 0.1]) and colors[4] == pytest.approx([0.7, 0.2, 0.7])
    assert colors[0] == pytest.approx([0.3, 0.3, 0.0])
    assert np.linalg.norm(np.array(rc.light)) == pytest.approx(1.0, abs=1e-6)


def _shade(rc, rgb, ndl):
    s = rc.ambient + rc.diffuse * max(0.0, ndl)
    return [int(min(1.0, max(0.0, c * s)) * 255.0 + 0.5) for c in rgb]


def test_center_ray_hits_the_pole(oracle_mod):
    """Both cameras aim at (0, 0, 0.3), inside the spawned pole: the centre pixels see
    the pole; camera 0 looks along -y, so it sees the pole's +y face."""
    rc = native.default_raster_config(num_cameras=2)
    phys = native.default_config().phys
    img = oracle_mod.render_frame(rc, phys, SPAWN, 0)
    assert img.shape == (50, 50, 3)
    exp = _shade(rc, rc.color[2], rc.light[1])       # face normal +y
    for p in [(24, 24), (25, 25), (24, 25), (25, 24)]:
        assert list(img[p]) == pytest.approx(exp, abs=1)
    img1 = oracle_mod.render_frame(rc, phys, SPAWN, 1)
    exp1 = _shade(rc, rc.color[2], rc.light[0])      # camera 1 looks along -x: face +x
    assert list(img1[25, 25]) == pytest.approx(exp1, abs=1)


def test_background_above_and_ground_below(oracle_mod):
    rc = native.default_raster_config()
    phys = native.default_config().phys
    img = oracle_mod.render_frame(rc, phys, SPAWN, 0)
    bg = [int(c * 255 + 0.5) for c in rc.background]
    assert (img[0, 0] == bg).all() and (img[0, -1] == bg).all()      # top corners: sky
    ground = _shade(rc, rc.color[0], rc.light[2])                    # ground top face, normal +z
    assert list(img[-1, 0]) == pytest.approx(ground, abs=1)
    cart = _shade(rc, rc.color[1], rc.light[2])                      # the cart's top is in view
    assert any(list(img[r, 25]) == cart for r in range(30, 50))


def test_moving_the_pole_moves_its_pixels(oracle_mod):
    """Shift the pole by +0.1 m in x.  Camera 0 looks along -y, so the image's right
    is world -x: the pole's column moves left."""
    rc = native.default_raster_config()
    phys = native.default_config().phys
    green = lambda img: np.where((img[:, :, 1] > img[:, :, 0]) & (img[:, :, 1] > img[:, :, 2] + 40))[1]
    p0 = green(oracle_mod.render_frame(rc, phys, SPAWN, 0))
    moved = SPAWN.copy()
    moved[1, 0] += 0.1
    p1 = green(oracle_mod.render_frame(rc, phys, moved, 0))
    assert len(p0) and len(p1)
    assert p1.mean() < p0.mean() - 3


def test_reference_pixel_conversion():
    """float16(uint8) /= 255 in float16 (bullet_cartpole.py:289-294) -> the kernel's
    half(float32(u8) / 255): the same for all 256 bytes."""
    from oracle import oracle as O
    u = np.arange(256, dtype=np.uint8)
    ref = O.u8_to_f16(u)
    mine = (u.astype(np.float32) / np.float32(255)).astype(np.float16)
    assert np.array_equal(ref.view(np.uint16), mine.view(np.uint16))
