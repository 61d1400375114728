"""bench.py helpers that need no GPU: the C5 roofline names the render kernel launch_render picks."""
import os
import re

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_small2_pairs_match_the_launcher():
    src = open(os.path.join(ROOT, "cartpoleplusplus_amd", "csrc", "cp_kernels.hip")).read()
    body = src[src.index("static int launch_render"):]
    body = body[:body.index("cp_render_small_kernel, dim3")]
    body = re.sub(r"std::integral_constant<int, (\d)>\{\}", r"I\1{}", body)
    pairs = {(int(a), int(b)) for a, b in re.findall(r"small2\(I(\d)\{\}, I(\d)\{\}\)", body)}
    assert pairs == bench.SMALL2_PAIRS, pairs


def test_render_kernel_name(monkeypatch):
    monkeypatch.delenv("CP_RENDER_V1", raising=False)
    assert bench.render_kernel_name(50, 50, 1, 3) == "cp_render_small2_kernel"      # C5
    assert bench.render_kernel_name(50, 50, 2, 3) == "cp_render_small2_kernel"
    assert bench.render_kernel_name(50, 50, 1, 5) == "cp_render_small_kernel"       # no (1, 5) instance
    assert bench.render_kernel_name(120, 160, 1, 2) == "cp_render_small_kernel"     # LDS over 48 KB
    monkeypatch.setenv("CP_RENDER_V1", "1")
    assert bench.render_kernel_name(50, 50, 1, 3) == "cp_render_small_kernel"
