"""bench.py's C5 roofline names the render kernel the library itself launches (cp_render_kernel_name,
ADVICE r4): no re-derivation of launch_render's LDS layout in Python."""
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_asks_the_library_for_the_render_kernel():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "env.render_kernel_name()" in src
    assert not hasattr(bench, "SMALL2_PAIRS") and not hasattr(bench, "render_kernel_name")
