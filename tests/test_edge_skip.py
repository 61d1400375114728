"""The edge-axis root skip in box_box (cp_physics.h) changes no decision.

For an edge axis of the SAT the oracle (oracle/cp_oracle.c box_box, the edge loop) computes L = sqrt(L2) and
tests  num > margin * L  (separation) and  num > (best + edge_bias) * L  (new best axis), each product
rounded to the working precision.  The throughput kernels skip both when

    num <= min(best + edge_bias, margin, 0) * (1 + 2^-10)          (lo below)

claiming both tests are false for every L in (0, 1 + 2^-11].  This test checks that claim in IEEE fp32 and
fp64 with numpy's correctly rounded arithmetic: adversarial num at and just below the bound, bounds of
every sign and magnitude (denormals included), L over the whole interval and at its ends.
"""
import numpy as np
import pytest


def _lo(x, margin, dt):
    lo = x if x < margin else margin
    lo = lo if lo < dt(0) else dt(0)
    return dt(lo * dt(1.0009765625))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_skip_implies_both_tests_false(dt):
    rng = np.random.default_rng(7)
    tiny = np.finfo(dt).tiny
    mags = [dt(0), tiny, dt(tiny * 3), dt(1e-30), dt(1e-7), dt(1e-4), dt(2e-2), dt(0.5), dt(3.0), dt(1e3)]
    lmax = dt(1) + dt(2.0 ** -11)
    Ls = [dt(1e-3), dt(0.25), dt(0.7071067811865476), dt(1), np.nextafter(dt(1), dt(2)), lmax]
    Ls += [dt(v) for v in rng.uniform(1e-3, float(lmax), 200)]
    checked = 0
    with np.errstate(all="ignore"):
        for mx in mags:
            for sx in (1, -1):
                x = dt(sx * mx)
                for margin in (dt(0.02), dt(0), dt(-1e-3), dt(1e-6)):
                    lo = _lo(x, margin, dt)
                    nums = [lo, np.nextafter(lo, dt(-np.inf)), dt(lo * dt(1.5)), dt(lo - dt(1e-3))]
                    for num in nums:
                        if not num <= lo:
                            continue
                        for L in Ls:
                            sep = num > dt(margin * L)
                            better = num > dt(x * L)
                            assert not sep and not better, (x, margin, num, L)
                            checked += 1
    assert checked > 5000


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_skip_bound_is_tight_enough_to_matter(dt):
    """The skip fires for the resting-stack case it is there for: a deeply negative num (the ground's half
    extents dwarf it) against a small negative best, and not for num above the bound."""
    x, margin = dt(-5e-4 + 1e-4), dt(0.02)
    lo = _lo(x, margin, dt)
    assert dt(-10.0) <= lo                      # ground pair: num ~ -(ra + rb) ~ -10
    assert not (dt(-3e-4) <= lo)               # a tie-breaking edge axis takes the full path
