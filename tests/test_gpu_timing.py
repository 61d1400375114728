"""cp_timing_begin / cp_timing_stride / cp_timing_end (bench.py's live kernel timing):
event pairs land on every stride-th launch and the durations are sane.  Fixed-length episodes
(no bounds termination) launch the reset kernel only on the calls where episodes end
(cp_kernels.hip may_finish): every max_episode_len-th call after a full reset."""
import pytest
import torch

from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.native import CartpoleError

pytestmark = pytest.mark.gpu


def test_timing_stride_samples_launches():
    B, L = 256, 4
    env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True, seed=3, max_episode_len=L)
    env.reset()
    acts = torch.zeros((B, 2), dtype=torch.int8, device="cuda")
    calls = 0
    for stride, steps, want in ((1, 6, 6), (2, 6, 3), (4, 9, 3)):
        env.timing_begin(steps)
        env.timing_stride(stride, 1)
        for _ in range(steps):
            env.step(acts)
        ends = sum(1 for c in range(calls + 1, calls + steps + 1) if c % L == 0)
        calls += steps
        tm = env.timing_end()
        assert tm["step_launches"] == want, (stride, tm)
        assert tm["reset_launches"] == ends, (stride, tm)
        assert 0.0 < tm["step_ms"] / want < 100.0
    env.close()


def test_timing_reset_launch_every_call_under_bounds():
    """Episodes that can end early (bounds termination) keep one reset launch per call."""
    B = 256
    env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True, seed=3, done_on_bounds=True)
    env.reset()
    acts = torch.zeros((B, 2), dtype=torch.int8, device="cuda")
    env.timing_begin(5)
    for _ in range(5):
        env.step(acts)
    assert env.timing_end()["reset_launches"] == 5
    env.close()


def test_timing_stride_rejects_bad_arguments():
    env = BatchedCartpole(64, 0, action_repeats=2, seed=1)
    with pytest.raises(CartpoleError):
        env.timing_stride(0, 1)
    env.close()
