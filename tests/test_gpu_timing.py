"""cp_timing_begin / cp_timing_stride / cp_timing_end (bench.py's live kernel timing):
event pairs land on every stride-th launch and the durations are sane."""
import pytest
import torch

from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.native import CartpoleError

pytestmark = pytest.mark.gpu


def test_timing_stride_samples_launches():
    B = 256
    env = BatchedCartpole(B, 0, action_repeats=3, initial_force=55.0, autoreset=True, seed=3)
    env.reset()
    acts = torch.zeros((B, 2), dtype=torch.int8, device="cuda")
    for stride, steps, want in ((1, 6, 6), (2, 6, 3), (4, 9, 3)):
        env.timing_begin(steps)
        env.timing_stride(stride, 1)
        for _ in range(steps):
            env.step(acts)
        tm = env.timing_end()
        assert tm["step_launches"] == want, (stride, tm)
        assert tm["reset_launches"] == steps, (stride, tm)
        assert 0.0 < tm["step_ms"] / want < 100.0
    env.close()


def test_timing_stride_rejects_bad_arguments():
    env = BatchedCartpole(64, 0, action_repeats=2, seed=1)
    with pytest.raises(CartpoleError):
        env.timing_stride(0, 1)
    env.close()
