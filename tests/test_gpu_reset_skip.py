"""cp_step launches no reset kernel on calls where no episode can end (cp_kernels.hip may_finish,
DESIGN.md §5 round 5): the host tracks the calls since every env's step counter was 0 and, for
fixed-length episodes without early termination, skips the launch unless (calls + 1) %
max_episode_len == 0.  A handle created with CP_RESET_EVERY_CALL=1 launches it on every call (the
behaviour before); both must agree bit for bit through everything that moves the step counters:
full and masked resets, cp_set_state, cp_rollout between cp_step calls, and a full reset that
brings the tracking back."""
import os

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd.batched import BatchedCartpole

pytestmark = pytest.mark.gpu

B, L = 384, 5


def _make(every_call, **kw):
    old = os.environ.get("CP_RESET_EVERY_CALL")
    os.environ["CP_RESET_EVERY_CALL"] = "1" if every_call else "0"
    try:
        return BatchedCartpole(B, 0, action_repeats=2, initial_force=55.0, autoreset=True, seed=41,
                               max_episode_len=L, **kw)
    finally:
        if old is None:
            del os.environ["CP_RESET_EVERY_CALL"]
        else:
            os.environ["CP_RESET_EVERY_CALL"] = old


def _same(a, b, what):
    a, b = a.cpu().numpy(), b.cpu().numpy()
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), what


@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency")], ids=["tp", "lat"])
def test_reset_skip_matches_reset_every_call(shape):
    envs = [_make(False), _make(True)]
    for e in envs:
        e.set_kernel_shape(*shape)
    rng = np.random.default_rng(43)
    n_done = 0

    def step(tag):
        nonlocal n_done
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        outs = [tuple(t.clone() for t in e.step(a)) for e in envs]
        for k, name in enumerate(("obs", "reward", "done")):
            _same(outs[0][k], outs[1][k], f"{tag} {name}")
        n_done += int(outs[0][2].sum().item())

    def state(tag):
        _same(envs[0].get_state(), envs[1].get_state(), f"{tag} state")

    for e in envs:
        e.reset()
    for t in range(2 * L + 2):                       # two bursts (calls 5 and 10), tracked
        step(f"tracked {t}")
    assert n_done == 2 * B
    mask = torch.from_numpy((np.arange(B) % 3 == 0).astype(np.uint8)).cuda()
    for e in envs:
        e.reset(mask)                                # desynchronised episodes: tracking off
    for t in range(2 * L):
        step(f"masked {t}")
    state("after masked")
    st = envs[0].get_state().clone()
    for e in envs:
        e.set_state(st)
    for t in range(L):
        step(f"set_state {t}")
    for e in envs:
        e.reset()                                    # tracked again from 0
    for t in range(3):
        step(f"re-tracked {t}")
    acts = torch.from_numpy(rng.integers(0, 5, (L + 1, B, 2)).astype(np.int8)).cuda()
    rolls = [tuple(t.clone() for t in e.rollout(acts)) for e in envs]   # calls 4 .. 9: a burst inside
    for k in range(3):
        _same(rolls[0][k], rolls[1][k], f"rollout {k}")
    for t in range(2 * L):                           # bursts at calls 10 and 15
        step(f"after rollout {t}")
    state("final")
    for e in envs:
        e.close()
