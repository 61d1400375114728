"""cp_step launches no reset kernel on calls where no episode can end (cp_kernels.hip may_finish,
DESIGN.md §5 round 5): the host tracks the calls since every env's step counter was 0 and, for
fixed-length episodes without early termination, skips the launch unless (calls + 1) %
max_episode_len == 0.  A handle created with CP_RESET_EVERY_CALL=1 launches it on every call (the
behaviour before); both must agree bit for bit through everything that moves the step counters:
full and masked resets, cp_set_state, cp_rollout between cp_step calls, and a full reset that
brings the tracking back.  Every kernel instantiation shares the step kernel's counter zeroing, so
the equivalence runs on both fp32 shapes, fp64, the sleeping model and a raster-on handle (pixels
compared too); plus the two edge cases ADVICE r5 named: max_episode_len <= 0 (every call ends every
episode) and a graph-captured step replayed behind the host's back."""
import os

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi
from cartpoleplusplus_amd.batched import BatchedCartpole

pytestmark = pytest.mark.gpu

B, L = 384, 5


def _make(every_call, L=L, **kw):
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


VARIANTS = {
    "tp": dict(shape=("throughput", "throughput"), kw={}),
    "lat": dict(shape=("latency", "latency"), kw={}),
    "wide": dict(shape=("wide", "wide"), kw={}),
    "f64": dict(shape=None, kw=dict(precision="f64")),
    "sleeping": dict(shape=None, kw=dict(model_flags=abi.CP_MODEL_SLEEPING)),
    "raster": dict(shape=None, kw={}, raster=True),
}


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_reset_skip_matches_reset_every_call(variant):
    v = VARIANTS[variant]
    envs = [_make(False, **v["kw"]), _make(True, **v["kw"])]
    raster = v.get("raster", False)
    for e in envs:
        if v["shape"]:
            e.set_kernel_shape(*v["shape"])
        if raster:
            e.enable_raster(True)
    rng = np.random.default_rng(43)
    n_done = 0

    def step(tag):
        nonlocal n_done
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        outs = [tuple(t.clone() for t in e.step(a)) for e in envs]
        for k, name in enumerate(("obs", "reward", "done")):
            _same(outs[0][k], outs[1][k], f"{tag} {name}")
        if raster:
            _same(envs[0].pixels, envs[1].pixels, f"{tag} pixels")
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
    if not raster:                                   # cp_rollout is cp_step-only with raster obs on
        acts = torch.from_numpy(rng.integers(0, 5, (L + 1, B, 2)).astype(np.int8)).cuda()
        rolls = [tuple(t.clone() for t in e.rollout(acts)) for e in envs]   # calls 4 .. 9: a burst inside
        for k in range(3):
            _same(rolls[0][k], rolls[1][k], f"rollout {k}")
    for t in range(2 * L):                           # bursts at calls 10 and 15
        step(f"after rollout {t}")
    state("final")
    for e in envs:
        e.close()


def test_reset_skip_max_episode_len_zero():
    """max_episode_len <= 0: done = steps >= limit holds after every step, so every call must reset
    every env (the skip used to launch no reset at all, leaving envs done for good)."""
    envs = [_make(False, L=0), _make(True, L=0)]
    rng = np.random.default_rng(44)
    for e in envs:
        e.reset()
    for t in range(3):
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        outs = [tuple(x.clone() for x in e.step(a)) for e in envs]
        for k, name in enumerate(("obs", "reward", "done")):
            _same(outs[0][k], outs[1][k], f"L=0 step {t} {name}")
        assert bool((outs[0][2] == 1).all()), "every env finishes every step"
        assert bool((outs[0][1] == 1.0).all()), "each step was simulated (reward 1), not a step-after-done"
    _same(envs[0].get_state(), envs[1].get_state(), "L=0 state")
    for e in envs:
        e.close()


def test_reset_skip_off_after_graph_capture():
    """A captured cp_step replayed behind the host's back moves the step counters: capture a step,
    reset eagerly, replay the graph twice, then step eagerly through an episode end; the skipping
    handle must stay bit-identical to the every-call one."""
    envs = [_make(False), _make(True)]
    rng = np.random.default_rng(45)
    ga = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
    for e in envs:
        e.reset()
    for t in range(2):
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        for e in envs:
            e.step(a)
    graphs = []
    for e in envs:
        g = torch.cuda.CUDAGraph()
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            with torch.cuda.graph(g, stream=stream):
                e.step(ga)
        torch.cuda.current_stream().wait_stream(stream)
        graphs.append(g)
    for e in envs:
        e.reset()
    for r in range(2):
        for g in graphs:
            g.replay()
        torch.cuda.synchronize()
        for k, name in enumerate(("obs", "reward", "done")):
            _same((envs[0].obs, envs[0].reward, envs[0].done)[k], (envs[1].obs, envs[1].reward, envs[1].done)[k],
                  f"replay {r} {name}")
    n_done = 0
    for t in range(2 * L + 1):                       # the eager calls cross episode ends
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        outs = [tuple(x.clone() for x in e.step(a)) for e in envs]
        for k, name in enumerate(("obs", "reward", "done")):
            _same(outs[0][k], outs[1][k], f"after replay {t} {name}")
        n_done += int(outs[0][2].sum().item())
    assert n_done >= 2 * B, n_done
    _same(envs[0].get_state(), envs[1].get_state(), "after replay state")
    del graphs
    for e in envs:
        e.close()
