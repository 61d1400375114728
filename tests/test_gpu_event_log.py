"""Event log on the MI355X: the HIP encoder's records and the native
writer's episodes against the env's own outputs, and the gym mirror's
--event-log-out, read back with the reference-format reader."""
import argparse

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, event_log as EL
from cartpoleplusplus_amd.batched import BatchedCartpole

pytestmark = pytest.mark.gpu


def test_gpu_records_equal_python_encoder():
    B, R = 40, 3
    env = BatchedCartpole(B, 0, action_repeats=R, initial_force=55.0, seed=4)
    env.reset()
    for kind in (abi.CP_ACTION_CONTINUOUS, abi.CP_ACTION_DISCRETE):
        log_bufs = {}
        lib = env.lib
        sb, rb = lib.cp_event_record_bytes(kind, R, 1), lib.cp_event_record_bytes(kind, R, 0)
        if kind == abi.CP_ACTION_CONTINUOUS:
            a = torch.rand((B, 2, 2), device="cuda") * 2 - 1
        else:
            a = torch.randint(0, 5, (B, 2), dtype=torch.int8, device="cuda")
        env.step(a)
        import ctypes as C
        step_rec = torch.zeros((B, sb), dtype=torch.uint8, device="cuda")
        flags = torch.zeros(B, dtype=torch.uint8, device="cuda")
        rc = lib.cp_encode_events(env.h, 0, C.c_void_p(a.data_ptr()), kind, C.c_void_p(env.obs.data_ptr()), None,
                                  C.c_void_p(env.reward.data_ptr()), C.c_void_p(env.done.data_ptr()), None,
                                  C.c_void_p(step_rec.data_ptr()), None, C.c_void_p(flags.data_ptr()),
                                  env._stream())
        assert rc == 0
        obs = env.obs.cpu().numpy()
        act = a.cpu().numpy().reshape(B, -1).astype(np.float32)
        recs = step_rec.cpu().numpy()
        assert (flags.cpu().numpy() == 1).all()
        for i in range(0, B, 7):
            exp = EL.episode_entry(EL.encode_event([EL.encode_state_lowdim(obs[i, r, 0], obs[i, r, 1])
                                                    for r in range(R)], act[i], 1.0))
            assert recs[i].tobytes() == exp


def test_batched_log_with_autoreset(tmp_path):
    B, R, L = 16, 2, 5
    env = BatchedCartpole(B, 0, action_repeats=R, initial_force=55.0, seed=6, autoreset=True,
                          max_episode_len=L, discrete_actions=True)
    path = str(tmp_path / "batched.log")
    log = EL.BatchedEventLog(env, path)
    history = {i: [] for i in range(B)}
    obs = env.reset().cpu().numpy().copy()
    log.after_reset()
    for i in range(B):
        history[i].append((None, obs[i], None))
    rng = np.random.default_rng(0)
    n_steps = 2 * L + 2
    for t in range(n_steps):
        a = torch.from_numpy(rng.integers(0, 5, (B, 2)).astype(np.int8)).cuda()
        o, r, d = env.step(a)
        log.after_step(a)
        o, d, term = o.cpu().numpy(), d.cpu().numpy(), env.terminal_obs.cpu().numpy()
        for i in range(B):
            history[i].append((a[i].cpu().numpy().astype(np.float32), term[i] if d[i] else o[i], 1.0))
            if d[i]:
                history[i].append(("reset", o[i].copy(), None))
    log.close()
    episodes = list(EL.EventLogReader(path).entries())
    # every env: 2 finished episodes of L steps + the open one (closed by close())
    assert len(episodes) == 3 * B
    assert sum(len(e.event) == L + 1 for e in episodes) == 2 * B
    # rebuild each env's expected episodes and match them as multisets of event lists
    exp = []
    for i in range(B):
        cur = []
        for a, s, r in history[i]:
            if isinstance(a, str):
                exp.append(cur)
                cur = [(None, s, None)]
            else:
                cur.append((a, s, r))
        exp.append(cur)
    key = lambda evs: tuple(np.asarray(s, np.float32).tobytes() for _, s, _ in evs)
    got = {}
    for e in episodes:
        got.setdefault(tuple(np.asarray(EL.read_state_from_event(ev), np.float32).tobytes() for ev in e.event),
                       []).append(e)
    for evs in exp:
        k = key(evs)
        assert k in got, "episode missing from the log"
        e = got[k].pop()
        assert len(e.event[0].action) == 0 and not e.event[0].HasField("reward")
        for ev, (a, s, r) in zip(e.event[1:], evs[1:]):
            assert ev.action == list(a) and ev.reward == r


def test_gym_mirror_event_log_out(tmp_path):
    from cartpoleplusplus_amd import bullet_cartpole as bc
    p = argparse.ArgumentParser()
    bc.add_opts(p)
    path = str(tmp_path / "gym.log")
    opts = p.parse_args(["--event-log-out", path, "--max-episode-len", "3", "--action-repeats", "2"])
    env = bc.BulletCartpole(opts, discrete_actions=False)
    states = [env.reset()]
    for _ in range(3):
        s, r, d, _ = env.step(np.array([[0.5, -0.25], [0.0, 0.1]], np.float32))
        states.append(s)
    env.reset()                       # writes the first episode (event_log.py:48-58)
    ep = next(EL.EventLogReader(path).entries())
    assert len(ep.event) == 4
    for ev, s in zip(ep.event, states):
        np.testing.assert_array_equal(EL.read_state_from_event(ev).astype(np.float32), s)
    assert ep.event[1].action == pytest.approx([0.5, -0.25, 0.0, 0.1])
