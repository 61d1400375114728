"""Replay memory, CPU side: the oracle restatement pinned by the
reference's own known answers (replay_memory_test.py:20-83) and its soak-test
consistency check (replay_memory.py:165-199); the product module's host logic
that needs no GPU."""
import random

import numpy as np
import pytest

from oracle.replay_oracle import ReplayOracle


def s_for(i):
    return (np.array(range(1, 7)) + (10 * i)).reshape(2, 3)


def test_oracle_empty_memory():
    # replay_memory_test.py:20-31
    rm = ReplayOracle(3, (2, 3), 2, load_factor=2)
    assert rm.size() == 0 and rm.insert == 0 and rm.full is False
    b = rm.batch_idxs([])
    assert len(b) == 5 and all(len(x) == 0 for x in b)


def test_oracle_adds_to_full():
    # replay_memory_test.py:33-59
    rm = ReplayOracle(3, (2, 3), 2, load_factor=2)
    rm.add_episode([[11, 12, 13], [14, 15, 16]],
                   [(17, 18, [[21, 22, 23], [24, 25, 26]]), (27, 28, [[31, 32, 33], [34, 35, 36]]),
                    (37, 38, [[41, 42, 43], [44, 45, 46]])])
    assert rm.size() == 3 and rm.insert == 0 and rm.full is True
    assert [rm.state[k][0][0] for k in range(4)] == [11, 21, 31, 41]


def test_oracle_adds_over_full():
    # replay_memory_test.py:61-83
    rm = ReplayOracle(3, (2, 3), 2, load_factor=2)
    rm.add_episode(s_for(0), [((i * 10) + 7, (i * 10) + 8, s_for(i)) for i in range(1, 5)])
    rm.add_episode(s_for(5), [((i * 10) + 7, (i * 10) + 8, s_for(i)) for i in range(6, 9)])
    assert rm.size() == 3
    b = rm.batch_idxs([0, 1, 2])
    assert np.array_equal(b[2], [[88], [68], [78]])
    assert np.array_equal(b[3], [[0], [1], [1]])


def soak_episodes(n_episodes, seed):
    """The reference's soak workload (replay_memory.py:167-199): state s(i), event i has
    action (i, 0), reward i, state_2 s(i)."""
    rnd = random.Random(seed)

    def s(i):
        i = (i * 10) % 199
        return [[i + 1, 0, 0], [0, 0, 0]]
    i, terminals, eps = 0, set(), []
    for _ in range(n_episodes):
        init = s(i)
        seq = []
        for _ in range(int(3 + rnd.random() * 5)):
            i += 1
            seq.append(((i, 0), i, s(i)))
        eps.append((init, seq))
        terminals.add(i)
        i += 1
    return eps, terminals


def check_soak_batch(state_1, action, reward, terminal_mask, state_2, terminals):
    """replay_memory.py:177-183"""
    for k in range(len(reward)):
        r = int(reward[k][0])
        assert state_1[k][0][0] == (((r - 1) * 10) % 199) + 1
        assert action[k][0] == r
        assert terminal_mask[k][0] == (0 if r in terminals else 1)
        assert state_2[k][0][0] == ((r * 10) % 199) + 1


def test_oracle_soak_consistency():
    eps, terminals = soak_episodes(120, seed=3)
    rm = ReplayOracle(43, (2, 3), 2)
    rng = np.random.default_rng(0)
    for init, seq in eps:
        rm.add_episode(init, seq)
        for _ in range(7):
            check_soak_batch(*rm.batch_idxs(rng.integers(0, rm.size(), 13)), terminals)
    # slot accounting: every slot is either free or referenced
    used = set(rm.state_1_idx.tolist()) | set(rm.state_2_idx.tolist())
    assert used.isdisjoint(rm.state_free_slots)


def test_oracle_batched_equals_sequential_adds():
    """add_step_batch is, by statement, _add per env in env order: check against calling
    the reference-order operations by hand."""
    B, N = 5, 12
    rng = np.random.default_rng(1)
    a, b = ReplayOracle(N, (3,), 1, 2.0), ReplayOracle(N, (3,), 1, 2.0)
    obs = rng.random((B, 3)).astype(np.float32)
    a.add_step_batch(None, None, None, None, None, np.ones(B, bool), obs)
    cur = []
    for j in range(B):
        slot = b.state_free_slots.pop(0)
        b.state[slot] = obs[j]
        cur.append(slot)
    for _ in range(9):
        valid = rng.random(B) < 0.8
        done = rng.random(B) < 0.3
        act, rew = rng.random((B, 1)), rng.random(B)
        s2, new = rng.random((B, 3)), rng.random((B, 3))
        a.add_step_batch(valid, act, rew, done, s2, valid & done, new)
        for j in range(B):
            if valid[j]:
                cur[j] = b._add(cur[j], act[j], rew[j], bool(done[j]), s2[j])
                if done[j]:
                    slot = b.state_free_slots.pop(0)
                    b.state[slot] = new[j]
                    cur[j] = slot
    assert a.state_free_slots == b.state_free_slots and list(a.cur) == cur
    for f in ("state_1_idx", "action", "reward", "terminal_mask", "state_2_idx", "state"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_product_replay_needs_gpu():
    """No GPU here: the device memory refuses a CPU device (no fallback)."""
    import torch
    from cartpoleplusplus_amd import native
    from cartpoleplusplus_amd.replay_memory import ReplayMemory
    with pytest.raises(native.CartpoleError):
        ReplayMemory(8, (2,), 1, device="cpu")
    if not torch.cuda.is_available():
        with pytest.raises(Exception):
            ReplayMemory(8, (2,), 1, device=0)


def test_replay_abi_rejects_bad_sizes():
    import ctypes as C
    from cartpoleplusplus_amd import abi, native
    lib = native.load()
    rm = abi.cp_replay(10, 12, 4, 1, *([8] * 10))   # S < 1.5 N; non-null fake pointers, no launch
    assert lib.cp_replay_init(C.byref(rm), None, 0, None) != 0
    assert b"1.5" in lib.cp_last_error(None)
    assert lib.cp_replay_add(None, None, 0, None, None, 0, None, None, None, None, None, 0, None) != 0
    assert b"null" in lib.cp_last_error(None)
