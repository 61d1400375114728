"""Replay memory in HBM on the MI355X against the oracle restatement:
the reference's known answers, its soak consistency check, batched ingestion bit-exact
against the sequential reference order (ring, slot FIFO, float16 states), the env feed,
and sampling."""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi
from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.replay_memory import ReplayError, ReplayMemory
from oracle.replay_oracle import ReplayOracle
from tests.test_replay_cpu import check_soak_batch, s_for, soak_episodes

pytestmark = pytest.mark.gpu


def same_as_oracle(rm, o):
    torch.cuda.synchronize()
    assert rm.insert == o.insert and rm.full == o.full
    assert rm.free_slots() == o.state_free_slots
    np.testing.assert_array_equal(rm.state_1_idx.cpu().numpy(), o.state_1_idx)
    np.testing.assert_array_equal(rm.state_2_idx.cpu().numpy(), o.state_2_idx)
    np.testing.assert_array_equal(rm.action.cpu().numpy(), o.action)
    np.testing.assert_array_equal(rm.reward.cpu().numpy(), o.reward)
    np.testing.assert_array_equal(rm.terminal_mask.cpu().numpy(), o.terminal_mask)
    np.testing.assert_array_equal(rm.state.cpu().numpy().view(np.uint16), o.state.view(np.uint16))
    rm.check()


def test_empty_memory():
    rm = ReplayMemory(3, (2, 3), 2, load_factor=2)
    assert rm.size() == 0 and rm.random_indexes() == []
    b = rm.batch(4)
    assert len(b) == 5 and all(len(x) == 0 for x in b)
    assert rm.insert == 0 and rm.full is False


def test_adds_to_full():
    rm = ReplayMemory(3, (2, 3), 2, load_factor=2)
    rm.add_episode([[11, 12, 13], [14, 15, 16]],
                   [(17, 18, [[21, 22, 23], [24, 25, 26]]), (27, 28, [[31, 32, 33], [34, 35, 36]]),
                    (37, 38, [[41, 42, 43], [44, 45, 46]])])
    assert rm.size() == 3 and rm.insert == 0 and rm.full
    idxs = rm.random_indexes(n=100).cpu().tolist()
    assert len(idxs) == 100 and sorted(set(idxs)) == [0, 1, 2]
    st = rm.state.cpu().numpy()
    assert [st[k][0][0] for k in range(4)] == [11, 21, 31, 41]


def test_adds_over_full():
    rm = ReplayMemory(3, (2, 3), 2, load_factor=2)
    o = ReplayOracle(3, (2, 3), 2, load_factor=2)
    for m in (rm, o):
        m.add_episode(s_for(0), [((i * 10) + 7, (i * 10) + 8, s_for(i)) for i in range(1, 5)])
        m.add_episode(s_for(5), [((i * 10) + 7, (i * 10) + 8, s_for(i)) for i in range(6, 9)])
    assert rm.size() == 3
    b = rm.batch(idxs=[0, 1, 2])
    assert np.array_equal(b.reward.cpu().numpy(), [[88], [68], [78]])
    assert np.array_equal(b.terminal_mask.cpu().numpy(), [[0], [1], [1]])
    same_as_oracle(rm, o)


def test_soak_consistency_and_oracle():
    eps, terminals = soak_episodes(60, seed=5)
    rm, o = ReplayMemory(43, (2, 3), 2), ReplayOracle(43, (2, 3), 2)
    for init, seq in eps:
        rm.add_episode(init, seq)
        o.add_episode(init, seq)
        b = rm.batch(13)
        check_soak_batch(*(x.cpu().numpy() for x in b), terminals)
    same_as_oracle(rm, o)
    st = rm.current_stats()
    assert st[">add"] == sum(len(s) for _, s in eps) and st["free_slots"] == len(o.state_free_slots)


@pytest.mark.parametrize("B,N,load,D,f16", [(37, 100, 2.0, 6, False), (1500, 4000, 2.0, 42, False),
                                             (300, 700, 3.0, 16, True), (5, 12, 2.5, 7, False)])
def test_batched_ingestion_matches_sequential_reference(B, N, load, D, f16):
    g = torch.Generator().manual_seed(B + N)
    rm = ReplayMemory(N, (D,), 3, load, num_envs=B)
    o = ReplayOracle(N, (D,), 3, load)
    dt = torch.float16 if f16 else torch.float32

    def rnd(*shape):
        return (torch.rand(shape, generator=g) * 200 - 100).to(dt)
    obs = rnd(B, D)
    rm.begin_episodes(obs.cuda())
    o.add_step_batch(None, None, None, None, None, np.ones(B, bool), obs.numpy())
    for step in range(12):
        valid = torch.rand(B, generator=g) < 0.9
        done = (torch.rand(B, generator=g) < 0.25) & valid
        restart = done.clone()
        act, rew = torch.rand((B, 3), generator=g), torch.rand(B, generator=g)
        s2, new = rnd(B, D), rnd(B, D)
        rm.add_steps(act.cuda(), rew.cuda(), done.cuda(), new.cuda(), s2.cuda(), valid=valid.cuda(),
                     restart=restart.cuda())
        s2_o = np.where(restart.numpy()[:, None], s2.numpy(), new.numpy())   # s2: terminal state if restarted
        o.add_step_batch(valid.numpy(), act.numpy(), rew.numpy(), done.numpy(), s2_o, restart.numpy(), new.numpy())
        if step % 4 == 3:
            same_as_oracle(rm, o)
    assert rm.cur[:B].cpu().tolist() == list(o.cur)


def test_env_feed_matches_oracle():
    """BatchedCartpole (autoreset) -> after_step: the memory equals the oracle fed from
    the same device outputs; sampled pairs are consecutive states of one env."""
    B, R = 96, 2
    env = BatchedCartpole(B, 0, action_repeats=R, autoreset=True, max_episode_len=15, seed=9)
    rm = ReplayMemory(600, (R, 2, 7), 4, 1.5, num_envs=B)
    o = ReplayOracle(600, (R, 2, 7), 4, 1.5)
    obs = env.reset()
    rm.after_reset(env)
    o.add_step_batch(None, None, None, None, None, np.ones(B, bool), obs.cpu().numpy())
    g = torch.Generator(device="cuda").manual_seed(2)
    stepped = torch.zeros(B, dtype=torch.uint8, device="cuda")
    for _ in range(40):
        a = torch.rand((B, 2, 2), device="cuda", generator=g) * 2 - 1
        env.step(a)
        rm.after_step(env, a)
        env.lib.cp_get_stepped(env.h, stepped.data_ptr(), env._stream())
        d = env.done.cpu().numpy().astype(bool)
        s2 = np.where(d[:, None, None, None], env.terminal_obs.cpu().numpy(), env.obs.cpu().numpy())
        o.add_step_batch(stepped.cpu().numpy().astype(bool), a.reshape(B, 4).cpu().numpy(),
                         env.reward.cpu().numpy(), d, s2, d, env.obs.cpu().numpy())
    same_as_oracle(rm, o)
    b, idx, (s1i, s2i) = rm.sample(512, with_slots=True)
    idx = idx.cpu().numpy()
    assert idx.min() >= 0 and idx.max() < rm.size()
    ob = o.batch_idxs(idx)
    for got, exp in zip(b, ob):
        np.testing.assert_array_equal(got.cpu().numpy(), exp)
    np.testing.assert_array_equal(s1i.cpu().numpy(), o.state_1_idx[idx])


def test_non_autoreset_env_skips_finished_envs():
    B = 50
    env = BatchedCartpole(B, 0, action_repeats=2, max_episode_len=6, seed=3)
    rm = ReplayMemory(1000, (2, 2, 7), 2, num_envs=B)
    env.reset()
    rm.after_reset(env)
    a = torch.zeros((B, 2), dtype=torch.int8, device="cuda")
    for _ in range(10):           # episodes end at 6 steps; steps 7..10 are not simulated
        env.step(a)
        rm.after_step(env, a)
    assert bool(env.done.bool().all())
    _, lengths = env.episode_returns()
    n = int(lengths.sum())
    assert rm.size() == n and n <= 6 * B
    tm = rm.terminal_mask[:n].cpu().numpy()
    assert (tm == 0).sum() == B
    rm.check()


def test_sample_random_indexes_cover_and_errors():
    rm = ReplayMemory(64, (4,), 1, 1.5, num_envs=16, seed=11)
    x = torch.arange(64, dtype=torch.float32, device="cuda").reshape(16, 4)
    rm.begin_episodes(x)
    for k in range(3):
        rm.add_steps(torch.ones(16, 1, device="cuda"), torch.full((16,), float(k), device="cuda"),
                     torch.zeros(16, dtype=torch.uint8, device="cuda"), x + k + 1)
    assert rm.size() == 48
    idx = rm.random_indexes(20000).cpu().numpy()
    counts = np.bincount(idx, minlength=48)
    assert idx.max() < 48 and counts.min() > 0.5 * 20000 / 48
    with pytest.raises(ReplayError):
        rm.batch(idxs=[0, 48])


def test_slot_underflow_is_loud():
    rm = ReplayMemory(4, (2,), 1, 1.5, num_envs=4)     # 6 slots, 4 episodes, length-1 episodes
    x = torch.zeros((4, 2), device="cuda")
    rm.begin_episodes(x)
    one = torch.ones(4, dtype=torch.uint8, device="cuda")
    rm.add_steps(torch.zeros(4, 1, device="cuda"), torch.zeros(4, device="cuda"), one, x, x, restart=one)
    with pytest.raises(ReplayError, match="no free state slot"):
        rm.check()


def test_large_ring_invariants():
    """At a production size (2^20 events, 65536 envs): slot accounting and the stored
    rows of a sample equal the float16 rounding of what was added."""
    B, N, D = 65536, 1 << 20, 42
    rm = ReplayMemory(N, (D,), 4, 1.5, num_envs=B)
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((B, D), device="cuda", generator=g)
    rm.begin_episodes(x)
    keep = {}
    for step in range(24):
        nxt = torch.randn((B, D), device="cuda", generator=g)
        done = (torch.rand(B, device="cuda", generator=g) < 0.05).to(torch.uint8)
        term = torch.randn((B, D), device="cuda", generator=g)
        rm.add_steps(torch.randn((B, 4), device="cuda", generator=g), torch.full((B,), float(step), device="cuda"),
                     done, nxt, term, restart=done)
        keep[step] = (torch.where(done.bool()[:, None], term, nxt).half(), done.clone())
    rm.check()
    assert rm.size() == N and rm.full
    st = rm.current_stats()
    assert st[">add"] == 24 * B
    c = rm.ctrl.cpu().tolist()
    # every state slot is free, or referenced by an event in the ring, or an env's current slot
    used = torch.zeros(rm.state_buffer_size, dtype=torch.int32, device="cuda")
    used[rm.state_1_idx.long()] = 1
    used[rm.state_2_idx.long()] = 1
    used[rm.cur[:B].long()] = 1
    free = torch.tensor(rm.free_slots(), device="cuda", dtype=torch.long)
    assert int(used[free].sum()) == 0
    assert int(used.sum()) + free.numel() == rm.state_buffer_size
    assert c[abi.CP_RM_TAIL] - c[abi.CP_RM_HEAD] == free.numel()
    # the last 16 steps are in the ring in env order: event (step, env j) at (step*B + j) % N
    b, idx = rm.sample(4096)
    idx = idx.long()
    step = rm.reward[idx, 0].long()
    env = (idx - (step * B) % N) % N
    assert bool((env < B).all()) and bool((step >= 8).all())
    for s_ in range(8, 24):
        m = step == s_
        exp, dn = keep[s_]
        assert torch.equal(b.state_2[m], exp[env[m]])
        assert torch.equal(b.terminal_mask[m, 0], 1.0 - dn[env[m]].float())


def test_reset_from_event_log(tmp_path):
    """replay_memory.py:40-61 over a log written by the GPU event-log path (f2)."""
    from cartpoleplusplus_amd import event_log as EL
    B, R = 8, 2
    env = BatchedCartpole(B, 0, action_repeats=R, autoreset=True, max_episode_len=7, seed=4)
    path = str(tmp_path / "roll.log")
    log = EL.BatchedEventLog(env, path)
    env.reset()
    log.after_reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(20):
        a = torch.rand((B, 2, 2), device="cuda", generator=g) * 2 - 1
        env.step(a)
        log.after_step(a)
    log.close()
    rm = ReplayMemory(100, (R, 2, 7), 4, 1.5)
    o = ReplayOracle(100, (R, 2, 7), 4, 1.5)
    rm.reset_from_event_log(path)
    for ep in EL.EventLogReader(path).entries():
        init = EL.read_state_from_event(ep.event[0])
        o.add_episode(init, [(e.action, e.reward, EL.read_state_from_event(e)) for e in ep.event[1:]])
        if o.full:
            break
    assert rm.size() > 0
    same_as_oracle(rm, o)
