"""CP_AUTORESET_NEXT_STEP in the oracle (the checker of the HIP path's pipelined resets), on the CPU.

NEXT_STEP must be SAME_STEP with each reset handed out one call later: a finishing env returns its
finishing obs with done 1, the next call returns the new episode's first obs with reward 0 and
done 0 and ignores that env's action, and from then on the env replays SAME_STEP's episode.  The
check feeds NEXT_STEP every env's SAME_STEP action stream shifted by the calls it spent in resets,
and requires every output bit for bit; bounds termination makes the episodes end at different
steps (bullet_cartpole.py:243-253), so envs are in different phases in every call."""
import numpy as np
import pytest

from cartpoleplusplus_amd import abi


def _cfg(O, mode, B):
    return O.default_config(num_envs=B, action_repeats=2, initial_force=55.0, seed=5, autoreset=mode,
                            done_on_bounds=1, max_episode_len=25)


def _done_field(env):
    return abi.state_ints(env.get_state()[abi.CP_SF_DONE])


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_next_step_is_same_step_one_call_later(oracle_mod, precision):
    O = oracle_mod
    B, K = 24, 90
    rng = np.random.default_rng(3)
    A = rng.integers(0, 5, (K, B, 2)).astype(np.int8)
    same = O.Envs(_cfg(O, abi.CP_AUTORESET_SAME_STEP, B), precision=precision)
    nxt = O.Envs(_cfg(O, abi.CP_AUTORESET_NEXT_STEP, B), precision=precision)
    r0, r1 = same.reset(), nxt.reset()
    assert np.array_equal(r0.view(np.uint32), r1.view(np.uint32))
    S = [same.step(A[k], terminal=True) for k in range(K)]   # (obs, reward, done, terminal obs)
    ptr = np.zeros(B, np.int64)      # SAME_STEP call each env replays next
    handed = 0
    for _ in range(K + 40):
        if ptr.min() >= K:
            break
        pending = _done_field(nxt) >= 2
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)        # pending envs ignore theirs
        live = ~pending & (ptr < K)
        a[live] = A[ptr[live], np.nonzero(live)[0]]
        obs, rew, done = nxt.step(a)
        for i in range(B):
            if ptr[i] >= K:
                continue
            if pending[i]:   # the reset obs SAME_STEP returned in the call that ended the episode
                k = ptr[i] - 1
                assert np.array_equal(obs[i].view(np.uint32), S[k][0][i].view(np.uint32)), (i, k)
                assert rew[i] == 0.0 and done[i] == 0
                handed += 1
                continue
            k = ptr[i]
            want = S[k][3][i] if S[k][2][i] else S[k][0][i]   # finishing obs, or the step's obs
            assert np.array_equal(obs[i].view(np.uint32), want.view(np.uint32)), (i, k)
            assert rew[i] == S[k][1][i] and done[i] == S[k][2][i], (i, k)
            ptr[i] += 1
    assert ptr.min() >= K and handed >= B, (ptr.min(), handed)   # every env replayed; several resets each


def test_reset_of_a_pending_env_returns_its_reset(oracle_mod):
    """cp_reset on an env whose reset already ran (NEXT_STEP, pending) hands out that reset's obs
    and does not reset again (one reset from the terminal state, as a lazy reset would); a
    non-pending env in the mask is reset normally.  Same state as SAME_STEP's after its reset."""
    O = oracle_mod
    B = 16
    rng = np.random.default_rng(11)
    same = O.Envs(_cfg(O, abi.CP_AUTORESET_SAME_STEP, B))
    nxt = O.Envs(_cfg(O, abi.CP_AUTORESET_NEXT_STEP, B))
    same.reset(), nxt.reset()
    for k in range(200):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        s_obs, _, s_done = same.step(a)
        n_obs, _, n_done = nxt.step(a)
        assert np.array_equal(s_done, n_done)
        if s_done.any():
            break
    assert s_done.any(), "no episode ended"
    pending = _done_field(nxt) >= 2
    assert np.array_equal(pending, s_done.astype(bool))
    st_same, st_next = same.get_state(), nxt.get_state()
    other = np.arange(abi.CP_STATE_FIELDS) != abi.CP_SF_DONE
    assert np.array_equal(st_same[other].view(np.uint32), st_next[other].view(np.uint32))   # eager reset
    mask = np.zeros(B, np.uint8)
    mask[np.nonzero(pending)[0][:1]] = 1      # one pending env
    mask[np.nonzero(~pending)[0][:2]] = 1     # two running envs
    obs = nxt.reset(mask)
    i = np.nonzero(pending)[0][0]
    assert np.array_equal(obs[i].view(np.uint32), s_obs[i].view(np.uint32))
    d = _done_field(nxt)
    assert (d[mask == 1] == 0).all() and (d[pending & (mask == 0)] >= 2).all()
