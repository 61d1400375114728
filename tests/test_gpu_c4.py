"""BASELINE configs[3] (C4) on one GPU: the 524,288-env job as its 8 shards, each a 65,536-env
handle with env_id_offset = r * 65,536 (the rank-r shard of `bench.py --gpus 8`, SURVEY.md §8e,
dist.py), driven by bench.py's own action stream, across one step-200 autoreset burst.

  - every step, the 8 shards' obs / reward / done concatenated equal bit for bit one handle of the
    whole 524,288-env batch (the unsharded job);
  - finiteness and unit quaternions on all 524,288 envs at every step, and cp_nonfinite_counts 0
    everywhere: the coordinate-velocity clamp (btMultiBody's m_maxCoordinateVelocity)
    bounds the loose-pole yaw spin whose explicit gyroscopic term used to diverge (before it, env
    138,554 went NaN at step 44 and 18 envs by step 203);
  - 6 blocks of 128 envs, two of them in the top shard (global ids >= 458,752) and two holding the
    envs that used to diverge (their poles now spin at the clamp), re-simulated on the oracle from
    reset: obs, done, terminal obs and the non-finite counters, bit for bit;
  - the episode-return histogram of the concatenated shards (what bench's RCCL all-gather feeds
    return_histogram) equals the unsharded batch's, with all 524,288 episodes of length 200.
The reference runs one env per process (bullet_cartpole.py:151, p.connect(p.DIRECT)); the shard
rule is what makes N processes one job."""
import os

import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from cartpoleplusplus_amd.dist import return_histogram, shard_spec
from tests.test_gpu_parity import _assert_same, _np

pytestmark = pytest.mark.gpu

RANKS, B = 8, 65536
STEPS = 203          # from reset: steps 1..200, the burst at step 200, then 3 steps of episode 2
CLAMPED_ENVS = (138554, 485573)   # diverged before the clamp (oracle run of the whole batch); now finite


def test_c4_eight_shards_on_one_gpu_equal_the_unsharded_job(oracle_mod):
    import bench
    N = RANKS * B
    kw = dict(action_repeats=3, steps_per_repeat=1, max_episode_len=bench.WINDOW, initial_force=55.0,
              autoreset=True, seed=bench.SEED)
    specs = [shard_spec(B, r, RANKS, seed=bench.SEED) for r in range(RANKS)]
    shards = [BatchedCartpole(B, 0, env_id_offset=s["env_id_offset"], **kw) for s in specs]
    for sh in shards:
        assert sh.kernel_shape() == ("throughput", "throughput")   # what each rank's bench times
    whole = BatchedCartpole(N, 0, env_id_offset=0, **kw)
    acts = bench.make_actions(False, N, 0, STEPS, bench.SEED, whole.device)
    # a rank's own make_actions (env_id_offset = its shard) is the slice of the whole job's stream
    assert torch.equal(bench.make_actions(False, B, specs[-1]["env_id_offset"], 3, bench.SEED, whole.device),
                       acts[:3, N - B:])

    blocks = [0, 138496, 200000, 458752, 485504, N - 128]   # global env ids: the CLAMPED_ENVS' blocks, the top shard
    cfg = native.default_config(num_envs=128, **{k: (int(v) if isinstance(v, bool) else v) for k, v in kw.items()})
    orcs = []
    for lo in blocks:
        sub = abi.cp_config.from_buffer_copy(cfg)
        sub.env_id_offset = lo
        orcs.append(oracle_mod.Envs(sub))
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def cat_shards(xs):
        return torch.cat(xs, dim=0)

    o_sh = cat_shards([sh.reset() for sh in shards])
    o_wh = whole.reset()
    assert torch.equal(o_sh.view(torch.int32), o_wh.view(torch.int32)), "reset obs"
    for lo, orc in zip(blocks, orcs):
        _assert_same(_np(o_wh[lo:lo + 128]), orc.reset(), f"block {lo} reset obs")

    rew = np.zeros(128, np.float32)
    for t in range(STEPS):
        outs = [sh.step(acts[t, r * B:(r + 1) * B]) for r, sh in enumerate(shards)]
        o_wh, r_wh, d_wh = whole.step(acts[t])
        o_sh = cat_shards([o for o, _, _ in outs])
        assert torch.equal(o_sh.view(torch.int32), o_wh.view(torch.int32)), f"obs step {t}"
        assert torch.equal(cat_shards([r for _, r, _ in outs]), r_wh), f"reward step {t}"
        d_sh = cat_shards([d for _, _, d in outs])
        assert torch.equal(d_sh, d_wh), f"done step {t}"
        t_sh = cat_shards([sh.terminal_obs for sh in shards])
        burst = t == bench.WINDOW - 1
        if burst:
            assert bool(d_wh.all()), "every episode ends at step 200"
            assert torch.equal(t_sh.view(torch.int32), whole.terminal_obs.view(torch.int32)), "terminal obs"
        else:
            assert not bool(d_wh.any())
        fin = torch.isfinite(o_wh).flatten(1).all(1)
        bad = set(torch.nonzero(~fin).flatten().tolist())
        assert not bad, f"non-finite obs at step {t} in {len(bad)} envs {sorted(bad)[:8]}"
        if t % 25 == 0 or burst or t == STEPS - 1:
            q = o_wh[..., 3:7].double()
            assert bool(torch.allclose(q.norm(dim=-1), torch.ones_like(q[..., 0]), atol=1e-5)), f"quat norm step {t}"
        for lo, orc in zip(blocks, orcs):
            r, i = divmod(lo, B)
            go = _np(outs[r][0][i:i + 128])
            oo = np.zeros((128, 3, 2, 7), np.float32)
            od = np.zeros(128, np.uint8)
            if burst:
                oo, _, od, ot = orc.step(np.ascontiguousarray(_np(acts[t, lo:lo + 128])), terminal=True)
                _assert_same(_np(shards[r].terminal_obs[i:i + 128]), ot, f"block {lo} terminal obs")
            else:
                orc.step_omp(np.ascontiguousarray(_np(acts[t, lo:lo + 128])), abi.CP_ACTION_DISCRETE, oo, rew, od,
                             threads)
            _assert_same(go, oo, f"block {lo} obs step {t}")
            _assert_same(_np(outs[r][2][i:i + 128]), od, f"block {lo} done step {t}")

    ret_sh = cat_shards([sh.episode_returns()[0] for sh in shards])
    ret_wh, len_wh = whole.episode_returns()
    assert torch.equal(ret_sh, ret_wh)
    h_sh = return_histogram(ret_sh, bench.WINDOW)
    h_wh = return_histogram(ret_wh, bench.WINDOW)
    assert torch.equal(h_sh, h_wh)
    assert int(h_wh[bench.WINDOW]) == N and int(h_wh.sum()) == N
    assert bool((len_wh == bench.WINDOW).all())
    for lo, orc in zip(blocks, orcs):
        _assert_same(_np(ret_wh[lo:lo + 128]), orc.episode_returns()[0], f"block {lo} returns")
    nf_sh = cat_shards([sh.nonfinite_counts() for sh in shards])
    nf_wh = whole.nonfinite_counts()
    assert torch.equal(nf_sh, nf_wh)
    assert int(nf_wh.count_nonzero()) == 0, sorted(torch.nonzero(nf_wh).flatten().tolist())[:8]
    st_all = whole.get_state()
    assert bool(torch.isfinite(st_all[:abi.CP_SF_STEPS]).all()), "every body state and pending force finite"
    for lo, orc in zip(blocks, orcs):
        _assert_same(_np(nf_wh[lo:lo + 128]), orc.nonfinite(), f"block {lo} non-finite counters")
    st = _np(whole.get_state())
    eps = st.view(np.int32)[abi.CP_SF_EPISODE]
    assert (eps == 2).all()
    for sh in shards:
        sh.close()
    whole.close()
