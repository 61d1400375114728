"""Multi-process (world size 2, gloo, CPU) checks of the data-parallel path: the
sharded job (rank r owns global env ids r*B..) reproduces the unsharded job exactly,
and the episode-return gather / histogram equals the single-process one.  The envs
are the CPU oracle here (no GPU); bench.py runs the same sharding on the HIP library
with backend "nccl" (RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B_PER_RANK = 24
STEPS = 45


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_envs(O, num_envs, env_id_offset, seed):
    from cartpoleplusplus_amd import abi
    cfg = O.default_config(num_envs=num_envs, action_repeats=3, initial_force=55.0, seed=seed,
                           env_id_offset=env_id_offset, autoreset=1, max_episode_len=20, done_on_bounds=1)
    e = O.Envs(cfg)
    obs0 = e.reset().copy()
    rng = np.random.default_rng(7)
    acts = rng.integers(0, 5, (STEPS, 2 * B_PER_RANK, 2)).astype(np.int8)   # global action stream
    lo = env_id_offset
    for t in range(STEPS):
        obs, _, _ = e.step(np.ascontiguousarray(acts[t, lo:lo + num_envs]), abi.CP_ACTION_DISCRETE)
    ret, _ = e.episode_returns()
    return obs0, obs.copy(), ret


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cartpoleplusplus_amd.dist import gather_returns, return_histogram, shard_spec
        from oracle import oracle as O
        spec = shard_spec(B_PER_RANK, rank, world)
        obs0, obs, ret = _run_envs(O, spec["num_envs"], spec["env_id_offset"], spec["seed"])
        allret = gather_returns(torch.from_numpy(ret))
        hist = return_histogram(allret, 20)
        parts = [torch.zeros_like(torch.from_numpy(obs)) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(obs))
        if rank == 0:
            q.put((allret.numpy(), hist.numpy(), torch.cat(parts).numpy(), spec["global_batch"]))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_equals_single_process(oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    allret, hist, obs, gb = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert gb == 2 * B_PER_RANK
    _, obs_ref, ret_ref = _run_envs(oracle_mod, 2 * B_PER_RANK, 0, 1234)
    assert np.array_equal(allret, ret_ref)
    assert np.array_equal(obs, obs_ref)
    assert np.array_equal(hist, np.bincount(ret_ref.astype(np.int64), minlength=21))
    assert hist.sum() == 2 * B_PER_RANK and (ret_ref > 0).all()


def test_shard_spec_covers_ids_once():
    from cartpoleplusplus_amd.dist import shard_spec
    ids = []
    for r in range(8):
        s = shard_spec(65536, r, 8)
        ids.append((s["env_id_offset"], s["env_id_offset"] + s["num_envs"]))
        assert s["global_batch"] == 8 * 65536
    assert ids[0][0] == 0 and all(ids[i][1] == ids[i + 1][0] for i in range(7)) and ids[-1][1] == 8 * 65536


def test_gather_without_process_group_is_identity():
    from cartpoleplusplus_amd.dist import gather_returns
    if dist.is_initialized():
        pytest.skip("process group active")
    t = torch.arange(5, dtype=torch.float32)
    assert torch.equal(gather_returns(t), t)
