"""C4's sharding on the HIP path: two processes on the one
GPU each drive a shard handle (common seed, env_id_offset = rank * B, autoreset, bounds
termination on, actions keyed by global env id as bench.py makes them); the obs, terminal
obs and episode returns gathered over gloo equal, bit for bit, a single-process run of the
2B-env batch.  The run crosses step 200 (fixed-length resets) and many bounds resets."""
import os
import socket

import numpy as np
import pytest
import torch

B_PER_RANK = 96
STEPS = 230


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(num_envs, env_id_offset, shape):
    """Envs [env_id_offset, env_id_offset + num_envs) of the global job: obs, terminal obs, done
    of every step, and the last episode returns (host numpy)."""
    import bench
    from cartpoleplusplus_amd.batched import BatchedCartpole
    env = BatchedCartpole(num_envs, 0, action_repeats=3, max_episode_len=200, initial_force=55.0, autoreset=True,
                          done_on_bounds=True, seed=bench.SEED, env_id_offset=env_id_offset)
    env.set_kernel_shape(*shape)
    acts = bench.make_actions(False, num_envs, env_id_offset, STEPS, bench.SEED, env.device)
    obs, term, done = [], [], []
    obs.append(env.reset().cpu().numpy().copy())
    for t in range(STEPS):
        o, _, d = env.step(acts[t])
        obs.append(o.cpu().numpy().copy())
        term.append(env.terminal_obs.cpu().numpy().copy())
        done.append(d.cpu().numpy().copy())
    ret, n = env.episode_returns()
    out = (np.stack(obs), np.stack(term), np.stack(done), ret.cpu().numpy(), n.cpu().numpy())
    env.close()
    return out


def _worker(rank, world, port, q, shape):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cartpoleplusplus_amd.dist import gather_returns, shard_spec
        torch.cuda.set_device(0)
        spec = shard_spec(B_PER_RANK, rank, world, seed=1234)
        obs, term, done, ret, n = _run(spec["num_envs"], spec["env_id_offset"], shape)
        allret = gather_returns(torch.from_numpy(ret))            # gloo on host copies
        gathered = []
        for a in (obs, term, done, n):
            parts = [torch.zeros_like(torch.from_numpy(a)) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(a)))
            gathered.append(torch.cat(parts, dim=1 if a.ndim > 1 else 0).numpy())
        if rank == 0:
            q.put((allret.numpy(), *gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [("throughput", "throughput"), ("latency", "latency")], ids=["tp", "lat"])
def test_two_shards_on_the_gpu_equal_one_process_of_2B_envs(shape):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, shape)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        allret, obs, term, done, n = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    r_obs, r_term, r_done, r_ret, r_n = _run(2 * B_PER_RANK, 0, shape[::-1] if shape[0] != shape[1] else shape)
    assert np.array_equal(done, r_done)
    assert done.sum() > 2 * B_PER_RANK     # bounds resets as well as the step-200 burst
    assert np.array_equal(obs.view(np.uint32), r_obs.view(np.uint32))
    assert np.array_equal(term.view(np.uint32), r_term.view(np.uint32))
    assert np.array_equal(allret, r_ret) and np.array_equal(n, r_n)
