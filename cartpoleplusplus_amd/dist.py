"""Data-parallel sharding of independent envs across ranks (one process per GPU).

Envs never interact, so a batch of N*B envs runs as N independent shards with no
per-step communication.  Rank r owns global env ids [r*B, (r+1)*B).  The seed rule:
every rank uses the SAME seed (the Philox key); the global env id is the Philox
counter's env word, so rank r's envs draw exactly the bump pushes envs r*B.. of one
unsharded N*B-env run draw, and a sharded job given the same per-env actions
reproduces the unsharded one bit for bit (tests/test_dist.py on the oracle,
tests/test_gpu_shard.py on the HIP path).  bench.py keys its synthetic actions by
global env id as well.  The only collective is the gather of per-env episode returns
once per reporting window (RCCL over xGMI with backend "nccl"; gloo on CPU in tests).
"""
import torch
import torch.distributed as dist


def shard_spec(envs_per_rank, rank, world, seed=1234):
    """Config fields of rank `rank`'s shard."""
    return {"num_envs": int(envs_per_rank), "env_id_offset": int(rank) * int(envs_per_rank),
            "seed": int(seed), "global_batch": int(envs_per_rank) * int(world)}


def gather_returns(returns, group=None):
    """All-gather a (B,) float tensor of episode returns from every rank -> (world*B,)."""
    if not dist.is_available() or not dist.is_initialized():
        return returns
    world = dist.get_world_size(group)
    out = torch.empty(world * returns.numel(), dtype=returns.dtype, device=returns.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, returns.contiguous(), group=group)
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, returns.contiguous(), group=group)
        out = torch.cat(parts)
    return out


def return_histogram(returns, max_len=200):
    """Histogram of integer episode returns (reward 1.0 per step), bins 0..max_len."""
    return torch.bincount(returns.to(torch.int64).clamp(0, max_len), minlength=max_len + 1)
