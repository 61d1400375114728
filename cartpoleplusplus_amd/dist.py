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
    """Histogram of integer episode returns (reward 1.0 per step), bins 0..max_len.  A scatter-add into
    a fixed-size histogram: torch.bincount sizes its output from the input's maximum, which waits on
    the device from the host in the middle of the caller's stream."""
    idx = returns.to(torch.int64).clamp(0, max_len)
    hist = torch.zeros(max_len + 1, dtype=torch.int64, device=returns.device)
    return hist.scatter_add_(0, idx, torch.ones_like(idx))


def _visible_filters():
    """The device filters a HIP process applies, in the order the ROCm runtime applies them:
    ROCR_VISIBLE_DEVICES first (the ROCr runtime's list of agents), then HIP_VISIBLE_DEVICES and
    CUDA_VISIBLE_DEVICES (HIP's alias for it), each an index list into what the one before left.
    Returns [(var, [entries])] for every variable that is set."""
    import os
    out = []
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            out.append((var, [x.strip() for x in v.split(",") if x.strip() != ""]))
    return out


def _apply_filter(count, entries):
    """Devices left after one filter over `count` devices: integer indices count only when they
    are in range (and once each); a UUID ("GPU-...") may only be counted, not checked."""
    seen = set()
    n = 0
    for x in entries:
        try:
            k = int(x, 0)
        except ValueError:
            if x.upper().startswith("GPU-") and x not in seen:
                seen.add(x)
                n += 1
            continue
        if 0 <= k < count and k not in seen:
            seen.add(k)
            n += 1
    return min(n, count)


def visible_gpu_count(sysfs="/sys/class/kfd/kfd/topology/nodes", dev_dri="/dev/dri"):
    """Count the GPUs this process could open WITHOUT initialising the HIP runtime (bench.py's
    --gpus N launcher runs it in the parent, which must never initialise the GPU before starting
    the ranks).  Source, in order:
      1. the KFD topology in sysfs: nodes with a non-zero gfx_target_version (CPU nodes have 0)
         whose render node /dev/dri/renderD<drm_render_minor> exists and is read/writable by this
         process (a container lists every GPU of the host in sysfs but maps only its own render
         nodes);
      2. amdsmi (the kernel driver's SMI interface, no HIP), when sysfs has no topology;
    then filtered by ROCR_VISIBLE_DEVICES, HIP_VISIBLE_DEVICES and CUDA_VISIBLE_DEVICES in turn
    (every one that is set; out-of-range indices dropped, _apply_filter).
    Never torch.cuda.device_count(): on ROCm it falls back to hipGetDeviceCount, which initialises
    the runtime, whenever amdsmi does not answer.  Returns (count, source)."""
    import os
    count, source = None, None
    if os.path.isdir(sysfs):
        n = 0
        for node in sorted(os.listdir(sysfs)):
            props = {}
            try:
                with open(os.path.join(sysfs, node, "properties")) as f:
                    for line in f:
                        k, _, v = line.strip().partition(" ")
                        props[k] = v.strip()
            except OSError:
                continue
            if int(props.get("gfx_target_version", "0") or 0) == 0:
                continue
            minor = props.get("drm_render_minor")
            if minor is None:
                continue
            path = os.path.join(dev_dri, f"renderD{int(minor)}")
            if os.path.exists(path) and os.access(path, os.R_OK | os.W_OK):
                n += 1
        count, source = n, "kfd-sysfs"
    else:
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            try:
                count = len(amdsmi.amdsmi_get_processor_handles())
            finally:
                amdsmi.amdsmi_shut_down()
            source = "amdsmi"
        except Exception:   # no driver interface at all: nothing visible
            count, source = 0, "none"
    for var, lst in _visible_filters():
        count = _apply_filter(count, lst)
        source += f"+{var}"
    return count, source
