"""The RCCL branch of the C4 collective (dist.gather_returns: all_gather_into_tensor under backend
"nccl" = RCCL on ROCm) executed on the MI355X with one rank: the GPU box has one GPU, RCCL refuses two
ranks on one device, and the driver runs the 8-GPU scaling bench itself.  The gathered returns and
the histogram equal the local ones, and bench.py's per-window gather runs inside a timed window."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_all_gather_of_episode_returns_world_size_1():
    import torch.distributed as dist

    from cartpoleplusplus_amd.batched import BatchedCartpole
    from cartpoleplusplus_amd.dist import gather_returns, return_histogram
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        env = BatchedCartpole(4096, 0, action_repeats=3, initial_force=55.0, autoreset=True, done_on_bounds=True,
                              max_episode_len=200, seed=1234)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        for _ in range(60):
            env.step(torch.randint(0, 5, (4096, 2), device="cuda", generator=g, dtype=torch.int8))
        r, n = env.episode_returns()
        allr = gather_returns(r)                      # RCCL all_gather_into_tensor
        torch.cuda.synchronize()
        assert allr.shape == (4096,) and torch.equal(allr, r)
        h = return_histogram(allr)
        assert int(h.sum()) == 4096 and torch.equal(h, return_histogram(r))
    finally:
        dist.destroy_process_group()
