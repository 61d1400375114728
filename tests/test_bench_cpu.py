"""bench.py's host logic on the CPU: the synthetic action stream is a pure function of
(seed, global env id, step, cart), so a shard's rows equal the unsharded job's rows for
its envs (the C4 seed rule), and the workload string follows the
arguments."""
import argparse

import numpy as np
import torch

import bench


def test_action_stream_shards_equal_unsharded_slices():
    dev = torch.device("cpu")
    for continuous in (False, True):
        full = bench.make_actions(continuous, 96, 0, 7, bench.SEED, dev)
        for r in range(3):
            part = bench.make_actions(continuous, 32, 32 * r, 7, bench.SEED, dev)
            assert torch.equal(part, full[:, 32 * r:32 * (r + 1)])
        # steps are independent of where the generation chunks start
        late = torch.cat([bench.action_block(continuous, torch.arange(96), t, 1, bench.SEED) for t in range(7)])
        assert torch.equal(late, full)


def test_action_stream_ranges_and_spread():
    dev = torch.device("cpu")
    d = bench.make_actions(False, 4096, 0, 4, bench.SEED, dev)
    assert d.dtype == torch.int8 and d.shape == (4, 4096, 2)
    counts = np.bincount(d.numpy().ravel(), minlength=5)
    assert counts.min() > 0.18 * d.numel() and counts.max() < 0.22 * d.numel() and len(counts) == 5
    c = bench.make_actions(True, 4096, 0, 4, bench.SEED, dev)
    assert c.dtype == torch.float32 and c.shape == (4, 4096, 2, 2)
    assert float(c.min()) >= -1.0 and float(c.max()) < 1.0 and abs(float(c.mean())) < 0.02
    # another seed, another stream
    assert not torch.equal(d, bench.make_actions(False, 4096, 0, 4, bench.SEED + 1, dev))


def _args(**kw):
    a = dict(batch=65536, repeats=3, continuous=False, raster=False, cameras=1, done_on_bounds=False,
             solver_iterations=None, dtype="f32")
    a.update(kw)
    return argparse.Namespace(**a)


def test_workload_names():
    assert bench.workload(_args(), 1)[0] == "C3"
    assert bench.workload(_args(), 8)[0] == "C4"
    assert bench.workload(_args(batch=4096, continuous=True), 1)[0] == "C2"
    assert bench.workload(_args(raster=True), 1)[0] == "C5"
    assert bench.workload(_args(batch=4096), 1)[0] == "custom"
    name, s = bench.workload(_args(batch=4096, continuous=True), 1)
    assert "4,096" in s and "continuous" in s and "configs[1]" in s


def test_step_kernel_bytes_formula():
    # 1,059 B per env-step at R = 3 with discrete actions
    assert bench.step_kernel_bytes(3, 2) == 1059
    assert bench.step_kernel_bytes(3, 16) == 1073
