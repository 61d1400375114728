"""bench.py's multi-GPU entry point on the CPU (VERDICT r3 "next round" 1): `--gpus N` without an
external launcher starts N ranks itself (torch.distributed.run as a child process, rendezvous on
127.0.0.1), each rank checks the process group's size against --gpus, and rank 0 prints the one
JSON line.  `--cpu-dry-run` runs that launch and the C4 collective path (gloo process group, shard
rule, return all-gather + histogram) with no GPU work; without it, too few visible GPUs is a
clear error before anything is launched."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _bench(*args, env=None, timeout=240):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env or _env(),
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks_itself():
    p = _bench("--gpus", "2", "--batch", "96", "--cpu-dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0 only
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 2 and d["rccl_world_size"] == 2
    assert d["global_batch"] == 192 and d["gathered"] == 192 and d["hist_equal_unsharded"]
    assert "torch.distributed.run" in p.stderr and "--nproc-per-node=2" in p.stderr


def _refusal(n):
    p = _bench("--gpus", str(n), "--steps", "1", "--warmup", "0")
    assert p.returncode == 2, p.stderr[-2000:]
    assert f"--gpus {n} needs {n} visible GPUs" in p.stderr
    assert "torch.distributed.run" not in p.stderr
    # the parent counted without the HIP runtime and left it uninitialised
    assert "hip_initialized=False" in p.stderr, p.stderr[-2000:]
    return p


def test_gpus_n_refuses_when_too_few_gpus_are_visible():
    from cartpoleplusplus_amd.dist import visible_gpu_count
    _refusal(max(2, visible_gpu_count()[0] + 1))


@pytest.mark.gpu
def test_gpus_2_on_a_one_gpu_box_refuses_hip_free():
    """On the one-GPU box: `bench.py --gpus 2` exits 2 with the refusal, the parent counted one
    GPU from the KFD topology (not the HIP runtime) and never initialised HIP."""
    from cartpoleplusplus_amd.dist import visible_gpu_count
    n, source = visible_gpu_count()
    assert n >= 1 and source.startswith("kfd-sysfs"), (n, source)
    if n >= 2:
        pytest.skip(f"{n} GPUs visible: the refusal needs fewer than 2")
    p = _refusal(2)
    assert "visible_gpus=1 source=kfd-sysfs" in p.stderr, p.stderr[-2000:]


def _fake_topology(tmp_path, nodes, render_minors_present):
    sysfs = tmp_path / "nodes"
    dri = tmp_path / "dri"
    dri.mkdir()
    for i, (gfx, minor) in enumerate(nodes):
        d = sysfs / str(i)
        d.mkdir(parents=True)
        lines = [f"cpu_cores_count {0 if gfx else 16}", f"gfx_target_version {gfx}"]
        if minor is not None:
            lines.append(f"drm_render_minor {minor}")
        (d / "properties").write_text("\n".join(lines) + "\n")
    for m in render_minors_present:
        (dri / f"renderD{m}").write_text("")
    return str(sysfs), str(dri)


def test_visible_gpu_count_from_kfd_topology(tmp_path, monkeypatch):
    """The launcher's device count: GPU nodes of the KFD topology (gfx_target_version != 0) whose
    render node this process can open; a container lists all 8 GPUs in sysfs but maps one."""
    from cartpoleplusplus_amd.dist import visible_gpu_count
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    nodes = [(0, None), (0, None)] + [(90500, 128 + 8 * k) for k in range(8)]
    sysfs, dri = _fake_topology(tmp_path, nodes, [136])
    assert visible_gpu_count(sysfs, dri) == (1, "kfd-sysfs")
    for k in range(8):
        open(os.path.join(dri, f"renderD{128 + 8 * k}"), "w").close()
    assert visible_gpu_count(sysfs, dri) == (8, "kfd-sysfs")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert visible_gpu_count(sysfs, dri) == (2, "kfd-sysfs+HIP_VISIBLE_DEVICES")
    # ROCR first, then HIP indexes into what ROCR left: "0,1" over one device is one device
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3")
    assert visible_gpu_count(sysfs, dri) == (1, "kfd-sysfs+ROCR_VISIBLE_DEVICES+HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    # out-of-range and repeated indices are no devices; UUIDs count once each
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,9,0,12")
    assert visible_gpu_count(sysfs, dri)[0] == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-aa,GPU-bb,7")
    assert visible_gpu_count(sysfs, dri)[0] == 3


def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = _bench("--gpus", "2", "--steps", "1", env=env)
    assert p.returncode != 0 and "must agree" in p.stderr
