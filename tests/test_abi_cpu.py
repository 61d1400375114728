"""C-ABI checks that need no GPU: the HIP library loads, exports every entry point
include/cartpole_amd.h declares, its defaults equal the oracle's and the reference's,
and the ctypes mirror (cartpoleplusplus_amd/abi.py) has the C layout."""
import ctypes as C
import os
import re
import subprocess

import pytest

from cartpoleplusplus_amd import abi, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cartpole_amd.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cp_[a-z0-9_]+)\s*\(", src)) - {"cp_handle"})


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(native.LIB_PATH)
    decl = _declared()
    assert len(decl) >= 15
    missing = [s for s in decl if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(native.EXPORTS) == decl
    nm = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True).stdout
    for s in decl:
        assert re.search(rf"\bT {s}\b", nm), f"{s} not a global text symbol"


def test_abi_version():
    assert native.load().cp_abi_version() == abi.CP_ABI_VERSION


def _fields(s, prefix=""):
    out = {}
    for name, typ in s._fields_:
        v = getattr(s, name)
        if isinstance(v, C.Structure):
            out.update(_fields(v, prefix + name + "."))
        elif isinstance(v, C.Array):
            out[prefix + name] = [list(x) if isinstance(x, C.Array) else x for x in v]
        else:
            out[prefix + name] = v
    return out


def test_default_config_matches_oracle(oracle_mod):
    a = _fields(native.default_config())
    b = _fields(oracle_mod.default_config())
    assert a == b


def test_default_config_matches_reference_defaults(golden):
    d = golden("init.json")["opts_defaults"]
    c = native.default_config()
    assert c.action_repeats == d["action_repeats"] and c.steps_per_repeat == d["steps_per_repeat"]
    assert c.max_episode_len == d["max_episode_len"]
    assert c.action_force == d["action_force"] and c.initial_force == d["initial_force"]
    assert c.random_theta == int(not d["no_random_theta"])
    k = golden("init.json")["constants"]
    assert c.initial_force_steps == k["initial_force_steps"]
    assert c.pos_threshold == pytest.approx(k["pos_threshold"]) and c.angle_threshold == pytest.approx(
        k["angle_threshold"])


def test_ctypes_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(cp_config), sizeof(cp_physics),
         offsetof(cp_config, seed), offsetof(cp_config, phys), offsetof(cp_physics, half_extents),
         offsetof(cp_physics, spawn_pos), offsetof(cp_physics, warmstart), offsetof(cp_physics, model_flags),
         offsetof(cp_config, precision));
  printf("%d %d\\n", CP_STATE_FIELDS, CP_SF_WS_LAM(1, 4, 3));
  printf("%zu %zu %zu %zu %zu\\n", sizeof(cp_replay), offsetof(cp_replay, state), offsetof(cp_replay, plan),
         sizeof(cp_replay_batch), offsetof(cp_replay_batch, state_2_idx));
  return 0;
}}""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = list(map(int, out[0].split()))
    exp = [C.sizeof(abi.cp_config), C.sizeof(abi.cp_physics), abi.cp_config.seed.offset,
           abi.cp_config.phys.offset, abi.cp_physics.half_extents.offset, abi.cp_physics.spawn_pos.offset,
           abi.cp_physics.warmstart.offset, abi.cp_physics.model_flags.offset, abi.cp_config.precision.offset]
    assert got == exp
    assert list(map(int, out[1].split())) == [abi.CP_STATE_FIELDS, abi.CP_SF_WS_LAM(1, 4, 3)]
    assert list(map(int, out[2].split())) == [C.sizeof(abi.cp_replay), abi.cp_replay.state.offset,
                                              abi.cp_replay.plan.offset, C.sizeof(abi.cp_replay_batch),
                                              abi.cp_replay_batch.state_2_idx.offset]


def test_create_without_gpu_fails_loudly():
    """No GPU in this container: cp_create must report an error, not fall back to CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = native.load()
    cfg = native.default_config(num_envs=4)
    h = C.c_void_p()
    rc = lib.cp_create(C.byref(cfg), 0, C.byref(h))
    assert rc != 0
    assert lib.cp_last_error(None)


def test_null_arguments_rejected():
    lib = native.load()
    assert lib.cp_create(None, 0, None) != 0
    assert b"null" in lib.cp_last_error(None)
    assert lib.cp_step(None, None, 0, None, None, None, None, None) != 0


def test_product_never_imports_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/."""
    pkg = os.path.join(ROOT, "cartpoleplusplus_amd")
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|#include\s*[<\"][^>\"]*oracle|libcp_oracle|orc_", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert not pat.search(src), f


def test_cp_create_rejects_inconsistent_derived_fields():
    """cp_create validates the host-computed fields before touching a GPU:
    dt / inv_dt, tan / sin of the angle threshold, the precision flag."""
    import ctypes as C
    from cartpoleplusplus_amd import native
    lib = native.load()
    h = C.c_void_p()
    cfg = native.default_config(num_envs=4)
    cfg.phys.dt = 1.0 / 120.0                     # inv_dt left at 240
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"inv_dt" in lib.cp_last_error(None)
    cfg = native.default_config(num_envs=4)
    cfg.angle_threshold = 0.5                     # tan/sin not recomputed
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"angle_threshold" in lib.cp_last_error(None)
    cfg = native.default_config(num_envs=4, precision=7)
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"precision" in lib.cp_last_error(None)
    cfg = native.default_config(num_envs=4)
    cfg.phys.inertia[2][0] = 0.2                  # inv_inertia left stale
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"inv_inertia" in lib.cp_last_error(None)
    cfg = native.default_config(num_envs=4)
    cfg.phys.model_flags = abi.CP_MODEL_SPLIT_ISLANDS   # an oracle-only model alternative
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"model_flags" in lib.cp_last_error(None)
    # a threshold near pi/2, built by default_config: accepted (relative tolerance on tan;
    # without a GPU cp_create then fails later, for another reason)
    cfg = native.default_config(num_envs=4)
    cfg.reset_flags = 0x80                        # an unknown CP_RESET_* bit
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"reset_flags" in lib.cp_last_error(None)
    cfg = native.default_config(num_envs=4)
    cfg.phys.max_coord_velocity = float("nan")    # NaN would silently turn the clamp off
    assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
    assert b"max_coord_velocity" in lib.cp_last_error(None)
    for field, bad in (("sleep_epsilon", float("nan")), ("sleep_timeout", -1.0), ("sleep_timeout", float("inf"))):
        cfg = native.default_config(num_envs=4)
        cfg.phys.model_flags = abi.CP_MODEL_SLEEPING
        setattr(cfg.phys, field, bad)
        assert lib.cp_create(C.byref(cfg), 0, C.byref(h)) != 0
        assert b"sleep_epsilon and sleep_timeout" in lib.cp_last_error(None), field
    cfg = native.default_config(num_envs=4, angle_threshold=1.45)
    if lib.cp_create(C.byref(cfg), 0, C.byref(h)) == 0:   # a GPU host: do not leak the handle
        lib.cp_destroy(h)
    assert b"angle_threshold" not in lib.cp_last_error(None)


def test_null_handle_shape_and_state_bytes_rejected():
    lib = native.load()
    assert lib.cp_set_kernel_shape(None, 0, 0) != 0
    assert lib.cp_get_kernel_shape(None, None, None) != 0
    assert lib.cp_state_bytes(None) < 0


def test_device_buffer_checks_shape_and_dtype():
    """Sizes the C-ABI trusts are checked with exceptions (not asserts) before any pointer
    reaches cp_step / cp_reset / cp_set_* (ADVICE r1)."""
    import torch
    from cartpoleplusplus_amd.batched import _device_buffer
    dev = torch.device("cpu")
    ok = _device_buffer(torch.zeros(8, 2, dtype=torch.int8), (8, 2), torch.int8, dev, "a")
    assert ok.shape == (8, 2) and ok.is_contiguous()
    with pytest.raises(ValueError):
        _device_buffer(torch.zeros(8, 2), (8, 2, 2), torch.float32, dev, "continuous actions")
    with pytest.raises(ValueError):
        _device_buffer(torch.zeros(7, 2, dtype=torch.int8), (8, 2), torch.int8, dev, "discrete actions")
    with pytest.raises(ValueError):
        _device_buffer(torch.zeros(8, 2, dtype=torch.float32), (8, 2), torch.int8, dev, "float as indices")
    f = _device_buffer(torch.zeros(8, 2, 2, dtype=torch.float64), (8, 2, 2), torch.float32, dev, "a")
    assert f.dtype == torch.float32
