"""ctypes binding of the HIP library (libcartpole_hip.so, C-ABI in include/cartpole_amd.h).

The product path has no CPU fallback: if the library is missing or no GPU is
visible, these calls raise.  (`tests/` compare against the CPU oracle, which is
never imported from here.)
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CP_LIB_PATH") or os.path.join(HERE, "libcartpole_hip.so")

# every entry point declared in include/cartpole_amd.h
EXPORTS = (
    "cp_default_config", "cp_create", "cp_destroy", "cp_last_error", "cp_abi_version",
    "cp_reset", "cp_step", "cp_set_readback", "cp_set_bump_forces", "cp_set_bump_forces64", "cp_get_state",
    "cp_set_state", "cp_episode_returns", "cp_overflow_counts", "cp_timing_begin", "cp_timing_end",
    "cp_timing_stride",
    "cp_debug_stamps", "cp_default_raster_config", "cp_set_raster", "cp_timing_render",
    "cp_event_record_bytes", "cp_encode_events", "cp_eventlog_open", "cp_eventlog_write", "cp_eventlog_close",
    "cp_set_lqr", "cp_get_stepped", "cp_replay_init", "cp_replay_add", "cp_replay_sample",
    "cp_state_bytes", "cp_set_kernel_shape", "cp_get_kernel_shape", "cp_rollout",
    "cp_nonfinite_counts", "cp_render_kernel_name",
)

_lib = None


class CartpoleError(RuntimeError):
    pass


def load():
    """Load the in-tree HIP library (does not touch the GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CartpoleError(
            f"{LIB_PATH} is missing: build it with `python -m cartpoleplusplus_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    P, VP, I = C.POINTER, C.c_void_p, C.c_int
    cfgp = P(abi.cp_config)
    sig = {
        "cp_default_config": (None, [cfgp]),
        "cp_create": (I, [cfgp, I, P(VP)]),
        "cp_destroy": (None, [VP]),
        "cp_last_error": (C.c_char_p, [VP]),
        "cp_abi_version": (I, []),
        "cp_reset": (I, [VP, VP, VP, VP]),
        "cp_step": (I, [VP, VP, I, VP, VP, VP, VP, VP]),
        "cp_set_readback": (I, [VP, VP, I]),
        "cp_set_bump_forces": (I, [VP, VP, VP]),
        "cp_set_bump_forces64": (I, [VP, VP, VP]),
        "cp_get_state": (I, [VP, VP, VP]),
        "cp_set_state": (I, [VP, VP, VP]),
        "cp_episode_returns": (I, [VP, VP, VP, VP]),
        "cp_overflow_counts": (I, [VP, VP, VP]),
        "cp_nonfinite_counts": (I, [VP, VP, VP]),
        "cp_timing_begin": (I, [VP, I]),
        "cp_timing_stride": (I, [VP, I, I]),
        "cp_debug_stamps": (I, [VP, P(C.c_uint64), I]),
        "cp_timing_end": (I, [VP, P(C.c_double), P(C.c_int32), P(C.c_double), P(C.c_int32)]),
        "cp_default_raster_config": (None, [P(abi.cp_raster_config)]),
        "cp_set_raster": (I, [VP, P(abi.cp_raster_config), VP]),
        "cp_timing_render": (I, [VP, P(C.c_double), P(C.c_int32)]),
        "cp_render_kernel_name": (C.c_char_p, [VP]),
        "cp_event_record_bytes": (I, [I, I, I]),
        "cp_encode_events": (I, [VP, I, VP, I, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
        "cp_eventlog_open": (I, [C.c_char_p, I, P(VP)]),
        "cp_eventlog_write": (I, [VP, VP, VP, I, VP, I]),
        "cp_eventlog_close": (I, [VP]),
        "cp_get_stepped": (I, [VP, VP, VP]),
        "cp_set_lqr": (I, [VP, VP, I, VP, C.c_float, C.c_float]),
        "cp_replay_init": (I, [P(abi.cp_replay), VP, I, VP]),
        "cp_replay_add": (I, [P(abi.cp_replay), VP, I, VP, VP, I, VP, VP, VP, VP, VP, I, VP]),
        "cp_replay_sample": (I, [P(abi.cp_replay), I, VP, C.c_uint64, C.c_uint64, P(abi.cp_replay_batch), VP]),
        "cp_state_bytes": (C.c_int64, [VP]),
        "cp_rollout": (I, [VP, I, VP, I, VP, VP, VP, VP, VP]),
        "cp_set_kernel_shape": (I, [VP, I, I]),
        "cp_get_kernel_shape": (I, [VP, P(I), P(I)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    if lib.cp_abi_version() != abi.CP_ABI_VERSION:
        raise CartpoleError("libcartpole_hip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def default_raster_config(**overrides):
    """cp_raster_config with the reference defaults (bullet_cartpole.py:27-37, :277-284)."""
    rc = abi.cp_raster_config()
    load().cp_default_raster_config(C.byref(rc))
    for k, v in overrides.items():
        if not hasattr(rc, k):
            raise AttributeError(f"cp_raster_config has no field {k!r}")
        setattr(rc, k, v)
    return rc


def default_config(**overrides):
    """cp_config with the reference defaults (bullet_cartpole.py:15-40), then overrides."""
    import math
    cfg = abi.cp_config()
    load().cp_default_config(C.byref(cfg))
    for k, v in overrides.items():
        if k == "angle_threshold":
            cfg.tan_angle_threshold = math.tan(v)
            cfg.sin_angle_threshold = math.sin(v)
        if not hasattr(cfg, k):
            raise AttributeError(f"cp_config has no field {k!r}")
        setattr(cfg, k, v)
    return cfg


def check(h, status, what):
    if status != 0:
        msg = load().cp_last_error(h)
        raise CartpoleError(f"{what} failed: {msg.decode() if msg else 'unknown error'}")


_hip = None


def mapped_device_pointer(t):
    """The device address of a pinned host tensor (hipHostGetDevicePointer): a kernel may read and write
    pinned host memory the runtime has mapped for the GPU directly, with no copy operation (the gym
    mirror's zero-copy step).  Raises CartpoleError when the memory is not mapped."""
    global _hip
    if not t.is_pinned():
        raise CartpoleError("mapped_device_pointer: the tensor is not in pinned host memory")
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
    p = C.c_void_p()
    rc = _hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not p.value:
        raise CartpoleError(f"hipHostGetDevicePointer failed ({rc}): pinned memory not mapped for the GPU")
    return C.c_void_p(p.value)
