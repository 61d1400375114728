"""ctypes wrapper of the CPU oracle (oracle/build/libcp_oracle*.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.  See cp_oracle.h for
what the oracle restates and how it is pinned.
"""
import ctypes as C
import math
import os
import subprocess

import numpy as np

from cartpoleplusplus_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")


def build(quiet=True):
    """Compile both oracle variants (gcc; seconds)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


class orc_world(C.Structure):
    _fields_ = [
        ("pos", (C.c_double * 3) * 4),
        ("quat", (C.c_double * 4) * 4),
        ("vel", (C.c_double * 3) * 4),
        ("omega", (C.c_double * 3) * 4),
        ("pending", (C.c_double * 3) * 4),
        ("ws_id", C.c_uint32 * 10),
        ("ws_lam", (C.c_double * 4) * 10),
        ("overflow", C.c_int32),
        ("last_iterations", C.c_int32),
        ("last_points", C.c_int32),
    ]


_LIBS = {}


def load(precision="f32"):
    """precision: "f32" (parity build), "f64", or "native" (fp32, -O3 -march=native: the
    CPU-baseline build of bench.py, same results as "f32")."""
    if precision == "native":
        name = native_path()
        if name in _LIBS:
            return _LIBS[name]
        path = name
        if not os.path.exists(path):
            out = subprocess.run(["make", "-C", HERE, "native", f"NATIVE_OUT={path}"], capture_output=True, text=True)
            if out.returncode != 0:
                raise RuntimeError("native oracle build failed:\n" + out.stdout + out.stderr)
    else:
        name = {"f32": "libcp_oracle.so", "f64": "libcp_oracle_f64.so"}[precision]
        if name in _LIBS:
            return _LIBS[name]
        path = os.environ.get("ORC_LIB_OVERRIDE") or os.path.join(BUILD, name)
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    P, VP = C.POINTER, C.c_void_p
    cfgp = P(abi.cp_config)
    wp = P(orc_world)
    sig = {
        "orc_default_config": (None, [cfgp]),
        "orc_world_spawn": (None, [wp, cfgp]),
        "orc_world_reset_pose": (None, [wp, C.c_int, P(C.c_double), P(C.c_double)]),
        "orc_world_step": (None, [wp, cfgp]),
        "orc_world_apply_force_link": (None, [wp, C.c_int, C.c_double, C.c_double, C.c_double]),
        "orc_world_get_pose": (None, [wp, C.c_int, P(C.c_double)]),
        "orc_world_get_velocity": (None, [wp, C.c_int, P(C.c_double)]),
        "orc_world_get_euler": (None, [wp, C.c_int, P(C.c_double)]),
        "orc_envs_create": (C.c_int, [cfgp, P(VP)]),
        "orc_envs_destroy": (None, [VP]),
        "orc_envs_set_bump_forces": (None, [VP, VP]),
        "orc_envs_set_bump_forces64": (None, [VP, VP]),
        "orc_envs_set_lqr": (None, [VP, VP, C.c_int, VP, C.c_float, C.c_float]),
        "orc_envs_get_state": (None, [VP, VP]),
        "orc_envs_set_state": (None, [VP, VP]),
        "orc_envs_reset": (None, [VP, VP, VP]),
        "orc_envs_step": (None, [VP, VP, C.c_int, VP, VP, VP, VP, VP, C.c_int]),
        "orc_envs_step_omp": (C.c_int, [VP, VP, C.c_int, VP, VP, VP, C.c_int]),
        "orc_envs_episode_returns": (None, [VP, VP, VP]),
        "orc_envs_sweeps": (None, [VP, VP]),
        "orc_envs_merged": (None, [VP, VP]),
        "orc_envs_nonfinite": (None, [VP, VP]),
        "orc_render_frame": (None, [VP, VP, VP, C.c_int, VP]),
        "orc_philox4x32_10": (None, [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]),
        "orc_sincos_turns": (None, [C.c_float, P(C.c_float), P(C.c_float)]),
        "orc_probe_transcendentals": (None, [C.c_double, C.c_double, C.c_double, P(C.c_double)]),
        "orc_sizeof_real": (C.c_int, []),
    }
    for fn, (res, args) in sig.items():
        f = getattr(lib, fn)
        f.restype, f.argtypes = res, args
    _LIBS[name] = lib
    return lib


def native_path():
    """Where the -march=native build for THIS host's CPU lives (keyed by the CPU model and
    flags, so a tree copied to another machine rebuilds instead of running foreign code)."""
    import hashlib
    import platform
    key = platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            lines = [ln for ln in f if ln.startswith(("model name", "flags"))][:2]
        key += "".join(lines)
    except OSError:
        pass
    tag = hashlib.sha1(key.encode()).hexdigest()[:12]
    return os.path.join(BUILD, f"native_{tag}", "libcp_oracle_native.so")


def default_config(**overrides):
    cfg = abi.cp_config()
    load().orc_default_config(C.byref(cfg))
    for k, v in overrides.items():
        if k == "angle_threshold":
            cfg.tan_angle_threshold = math.tan(v)
            cfg.sin_angle_threshold = math.sin(v)
        setattr(cfg, k, v)
    return cfg


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class World:
    """One scene driven exactly like the pybullet module (stepSimulation, ...)."""

    def __init__(self, cfg=None, precision="f32"):
        self.lib = load(precision)
        self.cfg = cfg if cfg is not None else default_config()
        self.w = orc_world()
        self.lib.orc_world_spawn(C.byref(self.w), C.byref(self.cfg))

    def reset_pose(self, body, pos, quat):
        p = (C.c_double * 3)(*pos)
        q = (C.c_double * 4)(*quat)
        self.lib.orc_world_reset_pose(C.byref(self.w), body, p, q)

    def step(self):
        self.lib.orc_world_step(C.byref(self.w), C.byref(self.cfg))

    def apply_force_link(self, body, f):
        self.lib.orc_world_apply_force_link(C.byref(self.w), body, *[float(x) for x in f])

    def pose(self, body):
        o = (C.c_double * 7)()
        self.lib.orc_world_get_pose(C.byref(self.w), body, o)
        return np.array(o[:])

    def velocity(self, body):
        o = (C.c_double * 6)()
        self.lib.orc_world_get_velocity(C.byref(self.w), body, o)
        return np.array(o[:])

    def euler(self, body):
        o = (C.c_double * 3)()
        self.lib.orc_world_get_euler(C.byref(self.w), body, o)
        return np.array(o[:])

    @property
    def last_iterations(self):
        return self.w.last_iterations

    @property
    def last_points(self):
        return self.w.last_points

    @property
    def overflow(self):
        return self.w.overflow


class Envs:
    """Batched env with the HIP library's semantics, on host numpy arrays."""

    def __init__(self, cfg, precision="f32"):
        self.lib = load(precision)
        self.cfg = cfg
        self.B, self.R, self.S = cfg.num_envs, cfg.action_repeats, cfg.steps_per_repeat
        self.h = C.c_void_p()
        rc = self.lib.orc_envs_create(C.byref(cfg), C.byref(self.h))
        if rc == -2:
            raise ValueError("orc_envs_create: non-finite max_coord_velocity, or a non-finite / negative "
                             "sleep_epsilon or sleep_timeout with CP_MODEL_SLEEPING (cp_create's checks)")
        if rc != 0:
            raise MemoryError("orc_envs_create failed")

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_envs_destroy(self.h)
            self.h = None

    def set_bump_forces(self, forces):
        """float64 input: cp_set_bump_forces64 (kept exact by the f64 build); else float32."""
        if np.asarray(forces).dtype == np.float64:
            f = np.ascontiguousarray(forces, dtype=np.float64)
            assert f.shape == (self.B, self.cfg.initial_force_steps, 2, 2)
            self.lib.orc_envs_set_bump_forces64(self.h, _ptr(f))
            return
        f = np.ascontiguousarray(forces, dtype=np.float32)
        assert f.shape == (self.B, self.cfg.initial_force_steps, 2, 2)
        self.lib.orc_envs_set_bump_forces(self.h, _ptr(f))

    def set_lqr(self, gains, per_env=False, state8=False, done_pos=0.0, done_angle=0.0):
        """cp_set_lqr restated (random_action_agent.py:60-135); gains None = off.
        With state8, later steps fill self.state8 (B, R, S, 2, 8)."""
        if gains is None:
            self._gains = self.state8 = None
            self.lib.orc_envs_set_lqr(self.h, None, 0, None, 0.0, 0.0)
            return
        self._gains = np.ascontiguousarray(gains, dtype=np.float32)
        assert self._gains.shape == ((self.B,) if per_env else ()) + (2, 2, 8), self._gains.shape
        self.state8 = np.zeros((self.B, self.R, self.S, 2, 8), np.float32) if state8 else None
        self.lib.orc_envs_set_lqr(self.h, _ptr(self._gains), int(bool(per_env)), _ptr(self.state8),
                                  float(done_pos), float(done_angle))

    @property
    def real(self):
        """numpy dtype of the state (float32, or float64 for the fp64 build)."""
        return np.float64 if self.lib.orc_sizeof_real() == 8 else np.float32

    def get_state(self):
        """State SoA (CP_STATE_FIELDS, B) in the build's real type; integer fields hold
        int32 bits in their first 4 bytes (read them with abi.state_ints)."""
        s = np.empty((abi.CP_STATE_FIELDS, self.B), self.real)
        self.lib.orc_envs_get_state(self.h, _ptr(s))
        return s

    def set_state(self, s):
        s = np.asarray(s)
        if s.dtype != self.real:
            raise ValueError(f"state dtype {s.dtype}, this oracle build keeps {np.dtype(self.real)}")
        s = np.ascontiguousarray(s)
        if s.shape != (abi.CP_STATE_FIELDS, self.B):
            raise ValueError(f"state shape {s.shape}")
        self.lib.orc_envs_set_state(self.h, _ptr(s))

    def reset(self, mask=None, obs=None):
        obs = np.zeros((self.B, self.R, 2, 7), np.float32) if obs is None else obs
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self.lib.orc_envs_reset(self.h, _ptr(m), _ptr(obs))
        return obs

    def step(self, actions, kind=None, terminal=False, readback=False, readback_bug=True, obs=None):
        if kind is None:
            kind = abi.CP_ACTION_DISCRETE if actions.dtype == np.int8 else abi.CP_ACTION_CONTINUOUS
        a = np.ascontiguousarray(actions, dtype=np.int8 if kind == abi.CP_ACTION_DISCRETE else np.float32)
        obs = np.zeros((self.B, self.R, 2, 7), np.float32) if obs is None else obs
        rew = np.zeros(self.B, np.float32)
        done = np.zeros(self.B, np.uint8)
        term = np.zeros_like(obs) if terminal else None
        rb = np.zeros(abi.readback_shape(self.B, self.R, self.S), np.float32) if readback else None
        self.lib.orc_envs_step(self.h, _ptr(a), kind, _ptr(obs), _ptr(rew), _ptr(done), _ptr(term),
                               _ptr(rb), int(readback_bug))
        out = [obs, rew, done]
        if terminal:
            out.append(term)
        if readback:
            out.append(rb)
        return tuple(out)

    def step_omp(self, actions, kind, obs, rew, done, threads=0):
        return self.lib.orc_envs_step_omp(self.h, _ptr(actions), kind, _ptr(obs), _ptr(rew), _ptr(done),
                                          int(threads))

    def episode_returns(self):
        r = np.zeros(self.B, np.float32)
        n = np.zeros(self.B, np.int32)
        self.lib.orc_envs_episode_returns(self.h, _ptr(r), _ptr(n))
        return r, n

    def merged(self):
        """(B,) diagnostic: substeps of the last step whose solve was merged (a cross-island
        contact: pairs 5-8, solved in the order 0 2 1 3 4 9 5 6 7 8)."""
        out = np.zeros(self.B, np.int32)
        self.lib.orc_envs_merged(self.h, _ptr(out))
        return out

    def nonfinite(self):
        """(B,) steps / resets that ended with a non-finite body state (cp_nonfinite_counts)."""
        out = np.zeros(self.B, np.int32)
        self.lib.orc_envs_nonfinite(self.h, _ptr(out))
        return out

    def sweeps(self):
        """(B, 2) diagnostic: max PGS sweeps per island over the last step."""
        out = np.zeros((self.B, 2), np.int32)
        self.lib.orc_envs_sweeps(self.h, _ptr(out))
        return out


def render_frame(raster_cfg, phys, poses, cam, precision="f32"):
    """One frame (H, W, 3) uint8 of camera `cam` for poses (4, 7) = (xyz, quat xyzw) of
    cart, pole, cart2, pole2 (the kernel's ray caster, restated)."""
    lib = load(precision)
    p = np.ascontiguousarray(poses, dtype=np.float32).reshape(4, 7)
    out = np.zeros((raster_cfg.height, raster_cfg.width, 3), np.uint8)
    lib.orc_render_frame(C.byref(raster_cfg), C.byref(phys), _ptr(p), int(cam), _ptr(out))
    return out


def u8_to_f16(u8):
    """The reference's conversion of TinyRenderer bytes (bullet_cartpole.py:289-294):
    float16(uint8), then /= 255 in float16 (numpy: float32 divide, round to half)."""
    a = np.asarray(u8, dtype=np.float16)
    a /= 255
    return a


def philox4x32_10(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    load().orc_philox4x32_10(c, k, o)
    return list(o)
