"""Batched cartpole++ env on one MI355X: B independent copies of the reference
scene (bullet_cartpole.py:154-160) stepped by the HIP library, with inputs and
outputs as PyTorch-ROCm tensors resident in HBM.

    env = BatchedCartpole(65536, device=0, action_repeats=3, autoreset=True)
    obs = env.reset()                                  # (B, R, 2, 7) float32
    obs, reward, done = env.step(actions)              # actions (B,2,2) f32 or (B,2) int8

One call of `step` is one env-step for every env: R x S physics substeps fused in
one kernel launch (plus one compacted reset launch when autoreset is on).

autoreset: False / "off"; True / "same_step" (a finishing env is reset in its step: obs holds
the new episode's first obs, terminal_obs the finishing obs); "next_step" (gymnasium >= 1.0 /
envpool: the step returns the finishing obs with done; the next step returns the new episode's
first obs with reward 0, done 0 and ignores that env's action; the reset itself runs on a
library stream in between, overlapped with the other envs' steps).
"""
import ctypes as C

import numpy as np
import torch

from . import abi, native

AUTORESET = {False: abi.CP_AUTORESET_OFF, "off": abi.CP_AUTORESET_OFF, True: abi.CP_AUTORESET_SAME_STEP,
             "same_step": abi.CP_AUTORESET_SAME_STEP, "next_step": abi.CP_AUTORESET_NEXT_STEP}


def autoreset_mode(x):
    """cp_config.autoreset for False / True / "off" / "same_step" / "next_step" (or the int itself)."""
    if isinstance(x, int) and not isinstance(x, bool) and x in AUTORESET.values():
        return x
    if x not in AUTORESET:
        raise ValueError(f"autoreset must be one of {sorted(map(str, AUTORESET))}, got {x!r}")
    return AUTORESET[x]


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _device_buffer(x, shape, dtype, device, name):
    """x as a contiguous tensor of exactly `shape` / `dtype` on `device`, or ValueError.
    The C-ABI trusts these sizes (it reads B rows through raw device pointers), so they
    are checked here, explicitly (not with assert, which python -O strips)."""
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(x)
    if t.dtype != dtype:
        if t.is_floating_point() != dtype.is_floating_point and dtype != torch.uint8:
            raise ValueError(f"{name}: dtype {t.dtype} cannot stand for {dtype}")
        t = t.to(dtype)
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if t.device != device:
        t = t.to(device)
    t = t.contiguous()
    if t.numel() != int(torch.Size(shape).numel()):
        raise ValueError(f"{name}: {t.numel()} elements, expected {torch.Size(shape).numel()}")
    return t


class BatchedCartpole:
    def __init__(self, num_envs, device=0, *, action_repeats=2, steps_per_repeat=1, max_episode_len=200,
                 action_force=50.0, initial_force=200.0, random_theta=True, done_on_bounds=False,
                 autoreset=False, seed=0, env_id_offset=0, bump_mode="philox", discrete_actions=False,
                 precision="f32", config=None, **phys):
        self.lib = native.load()
        if config is None:
            config = native.default_config(
                num_envs=int(num_envs), action_repeats=int(action_repeats),
                steps_per_repeat=int(steps_per_repeat), max_episode_len=int(max_episode_len),
                action_force=float(action_force), initial_force=float(initial_force),
                random_theta=int(bool(random_theta)), done_on_bounds=int(bool(done_on_bounds)),
                autoreset=autoreset_mode(autoreset), seed=int(seed), env_id_offset=int(env_id_offset),
                bump_mode=abi.CP_BUMP_HOST if bump_mode == "host" else abi.CP_BUMP_PHILOX)
            if precision not in ("f32", "f64"):
                raise ValueError(f"precision must be 'f32' or 'f64', got {precision!r}")
            config.precision = abi.CP_PRECISION_F64 if precision == "f64" else abi.CP_PRECISION_F32
            for k, v in phys.items():
                if not hasattr(config.phys, k):
                    raise ValueError(f"unknown physics parameter {k!r}")
                setattr(config.phys, k, v)
            if "dt" in phys and "inv_dt" not in phys:  # both are used by the kernels (cp_create checks)
                config.phys.inv_dt = 1.0 / float(phys["dt"])
            if "inertia" in phys and "inv_inertia" not in phys:  # the kernels read both (cp_create checks)
                for b in range(abi.CP_NUM_BODIES):
                    for k in range(3):
                        i_ = float(config.phys.inertia[b][k])
                        config.phys.inv_inertia[b][k] = 1.0 / i_ if i_ > 0 else 0.0
        self.cfg = config
        self.B, self.R, self.S = config.num_envs, config.action_repeats, config.steps_per_repeat
        # the state's real type (cp_config.precision); obs and all other outputs are float32
        self.real = torch.float64 if config.precision == abi.CP_PRECISION_F64 else torch.float32
        self.discrete_actions = bool(discrete_actions)
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type != "cuda":
            raise native.CartpoleError("BatchedCartpole runs on a GPU device (no CPU fallback)")
        self.h = C.c_void_p()
        native.check(None, self.lib.cp_create(C.byref(config), self.device.index or 0, C.byref(self.h)),
                     "cp_create")
        f32 = dict(device=self.device, dtype=torch.float32)
        self.obs = torch.zeros((self.B, self.R, 2, 7), **f32)
        self.reward = torch.zeros(self.B, **f32)
        self.done = torch.zeros(self.B, device=self.device, dtype=torch.uint8)
        self.terminal_obs = torch.zeros_like(self.obs) if config.autoreset else None
        self.readback = None
        self.pixels = None

    # -------------------------------------------------------------- plumbing
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None):
            self.lib.cp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    # ------------------------------------------------------------------- API
    def reset(self, mask=None):
        """Reset envs (all, or where mask != 0); returns the obs tensor (B,R,2,7)."""
        m = None
        if mask is not None:
            m = _device_buffer(torch.as_tensor(mask, device=self.device).reshape(-1).to(torch.uint8), (self.B,),
                               torch.uint8, self.device, "reset mask")
        native.check(self.h, self.lib.cp_reset(self.h, _ptr(m), _ptr(self.obs), self._stream()), "cp_reset")
        return self.obs

    def step(self, actions):
        """One env-step for all envs.  actions: (B,2,2) float32 in [-1,1] (continuous,
        bullet_cartpole.py:201-207) or (B,2) int8 indices into abi.DISCRETE_TABLE."""
        if not isinstance(actions, torch.Tensor):
            actions = torch.as_tensor(actions)
        if actions.dtype == torch.int8:
            kind = abi.CP_ACTION_DISCRETE
            actions = _device_buffer(actions, (self.B, 2), torch.int8, self.device, "discrete actions")
        else:
            kind = abi.CP_ACTION_CONTINUOUS
            if not actions.is_floating_point():
                raise ValueError(f"actions: int8 indices (B, 2) or float (B, 2, 2), got {actions.dtype}")
            actions = _device_buffer(actions, (self.B, 2, 2), torch.float32, self.device, "continuous actions")
        native.check(self.h, self.lib.cp_step(self.h, _ptr(actions), kind, _ptr(self.obs), _ptr(self.reward),
                                              _ptr(self.done), _ptr(self.terminal_obs), self._stream()),
                     "cp_step")
        return self.obs, self.reward, self.done

    def rollout(self, actions, terminal=None):
        """K env-steps in one kernel launch (cp_rollout): actions (K,B,2,2) float32 or (K,B,2)
        int8 -> (obs (K,B,R,2,7), reward (K,B), done (K,B)); bit for bit K step() calls.
        With autoreset, self.rollout_terminal_obs (K,B,R,2,7) holds the finishing obs of the
        episodes that ended (terminal=False skips it).  Afterwards self.obs / reward / done (and
        terminal_obs when collected) hold step K-1's values, as after K step() calls.  The returned
        tensors are views of buffers reused (overwritten) by the next rollout: clone them to keep them."""
        if not isinstance(actions, torch.Tensor):
            actions = torch.as_tensor(actions)
        if actions.dim() < 3:
            raise ValueError(f"actions: (K, B, 2) int8 or (K, B, 2, 2) float, got shape {tuple(actions.shape)}")
        K = int(actions.shape[0])
        if actions.dtype == torch.int8:
            kind = abi.CP_ACTION_DISCRETE
            actions = _device_buffer(actions, (K, self.B, 2), torch.int8, self.device, "discrete actions")
        else:
            kind = abi.CP_ACTION_CONTINUOUS
            if not actions.is_floating_point():
                raise ValueError(f"actions: int8 indices (K, B, 2) or float (K, B, 2, 2), got {actions.dtype}")
            actions = _device_buffer(actions, (K, self.B, 2, 2), torch.float32, self.device, "continuous actions")
        want_term = bool(self.cfg.autoreset if terminal is None else terminal)
        obs, rew, done, self.rollout_terminal_obs = self._roll_buffers(K, want_term)
        native.check(self.h, self.lib.cp_rollout(self.h, K, _ptr(actions), kind, _ptr(obs), _ptr(rew), _ptr(done),
                                                 _ptr(self.rollout_terminal_obs), self._stream()), "cp_rollout")
        # the handle is K steps on: the step()-level attributes follow it (the last step's values)
        self.obs.copy_(obs[-1])
        self.reward.copy_(rew[-1])
        self.done.copy_(done[-1])
        if self.terminal_obs is not None and self.rollout_terminal_obs is not None:
            # step() writes an env's terminal obs when it finishes: keep each env's last one
            d = done.bool()
            fin = d.any(0)
            k_last = (K - 1) - d.flip(0).to(torch.int32).argmax(0)
            last = self.rollout_terminal_obs[k_last.long(), torch.arange(self.B, device=self.device)]
            # a device-side select, no boolean-mask indexing: that calls nonzero and waits on the
            # host for the rollout kernel, which serialised StreamShards' rollouts
            torch.where(fin.view(-1, 1, 1, 1), last, self.terminal_obs, out=self.terminal_obs)
        return obs, rew, done

    def reserve_rollout(self, K, terminal=None):
        """Allocate rollout()'s output buffers for up to K steps now (a first allocation inside a timed
        region costs tens of milliseconds).  Size: K * B * (R * 56 + 5) bytes for obs, reward and done,
        plus K * B * R * 56 for the terminal obs when collected (autoreset on, the default): at C3 size
        (B = 65,536, R = 3) and K = 200 that is 2.27 GB + 2.20 GB = 4.5 GB.  The buffers only grow;
        release_rollout() frees them."""
        self._roll_buffers(int(K), bool(self.cfg.autoreset if terminal is None else terminal))

    def release_rollout(self):
        """Free rollout()'s grow-only output buffers (the next rollout allocates them again).  Tensors
        returned by earlier rollouts keep their storage alive until dropped."""
        self._roll_bufs = None
        self._roll_cap = (0, False)
        self.rollout_terminal_obs = None

    def _roll_buffers(self, K, want_term):
        """Views [:K] of grow-only output buffers (any rollout of at most the largest K so far reuses them)."""
        cap, term = getattr(self, "_roll_cap", (0, False))
        if K > cap or (want_term and not term):
            K_cap = max(K, cap)
            f32 = dict(device=self.device, dtype=torch.float32)
            self._roll_bufs = None   # free the old buffers before allocating the larger ones
            self._roll_bufs = (torch.empty((K_cap, self.B, self.R, 2, 7), **f32),
                               torch.empty((K_cap, self.B), **f32),
                               torch.empty((K_cap, self.B), device=self.device, dtype=torch.uint8),
                               torch.zeros((K_cap, self.B, self.R, 2, 7), **f32) if (want_term or term) else None)
            self._roll_cap = (K_cap, want_term or term)
        obs, rew, done, term_obs = self._roll_bufs
        return obs[:K], rew[:K], done[:K], (term_obs[:K] if want_term else None)

    def set_kernel_shape(self, step="auto", reset="auto"):
        """Override the step / autoreset kernel shapes ("auto", "throughput", "latency", "wide", "wide8"; the reset
        kernel also "wide64" and "list"; cp_set_kernel_shape).  Every shape computes the same numbers."""
        native.check(self.h, self.lib.cp_set_kernel_shape(self.h, abi.SHAPES[step], abi.SHAPES[reset]),
                     "cp_set_kernel_shape")

    def kernel_shape(self):
        """-> (step shape, reset shape) in use, by the names of abi.SHAPES."""
        st, rs = C.c_int(), C.c_int()
        native.check(self.h, self.lib.cp_get_kernel_shape(self.h, C.byref(st), C.byref(rs)), "cp_get_kernel_shape")
        names = {v: k for k, v in abi.SHAPES.items()}
        return names[st.value], names[rs.value]

    def enable_readback(self, on=True, reference_bug=True):
        """Per-substep 12-state pole readback (bullet_cartpole.py:212-234) into
        self.readback (B, 2, R, S, 4, 3) = (xyz, rpy, linvel, angvel)."""
        if on:
            self.readback = torch.zeros(abi.readback_shape(self.B, self.R, self.S), device=self.device,
                                        dtype=torch.float32)
        else:
            self.readback = None
        native.check(self.h, self.lib.cp_set_readback(self.h, _ptr(self.readback), int(bool(reference_bug))),
                     "cp_set_readback")

    def enable_raster(self, on=True, raster_config=None, **kw):
        """Raster obs (--use-raw-pixels, bullet_cartpole.py:277-306) into self.pixels,
        float16 (B, H, W, 3, C, R); rendered by every later step / reset."""
        if not on:
            self.pixels = None
            native.check(self.h, self.lib.cp_set_raster(self.h, None, None), "cp_set_raster")
            return None
        rc = raster_config if raster_config is not None else native.default_raster_config(**kw)
        self.raster_cfg = rc
        self.pixels = torch.zeros(abi.pixels_shape(self.B, rc.height, rc.width, rc.num_cameras, self.R),
                                  device=self.device, dtype=torch.float16)
        native.check(self.h, self.lib.cp_set_raster(self.h, C.byref(rc), _ptr(self.pixels)), "cp_set_raster")
        return self.pixels

    def render_kernel_name(self):
        """The render kernel the library launches for this raster configuration
        (cp_render_kernel_name); None with the raster obs off."""
        n = self.lib.cp_render_kernel_name(self.h)
        return n.decode() if n else None

    def enable_lqr(self, gains, per_env=False, state8=True, done_pos=0.0, done_angle=0.0):
        """Closed-loop LQR policy (random_action_agent.py:60-135; see cp_set_lqr): every
        substep pushes cart p with action_force * action_p + u_p, u_p = -K_p . s_p from pole
        p's 8-state.  gains (2, 2, 8) shared or (B, 2, 2, 8) per env (A/B gain search
        across envs); None turns it off.  state8: fill self.state8 (B, R, S, 2, 8).
        done_pos > 0: end an episode when both pairs leave the agent's bounds
        (random_action_agent.py:108-119, :908; the agent uses 3.0 m and pi/4)."""
        if gains is None:
            self.lqr_gains = self.state8 = None
            native.check(self.h, self.lib.cp_set_lqr(self.h, None, 0, None, 0.0, 0.0), "cp_set_lqr")
            return
        g = _device_buffer(torch.as_tensor(gains, dtype=torch.float32), ((self.B,) if per_env else ()) + (2, 2, 8),
                           torch.float32, self.device, "LQR gains")
        self.lqr_gains = g
        self.state8 = torch.zeros((self.B, self.R, self.S, 2, 8), device=self.device) if state8 else None
        native.check(self.h, self.lib.cp_set_lqr(self.h, _ptr(g), int(bool(per_env)), _ptr(self.state8),
                                                 float(done_pos), float(done_angle)), "cp_set_lqr")

    def set_bump_forces(self, forces):
        """Parity mode (bump_mode='host'): LINK-frame bump forces (B, 30, 2, 2).  float64 input goes
        through cp_set_bump_forces64 (an fp64 handle keeps the reference's doubles, an fp32 handle
        rounds them); anything else is taken as float32."""
        shape = (self.B, self.cfg.initial_force_steps, 2, 2)
        t = forces if isinstance(forces, torch.Tensor) else torch.as_tensor(np.asarray(forces))
        if t.dtype == torch.float64:
            f = _device_buffer(t, shape, torch.float64, self.device, "bump forces")
            native.check(self.h, self.lib.cp_set_bump_forces64(self.h, _ptr(f), self._stream()), "cp_set_bump_forces64")
        else:
            f = _device_buffer(t.to(torch.float32), shape, torch.float32, self.device, "bump forces")
            native.check(self.h, self.lib.cp_set_bump_forces(self.h, _ptr(f), self._stream()), "cp_set_bump_forces")

    def get_state(self):
        s = torch.empty((abi.CP_STATE_FIELDS, self.B), device=self.device, dtype=self.real)
        if s.numel() * s.element_size() != self.lib.cp_state_bytes(self.h):
            raise native.CartpoleError("state buffer size disagrees with cp_state_bytes")
        native.check(self.h, self.lib.cp_get_state(self.h, _ptr(s), self._stream()), "cp_get_state")
        return s

    def set_state(self, s):
        s = torch.as_tensor(s)
        if s.dtype != self.real:
            raise ValueError(f"state: this handle keeps {self.real} state, got {s.dtype}")
        s = _device_buffer(s, (abi.CP_STATE_FIELDS, self.B), self.real, self.device, "state")
        native.check(self.h, self.lib.cp_set_state(self.h, _ptr(s), self._stream()), "cp_set_state")

    def episode_returns(self):
        r = torch.empty(self.B, device=self.device, dtype=torch.float32)
        n = torch.empty(self.B, device=self.device, dtype=torch.int32)
        native.check(self.h, self.lib.cp_episode_returns(self.h, _ptr(r), _ptr(n), self._stream()),
                     "cp_episode_returns")
        return r, n

    def timing_begin(self, max_launches):
        """Record HIP events around every step / reset kernel launch (see cp_timing_begin)."""
        native.check(self.h, self.lib.cp_timing_begin(self.h, int(max_launches)), "cp_timing_begin")

    def timing_stride(self, step_stride=1, reset_stride=1):
        """Sample the events: every step_stride-th step launch, reset_stride-th reset launch."""
        native.check(self.h, self.lib.cp_timing_stride(self.h, int(step_stride), int(reset_stride)),
                     "cp_timing_stride")

    def timing_end(self):
        """-> dict(step_ms, step_launches, reset_ms, reset_launches); synchronises."""
        sm, rm = C.c_double(), C.c_double()
        sn, rn = C.c_int32(), C.c_int32()
        native.check(self.h, self.lib.cp_timing_end(self.h, C.byref(sm), C.byref(sn), C.byref(rm), C.byref(rn)),
                     "cp_timing_end")
        out = dict(step_ms=sm.value, step_launches=sn.value, reset_ms=rm.value, reset_launches=rn.value)
        pm, pn = C.c_double(), C.c_int32()
        native.check(self.h, self.lib.cp_timing_render(self.h, C.byref(pm), C.byref(pn)), "cp_timing_render")
        out.update(render_ms=pm.value, render_launches=pn.value)
        return out

    def overflow_counts(self):
        o = torch.empty(self.B, device=self.device, dtype=torch.int32)
        native.check(self.h, self.lib.cp_overflow_counts(self.h, _ptr(o), self._stream()), "cp_overflow_counts")
        return o

    def nonfinite_counts(self):
        """(B,) int32: env-steps and resets per env that ended with a non-finite body state."""
        o = torch.empty(self.B, device=self.device, dtype=torch.int32)
        native.check(self.h, self.lib.cp_nonfinite_counts(self.h, _ptr(o), self._stream()), "cp_nonfinite_counts")
        return o
