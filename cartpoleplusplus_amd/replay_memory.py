"""Replay memory resident in HBM, fed straight from the batched
env's device tensors.  Replaces replay_memory.ReplayMemory (replay_memory.py:11-163)
with the same API (add_episode, size, random_indexes, batch, current_stats,
reset_from_event_log) and the same storage model: a ring of `buffer_size` events
(state_1_idx, action, reward, terminal_mask, state_2_idx) and a float16 state buffer of
int(buffer_size * load_factor) rows shared by consecutive events, recycled through a
FIFO of free slots.  Kernels: include/cartpole_amd.h cp_replay_* (csrc/cp_replay.h).

    env = BatchedCartpole(4096, autoreset=True)
    rm = ReplayMemory(1 << 20, (env.R, 2, 7), 4, num_envs=env.B)
    obs = env.reset();            rm.after_reset(env)
    env.step(a);                  rm.after_step(env, a)      # B events, two launches
    b = rm.sample(256)            # device gather, no host sync

Batched ingestion applies the reference's per-event `_add` (:76-118) to env 0 .. B-1
in order each step (and add_episode's slot pop, :65-67, for every episode that
starts), so the ring, the slot FIFO and every stored value equal what the reference
holds after the same sequence of single adds.
"""
import collections
import ctypes as C

import numpy as np
import torch

from . import abi, native

Batch = collections.namedtuple("Batch", "state_1 action reward terminal_mask state_2")


class ReplayError(RuntimeError):
    pass


def _p(t, offset_bytes=0):
    return None if t is None else C.c_void_p(t.data_ptr() + offset_bytes)


class ReplayMemory:
    def __init__(self, buffer_size, state_shape, action_dim, load_factor=1.5, *, num_envs=0, device=0, seed=0):
        assert load_factor >= 1.5, "load_factor has to be at least 1.5"     # replay_memory.py:13
        self.lib = native.load()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type != "cuda":
            raise native.CartpoleError("ReplayMemory lives in GPU memory (no CPU fallback)")
        self.buffer_size = int(buffer_size)
        self.state_shape = tuple(int(s) for s in state_shape)
        self.action_dim = int(action_dim)
        self.state_buffer_size = int(buffer_size * load_factor)            # :30
        self.num_envs = int(num_envs)
        if self.num_envs > self.buffer_size:
            raise ValueError("num_envs must not exceed buffer_size (one step adds num_envs events)")
        self.state_dim = int(np.prod(self.state_shape))
        N, S, dev = self.buffer_size, self.state_buffer_size, self.device
        i32, f32 = dict(dtype=torch.int32, device=dev), dict(dtype=torch.float32, device=dev)
        self.state = torch.zeros((S,) + self.state_shape, dtype=torch.float16, device=dev)
        self.state_1_idx = torch.zeros(N, **i32)
        self.action = torch.zeros((N, self.action_dim), **f32)
        self.reward = torch.zeros((N, 1), **f32)
        self.terminal_mask = torch.zeros((N, 1), **f32)
        self.state_2_idx = torch.zeros(N, **i32)
        self.free_slot_ring = torch.zeros(S, **i32)
        self.ctrl = torch.zeros(abi.CP_RM_CTRL, dtype=torch.int64, device=dev)
        # cur[j]: env j's current state_1 slot; the extra last row serves add_episode
        self.cur = torch.full((self.num_envs + 1,), -1, **i32)
        self.plan = torch.zeros(2 * (self.num_envs + 1), **i32)
        self.scan = torch.zeros(2 * ((self.num_envs + 1024) // 1024) + abi.CP_RM_CTRL, dtype=torch.int64, device=dev)
        self._stepped = torch.zeros(max(self.num_envs, 1), dtype=torch.uint8, device=dev)
        self.rm = abi.cp_replay(N, S, self.state_dim, self.action_dim, *(
            t.data_ptr() for t in (self.state, self.state_1_idx, self.action, self.reward, self.terminal_mask,
                                   self.state_2_idx, self.free_slot_ring, self.ctrl, self.plan, self.scan)))
        self.seed, self._counter = int(seed), 0
        self.stats = collections.Counter()
        self._check(self.lib.cp_replay_init(C.byref(self.rm), _p(self.cur), self.num_envs + 1, self._stream()),
                    "cp_replay_init")

    # ------------------------------------------------------------ plumbing
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, status, what):
        if status != 0:
            msg = self.lib.cp_last_error(None)
            raise native.CartpoleError(f"{what} failed: {msg.decode() if msg else 'unknown error'}")

    def _ctrl(self):
        return self.ctrl.cpu().tolist()

    def check(self):
        """Raise if a kernel flagged an error (sticky; the memory is unusable after one)."""
        err = self._ctrl()[abi.CP_RM_ERROR]
        if err:
            what = [m for b, m in ((1, "no free state slot (load_factor too small for these episodes)"),
                                   (2, "event for an env with no episode (call after_reset / begin_episodes)"),
                                   (4, "batch index out of range")) if err & b]
            raise ReplayError("; ".join(what))

    def _add(self, rows, cur_off, valid, actions, action_kind, reward, done, restart, next_states,
             terminal_states, state_kind, offs=(0, 0, 0, 0, 0)):
        a_off, r_off, d_off, n_off, t_off = offs
        self._check(self.lib.cp_replay_add(
            C.byref(self.rm), _p(self.cur, 4 * cur_off), rows, _p(valid), _p(actions, a_off), action_kind,
            _p(reward, r_off), _p(done, d_off), _p(restart), _p(next_states, n_off), _p(terminal_states, t_off),
            state_kind, self._stream()), "cp_replay_add")

    def _states(self, x, rows):
        """-> (device tensor (rows, D) contiguous, state kind)."""
        if not torch.is_tensor(x):
            # the reference assigns into a float16 array: numpy's conversion (:67, :106)
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(x).astype(np.float16)))
        x = x.to(self.device)
        if x.dtype not in (torch.float16, torch.float32):
            x = x.float()
        if x.numel() != rows * self.state_dim:
            raise ValueError(f"states: {x.numel()} values for {rows} rows x state_dim {self.state_dim}")
        x = x.reshape(rows, self.state_dim).contiguous()
        return x, (abi.CP_STATES_F16 if x.dtype == torch.float16 else abi.CP_STATES_F32)

    # ------------------------------------------------- reference API (:40-163)
    def reset_from_event_log(self, log_file):
        """Fill from an event log (event_log.py format; :40-61)."""
        from . import event_log
        for episode in event_log.EventLogReader(log_file).entries():
            initial_state, seq = None, []
            for event_id, event in enumerate(episode.event):
                if event_id == 0:
                    assert len(event.action) == 0
                    assert not event.HasField("reward")
                    initial_state = event_log.read_state_from_event(event)
                else:
                    seq.append((event.action, event.reward, event_log.read_state_from_event(event)))
            self.add_episode(initial_state, seq)
            if self._ctrl()[abi.CP_RM_FULL]:
                break

    def add_episode(self, initial_state, action_reward_state_sequence):
        """:63-72: one episode; its last event is terminal."""
        self.stats[">add_episode"] += 1
        seq = list(action_reward_state_sequence)
        assert len(seq) > 0
        L, A, D = len(seq), self.action_dim, self.state_dim
        states = np.stack([np.asarray(initial_state)] + [np.asarray(s) for _, _, s in seq])
        states, kind = self._states(states, L + 1)
        actions = torch.from_numpy(np.stack([np.broadcast_to(np.asarray(a, dtype=np.float32).reshape(-1)
                                                              if np.ndim(a) else np.float32(a), (A,))
                                             for a, _, _ in seq]).astype(np.float32)).to(self.device)
        rewards = torch.tensor([float(r) for _, r, _ in seq], dtype=torch.float32, device=self.device)
        done = torch.zeros(L, dtype=torch.uint8, device=self.device)
        done[-1] = 1
        one = torch.ones(1, dtype=torch.uint8, device=self.device)
        row, es = self.num_envs, states.element_size() * D
        self._add(1, row, None, None, abi.CP_ACTION_CONTINUOUS, None, None, one, states, None, kind)
        for n in range(L):
            self._add(1, row, one, actions, abi.CP_ACTION_CONTINUOUS, rewards, done, None, states, None, kind,
                      offs=(4 * A * n, 4 * n, n, es * (n + 1), 0))

    def size(self):
        c = self._ctrl()
        return self.buffer_size if c[abi.CP_RM_FULL] else c[abi.CP_RM_INSERT]

    def random_indexes(self, n=1):
        """:120-126 (device int32 tensor; [] when empty)."""
        if self.size() == 0:
            return []
        idx = torch.empty(n, dtype=torch.int32, device=self.device)
        self._sample(n, None, abi.cp_replay_batch(idx.data_ptr()))
        return idx

    def batch(self, batch_size=None, idxs=None):
        """:128-135 (a float16 state pair per event); idxs picks events explicitly."""
        self.stats[">batch"] += 1
        if idxs is None and self.size() == 0:
            return self._empty()
        b, _ = self.sample(batch_size or 1, idxs)
        if idxs is not None:
            self.check()
        return b

    def current_stats(self):
        c = self._ctrl()
        s = dict(self.stats)
        s[">add"] = c[abi.CP_RM_ADDS]
        if c[abi.CP_RM_EVICTED_S2]:
            s["cache_evicted_s2"] = c[abi.CP_RM_EVICTED_S2]
        s["free_slots"] = c[abi.CP_RM_TAIL] - c[abi.CP_RM_HEAD]
        return s

    # ---------------------------------------------------- device-side API
    def sample(self, n, idxs=None, with_slots=False):
        """Gather n events (random, or idxs) into fresh device tensors without a host sync.
        -> (Batch, idx) [+ (state_1_idx, state_2_idx) with with_slots]."""
        dev, A = self.device, self.action_dim
        if idxs is not None:
            idxs = torch.as_tensor(idxs, device=dev).to(torch.int32).reshape(-1).contiguous()
            n = idxs.numel()
        idx = torch.empty(n, dtype=torch.int32, device=dev)
        s1 = torch.empty((n,) + self.state_shape, dtype=torch.float16, device=dev)
        s2 = torch.empty_like(s1)
        act = torch.empty((n, A), dtype=torch.float32, device=dev)
        rew = torch.empty((n, 1), dtype=torch.float32, device=dev)
        tm = torch.empty((n, 1), dtype=torch.float32, device=dev)
        slots = (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev)) \
            if with_slots else (None, None)
        out = abi.cp_replay_batch(*(None if t is None else t.data_ptr()
                                    for t in (idx, s1, act, rew, tm, s2) + slots))
        self._sample(n, idxs, out)
        b = Batch(s1, act, rew, tm, s2)
        return (b, idx, slots) if with_slots else (b, idx)

    def _sample(self, n, idxs, out):
        self._counter += 1
        self._check(self.lib.cp_replay_sample(C.byref(self.rm), n, _p(idxs), self.seed, self._counter,
                                              C.byref(out), self._stream()), "cp_replay_sample")

    def _empty(self):
        dev = self.device
        z = torch.zeros((0,) + self.state_shape, dtype=torch.float16, device=dev)
        return Batch(z, torch.zeros((0, self.action_dim), device=dev), torch.zeros((0, 1), device=dev),
                     torch.zeros((0, 1), device=dev), z.clone())

    def begin_episodes(self, states, mask=None):
        """Envs (all, or mask != 0) start an episode at states[j] (B, *state_shape)."""
        B = self.num_envs
        x, kind = self._states(states, B)
        m = torch.ones(B, dtype=torch.uint8, device=self.device) if mask is None else self._rows_u8(mask, B, "mask")
        self._add(B, 0, None, None, abi.CP_ACTION_CONTINUOUS, None, None, m, x, None, kind)

    def add_steps(self, actions, reward, done, next_states, terminal_states=None, valid=None, restart=None):
        """One transition per env (valid: which envs moved, default all); restart: envs whose
        episode restarted at next_states (then terminal_states holds their s2)."""
        B, dev = self.num_envs, self.device
        kind = abi.CP_ACTION_DISCRETE if actions.dtype == torch.int8 else abi.CP_ACTION_CONTINUOUS
        actions = actions.to(dev)
        if kind == abi.CP_ACTION_CONTINUOUS:
            actions = actions.float()
        if actions.numel() != B * self.action_dim:
            raise ValueError(f"actions: {actions.numel()} values for {B} rows x action_dim {self.action_dim}")
        actions = actions.reshape(B, self.action_dim).contiguous()
        x, skind = self._states(next_states, B)
        t = None
        if terminal_states is not None:
            t, tkind = self._states(terminal_states, B)
            if tkind != skind:
                raise ValueError("terminal_states and next_states must have the same dtype")
        u8 = lambda v, name: None if v is None else self._rows_u8(v, B, name)  # noqa: E731
        valid = torch.ones(B, dtype=torch.uint8, device=dev) if valid is None else u8(valid, "valid")
        reward = torch.as_tensor(reward, device=dev).float().reshape(-1).contiguous()
        if reward.numel() != B:
            raise ValueError(f"reward: {reward.numel()} values for {B} rows")
        self._add(B, 0, valid, actions, kind, reward, u8(done, "done"), u8(restart, "restart"), x, t, skind)

    def _rows_u8(self, v, rows, name):
        """(rows,) uint8 device mask; the C-ABI reads `rows` bytes through the pointer."""
        t = torch.as_tensor(v, device=self.device).to(torch.uint8).reshape(-1).contiguous()
        if t.numel() != rows:
            raise ValueError(f"{name}: {t.numel()} values for {rows} rows")
        return t

    # ----------------------------------------------- BatchedCartpole feed
    def _env_states(self, env):
        if self.state_shape == tuple(env.obs.shape[1:]):
            return env.obs, env.terminal_obs
        if env.pixels is not None and self.state_shape == tuple(env.pixels.shape[1:]):
            if env.cfg.autoreset:
                raise ValueError("pixel states with autoreset: the terminal frame is not rendered")
            return env.pixels, None
        raise ValueError(f"state_shape {self.state_shape} matches neither env.obs nor env.pixels")

    def after_reset(self, env, mask=None):
        """After env.reset(mask): those envs start new episodes."""
        if env.B != self.num_envs:
            raise ValueError(f"env has {env.B} envs, the replay memory {self.num_envs} rows")
        self.begin_episodes(self._env_states(env)[0], mask)

    def after_step(self, env, actions):
        """After env.step(actions): one event per simulated env (the done-before envs of a
        non-autoreset env are skipped); autoreset envs also start their next episode."""
        if env.B != self.num_envs:
            raise ValueError(f"env has {env.B} envs, the replay memory {self.num_envs} rows")
        native.check(env.h, self.lib.cp_get_stepped(env.h, _p(self._stepped), env._stream()), "cp_get_stepped")
        nxt, term = self._env_states(env)
        restart = env.done if env.cfg.autoreset else None
        self.add_steps(actions, env.reward, env.done, nxt, term, valid=self._stepped, restart=restart)

    # ----------------------------------------------------------- inspection
    def free_slots(self):
        """The free-slot FIFO in order (the reference's state_free_slots)."""
        c = self._ctrl()
        ring = self.free_slot_ring.cpu().tolist()
        S = self.state_buffer_size
        return [ring[i % S] for i in range(c[abi.CP_RM_HEAD], c[abi.CP_RM_TAIL])]

    @property
    def insert(self):
        return self._ctrl()[abi.CP_RM_INSERT]

    @property
    def full(self):
        return bool(self._ctrl()[abi.CP_RM_FULL])
