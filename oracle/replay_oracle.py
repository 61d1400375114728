"""CPU restatement of the reference's ReplayMemory (replay_memory.py:11-163) for the
device replay memory's parity tests.  TEST INFRASTRUCTURE ONLY: only tests/ may use it.

Follows replay_memory.py: events in a ring of `buffer_size` rows (state_1_idx, action,
reward, terminal_mask, state_2_idx), states in a float16 buffer of
int(buffer_size * load_factor) rows shared between consecutive events, free state slots
in a FIFO list (`pop(0)` / `append`).  `add_step_batch` is the batched ingestion of the
MI355X memory stated sequentially: for env j = 0 .. B-1 in order, the reference's `_add`
(:76-118) of env j's transition, then, for an env whose episode restarted, a popped slot
for the new episode's first state (what add_episode does at :65-67)."""
import collections

import numpy as np


class ReplayOracle:
    def __init__(self, buffer_size, state_shape, action_dim, load_factor=1.5):
        assert load_factor >= 1.5, "load_factor has to be at least 1.5"     # :13
        self.buffer_size = buffer_size
        self.state_shape = tuple(state_shape)
        self.insert = 0
        self.full = False
        self.state_1_idx = np.zeros(buffer_size, dtype=np.int32)
        self.action = np.zeros((buffer_size, action_dim), dtype=np.float32)
        self.reward = np.zeros((buffer_size, 1), dtype=np.float32)
        self.terminal_mask = np.zeros((buffer_size, 1), dtype=np.float32)
        self.state_2_idx = np.zeros(buffer_size, dtype=np.int32)
        self.state_buffer_size = int(buffer_size * load_factor)             # :30
        self.state = np.zeros([self.state_buffer_size] + list(state_shape), dtype=np.float16)
        self.state_free_slots = list(range(self.state_buffer_size))        # :35
        self.stats = collections.Counter()
        self.cur = None                                                     # per-env s1 slot (batched)

    # ---- replay_memory.py:63-118
    def add_episode(self, initial_state, action_reward_state_sequence):
        assert len(action_reward_state_sequence) > 0
        state_1_idx = self.state_free_slots.pop(0)
        self.state[state_1_idx] = initial_state
        for n, (action, reward, state_2) in enumerate(action_reward_state_sequence):
            terminal = n == len(action_reward_state_sequence) - 1
            state_1_idx = self._add(state_1_idx, action, reward, terminal, state_2)

    def _add(self, s1_idx, a, r, t, s2):
        if self.full:
            self.state_free_slots.append(int(self.state_1_idx[self.insert]))
            if self.terminal_mask[self.insert] == 0:
                self.state_free_slots.append(int(self.state_2_idx[self.insert]))
        self.state_1_idx[self.insert] = s1_idx
        self.action[self.insert] = a
        self.reward[self.insert] = r
        self.terminal_mask[self.insert] = 0.0 if t else 1.0
        s2_idx = self.state_free_slots.pop(0)
        self.state_2_idx[self.insert] = s2_idx
        self.state[s2_idx] = s2
        self.insert += 1
        if self.insert >= self.buffer_size:
            self.insert = 0
            self.full = True
        return s2_idx

    def size(self):
        return self.buffer_size if self.full else self.insert

    def batch_idxs(self, idxs):
        idxs = np.asarray(idxs, dtype=np.int64)
        return (self.state[self.state_1_idx[idxs]], self.action[idxs], self.reward[idxs],
                self.terminal_mask[idxs], self.state[self.state_2_idx[idxs]])

    # ---- batched ingestion (the device memory's semantics, stated sequentially)
    def add_step_batch(self, valid, actions, rewards, done, s2_obs, restarted, new_obs):
        """For env j = 0 .. B-1 in order: if valid[j], env j's transition (s2_obs[j] its next
        state: the terminal one when it restarted); then, if restarted[j], its new episode's
        first state new_obs[j] gets a slot (:65-67).  valid = None: no transitions (episode
        starts only); restarted = None: no restarts."""
        B = len(new_obs)
        if self.cur is None:
            self.cur = np.full(B, -1, np.int64)
        for j in range(B):
            if valid is not None and valid[j]:
                assert self.cur[j] >= 0, "event for an env with no episode"
                s2 = self._add(int(self.cur[j]), actions[j], rewards[j], bool(done[j]), s2_obs[j])
                self.cur[j] = s2
            if restarted is not None and restarted[j]:
                slot = self.state_free_slots.pop(0)
                self.state[slot] = new_obs[j]
                self.cur[j] = slot
