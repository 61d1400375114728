"""Drop-in for the reference's `bullet_cartpole` module, backed by the HIP library.

Same surface as /root/reference/bullet_cartpole.py so the agents
(lrpg/ddpg/naf_cartpole.py) run unchanged:

  add_opts(parser)                        same 13 flags and defaults (:15-40)
  BulletCartpole(opts, discrete_actions)  spaces as :91-94 and :125-141
  .reset() -> np.ndarray (R,2,7) f32      :313-346
  .step(action) -> (obs, reward, done, info)   :178-275
  .render(mode, close), .seed(), .configure()  no-ops (:169-176)
  .monkey_positions / .monkey_velocities  12-state pole readback (:212-234)

The env is one env of the batched kernel (B = 1) on a GPU.  A step is one cp_step launch whose
action, obs and readback buffers are pinned host memory mapped for the GPU (hipHostGetDevicePointer),
then one stream sync: no copy operations around the kernel (step_io "zero_copy"; "graph" replays
the H2D copy, cp_step and D2H copies as a captured hipGraph, "eager" issues them one by one).  Bump forces are
drawn from the global legacy `np.random` stream in the reference's order and with
its formula (:354-359: theta = U * 2 * pi, f = F (cos, sin)), so a given
`np.random.seed` produces the reference's pushes exactly (parity mode,
CP_BUMP_HOST).  Errors follow the reference: step before reset -> AttributeError,
bad --num-cameras -> ValueError, bad --reward-calc -> AssertionError, an int
action -> TypeError, a (1,2) action -> IndexError (the fork indexes action[1]).
"""
import ctypes as C
import sys
import time

import numpy as np
import torch

from . import abi, native
from .batched import BatchedCartpole
from .spaces import Box, Discrete, Env


def add_opts(parser):
    """Register the env's command-line flags (bullet_cartpole.py:15-40)."""
    a = parser.add_argument
    a('--gui', action='store_true')
    a('--delay', type=float, default=0.0)
    a('--action-force', type=float, default=50.0, help="magnitude of action force applied per step")
    a('--initial-force', type=float, default=200.0, help="magnitude of initial push, in random direction")
    a('--no-random-theta', action='store_true')
    a('--action-repeats', type=int, default=2, help="number of action repeats")
    a('--steps-per-repeat', type=int, default=1, help="number of sim steps per repeat")
    a('--num-cameras', type=int, default=1, help="how many camera points to render; 1 or 2")
    a('--event-log-out', type=str, default=None, help="path to record event log.")
    a('--max-episode-len', type=int, default=200, help="maximum episode len for cartpole")
    a('--use-raw-pixels', action='store_true', help="use raw pixels as state instead of cart/pole poses")
    a('--render-width', type=int, default=50, help="if --use-raw-pixels render with this width")
    a('--render-height', type=int, default=50, help="if --use-raw-pixels render with this height")
    a('--reward-calc', type=str, default='fixed',
      help="'fixed': 1 per step. 'angle': 2*max_angle - ox - oy. 'action': 1.5 - |action|. "
           "'angle_action': both angle and action")


def draw_bump_forces(initial_force, random_theta, steps=30):
    """The reset's pushes from the global legacy np.random stream, in the
    reference's order (per bump step: cart then cart2, bullet_cartpole.py:329-332)
    and formula (:354-359).  Returns float64 (steps, 2 carts, 2) LINK-frame (fx, fy)."""
    f = np.zeros((steps, 2, 2), np.float64)
    for k in range(steps):
        for c in range(2):
            theta = (np.random.random() * 2 * np.pi) if random_theta else 0.0
            f[k, c] = initial_force * np.cos(theta), initial_force * np.sin(theta)
    return f


class BulletCartpole(Env):
    """Single-env gym surface over the MI355X kernel (reference: bullet_cartpole.py:48)."""

    def __init__(self, opts, discrete_actions, device=0, precision="f32"):
        # precision (not a reference flag): "f64" steps the fp64 parity variant, fed the reset's float64
        # pushes unrounded (cp_set_bump_forces64, as pybullet receives them, :354-359)
        self.gui = opts.gui
        self.delay = opts.delay if self.gui else 0.0
        self.max_episode_len = opts.max_episode_len
        self.pos_threshold = 3.0        # :58 (check commented out in the fork)
        self.angle_threshold = 0.35     # :62
        self.action_force = opts.action_force
        self.initial_force = opts.initial_force
        self.initial_force_steps = 30   # :76
        self.random_theta = not opts.no_random_theta
        self.discrete_actions = discrete_actions
        self.action_space = Discrete(5) if discrete_actions else Box(-1.0, 1.0, shape=(1, 2))
        if opts.event_log_out:  # :97-100 (protobuf wire format, cartpoleplusplus_amd/event_log.py)
            from . import event_log
            self.event_log = event_log.EventLog(opts.event_log_out, opts.use_raw_pixels)
        else:
            self.event_log = None
        self.repeats = opts.action_repeats
        self.steps_per_repeat = opts.steps_per_repeat
        if opts.num_cameras not in (1, 2):
            raise ValueError("--num-cameras must be 1 or 2")
        self.num_cameras = opts.num_cameras
        self.use_raw_pixels = opts.use_raw_pixels
        self.render_width, self.render_height = opts.render_width, opts.render_height
        if self.use_raw_pixels:
            # (H, W, 3, C, R), :121-126; filled by the in-kernel ray caster (cp_set_raster)
            state_shape = (self.render_height, self.render_width, 3, self.num_cameras, self.repeats)
        else:
            state_shape = (self.repeats, 2, 7)
        fmax = np.finfo(np.float32).max
        self.observation_space = Box(-fmax, fmax, state_shape)
        assert opts.reward_calc in ['fixed', 'angle', 'action', 'angle_action']
        self.reward_calc = opts.reward_calc
        self.state = np.empty(state_shape, dtype=np.float32)
        # p.connect / setGravity / 5 x loadURDF -> one env of the batched kernel
        self._env = BatchedCartpole(
            1, device, action_repeats=self.repeats, steps_per_repeat=self.steps_per_repeat,
            max_episode_len=self.max_episode_len, action_force=self.action_force,
            initial_force=self.initial_force, random_theta=self.random_theta, bump_mode="host",
            precision=precision)
        self._env.enable_readback(True, reference_bug=True)
        if self.use_raw_pixels:
            self._env.enable_raster(True, width=self.render_width, height=self.render_height,
                                    num_cameras=self.num_cameras)
        self._act = torch.zeros((1, 2, 2), dtype=torch.float32, device=self._env.device)
        # pinned host buffers: the zero-copy step's own (mapped) and the graph / eager steps' staging
        self._h_act = torch.zeros((1, 2, 2), dtype=torch.float32).pin_memory()
        self._h_obs = torch.zeros((1, self.repeats, 2, 7), dtype=torch.float32).pin_memory()
        self._h_rb = torch.zeros(abi.readback_shape(1, self.repeats, self.steps_per_repeat),
                                 dtype=torch.float32).pin_memory()
        self._h_rew = torch.zeros(1, dtype=torch.float32).pin_memory()
        self._h_done = torch.zeros(1, dtype=torch.uint8).pin_memory()
        self._graph = None
        # How a step crosses the host boundary: "zero_copy" (the kernel reads the action from and writes
        # its obs and readback to pinned host memory mapped for the GPU: one launch and a stream sync, no
        # copy operations), "graph" (H2D copy, step, D2H copies replayed as a captured hipGraph) or "eager"
        # (the same as separate calls).  Raster obs stay on the device (eager).
        self._zc = None
        if not self.use_raw_pixels:
            try:
                self._zc = tuple(native.mapped_device_pointer(t)
                                 for t in (self._h_act, self._h_obs, self._h_rew, self._h_done, self._h_rb))
            except native.CartpoleError:
                self._zc = None
        self.step_io = "zero_copy" if self._zc else ("eager" if self.use_raw_pixels else "graph")
        self._rb_host = False    # the handle's readback pointer: the pinned buffer (zero_copy) or the device one

    @property
    def use_graph(self):
        return self.step_io == "graph"

    @use_graph.setter
    def use_graph(self, on):
        self.step_io = "graph" if on else "eager"

    def _capture(self, obs):
        # set_state_element_for_repeat (:298-311): pixels (float16 values, float32 state)
        # or the (R, 2, 7) poses
        if self.use_raw_pixels:
            self.state[...] = self._env.pixels[0].float().cpu().numpy()
        else:
            self.state[...] = obs[0].cpu().numpy()

    def configure(self, display=None):
        pass

    def seed(self, seed=None):
        pass

    def render(self, mode, close):
        pass

    def close(self):
        """gym.Env.close (the reference relies on p.disconnect at exit): drop the captured step
        graph, then the library handle and its device buffers."""
        self._graph = None
        self._env.close()

    def _readback_to(self, host):
        if host != self._rb_host:
            ptr = self._zc[4] if host else C.c_void_p(self._env.readback.data_ptr())
            native.check(self._env.h, self._env.lib.cp_set_readback(self._env.h, ptr, 1), "cp_set_readback")
            self._rb_host = host

    def _step_zero_copy(self, a):
        """One env step in one launch: action, obs and readback in pinned host memory (mapped), then a
        stream sync; the same kernel and numbers as the other paths."""
        self._readback_to(True)
        self._h_act.numpy()[...] = a.reshape(1, 2, 2)
        d_act, d_obs, d_rew, d_done, _ = self._zc
        st = torch.cuda.current_stream(self._env.device)
        native.check(self._env.h, self._env.lib.cp_step(self._env.h, d_act, abi.CP_ACTION_CONTINUOUS, d_obs, d_rew,
                                                         d_done, None, C.c_void_p(st.cuda_stream)), "cp_step")
        st.synchronize()

    def _step_eager(self, a):
        self._readback_to(False)
        self._act.copy_(torch.from_numpy(a).view(1, 2, 2))
        obs, _, _ = self._env.step(self._act)
        self._h_obs.copy_(obs)
        self._h_rb.copy_(self._env.readback)

    def _step_graph(self, a):
        """One env step as a replay of the captured graph (H2D action, cp_step, D2H obs and
        readback); the handle has no autoreset and no timing, so the launches are the same on
        every call and capture once."""
        self._readback_to(False)
        self._h_act.numpy()[...] = a.reshape(1, 2, 2)
        if self._graph is None:
            self._graph = torch.cuda.CUDAGraph()
            stream = torch.cuda.Stream(self._env.device)
            stream.wait_stream(torch.cuda.current_stream(self._env.device))
            with torch.cuda.stream(stream):
                with torch.cuda.graph(self._graph, stream=stream):
                    self._act.copy_(self._h_act, non_blocking=True)
                    obs, _, _ = self._env.step(self._act)
                    self._h_obs.copy_(obs, non_blocking=True)
                    self._h_rb.copy_(self._env.readback, non_blocking=True)
            torch.cuda.current_stream(self._env.device).wait_stream(stream)
        self._graph.replay()
        torch.cuda.current_stream(self._env.device).synchronize()

    def reset(self):
        self.steps = 0
        self.done = False
        self._env.set_bump_forces(
            draw_bump_forces(self.initial_force, self.random_theta, self.initial_force_steps)[None])
        obs = self._env.reset()
        self._capture(obs)
        if self.event_log:  # :342-344
            self.event_log.reset()
            self.event_log.add_just_state(self.state)
        return np.copy(self.state)

    def step(self, action):
        if self.done:
            print("calling step after done????", file=sys.stderr)
            return np.copy(self.state), 0, True, {}
        info = {}
        # the fork's indexing (:201, :205): action[0] -> cart, action[1] -> cart2
        if self.discrete_actions and not isinstance(action, (int, np.integer)):
            a = np.asarray([abi.DISCRETE_TABLE[int(action[0])], abi.DISCRETE_TABLE[int(action[1])]],
                           np.float32)
        else:
            fx, fy = action[0]
            fx2, fy2 = action[1]
            a = np.asarray([[fx, fy], [fx2, fy2]], np.float32)
        if self.step_io == "zero_copy":
            self._step_zero_copy(a)
        elif self.step_io == "graph":
            self._step_graph(a)
        else:
            self._step_eager(a)
        if self.delay > 0:
            time.sleep(self.delay * self.repeats * self.steps_per_repeat)
        if self.use_raw_pixels:
            self._capture(None)
        else:
            self.state[...] = self._h_obs.numpy()[0]
        rb = self._h_rb.numpy()[0]     # (2, R, S, 4, 3)
        self.monkey_positions = np.ascontiguousarray(rb[:, :, :, 0:2, :]).astype(np.float64)
        self.monkey_velocities = np.ascontiguousarray(rb[:, :, :, 2:4, :]).astype(np.float64)
        self.steps += 1
        if self.steps >= self.max_episode_len:
            info['done_reason'] = 'episode length'
            self.done = True
        reward = 1.0
        if self.event_log:  # :272-273; a 2-cart action is logged flattened (the fork's assert on
            self.event_log.add(self.state, action, reward)  # action.shape[0] == 1 cannot hold)
        return np.copy(self.state), reward, self.done, info
