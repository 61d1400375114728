#!/usr/bin/env python3
"""Generate the control-flow golden fixtures from the reference env.

Run ONLY in the build container (the reference tree is not on the GPU box):

    python tests/golden/make_fixtures.py            # writes tests/golden/*.json

What this does: `bullet_cartpole.py` (reference, /root/reference) imports `gym` and
`pybullet`, neither of which exists here.  We inject two *recording
stubs* into `sys.modules`, import the reference module from its own file, drive
`__init__` / `reset()` / `step()` exactly as an agent would, and write down:

  * the exact pybullet call sequence (name + arguments) of `__init__`, `reset()`
    and `step()` for several (action_repeats, steps_per_repeat) settings;
  * the 60 bump forces of a reset for seeds {0, 1, 1234} x initial_force {55, 200},
    with and without --no-random-theta (they come from the legacy global
    `np.random` stream, bullet_cartpole.py:354-359);
  * the observation layout: the stub's getBasePositionAndOrientation returns a
    pose that encodes (call index, body id), so the fixture shows which readback
    lands in which obs slot (bullet_cartpole.py:298-311);
  * spaces, reward/done sequence to max_episode_len, step-after-done behaviour
    and the fork's action-shape errors.

These pin CONTROL FLOW, not physics (pybullet is absent, parity vs pybullet is
unpinned: DESIGN.md §Oracle).  The output files are data (inputs + expected
outputs); no reference source is copied into the repo.
"""
import argparse
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = os.environ.get("CARTPOLE_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- stubs
class _Discrete:
    def __init__(self, n):
        self.n = n
        self.shape = ()


class _Box:
    def __init__(self, low, high, shape):
        self.low, self.high, self.shape = low, high, tuple(shape)


class _Env:
    pass


def _make_gym():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    spaces.Discrete, spaces.Box = _Discrete, _Box
    gym.Env, gym.spaces = _Env, spaces
    return gym, spaces


class Recorder:
    """Recording stand-in for the pybullet module (only what bullet_cartpole uses)."""

    GUI, DIRECT, LINK_FRAME, WORLD_FRAME = 1, 2, 1, 2

    def __init__(self):
        self.calls = []
        self.n_bodies = 0
        self.pose_calls = 0

    def _rec(self, name, *args, **kw):
        self.calls.append([name, [_plain(a) for a in args],
                           {k: _plain(v) for k, v in kw.items()}])

    # world / scene
    def connect(self, mode):
        self._rec("connect", mode)
        return 0

    def setGravity(self, *a):
        self._rec("setGravity", *a)

    def loadURDF(self, *a):
        self._rec("loadURDF", *a)
        bid = self.n_bodies
        self.n_bodies += 1
        return bid

    def resetDebugVisualizerCamera(self, **kw):
        self._rec("resetDebugVisualizerCamera", **kw)

    # dynamics
    def stepSimulation(self):
        self._rec("stepSimulation")

    def applyExternalForce(self, *a):
        self._rec("applyExternalForce", *a)

    def resetBasePositionAndOrientation(self, *a):
        self._rec("resetBasePositionAndOrientation", *a)

    # readback: encode (call index, body) into exactly representable f32 values
    def getBasePositionAndOrientation(self, body):
        k = self.pose_calls
        self.pose_calls += 1
        self._rec("getBasePositionAndOrientation", body)
        return (float(k), float(body), 7.0), (float(k) + 0.5, float(body) + 0.25, 3.0, 4.0)

    def getEulerFromQuaternion(self, q):
        self._rec("getEulerFromQuaternion", list(q))
        return (0.0, 0.0, 0.0)

    def getBaseVelocity(self, body):
        self._rec("getBaseVelocity", body)
        return (0.0, 0.0, 0.0), (0.0, 0.0, 0.0)


def _plain(a):
    if isinstance(a, (np.floating,)):
        return float(a)
    if isinstance(a, (np.integer,)):
        return int(a)
    if isinstance(a, (tuple, list, np.ndarray)):
        return [_plain(x) for x in a]
    return a


def load_reference(rec):
    gym, spaces = _make_gym()
    sys.modules["gym"], sys.modules["gym.spaces"] = gym, spaces
    sys.modules["pybullet"] = rec
    path = os.path.join(REF, "bullet_cartpole.py")
    spec = importlib.util.spec_from_file_location("ref_bullet_cartpole", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_opts(mod, argv):
    ap = argparse.ArgumentParser()
    mod.add_opts(ap)
    return ap.parse_args(argv)


def fresh(argv, discrete=False):
    rec = Recorder()
    mod = load_reference(rec)
    env = mod.BulletCartpole(make_opts(mod, argv), discrete_actions=discrete)
    return mod, rec, env


# ------------------------------------------------------------------------ fixtures
def fx_init():
    mod, rec, env = fresh([])
    ap = argparse.ArgumentParser()
    mod.add_opts(ap)
    defaults = vars(ap.parse_args([]))
    _, rec_d, env_d = fresh([], discrete=True)
    return {
        "calls": rec.calls,
        "body_ids": {"cart": env.cart, "pole": env.pole, "cart2": env.cart2, "pole2": env.pole2},
        "opts_defaults": defaults,
        "continuous": {"action_space": "Box", "action_shape": list(env.action_space.shape),
                       "obs_shape": list(env.observation_space.shape),
                       "obs_low": float(env.observation_space.low),
                       "obs_high": float(env.observation_space.high),
                       "state_dtype": str(env.state.dtype)},
        "discrete": {"action_space": "Discrete", "n": env_d.action_space.n,
                     "obs_shape": list(env_d.observation_space.shape)},
        "constants": {"initial_force_steps": env.initial_force_steps,
                      "pos_threshold": env.pos_threshold,
                      "angle_threshold": env.angle_threshold},
    }


def fx_reset_bumps():
    out = []
    for seed in (0, 1, 1234):
        for force in (55.0, 200.0):
            for no_theta in (False, True):
                argv = ["--initial-force", str(force)] + (["--no-random-theta"] if no_theta else [])
                _, rec, env = fresh(argv)
                rec.calls.clear()
                np.random.seed(seed)
                obs = env.reset()
                forces = [c[1] for c in rec.calls if c[0] == "applyExternalForce"]
                out.append({"seed": seed, "initial_force": force, "no_random_theta": no_theta,
                            "forces": forces, "n_calls": len(rec.calls),
                            "obs": obs.tolist()})
    return out


def fx_reset_calls():
    _, rec, env = fresh(["--initial-force", "55"])
    rec.calls.clear()
    np.random.seed(0)
    obs = env.reset()
    return {"argv": ["--initial-force", "55"], "seed": 0, "calls": rec.calls,
            "obs": obs.tolist(), "obs_dtype": str(obs.dtype)}


def fx_step_calls():
    out = []
    for R, S in ((2, 1), (3, 1), (3, 4)):
        argv = ["--initial-force", "55", "--action-repeats", str(R), "--steps-per-repeat", str(S)]
        _, rec, env = fresh(argv)
        np.random.seed(0)
        env.reset()
        rec.calls.clear()
        rec.pose_calls = 0
        action = np.array([[0.5, -0.25], [-1.0, 0.75]])
        obs, reward, done, info = env.step(action)
        out.append({"argv": argv, "R": R, "S": S, "action": action.tolist(),
                    "calls": rec.calls, "obs": obs.tolist(), "reward": reward,
                    "done": done, "info": info,
                    "monkey_positions_shape": list(env.monkey_positions.shape)})
    return out


def fx_episode():
    argv = ["--initial-force", "55", "--action-repeats", "3", "--max-episode-len", "200"]
    _, rec, env = fresh(argv)
    np.random.seed(0)
    env.reset()
    rewards, dones, infos = [], [], []
    act = np.zeros((2, 2))
    for _ in range(200):
        _, r, d, i = env.step(act)
        rewards.append(r)
        dones.append(d)
        infos.append(i)
    first_done = dones.index(True) + 1
    rec.calls.clear()
    after = env.step(act)
    calls_after = list(rec.calls)
    return {"argv": argv, "rewards": rewards, "dones": dones,
            "first_done_step": first_done, "info_at_done": infos[first_done - 1],
            "after_done": {"reward": after[1], "done": after[2], "info": after[3],
                           "obs_equals_last": bool(np.array_equal(after[0], env.state)),
                           "n_physics_calls": len(calls_after)}}


def fx_errors():
    res = {}
    _, _, env = fresh([])
    np.random.seed(0)
    env.reset()
    for name, act in (("declared_box_1x2", np.zeros((1, 2))), ("discrete_int", 3),
                      ("pair_2x2", np.zeros((2, 2)))):
        try:
            env.step(act)
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001 - recording the reference's error type
            res[name] = type(e).__name__
    # step before reset
    _, _, env2 = fresh([])
    try:
        env2.step(np.zeros((2, 2)))
        res["step_before_reset"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["step_before_reset"] = type(e).__name__
    try:
        fresh(["--num-cameras", "3"])
        res["num_cameras_3"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["num_cameras_3"] = type(e).__name__
    try:
        fresh(["--reward-calc", "bogus"])
        res["reward_calc_bogus"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["reward_calc_bogus"] = type(e).__name__
    return res


def main():
    fixtures = {
        "init.json": fx_init(),
        "reset_bumps.json": fx_reset_bumps(),
        "reset_calls.json": fx_reset_calls(),
        "step_calls.json": fx_step_calls(),
        "episode.json": fx_episode(),
        "errors.json": fx_errors(),
    }
    for name, data in fixtures.items():
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print("wrote", name, os.path.getsize(os.path.join(OUT, name)), "bytes")


if __name__ == "__main__":
    main()
