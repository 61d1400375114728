"""Replay a recorded pybullet call sequence (tests/golden/*.json) on the oracle's
world-level API, i.e. drive the CPU restatement exactly the way the reference
bullet_cartpole.py drives pybullet.  Used to pin the env-level control flow."""
import numpy as np

LINK_FRAME = 1  # value the recording stub gave p.LINK_FRAME


def replay(world, calls):
    """Execute `calls`; returns the list of poses returned by each
    getBasePositionAndOrientation call, in call order."""
    poses = []
    for name, args, _kw in calls:
        if name == "stepSimulation":
            world.step()
        elif name == "applyExternalForce":
            body, link, force, pos, flags = args
            assert link == -1 and list(pos) == [0, 0, 0] and flags == LINK_FRAME
            world.apply_force_link(body, force)
        elif name == "resetBasePositionAndOrientation":
            body, pos, quat = args
            world.reset_pose(body, pos, quat)
        elif name == "getBasePositionAndOrientation":
            poses.append(world.pose(args[0]))
        elif name in ("getEulerFromQuaternion", "getBaseVelocity"):
            pass  # side readback only (monkey_positions), not part of obs
        else:
            raise AssertionError(f"unexpected call {name}")
    return poses


def obs_from_fixture(fixture_obs, poses):
    """Map the stub-encoded obs (slot value 0 = call index) onto real poses."""
    enc = np.asarray(fixture_obs)
    out = np.zeros(enc.shape, np.float32)
    for idx in np.ndindex(enc.shape[:-1]):
        k = int(enc[idx][0])
        body = int(enc[idx][1])
        out[idx] = poses[k].astype(np.float32)
        assert enc[idx][2] == 7.0 and body in (1, 2)
    return out


def fixture_bumps(forces, steps=30):
    """Fixture applyExternalForce arg lists -> (1, steps, 2, 2) float32 (cart, cart2)."""
    f = np.zeros((1, steps, 2, 2), np.float64)
    for j, args in enumerate(forces):
        body, _, force, _, _ = args
        k, c = divmod(j, 2)
        assert body == (1 if c == 0 else 3)
        f[0, k, c] = force[0], force[1]
    return f.astype(np.float32)
