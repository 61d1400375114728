"""LQR controller of the reference's A/B experiment (random_action_agent.py:60-135,
:812-829), for the batched env's in-kernel closed-loop policy (BatchedCartpole.enable_lqr).

The 8-state per cart-pole pair is (x - x0, x', y, y', roll, roll', pitch, pitch') of
the pole; a controller is a (2, 8) gain matrix K whose rows give (fx, fy) = -K . s.
"""
import numpy as np

STATE_NAMES = ("x", "x_dot", "y", "y_dot", "roll", "roll_dot", "pitch", "pitch_dot")

# random_action_agent.py:812-829 ("ground truth" gains, keyboard command '6')
EXACT_GAINS_X = (-2.82843, -9.15175, 0.0, 0.0, -16.0987, -15.3304, 0.0, 0.0)
EXACT_GAINS_Y = (0.0, 0.0, -2.82843, -9.15175, 0.0, 0.0, -16.0987, -15.3304)

# game_factory thresholds (random_action_agent.py:694-695)
POSITION_THRESHOLD = 3.0
ANGLE_THRESHOLD = np.pi / 4


def exact_gains():
    """(2 pairs, 2, 8) float32: both pairs on the exact gains (:921-923)."""
    k = np.array([EXACT_GAINS_X, EXACT_GAINS_Y], dtype=np.float32)
    return np.stack([k, k])


def lqr_control_forces(controller, pole_state, lqr_zero_point=None):
    """random_action_agent.py:92-95 for one pair (host helper, float64 like the reference)."""
    residual = np.asarray(pole_state, dtype=np.float64)
    if lqr_zero_point is not None:
        residual = residual - np.asarray(lqr_zero_point, dtype=np.float64)
    return -np.dot(np.asarray(controller, dtype=np.float64), residual)
