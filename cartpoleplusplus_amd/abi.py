"""ctypes mirror of include/cartpole_amd.h (structs, constants, layouts).

Pure data definitions: no library is loaded here.  `native.py` binds the HIP
library's entry points with these types.
"""
import ctypes as C

CP_ABI_VERSION = 6

CP_BODY_GROUND, CP_BODY_CART, CP_BODY_POLE, CP_BODY_CART2, CP_BODY_POLE2 = range(5)
CP_NUM_BODIES = 5
CP_NUM_DYN = 4
CP_NUM_PAIRS = 10
CP_NUM_ISLANDS = 2
CP_ISLAND_PAIRS = 5
CP_BODY_FIELDS = 13
CP_ISLAND_POINTS = 10
CP_ISLAND_FRICTION = 5
# global pair index of island p's local pair j (own 3, then its 2 cross pairs)
ISLAND_PAIR = ((0, 1, 4, 5, 6), (2, 3, 9, 7, 8))
CP_NUM_DISCRETE = 5


def CP_SF_BODY(dyn, c):
    return dyn * CP_BODY_FIELDS + c


def CP_SF_PENDING(cart, c):
    return CP_NUM_DYN * CP_BODY_FIELDS + cart * 3 + c


CP_SF_STEPS = CP_NUM_DYN * CP_BODY_FIELDS + 6
CP_SF_EPISODE = CP_SF_STEPS + 1
CP_SF_DONE = CP_SF_STEPS + 2


def CP_SF_WS_ID(isl, j):
    return CP_SF_STEPS + 3 + isl * CP_ISLAND_PAIRS + j


def CP_SF_WS_LAM(isl, j, k):
    return CP_SF_STEPS + 3 + CP_NUM_PAIRS + (isl * CP_ISLAND_PAIRS + j) * 4 + k


def CP_SF_SLEEP_ACT(dyn):
    return CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + dyn


def CP_SF_SLEEP_TIMER(dyn):
    return CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + CP_NUM_DYN + dyn


CP_STATE_FIELDS = CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + 2 * CP_NUM_DYN
CP_ACT_ACTIVE, CP_ACT_SLEEPING, CP_ACT_WANTS, CP_ACT_AWAKE = 1, 2, 3, 16

CP_AUTORESET_OFF, CP_AUTORESET_SAME_STEP, CP_AUTORESET_NEXT_STEP = 0, 1, 2

CP_BUMP_PHILOX = 0
CP_BUMP_HOST = 1
CP_ACTION_CONTINUOUS = 0
CP_ACTION_DISCRETE = 1

# Discrete action table: order "no push, left, right, up, down"
# (bullet_cartpole.py:84,89); entry = unit (fx, fy) scaled by action_force.
DISCRETE_TABLE = ((0.0, 0.0), (-1.0, 0.0), (1.0, 0.0), (0.0, 1.0), (0.0, -1.0))

_F3 = C.c_float * 3


class cp_physics(C.Structure):
    _fields_ = [
        ("dt", C.c_float),
        ("inv_dt", C.c_float),
        ("gravity", _F3),
        ("lin_damping", C.c_float),
        ("ang_damping", C.c_float),
        ("erp", C.c_float),
        ("contact_margin", C.c_float),
        ("residual_threshold", C.c_float),
        ("solver_iterations", C.c_int32),
        ("edge_bias", C.c_float),
        ("max_angular_step", C.c_float),
        ("warmstart", C.c_float),
        ("half_extents", _F3 * CP_NUM_BODIES),
        ("inv_mass", C.c_float * CP_NUM_BODIES),
        ("inertia", _F3 * CP_NUM_BODIES),
        ("inv_inertia", _F3 * CP_NUM_BODIES),
        ("friction", C.c_float * CP_NUM_BODIES),
        ("spawn_pos", _F3 * CP_NUM_BODIES),
        ("model_flags", C.c_int32),
        ("max_coord_velocity", C.c_float),
        ("sleep_epsilon", C.c_float),
        ("sleep_timeout", C.c_float),
    ]


# cp_physics.model_flags: alternatives to the default contact model (oracle-only unless in
# CP_MODEL_GPU_FLAGS; DESIGN.md §3 sensitivity study)
CP_MODEL_SPLIT_ISLANDS = 0x1
CP_MODEL_VEL_FRICTION = 0x2
CP_MODEL_PERSISTENT = 0x4
CP_MODEL_SLEEPING = 0x8
CP_MODEL_GPU_FLAGS = 0xC

# kernel shapes (cp_set_kernel_shape)
CP_SHAPE_AUTO = -1
CP_SHAPE_THROUGHPUT = 0
CP_SHAPE_LATENCY = 1
CP_SHAPE_WIDE = 2
CP_SHAPE_WIDE8 = 3
CP_SHAPE_WIDE64 = 4
CP_SHAPE_LIST = 5   # reset lists: the layout picked on the device by the list's length (include/cartpole_amd.h)
SHAPES = {"auto": CP_SHAPE_AUTO, "throughput": CP_SHAPE_THROUGHPUT, "latency": CP_SHAPE_LATENCY, "wide": CP_SHAPE_WIDE,
          "wide8": CP_SHAPE_WIDE8, "wide64": CP_SHAPE_WIDE64, "list": CP_SHAPE_LIST}


class cp_config(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32),
        ("action_repeats", C.c_int32),
        ("steps_per_repeat", C.c_int32),
        ("max_episode_len", C.c_int32),
        ("action_force", C.c_float),
        ("initial_force", C.c_float),
        ("random_theta", C.c_int32),
        ("initial_force_steps", C.c_int32),
        ("settle_steps", C.c_int32),
        ("done_on_bounds", C.c_int32),
        ("pos_threshold", C.c_float),
        ("angle_threshold", C.c_float),
        ("tan_angle_threshold", C.c_float),
        ("sin_angle_threshold", C.c_float),
        ("autoreset", C.c_int32),
        ("bump_mode", C.c_int32),
        ("seed", C.c_uint64),
        ("env_id_offset", C.c_int64),
        ("phys", cp_physics),
        ("precision", C.c_int32),
        ("reset_flags", C.c_int32),
    ]


CP_RESET_CLEAR_NONFINITE_FORCE = 0x1


CP_PRECISION_F32 = 0
CP_PRECISION_F64 = 1


class cp_raster_config(C.Structure):
    """include/cartpole_amd.h: cp_raster_config (raster obs, bullet_cartpole.py:277-306)."""
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("num_cameras", C.c_int32),
        ("eye", _F3 * 2),
        ("target", _F3),
        ("up", _F3),
        ("tan_half_fov", C.c_float),
        ("far_plane", C.c_float),
        ("light", _F3),
        ("ambient", C.c_float),
        ("diffuse", C.c_float),
        ("background", _F3),
        ("color", _F3 * CP_NUM_BODIES),
    ]


def pixels_shape(B, H, W, C_, R):
    """Raster obs per env (H, W, 3, C, R), bullet_cartpole.py:299-306 (camera before repeat)."""
    return (B, H, W, 3, C_, R)


def obs_shape(B, R):
    return (B, R, 2, 7)


def readback_shape(B, R, S):
    return (B, 2, R, S, 4, 3)


# ---- replay memory (include/cartpole_amd.h: cp_replay)
CP_RM_INSERT, CP_RM_FULL, CP_RM_HEAD, CP_RM_TAIL, CP_RM_ERROR, CP_RM_ADDS, CP_RM_EVICTED_S2 = range(7)
CP_RM_CTRL = 8
CP_STATES_F32 = 0
CP_STATES_F16 = 1


class cp_replay(C.Structure):
    _fields_ = [
        ("buffer_size", C.c_int32),
        ("state_buffer_size", C.c_int32),
        ("state_dim", C.c_int32),
        ("action_dim", C.c_int32),
        ("state", C.c_void_p),
        ("state_1_idx", C.c_void_p),
        ("action", C.c_void_p),
        ("reward", C.c_void_p),
        ("terminal_mask", C.c_void_p),
        ("state_2_idx", C.c_void_p),
        ("free_slots", C.c_void_p),
        ("ctrl", C.c_void_p),
        ("plan", C.c_void_p),
        ("scan", C.c_void_p),
    ]


class cp_replay_batch(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("idx", "state_1", "action", "reward", "terminal_mask", "state_2",
                                          "state_1_idx", "state_2_idx")]


def state_ints(values):
    """Integer state fields (steps, episode, done, warm-start ids) from a state array:
    float32 holds the int32 bits; a float64 state (fp64 build) holds them in the first 4
    bytes (the low word on this little-endian ABI) of each 8-byte field."""
    import numpy as np
    a = np.ascontiguousarray(values)
    if a.dtype == np.float64:
        return a.view(np.int32)[..., 0::2]
    return a.view(np.int32)
