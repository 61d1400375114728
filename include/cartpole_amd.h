/*
 * cartpole_amd.h — C-ABI of the MI355X-native batched cartpole++ environment.
 *
 * Drop-in boundary for the reference's hot path: the `BulletCartpole` gym env
 * (bullet_cartpole.py:48-359) and the pybullet calls it makes per step / reset
 * (stepSimulation, applyExternalForce, getBasePositionAndOrientation,
 * resetBasePositionAndOrientation; call sites listed per entry point below).
 *
 * Conventions
 *   - extern "C", plain pointers and sizes; no torch/HIP types in signatures
 *     (streams are passed as `void*` = hipStream_t, NULL = default stream).
 *   - Every status is an int: 0 = ok, <0 = error; cp_last_error() explains.
 *   - All per-call buffers are CALLER-OWNED DEVICE pointers (e.g. torch-ROCm
 *     data_ptr()).  cp_step/cp_reset allocate nothing and never synchronise the
 *     host, so a caller may capture them into a hipGraph.
 *   - One handle per stream; a handle is not thread-safe, distinct handles are
 *     independent (one process per GPU: each rank creates its own handle).
 *
 * Layouts (B = num_envs, R = action_repeats)
 *   obs           float32 [B][R][2][7]   (cart pose, pole pose; xyz + quat xyzw),
 *                 bullet_cartpole.py:298-311 + :43-45, (R,2,7) per env
 *   actions       kind 0: float32 [B][2][2]  (action[0] -> cart, action[1] -> cart2,
 *                         bullet_cartpole.py:201-207), scaled by action_force
 *                 kind 1: int8    [B][2]     discrete table (see CP_DISCRETE_TABLE)
 *   reward        float32 [B]            (1.0 per step, bullet_cartpole.py:260)
 *   done          uint8   [B]
 *   state (get/set) [CP_STATE_FIELDS][B] SoA of the handle's real type: float32, or
 *                 float64 when cfg.precision == CP_PRECISION_F64 (see CP_SF_* below)
 *   pixels        float16 [B][H][W][3][C][R]  raster obs (--use-raw-pixels,
 *                 bullet_cartpole.py:277-306; cp_set_raster)
 */
#ifndef CARTPOLE_AMD_H
#define CARTPOLE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CP_ABI_VERSION 6

/* Bodies, in the reference's loadURDF order (bullet_cartpole.py:154-160). */
#define CP_BODY_GROUND 0
#define CP_BODY_CART   1
#define CP_BODY_POLE   2
#define CP_BODY_CART2  3
#define CP_BODY_POLE2  4
#define CP_NUM_BODIES  5
#define CP_NUM_DYN     4          /* dynamic bodies: cart, pole, cart2, pole2 */
#define CP_NUM_PAIRS   10         /* all body pairs (a<b) */
/* Islands: {cart, pole} and {cart2, pole2} (the ground is static and joins nothing).
 * Each island owns 5 local pairs: (ground,cart_p) (ground,pole_p) (cart_p,pole_p) and
 * two cross pairs -- island 0: (cart,cart2) (cart,pole2); island 1: (pole,cart2)
 * (pole,pole2).  The kernel runs one island per lane (2 lanes per env). */
#define CP_NUM_ISLANDS  2
#define CP_ISLAND_PAIRS 5

/* Per-body dynamic state: pos(3) quat xyzw(4) linvel(3) angvel(3). */
#define CP_BODY_FIELDS 13
/* SoA state fields for get/set: 4 dynamic bodies x 13, then pending world
 * forces on cart and cart2 (3 each), then integer counters stored as float
 * bit patterns (steps, episode, done). */
#define CP_SF_BODY(dyn, c)  ((dyn) * CP_BODY_FIELDS + (c))
#define CP_SF_PENDING(cart, c) (CP_NUM_DYN * CP_BODY_FIELDS + (cart) * 3 + (c))
#define CP_SF_STEPS   (CP_NUM_DYN * CP_BODY_FIELDS + 6)
#define CP_SF_EPISODE (CP_SF_STEPS + 1)
#define CP_SF_DONE    (CP_SF_STEPS + 2)
/* warm-start cache (persistent contact impulses, DESIGN.md §Physics model): per
 * island and local pair one packed word of 4 feature ids (bytes, 0xFF = empty
 * slot), and the 4 accumulated normal impulses of the last substep */
#define CP_SF_WS_ID(isl, j)      (CP_SF_STEPS + 3 + (isl) * CP_ISLAND_PAIRS + (j))
#define CP_SF_WS_LAM(isl, j, k)  (CP_SF_STEPS + 3 + CP_NUM_PAIRS + ((isl) * CP_ISLAND_PAIRS + (j)) * 4 + (k))
/* CP_MODEL_SLEEPING state per dynamic body (untouched by the other models): the activation word
 * (int bits: CP_ACT_* | CP_ACT_AWAKE) and the sleep timer (seconds) */
#define CP_SF_SLEEP_ACT(dyn)    (CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + (dyn))
#define CP_SF_SLEEP_TIMER(dyn)  (CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + CP_NUM_DYN + (dyn))
#define CP_STATE_FIELDS (CP_SF_STEPS + 3 + CP_NUM_PAIRS * 5 + 2 * CP_NUM_DYN)
/* activation states (btCollisionObject.h: ACTIVE_TAG 1, ISLAND_SLEEPING 2, WANTS_DEACTIVATION 3) and
 * btMultiBody::m_awake as bit 4 */
#define CP_ACT_ACTIVE   1
#define CP_ACT_SLEEPING 2
#define CP_ACT_WANTS    3
#define CP_ACT_AWAKE    16

/* Contact pools per island (LDS-resident in the kernel; same caps in the oracle). */
#define CP_ISLAND_POINTS   10     /* normal-contact rows per island per substep */
#define CP_ISLAND_FRICTION 5      /* contact points that carry 2 friction rows */

/* Discrete action table (the fork dropped upstream's mapping; the comment at
 * bullet_cartpole.py:84,89 names the order "no push, left, right, up, down").
 * Entry k is the unit (fx, fy) pushed on a cart, scaled by action_force. */
#define CP_NUM_DISCRETE 5

/* Physics parameters.  Defaults (cp_default_config) restate the Bullet /
 * pybullet defaults as documented in DESIGN.md §Physics model; every one of
 * them is an [ext] hypothesis (pybullet is not available to pin them). */
typedef struct cp_physics {
    float dt;                 /* fixed step, 1/240 s                           */
    float inv_dt;             /* 1/dt (host-computed so all paths agree)       */
    float gravity[3];         /* (0,0,-9.81), bullet_cartpole.py:152           */
    float lin_damping;        /* k1 = k2 = 0.04 (btMultiBody default)          */
    float ang_damping;        /* k1 = k2 = 0.04                                */
    float erp;                /* contact error reduction, 0.2                  */
    float contact_margin;     /* speculative contact distance, 0.02 m          */
    float residual_threshold; /* PGS early-exit threshold, 1e-7                */
    int32_t solver_iterations;/* PGS iterations, 50                            */
    float edge_bias;          /* SAT: edge axis must beat faces by this, 1e-4 m */
    float max_angular_step;   /* quaternion-integration clamp, pi/4 rad/step   */
    float warmstart;          /* warm-start factor on cached impulses, 0.85    */
    /* per body (ground, cart, pole, cart2, pole2) from the models/ URDF files */
    float half_extents[CP_NUM_BODIES][3];
    float inv_mass[CP_NUM_BODIES];
    float inertia[CP_NUM_BODIES][3];      /* local principal inertia            */
    float inv_inertia[CP_NUM_BODIES][3];
    float friction[CP_NUM_BODIES];        /* lateral friction; pair mu = product */
    float spawn_pos[CP_NUM_BODIES][3];    /* bullet_cartpole.py:154-160,319-323  */
    int32_t model_flags;      /* CP_MODEL_* alternatives to the default model (0) */
    /* btMultiBody::m_maxCoordinateVelocity (100): applyDeltaVeeMultiDof clamps every base
     * velocity coordinate (world angular x,y,z and linear x,y,z) to +-this after the
     * unconstrained update and after the solver's write-back [ext]; <= 0: off */
    float max_coord_velocity;
    /* CP_MODEL_SLEEPING only: btMultiBody::checkMotionAndSleepIfRequired's constants [ext] -- a
     * body whose motion |w|^2 + |v|^2 stays below sleep_epsilon (0.05, a squared velocity) for more
     * than sleep_timeout (2 s) stops being awake; an island of bodies none of which is awake sleeps */
    float sleep_epsilon;
    float sleep_timeout;
} cp_physics;

/* Alternatives to the default contact model (cp_physics.model_flags), for the sensitivity
 * study of the [ext] choices.  cp_create rejects a flag the HIP kernels do
 * not implement (the oracle implements all of them). */
#define CP_MODEL_SPLIT_ISLANDS   0x1  /* the two islands as separate solver groups, one stopping
                                         decision each (instead of one group per env)          */
#define CP_MODEL_VEL_FRICTION    0x2  /* velocity-dependent first friction direction (Bullet's
                                         convertContact default) instead of btPlaneSpace1 only  */
#define CP_MODEL_PERSISTENT      0x4  /* Bullet's persistent manifold (getCacheEntry matching,
                                         replaceContactPoint, sortCachedPoints,
                                         refreshContactPoints) instead of feature-id matching   */
#define CP_MODEL_SLEEPING        0x8  /* Bullet's deactivation (sleeping) of resting bodies, on when pybullet
                                         loads a URDF with URDF_ENABLE_SLEEPING (off by default in pybullet
                                         since that flag exists; bullet_cartpole.py:154-160 passes no flags):
                                         per body a sleep timer and an activation state in the state SoA
                                         (CP_SF_SLEEP_*), islands from the bodies' contact-threshold AABBs,
                                         a sleeping island is neither integrated nor solved */
#define CP_MODEL_GPU_FLAGS       0xC  /* the flags the HIP kernels implement (PERSISTENT, SLEEPING: latency-
                                         shaped kernels only, not together, no LQR policy; the persistent
                                         manifolds are not part of the state SoA) */

typedef struct cp_config {
    int32_t num_envs;            /* B                                          */
    int32_t action_repeats;      /* --action-repeats (ref default 2)           */
    int32_t steps_per_repeat;    /* --steps-per-repeat (1)                     */
    int32_t max_episode_len;     /* --max-episode-len (200)                    */
    float   action_force;        /* --action-force (50)                        */
    float   initial_force;       /* --initial-force (200)                      */
    int32_t random_theta;        /* !--no-random-theta                         */
    int32_t initial_force_steps; /* 30, bullet_cartpole.py:76                  */
    int32_t settle_steps;        /* 100, bullet_cartpole.py:326                */
    int32_t done_on_bounds;      /* restore the commented check :243-253 (0)   */
    float   pos_threshold;       /* 3.0, :58                                   */
    float   angle_threshold;     /* 0.35, :62                                  */
    float   tan_angle_threshold; /* tan(angle_threshold), host-computed        */
    float   sin_angle_threshold; /* sin(angle_threshold), host-computed        */
    int32_t autoreset;           /* CP_AUTORESET_* (0: off)                    */
    int32_t bump_mode;           /* CP_BUMP_PHILOX or CP_BUMP_HOST             */
    uint64_t seed;               /* Philox key                                 */
    int64_t env_id_offset;       /* global id of env 0 (rank * B when sharded) */
    cp_physics phys;
    int32_t precision;           /* CP_PRECISION_F32 (the product path) or _F64  */
    int32_t reset_flags;         /* CP_RESET_* (0: the reference's behaviour)   */
} cp_config;

/* cp_config.reset_flags.  CLEAR_NONFINITE_FORCE: a reset (cp_reset, autoreset, cp_rollout's
 * inline reset) zeroes a cart's pending external force if any component of it is not finite.
 * Off by default: pybullet keeps pending forces across resetBasePositionAndOrientation
 * (bullet_cartpole.py:313-323), so an env whose state went NaN (the explicit
 * gyroscopic term of a spinning loose pole) carries its NaN force into every later episode;
 * with the flag the next reset brings it back.  cp_nonfinite_counts shows such envs either way. */
#define CP_RESET_CLEAR_NONFINITE_FORCE 0x1

/* Arithmetic type of a handle (cp_config.precision).  F32: the fp32 kernels, state float32.
 * F64: the same algorithm in double precision (the parity variant: bit-exact against the
 * oracle's fp64 build, the precision of pybullet's double btScalar), state float64 (the
 * integer fields' int32 bits in the first 4 bytes of their 8-byte field); obs, terminal
 * obs, readback, 8-states and pixels stay float32, as the reference's state array
 * (bullet_cartpole.py:148).  The fp64 kernels run one 512-register wave per SIMD. */
#define CP_PRECISION_F32 0
#define CP_PRECISION_F64 1

/* cp_config.autoreset: who resets an env whose episode ended, and when.
 *   OFF        the caller (cp_reset); cp_step on a done env returns its last obs, reward 0,
 *              done 1 (bullet_cartpole.py:179-181).
 *   SAME_STEP  cp_step resets it in the call where it ends: obs_out holds the new episode's
 *              first obs, terminal_obs_out the finishing obs (gym 0.x vector envs).
 *   NEXT_STEP  cp_step returns the finishing obs in obs_out with done 1; the NEXT cp_step
 *              returns the new episode's first obs for it, reward 0, done 0, and ignores its
 *              action (gymnasium >= 1.0 vector envs, envpool).  The reset runs on a library
 *              stream between the two calls, overlapped with the other envs' steps and the
 *              caller's own work; every entry point that reads the state first
 *              waits for it.  A cp_reset of a pending env returns that reset's obs.  Not for
 *              hipGraph capture, cp_rollout, the raster obs or the event log. */
#define CP_AUTORESET_OFF       0
#define CP_AUTORESET_SAME_STEP 1
#define CP_AUTORESET_NEXT_STEP 2

#define CP_BUMP_PHILOX 0   /* theta = 2*pi*U, U from Philox4x32-10(seed; env, episode, k) */
#define CP_BUMP_HOST   1   /* parity mode: host supplies the 60 bump forces per env      */

#define CP_ACTION_CONTINUOUS 0
#define CP_ACTION_DISCRETE   1

typedef struct cp_handle cp_handle;

/* Fill `cfg` with the reference defaults (bullet_cartpole.py:15-40 + URDFs). */
void cp_default_config(cp_config* cfg);

/* Replaces BulletCartpole.__init__ (bullet_cartpole.py:50-167): p.connect,
 * p.setGravity, 5x p.loadURDF.  Allocates the per-env SoA state on `device`
 * (HBM) and puts every env at its spawn pose with zero pending force. */
int  cp_create(const cp_config* cfg, int device, cp_handle** out);
void cp_destroy(cp_handle* h);
const char* cp_last_error(const cp_handle* h);   /* h may be NULL */
int  cp_abi_version(void);

/* Replaces BulletCartpole.reset (bullet_cartpole.py:313-346): for every env with
 * env_mask[i] != 0 (env_mask NULL = all): 4x resetBasePositionAndOrientation,
 * 100 settle stepSimulation, 30x (stepSimulation + bump cart + bump cart2),
 * then obs[r] = (pose cart, pose pole) for all r.  Pending forces survive the
 * reset, as in pybullet.  obs_out [B][R][2][7] (rows of unmasked envs are left
 * untouched).  env_mask is a device pointer. */
int cp_reset(cp_handle* h, const uint8_t* env_mask, float* obs_out, void* stream);

/* Replaces BulletCartpole.step (bullet_cartpole.py:178-275): R x S substeps,
 * each followed by applyExternalForce on cart/cart2 (LINK_FRAME, at the COM),
 * obs captured at the end of each repeat, steps += 1, done at max_episode_len
 * (and bounds if enabled), reward 1.0.  An env that is already done returns
 * its last obs, reward 0, done 1 and is not simulated (:179-181).  With
 * autoreset, envs that finish are reset in the same call: obs_out then holds
 * the fresh episode's first obs and terminal_obs_out (may be NULL) the
 * finishing obs.  All pointers are device pointers; terminal_obs_out and
 * pole_readback_out may be NULL.  With CP_AUTORESET_SAME_STEP and no early termination
 * (no bounds, no LQR done thresholds) the handle counts the calls since every env's step
 * counter was 0 (cp_create, cp_reset with env_mask NULL, cp_rollout adds its steps) and
 * launches the reset kernel only on calls where episodes end; a masked cp_reset or
 * cp_set_state stops that until the next full reset, and a cp_step / cp_reset / cp_rollout
 * under stream capture stops it for the handle's lifetime (graph replays move the step
 * counters unseen); max_episode_len <= 0 launches it on every call
 * (CP_RESET_EVERY_CALL=1 in the environment at cp_create: a launch on every call). */
int cp_step(cp_handle* h, const void* actions, int action_kind,
            float* obs_out, float* reward_out, uint8_t* done_out,
            float* terminal_obs_out, void* stream);

/* K consecutive env-steps in ONE kernel launch: the outputs and the final state are bit for bit
 * those of K cp_step calls with actions[k] (k = 0..K-1), autoreset included (an episode that
 * ends in step k is reset in step k: obs_out[k] holds the new episode's first obs and
 * terminal_obs_out[k] the finishing obs).  Replaces the agents' per-step loop over
 * BulletCartpole.step (bullet_cartpole.py:178-275; e.g. the reference's random / LQR rollouts,
 * random_action_agent.py:876-906) when the actions are known in advance or come from the
 * in-kernel LQR policy (cp_set_lqr, without the 8-state output).  Each env advances through its
 * own substeps without waiting for the other envs between steps.
 * Layouts: actions [K][B][2][2] f32 or [K][B][2] i8; obs_out and terminal_obs_out (may be NULL)
 * [K][B][R][2][7]; reward_out [K][B]; done_out [K][B] (device pointers).  The per-step side
 * outputs (readback, 8-states, raster) must be disabled.  With cp_timing_begin active the
 * launch is timed as one step-kernel launch. */
int cp_rollout(cp_handle* h, int steps, const void* actions, int action_kind, float* obs_out,
               float* reward_out, uint8_t* done_out, float* terminal_obs_out, void* stream);

/* Optional per-substep 12-state readback of both poles (bullet_cartpole.py:212-234,
 * exposed there as monkey_positions / monkey_velocities):
 * float32 [B][2 poles][R][S][4][3] = (xyz, rpy, linvel, angvel).  Enabled when
 * `readback_out` is non-NULL on the next cp_step; pass NULL to disable.
 * `reference_bug` != 0 reproduces :224 (pole2 rows read pole's velocity). */
int cp_set_readback(cp_handle* h, float* readback_out, int reference_bug);

/* Parity mode (bump_mode == CP_BUMP_HOST): the 2*initial_force_steps bump
 * forces per env in LINK frame, float32 [B][initial_force_steps][2 carts][2],
 * in the reference's draw order (cart then cart2 per bump step, :331-332).
 * Device pointer; copied into the handle (used by every later reset). */
int cp_set_bump_forces(cp_handle* h, const float* forces, void* stream);

/* The same in float64, as the reference draws them (bullet_cartpole.py:354-359: np.random
 * doubles through cos/sin, handed to pybullet's applyExternalForce as doubles).  A
 * CP_PRECISION_F64 handle keeps them exact; an fp32 handle rounds each to the nearest float
 * (what cp_set_bump_forces of the rounded array gives).  cp_set_bump_forces on an fp64 handle
 * widens its floats exactly.  Device pointer, [B][initial_force_steps][2 carts][2]. */
int cp_set_bump_forces64(cp_handle* h, const double* forces, void* stream);

/* Closed-loop LQR policy (random_action_agent.py:60-135, gains :812-829; SURVEY.md
 * §8f row f4).  With gains != NULL every substep applies, per cart p,
 *     force_p = action_force * action_p + u_p,   u_p = -K_p . s_p   (:92-95, :897-901)
 * in the cart's LINK frame, where s_p is pole p's 8-state observed after the
 * previous substep: (x - x0, x', y, y', roll, roll', pitch, pitch') with x0 the pole's
 * spawn x (:121-135).  gains: device float [per_env ? B : 1][2 pairs][2 (fx, fy)][8].
 * state8_out (device, may be NULL): [B][R][S][2 pairs][8], the 8-states after every
 * substep.  done_pos > 0 adds the agent's termination (:108-119, :908): the episode
 * ends when both pairs have |x - x0| or |y| > done_pos or |roll| or |pitch| >
 * done_angle after the same substep.  gains = NULL turns the policy off. */
int cp_set_lqr(cp_handle* h, const float* gains, int per_env, float* state8_out, float done_pos,
               float done_angle);

/* Full env state, SoA [CP_STATE_FIELDS][B] of the handle's real type (float32, or float64
 * for CP_PRECISION_F64 handles), device pointers of cp_state_bytes(h) bytes.
 * CP_MODEL_PERSISTENT handles: the persistent contact manifolds are not part of this state;
 * cp_set_state clears them (a teleport, as resetBasePositionAndOrientation in cp_reset), so a
 * get_state -> set_state round trip mid-episode rebuilds the contacts from the poses. */
int cp_get_state(cp_handle* h, void* state_out, void* stream);
int cp_set_state(cp_handle* h, const void* state_in, void* stream);
int64_t cp_state_bytes(const cp_handle* h);   /* CP_STATE_FIELDS * B * sizeof(real); <0: error */

/* Kernel shapes.  The step and autoreset kernels each come in two register budgets:
 * THROUGHPUT (2 waves per SIMD; bursts and batches above 32,768 envs) and LATENCY (1 wave
 * per SIMD with 512 registers and fast-form solver rows; short reset lists and small
 * batches), and the latency budget in a third layout, WIDE (16 lanes per env instead of 2:
 * the env's 10 contact pairs found side by side, for batches and reset lists that leave
 * most SIMDs idle; fp32 default-model handles).  All compute the same numbers (the GPU
 * parity suite runs every case on every shape).  cp_create picks them (CP_SHAPE_AUTO:
 * DESIGN.md §5); this call overrides either (fp64 handles have only the latency shape and
 * reject THROUGHPUT and WIDE; persistent-manifold and sleeping-model handles likewise). */
#define CP_SHAPE_AUTO       (-1)
#define CP_SHAPE_THROUGHPUT 0
#define CP_SHAPE_LATENCY    1
#define CP_SHAPE_WIDE       2
#define CP_SHAPE_WIDE8      3   /* the WIDE layout on 8 lanes per env (both cross pairs on one lane pair) */
#define CP_SHAPE_WIDE64     4   /* the reset kernel on 64 lanes per env: one env per wave (reset lists;
                                   rejected as a step shape) */
#define CP_SHAPE_LIST       5   /* reset lists whose length only the device knows (bounds / LQR termination):
                                   one launch per layout, each serving one range of the list's length and
                                   exiting at once outside it -- one env per wave up to 1,024 envs, 16 lanes
                                   up to 4,096, the two-lane latency layout up to 32,768, THROUGHPUT above
                                   (rejected as a step shape) */
int cp_set_kernel_shape(cp_handle* h, int step_shape, int reset_shape);
int cp_get_kernel_shape(const cp_handle* h, int* step_shape, int* reset_shape);   /* the shapes in use */

/* Last completed episode per env: return (float32 [B]) and length (int32 [B]);
 * either pointer may be NULL.  Feeds the RCCL return histogram. */
int cp_episode_returns(cp_handle* h, float* returns_out, int32_t* lengths_out, void* stream);

/* Diagnostics: per-env count of contact rows dropped by the CP_ISLAND_* caps since
 * creation (int32 [B], device).  0 everywhere in normal operation. */
int cp_overflow_counts(cp_handle* h, int32_t* out, void* stream);

/* Diagnostics: per-env count (int32 [B], device) of env-steps and resets since creation that
 * ended with a non-finite body state (a NaN or inf in any position, quaternion, linear or
 * angular velocity of cart, pole, cart2, pole2).  0 everywhere in normal operation; an env
 * that went NaN keeps counting up (one per step) until a reset brings it back (see
 * CP_RESET_CLEAR_NONFINITE_FORCE).  The oracle counts the same (oracle/cp_oracle.c). */
int cp_nonfinite_counts(cp_handle* h, int32_t* out, void* stream);

/* Kernel timing with HIP events recorded on the launch stream around every
 * step-kernel and reset-kernel launch of the next `max_launches` cp_step /
 * cp_reset calls (bench.py's roofline).  cp_timing_end synchronises on the last
 * event and returns the summed durations (ms) and launch counts.  Not for use
 * inside hipGraph capture. */
int cp_timing_begin(cp_handle* h, int max_launches);
int cp_timing_end(cp_handle* h, double* step_ms, int32_t* step_launches, double* reset_ms,
                  int32_t* reset_launches);
/* Record events around every `step_stride`-th step-kernel launch and every
 * `reset_stride`-th reset-kernel launch only (default 1, 1; set after cp_timing_begin,
 * which resets them): each recorded event costs the stream a few microseconds, so a
 * sampled average keeps that cost out of the timed throughput.  The launch counts
 * returned by cp_timing_end are the sampled ones. */
int cp_timing_stride(cp_handle* h, int step_stride, int reset_stride);

/* Diagnostics of a stamp build (-DCP_STAMPS): host array of CP_STAMP_SLOTS (64) counters
 * summed over waves since the last reset: slots 0-7 for the step kernel, 16-23 for the reset
 * kernel, each: s_memtime cycles in narrowphase + row setup, velocity update + warm start, PGS
 * sweeps, integration + cache; sweep count, substep count, total kernel cycles, waves;
 * slots 8-10 / 24-26 split the narrowphase (body selection, box_box, row setup); slots
 * 11-15 / 27-31 the longest wave (cycles) and, in 10 ns ticks of s_memrealtime, the latest
 * wave end, the complement of the earliest wave start, the sum and the max of the wave
 * durations; slots 32-47 (step kernel) wave count and summed duration per set of slow paths
 * taken (bit 0 merged solve, bit 1 / 2 ground-cart / ground-pole rows not +z), slots 48-63 a
 * histogram of step-kernel wave durations in 50 us bins (the last open-ended).
 * Synchronises the device.  Returns 1 in a stamp build, 0 otherwise (counters then stay 0). */
#define CP_STAMP_SLOTS 64
int cp_debug_stamps(cp_handle* h, uint64_t* out64, int reset);

/* ---- Raster observation (--use-raw-pixels) ----------
 * Replaces render_rgb + set_state_element_for_repeat (bullet_cartpole.py:277-306):
 * per env, per repeat r and camera c, an RGB image of the scene from the
 * reference's cameras, converted as the reference converts TinyRenderer's
 * uint8 RGBA: float16(uint8) / 255 in float16 (:289-294).  The image is ray cast
 * (DESIGN.md §Raster): flat-shaded boxes with the URDF colours; pixel parity with
 * pybullet's TinyRenderer is unpinned (no pybullet here), the oracle's
 * restatement of this renderer is pinned bit for bit. */
typedef struct cp_raster_config {
    int32_t width, height;     /* --render-width / --render-height (50, 50)          */
    int32_t num_cameras;       /* --num-cameras, 1 or 2 (:111-114)                   */
    float eye[2][3];           /* camera positions, (0,.75,.75) and (.75,0,.75) :279 */
    float target[3];           /* (0, 0, 0.3) :280                                    */
    float up[3];               /* (0, 0, 1) :281                                      */
    float tan_half_fov;        /* tan(fov/2), fov = 30 deg vertical (:283)            */
    float far_plane;           /* 20 (:282); rays stop there (near plane: DESIGN.md)  */
    float light[3];            /* unit direction towards the light                   */
    float ambient, diffuse;    /* shade = ambient + diffuse * max(0, n . light)       */
    float background[3];       /* colour of a ray that hits nothing                  */
    float color[CP_NUM_BODIES][3]; /* visual RGB of ground, cart, pole, cart2, pole2  */
} cp_raster_config;

/* Reference defaults (bullet_cartpole.py:15-40, :277-284, the models/ URDF colours). */
void cp_default_raster_config(cp_raster_config* rc);

/* Enable (pixels_out != NULL) or disable the raster obs.  When enabled, every
 * later cp_step renders the R repeat-end frames of each simulated env into
 * pixels_out float16 [B][H][W][3][C][R] (device), and cp_reset renders the reset
 * envs' first frame into all R slots.  Envs that are done before a step keep
 * their pixels (the last obs, :179-181).  With autoreset, a finishing env's
 * pixels hold the new episode's first frame (its terminal frame is not kept). */
int cp_set_raster(cp_handle* h, const cp_raster_config* rc, uint16_t* pixels_out);

/* Timing of the render kernel launches (one per cp_step / cp_reset with raster on)
 * of the last cp_timing_begin .. cp_timing_end window: summed ms and launch count. */
int cp_timing_render(cp_handle* h, double* render_ms, int32_t* render_launches);

/* The name of the render kernel cp_step / cp_reset launch for the handle's raster configuration
 * (the library's own choice, for profiling: "cp_render_small2_kernel", "cp_render_small_kernel" or
 * "cp_render_kernel"); NULL when the raster obs is off.  The environment variable CP_RENDER_V1=1 at
 * cp_create is a diagnostic that forces the round-3 kernel (A/B measurements only). */
const char* cp_render_kernel_name(cp_handle* h);

/* ---- Event log (--event-log-out) ---------------------
 * Replaces event_log.EventLog (event_log.py:42-99) for B envs: episodes of events
 * in the protobuf wire format of event.proto:1-35, each episode framed by a
 * native int32 length ('=l', event_log.py:53-57), appended to one file.
 *
 * Record = one `event` field of an Episode (tag, length, Event), fixed size per
 * (action kind, R): a step record holds the action (continuous: 4 floats
 * a00 a01 a10 a11; discrete: the 2 indices as floats), R States (cart_pose[7],
 * pole_pose[7]) and the reward; a reset record holds the R States only
 * (event_log.py:95-97, bullet_cartpole.py:342-344). */
int cp_event_record_bytes(int action_kind, int repeats, int with_action);

/* GPU encoder (device pointers).  mode 0, after cp_step: for every env simulated by
 * the last cp_step (not the done-before ones, which the reference does not log,
 * :179-181) a step record from obs (or terminal_obs for an env that finished and
 * was auto-reset) and flags |= 1; an auto-reset env also gets a reset record from
 * obs and flags |= 2.  mode 1, after cp_reset: a reset record and flags = 2 for
 * every env with env_mask != 0 (NULL = all).  step_records [B][step bytes],
 * reset_records [B][reset bytes], flags uint8 [B]; unused pointers may be NULL. */
int cp_encode_events(cp_handle* h, int mode, const void* actions, int action_kind, const float* obs,
                     const float* terminal_obs, const float* reward, const uint8_t* done,
                     const uint8_t* env_mask, uint8_t* step_records, uint8_t* reset_records,
                     uint8_t* flags, void* stream);

/* Host writer (host pointers; no GPU).  cp_eventlog_write, per env i: flags & 1
 * appends step_records[i] to the env's open episode; flags & 2 writes the open
 * episode (if not empty) and starts a new one with reset_records[i].  Close
 * writes every non-empty open episode, then closes the file (the reference
 * drops the last episode; writing it is the one extension). */
typedef struct cp_eventlog cp_eventlog;
int cp_eventlog_open(const char* path, int num_envs, cp_eventlog** out);
int cp_eventlog_write(cp_eventlog* log, const uint8_t* flags, const uint8_t* step_records, int step_bytes,
                      const uint8_t* reset_records, int reset_bytes);
int cp_eventlog_close(cp_eventlog* log);

/* Envs simulated by the last cp_step (uint8 [B], 1 = its transition is real; the
 * done-before envs of a non-autoreset handle are 0).  Device copy on `stream`. */
int cp_get_stepped(cp_handle* h, uint8_t* out, void* stream);

/* ---- Replay memory in HBM ------------------------------
 * Replaces replay_memory.ReplayMemory (replay_memory.py:11-163): a ring of
 * buffer_size events (state_1_idx, action, reward, terminal_mask, state_2_idx) and
 * a float16 state buffer of state_buffer_size = int(buffer_size * load_factor)
 * rows shared by consecutive events, free state slots in a FIFO ring (the
 * reference's state_free_slots list, pop(0) / append).  All storage is caller
 * owned device memory (the struct holds device pointers); the functions below
 * launch kernels on `stream` and never synchronise.
 *
 * Transitions arrive in "rows" (one per env; cur[row] holds the row's current
 * state_1 slot, -1 before its first episode).  cp_replay_add applies, for row
 * j = 0 .. rows-1 in order, exactly the reference's _add (:76-118) for every row
 * with valid[j] (s1 = cur[j], terminal = done[j], s2 = terminal_states[j] when
 * restart[j] and terminal_states != NULL, else next_states[j]) and then, for every
 * row with restart[j], add_episode's slot pop for the new episode's first state
 * next_states[j] (:65-67).  valid = NULL adds no events (episode starts only);
 * restart = NULL restarts none.  rows <= buffer_size.
 * A free-slot underflow (the reference's pop from an empty list), an event for a
 * row with no episode, or a sample index out of range sets a sticky error bit in
 * ctrl[CP_RM_ERROR] (read it back; the memory is unusable after one). */
#define CP_RM_INSERT 0   /* ctrl[]: int64 insert pointer */
#define CP_RM_FULL 1     /* 1 once the ring wrapped */
#define CP_RM_HEAD 2     /* free-slot ring: pops so far */
#define CP_RM_TAIL 3     /* free-slot ring: pushes so far (+ state_buffer_size initial) */
#define CP_RM_ERROR 4    /* bit 0 slot underflow, bit 1 row without episode, bit 2 bad index */
#define CP_RM_ADDS 5     /* events added ('>add' stat) */
#define CP_RM_EVICTED_S2 6 /* 'cache_evicted_s2' stat */
#define CP_RM_CTRL 8

#define CP_STATES_F32 0  /* state inputs float32 (converted round-to-nearest-even) */
#define CP_STATES_F16 1  /* state inputs float16 bits, stored as is */

typedef struct cp_replay {
    int32_t buffer_size;        /* N events */
    int32_t state_buffer_size;  /* S state slots */
    int32_t state_dim;          /* D: float16 elements per state */
    int32_t action_dim;         /* A */
    uint16_t* state;            /* [S][D] float16 */
    int32_t* state_1_idx;       /* [N] */
    float* action;              /* [N][A] */
    float* reward;              /* [N] */
    float* terminal_mask;       /* [N] 0 = terminal */
    int32_t* state_2_idx;       /* [N] */
    int32_t* free_slots;        /* [S] FIFO ring */
    int64_t* ctrl;              /* [CP_RM_CTRL] */
    int32_t* plan;              /* [2 * max rows] scratch */
    int64_t* scan;              /* [2 * ceil(max rows / 1024) + CP_RM_CTRL] scratch */
} cp_replay;

/* Empty memory: free_slots = 0..S-1 in order (:35), ctrl zeroed, cur[0..rows) = -1. */
int cp_replay_init(const cp_replay* rm, int32_t* cur, int rows, void* stream);
int cp_replay_add(const cp_replay* rm, int32_t* cur, int rows, const uint8_t* valid, const void* actions,
                  int action_kind, const float* reward, const uint8_t* done, const uint8_t* restart,
                  const void* next_states, const void* terminal_states, int state_kind, void* stream);

/* Gather n events (batch(), :128-135): idxs (int32 [n], device) or, when NULL, uniform
 * random indexes in [0, size) from Philox4x32-10 (seed, counter) (random_indexes,
 * :120-126).  Outputs (each may be NULL): idx_out [n], state_1 [n][D] float16,
 * action [n][A], reward [n], terminal_mask [n], state_2 [n][D], state_1_idx [n],
 * state_2_idx [n]. */
typedef struct cp_replay_batch {
    int32_t* idx;
    uint16_t* state_1;
    float* action;
    float* reward;
    float* terminal_mask;
    uint16_t* state_2;
    int32_t* state_1_idx;
    int32_t* state_2_idx;
} cp_replay_batch;
int cp_replay_sample(const cp_replay* rm, int n, const int32_t* idxs, uint64_t seed, uint64_t counter,
                     const cp_replay_batch* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CARTPOLE_AMD_H */
