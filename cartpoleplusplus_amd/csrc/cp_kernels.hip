// cp_kernels.hip — batched cartpole++ env on MI355X (gfx950): the fp32 kernels + C-ABI.
//
// Replaces bullet_cartpole.py's hot path (BulletCartpole.step/reset and the
// pybullet calls behind them) for B independent envs, two lanes per env (lane
// 2e+p owns contact island p; cp_physics.h), or 16 / 8 for the latency-shaped kernels of small
// batches and reset lists (the WIDE layout: replicas of the lane pair that split the narrowphase).  The env kernels (cp_env.h) are written
// over `real` and instantiated here for fp32 (namespace cp, the product path) and in
// cp_kernels64.hip for fp64 (namespace cp64, the parity variant, cp_config.precision).
// This file also holds the fp32-only kernels (reset-mask compaction, raster obs, event
// log records, replay memory) and every C-ABI entry point (include/cartpole_amd.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/cartpole_amd.h"
#include "cp_common.h"

#define CP_NS cp
#define CP_REAL float
#include "cp_math.h"
#include "cp_physics.h"
#include "cp_env.h"
#undef CP_NS
#undef CP_REAL

#include "cp_raster.h"
#include "cp_replay.h"

namespace cp {

// env_mask -> compacted list (wave ballot + one atomic per wave)
__global__ void __launch_bounds__(256) cp_mask_to_list_kernel(int B, const uint8_t* mask, int32_t* list,
                                                               int32_t* count) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool want = i < B && (mask == nullptr || mask[i] != 0);
    uint64_t bal = __ballot(want);
    int lane = threadIdx.x & (WAVE - 1);
    int n = __popcll(bal);
    int base = 0;
    if (lane == 0 && n) base = atomicAdd(count, n);
    base = __shfl(base, 0);
    if (want) list[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
}

// ---------------------------------------------------------------------------
// Event log records (protobuf wire format of event.proto; see cp_encode_events).
CP_DEV void put_u8(uint8_t*& p, uint32_t v) { *p++ = (uint8_t)v; }
CP_DEV void put_varint(uint8_t*& p, uint32_t v) {
    while (v >= 0x80u) { put_u8(p, (v & 0x7Fu) | 0x80u); v >>= 7; }
    put_u8(p, v);
}
CP_DEV void put_f32(uint8_t*& p, uint32_t key, float x) {  // fixed32 field, little endian
    put_u8(p, key);
    const uint32_t u = __float_as_uint(x);
    put_u8(p, u); put_u8(p, u >> 8); put_u8(p, u >> 16); put_u8(p, u >> 24);
}
__host__ __device__ inline int varint_len(uint32_t v) { int n = 1; while (v >= 0x80u) { v >>= 7; ++n; } return n; }
__host__ __device__ inline int event_len(int kind, int R, int with_action) {
    // State: 7 cart_pose + 7 pole_pose fixed32 fields = 70 B, wrapped (tag, len 70) = 72 B
    return (with_action ? (kind == CP_ACTION_CONTINUOUS ? 4 : 2) * 5 + 5 : 0) + R * 72;
}
__host__ __device__ inline int record_len(int kind, int R, int with_action) {
    const int n = event_len(kind, R, with_action);
    return 1 + varint_len((uint32_t)n) + n;
}
// one Episode.event entry: tag 1 (length-delimited), Event { action*, state*, reward }
CP_DEV void put_record(uint8_t* p, int kind, int R, bool with_action, const void* actions, int i, const float* obs,
                       float reward) {
    put_u8(p, 0x0A);
    put_varint(p, (uint32_t)event_len(kind, R, with_action ? 1 : 0));
    if (with_action) {
        if (kind == CP_ACTION_CONTINUOUS) {
            const float* a = reinterpret_cast<const float*>(actions) + (size_t)i * 4;
            for (int k = 0; k < 4; ++k) put_f32(p, 0x0D, a[k]);
        } else {
            const int8_t* a = reinterpret_cast<const int8_t*>(actions) + (size_t)i * 2;
            put_f32(p, 0x0D, (float)a[0]);
            put_f32(p, 0x0D, (float)a[1]);
        }
    }
    for (int r = 0; r < R; ++r) {
        put_u8(p, 0x12);
        put_u8(p, 70);
        const float* o = obs + ((size_t)i * R + r) * 14;
        for (int k = 0; k < 7; ++k) put_f32(p, 0x0D, o[k]);       // cart_pose = 1
        for (int k = 0; k < 7; ++k) put_f32(p, 0x15, o[7 + k]);   // pole_pose = 2
    }
    if (with_action) put_f32(p, 0x1D, reward);                    // reward = 3
}

__global__ void __launch_bounds__(256) cp_event_kernel(int B, int R, int mode, int kind, int autoreset,
                                                        const void* actions, const float* obs, const float* term,
                                                        const float* reward, const uint8_t* done,
                                                        const uint8_t* mask, const uint8_t* stepped,
                                                        uint8_t* step_rec, uint8_t* reset_rec, uint8_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const int sb = record_len(kind, R, 1), rb = record_len(kind, R, 0);
    uint8_t fl = 0;
    if (mode == 0) {
        if (stepped[i]) {
            fl = 1;
            const bool fresh = autoreset && done[i];   // finished and auto-reset in that cp_step
            put_record(step_rec + (size_t)i * sb, kind, R, true, actions, i, fresh && term ? term : obs,
                       reward[i]);
            if (fresh && reset_rec) {
                fl |= 2;
                put_record(reset_rec + (size_t)i * rb, kind, R, false, nullptr, i, obs, 0.0f);
            }
        }
    } else if (!mask || mask[i]) {
        fl = 2;
        put_record(reset_rec + (size_t)i * rb, kind, R, false, nullptr, i, obs, 0.0f);
    }
    flags[i] = fl;
}

__global__ void __launch_bounds__(256) cp_copy_kernel(const float* src, float* dst, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

// host bump forces into the handle's real type: widening is exact, narrowing rounds to nearest (as
// numpy's astype(float32) does)
template <typename S, typename D>
__global__ void __launch_bounds__(256) cp_convert_kernel(const S* src, D* dst, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (D)src[i];
}

}  // namespace cp

// ============================================================================ C-ABI
struct cp_timing {
    int cap = 0;                             // event pairs per kind
    int nstep = 0, nreset = 0, nrender = 0;  // pairs recorded
    int stride[3] = {1, 1, 1};               // record every stride-th launch of a kind
    int seen[3] = {0, 0, 0};                 // launches of a kind since cp_timing_begin
    double render_ms = 0.0;                  // summed by cp_timing_end
    int render_launches = 0;
    std::vector<hipEvent_t> ev;  // [0, 2cap): step pairs, [2cap, 4cap): reset, [4cap, 6cap): render
};

struct cp_handle {
    cp_config cfg;
    int device;
    cpc::Bufs b;
    int f64;           // cfg.precision == CP_PRECISION_F64: real = double (namespace cp64)
    float* readback;
    int readback_bug;
    cpc::Lqr lqr;
    cp_timing timing;
    cp_raster_config raster;
    uint16_t* pixels;  // raster obs output (NULL: raster off)
    bool render_v1;    // CP_RENDER_V1=1 at cp_create: the round-3 small-frame render kernel (A/B diagnostic)
    int32_t* count2;   // [3] reset-list counters: [0] [1] alternating by call (SAME_STEP: each step kernel
                       // and reset launch zeroes the other one; NEXT_STEP: one per reset list), [2] NEXT_STEP's cp_reset list
    int par;           // counter the next call appends to
    // CP_AUTORESET_NEXT_STEP: the two reset lists (by call parity), the side stream each one's reset
    // kernel runs on, the events that fork it after the step kernel and join it back, the reset obs
    // the fixup kernel hands out, and the list whose reset is in flight (-1: none)
    int32_t* nlist[2];
    hipStream_t nstream[2];
    hipEvent_t nfork[2], njoin[2];
    float* nobs;
    int npar;
    int ninflight;
    int reset_lat;     // CP_SHAPE_* of the autoreset kernel: 1 latency (episodes end at different steps), 2 its WIDE layout
    int step_lat;      // CP_SHAPE_* of the step kernel: 1 latency (every wave gets a SIMD of its own), 2 WIDE
    int reset_req;     // cp_set_kernel_shape request (CP_SHAPE_AUTO: choose_reset_shape decides)
    int step_req;
    // SAME_STEP autoreset without early termination: the number of cp_step calls since every env's
    // step counter was 0 (cp_create, cp_reset of all envs), -1 when unknown (a masked reset,
    // cp_set_state, a call captured into a graph).  Fixed-length episodes then end only on calls n
    // with (n + 1) % max_episode_len == 0, and the other calls launch no reset kernel
    // (may_finish; their list is empty).  CP_RESET_EVERY_CALL=1 turns the skip off (diagnostic).
    int64_t phase;
    bool reset_every_call;
    bool captured;     // some call on this handle was captured into a graph: phase tracking off until cp_destroy
    std::string err;
};

static void choose_reset_shape(cp_handle* h);
// CP_SHAPE_AUTO picks, for the latency-shaped kernels, the widest layout whose waves still fit the chip once
// (1,024 SIMDs x 64 lanes): for the step kernel 16 lanes per env up to 4,096 envs (C2), 8 up to 8,192, else
// the two-lane layout; for the reset kernel also one env per wave (64 lanes) up to 1,024 envs.  The reset lists
// of desynchronised episodes (bounds / LQR termination) have a length only the device knows: tens to hundreds
// of envs per step, thousands where many episodes reach max_episode_len together, the whole batch at the first
// cp_reset; CP_SHAPE_LIST launches one kernel per layout and the list's length picks the one that runs
// (one env per wave for short lists).  Measured in profiles/rd7d_wide, rd7e_wide, rd7m_reset, rd7z_bench,
// rd8f_list.
static int wide_shape_for(int envs) {
    return envs <= 4096 ? CP_SHAPE_WIDE : (envs <= 8192 ? CP_SHAPE_WIDE8 : CP_SHAPE_LATENCY);
}
static int wide_reset_shape_for(int envs) { return envs <= 1024 ? CP_SHAPE_WIDE64 : wide_shape_for(envs); }

static void timing_free(cp_timing& t) {
    for (hipEvent_t e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
    t.cap = t.nstep = t.nreset = t.nrender = 0;
    for (int k = 0; k < 3; ++k) t.stride[k] = 1, t.seen[k] = 0;
}
// returns the event pair to record around a launch of `kind` (0 step, 1 reset, 2 render), or nullptr
static hipEvent_t* timing_slot(cp_handle* h, int kind) {
    cp_timing& t = h->timing;
    if (t.cap == 0) return nullptr;
    if (t.seen[kind]++ % t.stride[kind] != 0) return nullptr;
    int& n = kind == 0 ? t.nstep : (kind == 1 ? t.nreset : t.nrender);
    if (n >= (kind == 2 ? 2 * t.cap : t.cap)) return nullptr;  // up to 2 render launches per step
    hipEvent_t* p = &t.ev[(size_t)(kind * t.cap + n) * 2];
    ++n;
    return p;
}

static thread_local std::string g_err;

static int fail(cp_handle* h, const std::string& msg) {
    if (h) h->err = msg;
    g_err = msg;
    return -1;
}
static int check(cp_handle* h, hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(h, std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}
#define CP_TRY(h, call)                                   \
    do {                                                  \
        if (check((h), (call), #call)) return -1;         \
    } while (0)

static inline unsigned grid_for(int n, int block) { return (unsigned)((n + block - 1) / block); }

extern "C" {

int cp_abi_version(void) { return CP_ABI_VERSION; }

void cp_default_config(cp_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->num_envs = 1;
    c->action_repeats = 2;       // bullet_cartpole.py:23
    c->steps_per_repeat = 1;     // :25
    c->max_episode_len = 200;    // :31
    c->action_force = 50.0f;     // :18
    c->initial_force = 200.0f;   // :20
    c->random_theta = 1;         // :22
    c->initial_force_steps = 30; // :76
    c->settle_steps = 100;       // :326
    c->done_on_bounds = 0;       // :243-253 are commented out in the fork
    c->pos_threshold = 3.0f;     // :58
    c->angle_threshold = 0.35f;  // :62
    c->tan_angle_threshold = (float)std::tan((double)0.35f);
    c->sin_angle_threshold = (float)std::sin((double)0.35f);
    c->autoreset = 0;
    c->bump_mode = CP_BUMP_PHILOX;
    c->seed = 0;
    c->env_id_offset = 0;
    cp_physics* p = &c->phys;
    p->dt = (float)(1.0 / 240.0);
    p->inv_dt = 240.0f;
    p->gravity[0] = 0.0f;
    p->gravity[1] = 0.0f;
    p->gravity[2] = -9.81f;  // :152
    p->lin_damping = 0.04f;
    p->ang_damping = 0.04f;
    p->erp = 0.2f;
    p->contact_margin = 0.02f;
    p->residual_threshold = 1e-7f;
    p->solver_iterations = 50;
    p->edge_bias = 1e-4f;
    p->max_angular_step = (float)(0.25 * 3.141592653589793);
    p->warmstart = 0.85f;
    p->max_coord_velocity = 100.0f;   /* btMultiBody m_maxCoordinateVelocity [ext] */
    p->sleep_epsilon = 0.05f;         /* btMultiBody SLEEP_EPSILON [ext] (CP_MODEL_SLEEPING) */
    p->sleep_timeout = 2.0f;          /* btMultiBody SLEEP_TIMEOUT [ext] */
    // models/ground.urdf, cart.urdf, pole.urdf, cart2.urdf, pole2.urdf
    static const double he[5][3] = {{1.5, 1.5, 0.05}, {0.1, 0.1, 0.025}, {0.005, 0.005, 0.25},
                                    {0.1, 0.1, 0.025}, {0.005, 0.005, 0.25}};
    static const double mass[5] = {0.0, 1.0, 5.0, 1.0, 5.0};
    static const double inert[5][3] = {{0, 0, 0},
                                       {0.0035416666666, 0.0035416666666, 0.0066666666666},
                                       {0.104208333333333, 0.104208333333333, 0.00008333333333},
                                       {0.0035416666666, 0.0035416666666, 0.0066666666666},
                                       {0.104208333333333, 0.104208333333333, 0.00008333333333}};
    static const double mu[5] = {0.5, 0.0, 1.0, 0.0, 1.0};
    static const double spawn[5][3] = {{0, 0, 0}, {0, 0, 0.08}, {0, 0, 0.35}, {1, 0, 0.08}, {1, 0, 0.35}};
    for (int b = 0; b < 5; ++b) {
        for (int k = 0; k < 3; ++k) {
            p->half_extents[b][k] = (float)he[b][k];
            p->inertia[b][k] = (float)inert[b][k];
            p->inv_inertia[b][k] = inert[b][k] > 0 ? (float)(1.0 / inert[b][k]) : 0.0f;
            p->spawn_pos[b][k] = (float)spawn[b][k];
        }
        p->inv_mass[b] = mass[b] > 0 ? (float)(1.0 / mass[b]) : 0.0f;
        p->friction[b] = (float)mu[b];
    }
}

const char* cp_last_error(const cp_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

int cp_create(const cp_config* cfg, int device, cp_handle** out) {
    if (!cfg || !out) return fail(nullptr, "cp_create: null argument");
    if (cfg->num_envs <= 0) return fail(nullptr, "cp_create: num_envs must be > 0");
    if (cfg->action_repeats <= 0 || cfg->steps_per_repeat <= 0)
        return fail(nullptr, "cp_create: action_repeats and steps_per_repeat must be > 0");
    if (cfg->initial_force_steps < 0 || cfg->settle_steps < 0)
        return fail(nullptr, "cp_create: negative step counts");
    if (cfg->phys.solver_iterations < 0) return fail(nullptr, "cp_create: negative solver_iterations");
    // host-computed derived fields must agree with their sources (the kernels use both)
    if (!(cfg->phys.dt > 0.0f) || std::fabs((double)cfg->phys.dt * (double)cfg->phys.inv_dt - 1.0) > 1e-6)
        return fail(nullptr, "cp_create: phys.inv_dt must be 1 / phys.dt (recompute it when dt changes)");
    {   // relative tolerance: near pi/2 tan's slope makes the float32 rounding of the angle visible
        const double a = (double)cfg->angle_threshold, t = std::tan(a), s = std::sin(a);
        if (std::fabs((double)cfg->tan_angle_threshold - t) > 1e-6 * std::max(1.0, std::fabs(t)) ||
            std::fabs((double)cfg->sin_angle_threshold - s) > 1e-6)
            return fail(nullptr, "cp_create: tan/sin_angle_threshold must be tan/sin(angle_threshold)");
    }
    for (int b = 0; b < CP_NUM_BODIES; ++b) {   // the kernels read both members of each pair
        for (int k = 0; k < 3; ++k) {
            const double I = cfg->phys.inertia[b][k], iI = cfg->phys.inv_inertia[b][k];
            if (I > 0.0 ? std::fabs(I * iI - 1.0) > 1e-6 : iI != 0.0)
                return fail(nullptr, "cp_create: phys.inv_inertia must be 1 / phys.inertia (0 for a static body)");
        }
    }
    if (cfg->phys.model_flags & ~CP_MODEL_GPU_FLAGS)
        return fail(nullptr, "cp_create: phys.model_flags names a model alternative the HIP kernels do not "
                             "implement (oracle-only, DESIGN.md §3)");
    if ((cfg->phys.model_flags & CP_MODEL_PERSISTENT) && (cfg->phys.model_flags & CP_MODEL_SLEEPING))
        return fail(nullptr, "cp_create: CP_MODEL_PERSISTENT and CP_MODEL_SLEEPING together are oracle-only");
    if (!(cfg->phys.residual_threshold >= 0.0f)) return fail(nullptr, "cp_create: negative residual_threshold");
    // NaN would silently turn the clamp off (the documented off switch is <= 0) or keep bodies awake
    if (!std::isfinite(cfg->phys.max_coord_velocity))
        return fail(nullptr, "cp_create: phys.max_coord_velocity must be finite (<= 0 turns the clamp off)");
    if ((cfg->phys.model_flags & CP_MODEL_SLEEPING) &&
        (!std::isfinite(cfg->phys.sleep_epsilon) || cfg->phys.sleep_epsilon < 0.0f ||
         !std::isfinite(cfg->phys.sleep_timeout) || cfg->phys.sleep_timeout < 0.0f))
        return fail(nullptr, "cp_create: CP_MODEL_SLEEPING needs a finite, non-negative sleep_epsilon and sleep_timeout");
    if (cfg->autoreset != CP_AUTORESET_OFF && cfg->autoreset != CP_AUTORESET_SAME_STEP &&
        cfg->autoreset != CP_AUTORESET_NEXT_STEP)
        return fail(nullptr, "cp_create: autoreset must be CP_AUTORESET_OFF, _SAME_STEP or _NEXT_STEP");
    if (cfg->precision != CP_PRECISION_F32 && cfg->precision != CP_PRECISION_F64)
        return fail(nullptr, "cp_create: precision must be CP_PRECISION_F32 or CP_PRECISION_F64");
    if (cfg->reset_flags & ~CP_RESET_CLEAR_NONFINITE_FORCE)
        return fail(nullptr, "cp_create: reset_flags holds an unknown CP_RESET_* bit");
    if ((unsigned long long)cfg->num_envs * CP_STATE_FIELDS * (cfg->precision == CP_PRECISION_F64 ? 8ull : 4ull) >= (1ull << 32) ||
        (unsigned long long)cfg->num_envs * cfg->action_repeats * 14ull * 4ull >= (1ull << 32))
        return fail(nullptr, "cp_create: num_envs too large for one handle (SoA arrays must stay below 4 GiB)");
    cp_handle* h = new (std::nothrow) cp_handle();
    if (!h) return fail(nullptr, "cp_create: out of memory");
    h->cfg = *cfg;
    h->device = device;
    h->readback = nullptr;
    h->readback_bug = 1;
    h->lqr = cpc::Lqr{nullptr, 0, nullptr, 0.0f, 0.0f};
    h->f64 = cfg->precision == CP_PRECISION_F64;
    h->pixels = nullptr;
    {
        const char* v1 = std::getenv("CP_RENDER_V1");
        h->render_v1 = v1 && v1[0] == '1';
    }
    h->npar = 0;
    h->ninflight = -1;
    h->phase = 0;  // every env's step counter is 0 (and done is 1: they do not step until reset)
    h->captured = false;
    {
        const char* rc = std::getenv("CP_RESET_EVERY_CALL");
        h->reset_every_call = rc && rc[0] == '1';
    }
    h->reset_req = h->step_req = CP_SHAPE_AUTO;
    choose_reset_shape(h);
    cp_default_raster_config(&h->raster);
    std::memset(&h->b, 0, sizeof(h->b));
    const size_t B = (size_t)cfg->num_envs;
    const int R = cfg->action_repeats;
    auto fail_free = [&](hipError_t e, const char* what) {
        std::string msg = std::string(what) + ": " + hipGetErrorString(e);
        cp_destroy(h);
        return fail(nullptr, msg);
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail_free(e, "hipSetDevice");
#define CP_ALLOC(ptr, bytes)                                   \
    e = hipMalloc((void**)&(ptr), (bytes));                    \
    if (e != hipSuccess) return fail_free(e, "hipMalloc " #ptr);
    const size_t rb = h->f64 ? sizeof(double) : sizeof(float);  // bytes of the handle's real type
    CP_ALLOC(h->b.state, (size_t)CP_STATE_FIELDS * B * rb);
    CP_ALLOC(h->b.term_obs, (size_t)R * 14 * B * sizeof(float));
    CP_ALLOC(h->b.bumps, B * (size_t)(cfg->initial_force_steps > 0 ? cfg->initial_force_steps : 1) * 4 * rb);
    CP_ALLOC(h->b.ret_acc, B * sizeof(float));
    CP_ALLOC(h->b.last_ret, B * sizeof(float));
    CP_ALLOC(h->b.last_len, B * sizeof(int32_t));
    CP_ALLOC(h->b.overflow, B * sizeof(int32_t));
    CP_ALLOC(h->b.nonfinite, B * sizeof(int32_t));
    CP_ALLOC(h->b.list, B * sizeof(int32_t));
    CP_ALLOC(h->count2, 3 * sizeof(int32_t));
    CP_ALLOC(h->b.scratch, (size_t)CP_SCR_FIELDS * 2 * B * rb);
    CP_ALLOC(h->b.stamps, CP_STAMP_SLOTS * sizeof(uint64_t));
    CP_ALLOC(h->b.stepped, B * sizeof(uint8_t));
    if (cfg->phys.model_flags & CP_MODEL_PERSISTENT) {  // the persistent manifolds, empty
        CP_ALLOC(h->b.pman, (size_t)CP_PM_FIELDS * 2 * B * rb);
        e = hipMemset(h->b.pman, 0, (size_t)CP_PM_FIELDS * 2 * B * rb);
        if (e != hipSuccess) return fail_free(e, "hipMemset");
    }
    if (cfg->autoreset == CP_AUTORESET_NEXT_STEP) {
        for (int k = 0; k < 2; ++k) {
            CP_ALLOC(h->nlist[k], B * sizeof(int32_t));
            // non-blocking: no implicit ordering against a caller's legacy default stream
            e = hipStreamCreateWithFlags(&h->nstream[k], hipStreamNonBlocking);
            if (e != hipSuccess) return fail_free(e, "hipStreamCreateWithFlags");
            e = hipEventCreateWithFlags(&h->nfork[k], hipEventDisableTiming);
            if (e != hipSuccess) return fail_free(e, "hipEventCreateWithFlags");
            e = hipEventCreateWithFlags(&h->njoin[k], hipEventDisableTiming);
            if (e != hipSuccess) return fail_free(e, "hipEventCreateWithFlags");
        }
        CP_ALLOC(h->nobs, (size_t)R * 14 * B * sizeof(float));
        e = hipMemset(h->nobs, 0, (size_t)R * 14 * B * sizeof(float));
        if (e != hipSuccess) return fail_free(e, "hipMemset");
    }
#undef CP_ALLOC
    e = hipMemset(h->count2, 0, 3 * sizeof(int32_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    h->b.count = h->count2;
    h->b.count_next = nullptr;
    e = hipMemset(h->b.stepped, 0, B * sizeof(uint8_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.stamps, 0, CP_STAMP_SLOTS * sizeof(uint64_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.term_obs, 0, (size_t)R * 14 * B * sizeof(float));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.bumps, 0, B * (size_t)(cfg->initial_force_steps > 0 ? cfg->initial_force_steps : 1) * 4 * rb);
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    if (h->f64) cp64::launch_init(h->cfg, h->b, 0);
    else cp::launch_init(h->cfg, h->b, 0);
    e = hipGetLastError();
    if (e != hipSuccess) return fail_free(e, "cp_init_kernel");
    e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail_free(e, "hipDeviceSynchronize");
    *out = h;
    return 0;
}

void cp_destroy(cp_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (int k = 0; k < 2; ++k) {  // NEXT_STEP: a reset may still be in flight on a side stream
        if (h->nstream[k]) {
            (void)hipStreamSynchronize(h->nstream[k]);
            (void)hipStreamDestroy(h->nstream[k]);
        }
        if (h->nfork[k]) (void)hipEventDestroy(h->nfork[k]);
        if (h->njoin[k]) (void)hipEventDestroy(h->njoin[k]);
        (void)hipFree(h->nlist[k]);
    }
    (void)hipFree(h->nobs);
    timing_free(h->timing);
    (void)hipFree(h->b.state);
    (void)hipFree(h->b.term_obs);
    (void)hipFree(h->b.bumps);
    (void)hipFree(h->b.ret_acc);
    (void)hipFree(h->b.last_ret);
    (void)hipFree(h->b.last_len);
    (void)hipFree(h->b.overflow);
    (void)hipFree(h->b.nonfinite);
    (void)hipFree(h->b.list);
    (void)hipFree(h->count2);
    (void)hipFree(h->b.scratch);
    (void)hipFree(h->b.stamps);
    (void)hipFree(h->b.stepped);
    (void)hipFree(h->b.pman);
    (void)hipFree(h->b.rposes);
    (void)hipFree(h->b.rlist);
    (void)hipFree(h->b.rcount);
    (void)hipFree(h->b.rtable);
    delete h;
}

// raster obs of the envs in list[0 .. *count) (a device count: the grid covers B).  launch = false only
// names the kernel the handle would launch (cp_render_kernel_name): 0 small2, 1 small, 2 wave kernel.
static int launch_render(cp_handle* h, const int32_t* list, const int32_t* count, hipStream_t st,
                         bool launch = true, int* kind = nullptr) {
    hipEvent_t* ev = launch ? timing_slot(h, 2) : nullptr;
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    const int C = h->raster.num_cameras, R = h->cfg.action_repeats, npx = h->raster.width * h->raster.height;
    const uint8_t* cls = launch ? reinterpret_cast<const uint8_t*>(h->b.rtable + (size_t)C * npx) : nullptr;
    const size_t small = (size_t)cp::render_small_lds(C, R, npx).total;
    // v2 of the small-frame kernel for the common (cameras, repeats) pairs, both compile-time
    auto small2 = [&](auto cc, auto rr) -> bool {
        constexpr int CC = decltype(cc)::value, RR = decltype(rr)::value;
        if (C != CC || R != RR || h->render_v1) return false;
        const size_t lds = (size_t)cp::render_small2_lds<CC * RR>(C, R, npx).total;
        if (lds > (size_t)cp::SMALL_LDS_MAX) return false;
        if (launch)
            hipLaunchKernelGGL((cp::cp_render_small2_kernel<CC, RR>), dim3((unsigned)h->cfg.num_envs),
                               dim3(cp::RENDER_WAVES * cp::WAVE_R), lds, st, h->raster, h->cfg.phys, list, count,
                               h->b.rposes, h->b.rtable, cls, h->pixels);
        return true;
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I6 = std::integral_constant<int, 6>;
    if (small2(I1{}, I3{}) || small2(I1{}, I2{}) || small2(I1{}, I1{}) || small2(I1{}, I4{}) || small2(I1{}, I6{}) ||
        small2(I2{}, I1{}) || small2(I2{}, I2{}) || small2(I2{}, I3{})) {
        if (kind) *kind = 0;  // launched
    } else if (!launch) {
        if (kind) *kind = small <= (size_t)cp::SMALL_LDS_MAX ? 1 : 2;
        return 0;
    } else if (small <= (size_t)cp::SMALL_LDS_MAX) {  // one block per env, dense ray tests
        hipLaunchKernelGGL(cp::cp_render_small_kernel, dim3((unsigned)h->cfg.num_envs),
                           dim3(cp::RENDER_WAVES * cp::WAVE_R), small, st, h->raster, h->cfg.phys, R, list, count,
                           h->b.rposes, h->b.rtable, cls, h->pixels);
    } else {  // large frames: one wave per env
        const size_t lds = (size_t)cp::RENDER_WAVES * cp::render_lds(C, R).total;
        const unsigned grid = (unsigned)((h->cfg.num_envs + cp::RENDER_WAVES - 1) / cp::RENDER_WAVES);
        hipLaunchKernelGGL(cp::cp_render_kernel, dim3(grid), dim3(cp::RENDER_WAVES * cp::WAVE_R), lds, st, h->raster,
                           h->cfg.phys, R, list, count, h->b.rposes, h->b.rtable, cls, h->pixels);
    }
    if (!launch) return 0;
    if (check(h, hipGetLastError(), "cp_render_kernel")) return -1;
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    return 0;
}

const char* cp_render_kernel_name(cp_handle* h) {
    if (!h || !h->pixels) return nullptr;
    int kind = -1;
    if (launch_render(h, nullptr, nullptr, nullptr, false, &kind) != 0) return nullptr;
    static const char* const names[3] = {"cp_render_small2_kernel", "cp_render_small_kernel", "cp_render_kernel"};
    return kind >= 0 && kind < 3 ? names[kind] : nullptr;
}

// the reset list's counter for this call: the one the previous call's step kernel (and reset launch) zeroed
static void use_counter(cp_handle* h) {
    h->b.count = h->count2 + h->par;
    h->b.count_next = h->count2 + (h->par ^ 1);
    h->par ^= 1;
}

// Which autoreset kernel shape (cp_reset_kernel<LAT>): episodes that can end early (bounds
// termination, LQR done thresholds) end at different steps, so every step resets a short list
// and its latency is the step's; fixed-length episodes end together in bursts (throughput),
// except in batches small enough that a burst fits one wave per SIMD.
// The step kernel has the same two shapes, chosen by batch size alone.  CP_RESET_LATENCY=0/1 and
// CP_STEP_LATENCY=0/1 override (diagnostics).
static void choose_reset_shape(cp_handle* h) {
    const bool lqr_done = h->lqr.gains && (h->lqr.done_pos > 0.0f || h->lqr.done_angle > 0.0f);
    // up to 32,768 envs every wave gets a SIMD of its own even in a full burst (1,024 SIMDs), so
    // the latency shape is never the slower one there
    const bool small = h->cfg.num_envs <= 32768;
    const char* e = std::getenv("CP_RESET_LATENCY");
    h->reset_lat = (e && (e[0] == '0' || e[0] == '1')) ? e[0] == '1' : (h->cfg.done_on_bounds || lqr_done || small);
    const char* es = std::getenv("CP_STEP_LATENCY");
    h->step_lat = (es && (es[0] == '0' || es[0] == '1')) ? es[0] == '1' : small;
    // the WIDE layout (16 lanes per env) where its extra waves still leave SIMDs idle
    const bool wide_ok = !h->f64 && !(h->cfg.phys.model_flags & (CP_MODEL_PERSISTENT | CP_MODEL_SLEEPING));
    if (wide_ok && h->step_lat) h->step_lat = wide_shape_for(h->cfg.num_envs);
    // Lists of desynchronised episodes: CP_SHAPE_LIST under either autoreset mode (bounds regime, steps 61-260:
    // SAME_STEP 10.9 M with one env per wave whatever the list's length, 11.1 M two-lane, 13.2 M by the length;
    // NEXT_STEP 17.6 / 21.5 / 24.9 M; profiles/rd8f_list).  Fixed-length episodes under NEXT_STEP keep the
    // two-lane reset beside the next call's step kernel.
    if (wide_ok && h->reset_lat && (h->cfg.done_on_bounds || lqr_done))
        h->reset_lat = CP_SHAPE_LIST;
    else if (wide_ok && h->reset_lat && h->cfg.autoreset != CP_AUTORESET_NEXT_STEP)
        h->reset_lat = wide_reset_shape_for(h->cfg.num_envs);
    if (h->reset_req != CP_SHAPE_AUTO) h->reset_lat = h->reset_req;
    if (h->step_req != CP_SHAPE_AUTO) h->step_lat = h->step_req;
    if (h->f64) h->reset_lat = h->step_lat = 1;  // fp64: the 512-register shape only
    if (h->cfg.phys.model_flags & (CP_MODEL_PERSISTENT | CP_MODEL_SLEEPING))
        h->reset_lat = h->step_lat = 1;  // PM, SLEEPING: latency shape only
}

static int launch_reset_list(cp_handle* h, const cpc::Bufs& b, float* obs_out, hipStream_t st) {
    hipEvent_t* ev = timing_slot(h, 1);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    if (h->f64) cp64::launch_reset(true, h->cfg, b, obs_out, st);
    else cp::launch_reset(h->reset_lat, h->cfg, b, obs_out, st);
    if (check(h, hipGetLastError(), "cp_reset_kernel")) return -1;
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    return 0;
}

// A graph replays a captured call any number of times without the host seeing it, so once any entry
// point that moves the step counters (cp_step, cp_reset, cp_rollout) has been captured on this handle,
// the phase is unknown for good: every later cp_step launches its reset kernel.
static bool note_capture(cp_handle* h, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        h->captured = true;
        h->phase = -1;
        return true;
    }
    return false;
}

// false when no env can finish in this cp_step call (see cp_handle::phase): every env that steps
// enters it with a step counter of phase % max_episode_len, so it reaches the limit only when
// (phase + 1) % max_episode_len == 0, and nothing else ends an episode.  The step kernel zeroes the next call's counter itself, so a skipped reset launch
// leaves the counters as a launched one would.
static bool may_finish(cp_handle* h, hipStream_t st) {
    const bool lqr_done = h->lqr.gains && (h->lqr.done_pos > 0.0f || h->lqr.done_angle > 0.0f);
    if (h->reset_every_call || h->captured || h->phase < 0 || h->cfg.done_on_bounds || lqr_done) return true;
    if (h->cfg.max_episode_len <= 0) return true;  // every step ends the episode (done = steps >= limit)
    return (h->phase + 1) % h->cfg.max_episode_len == 0;
}

static int launch_reset_from_list(cp_handle* h, float* obs_out, hipStream_t st, bool render) {
    if (launch_reset_list(h, h->b, obs_out, st)) return -1;
    if (render && h->pixels) return launch_render(h, h->b.list, h->b.count, st);
    return 0;
}

// CP_AUTORESET_NEXT_STEP: make `st` wait for the reset in flight on a side stream (every entry point
// that reads or writes the state or the per-env outputs of the last call does this first)
static int join_next_step(cp_handle* h, hipStream_t st) {
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP && h->ninflight >= 0)
        CP_TRY(h, hipStreamWaitEvent(st, h->njoin[h->ninflight], 0));
    return 0;
}

// cp_step of a NEXT_STEP handle.  Call n appends its finishing envs to list q = n % 2
// (their done field becomes 2 + q) and starts their reset on side stream q as soon as its step kernel
// is done; call n + 1 steps every other env meanwhile (the step kernel skips done fields >= 2), then
// waits for that reset and hands out its obs (fixup kernel).  Two resets can be in flight at once:
// list q's reset overlaps call n + 1's step kernel and the caller's work between the calls.
static int step_next_step(cp_handle* h, const void* actions, int action_kind, float* obs_out, float* reward_out,
                          uint8_t* done_out, float* terminal_obs_out, hipStream_t st) {
    const int q = h->npar;
    cpc::Bufs b = h->b;
    b.list = h->nlist[q];
    b.count = h->count2 + q;  // zeroed by the fixup of its previous use (or at cp_create)
    b.count_next = nullptr;
    b.npar = q;
    b.keep_done = 1;
    hipEvent_t* ev = timing_slot(h, 0);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    if (h->f64)
        cp64::launch_step(true, action_kind, h->cfg, b, actions, obs_out, reward_out, done_out, terminal_obs_out,
                          h->readback, h->readback_bug, h->lqr, st);
    else
        cp::launch_step(h->step_lat, action_kind, h->cfg, b, actions, obs_out, reward_out, done_out,
                        terminal_obs_out, h->readback, h->readback_bug, h->lqr, st);
    CP_TRY(h, hipGetLastError());
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    CP_TRY(h, hipEventRecord(h->nfork[q], st));
    if (h->ninflight >= 0) {  // the previous call's list: its reset obs are this call's obs
        const int p = h->ninflight;
        CP_TRY(h, hipStreamWaitEvent(st, h->njoin[p], 0));
        if (h->f64)
            cp64::launch_nextstep_fixup(h->cfg, h->b, h->nlist[p], h->count2 + p, p, h->nobs, obs_out, reward_out,
                                        done_out, st);
        else
            cp::launch_nextstep_fixup(h->cfg, h->b, h->nlist[p], h->count2 + p, p, h->nobs, obs_out, reward_out,
                                      done_out, st);
        CP_TRY(h, hipGetLastError());
        CP_TRY(h, hipMemsetAsync(h->count2 + p, 0, sizeof(int32_t), st));
    }
    CP_TRY(h, hipStreamWaitEvent(h->nstream[q], h->nfork[q], 0));
    if (launch_reset_list(h, b, h->nobs, h->nstream[q])) return -1;
    CP_TRY(h, hipEventRecord(h->njoin[q], h->nstream[q]));
    h->ninflight = q;
    h->npar = q ^ 1;
    return 0;
}

int cp_reset(cp_handle* h, const uint8_t* env_mask, float* obs_out, void* stream) {
    if (!h || !obs_out) return fail(h, "cp_reset: null argument");
    hipStream_t st = (hipStream_t)stream;
    const int B = h->cfg.num_envs;
    CP_TRY(h, hipSetDevice(h->device));
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP) {  // envs whose reset already ran keep it
        if (join_next_step(h, st)) return -1;
        cpc::Bufs b = h->b;
        b.count = h->count2 + 2;
        b.count_next = nullptr;
        CP_TRY(h, hipMemsetAsync(b.count, 0, sizeof(int32_t), st));
        if (h->f64) cp64::launch_nextstep_resolve(h->cfg, b, env_mask, h->nobs, obs_out, st);
        else cp::launch_nextstep_resolve(h->cfg, b, env_mask, h->nobs, obs_out, st);
        CP_TRY(h, hipGetLastError());
        return launch_reset_list(h, b, obs_out, st);
    }
    use_counter(h);
    h->phase = env_mask ? -1 : 0;
    note_capture(h, st);
    CP_TRY(h, hipMemsetAsync(h->b.count, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(cp::cp_mask_to_list_kernel, dim3(grid_for(B, 256)), dim3(256), 0, st, B, env_mask, h->b.list,
                       h->b.count);
    CP_TRY(h, hipGetLastError());
    return launch_reset_from_list(h, obs_out, st, true);
}

int cp_step(cp_handle* h, const void* actions, int action_kind, float* obs_out, float* reward_out,
            uint8_t* done_out, float* terminal_obs_out, void* stream) {
    if (!h || !actions || !obs_out || !reward_out || !done_out) return fail(h, "cp_step: null argument");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(h, "cp_step: action_kind must be CP_ACTION_CONTINUOUS or CP_ACTION_DISCRETE");
    hipStream_t st = (hipStream_t)stream;
    CP_TRY(h, hipSetDevice(h->device));
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP)
        return step_next_step(h, actions, action_kind, obs_out, reward_out, done_out, terminal_obs_out, st);
    if (h->cfg.autoreset) use_counter(h);  // zeroed by the previous call's step kernel (and reset launch)
    const bool capturing = note_capture(h, st);
    const bool reset = h->cfg.autoreset && may_finish(h, st);
    if (h->pixels) CP_TRY(h, hipMemsetAsync(h->b.rcount, 0, sizeof(int32_t), st));
    hipEvent_t* ev = timing_slot(h, 0);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    if (h->f64)
        cp64::launch_step(true, action_kind, h->cfg, h->b, actions, obs_out, reward_out, done_out, terminal_obs_out,
                          h->readback, h->readback_bug, h->lqr, st);
    else
        cp::launch_step(h->step_lat, action_kind, h->cfg, h->b, actions, obs_out, reward_out, done_out,
                        terminal_obs_out, h->readback, h->readback_bug, h->lqr, st);
    CP_TRY(h, hipGetLastError());
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    // autoreset envs were simulated this step, so they are in the render list; the reset
    // kernel rewrites their poses first, and the one render launch draws the new episode
    if (reset && launch_reset_from_list(h, obs_out, st, false)) return -1;
    if (h->phase >= 0) ++h->phase;
    if (h->pixels && launch_render(h, h->b.rlist, h->b.rcount, st)) return -1;
    // a graph replays this call with the same counter every time: leave it empty for the next replay
    // (eagerly the next call's step kernel zeroes it, as the other counter)
    if (capturing && h->cfg.autoreset) CP_TRY(h, hipMemsetAsync(h->b.count, 0, sizeof(int32_t), st));
    return 0;
}

int cp_rollout(cp_handle* h, int steps, const void* actions, int action_kind, float* obs_out, float* reward_out,
               uint8_t* done_out, float* terminal_obs_out, void* stream) {
    if (!h || !actions || !obs_out || !reward_out || !done_out) return fail(h, "cp_rollout: null argument");
    if (steps <= 0) return fail(h, "cp_rollout: steps must be > 0");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(h, "cp_rollout: action_kind must be CP_ACTION_CONTINUOUS or CP_ACTION_DISCRETE");
    if (h->readback || h->lqr.state8 || h->pixels)
        return fail(h, "cp_rollout: the per-step side outputs (readback, LQR 8-states, raster obs) are cp_step-only; "
                       "disable them first");
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP)
        return fail(h, "cp_rollout: CP_AUTORESET_NEXT_STEP handles step through cp_step only");
    hipStream_t st = (hipStream_t)stream;
    CP_TRY(h, hipSetDevice(h->device));
    hipEvent_t* ev = timing_slot(h, 0);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    if (h->f64)
        cp64::launch_rollout(true, action_kind, h->cfg, h->b, steps, actions, obs_out, reward_out, done_out,
                             terminal_obs_out, h->lqr, st);
    else
        cp::launch_rollout(h->step_lat != 0, action_kind, h->cfg, h->b, steps, actions, obs_out, reward_out, done_out,
                           terminal_obs_out, h->lqr, st);
    CP_TRY(h, hipGetLastError());
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    note_capture(h, st);
    if (h->phase >= 0) h->phase += steps;  // the kernel resets finishing envs inline
    return 0;
}

int cp_set_readback(cp_handle* h, float* readback_out, int reference_bug) {
    if (!h) return fail(h, "cp_set_readback: null handle");
    h->readback = readback_out;
    h->readback_bug = reference_bug ? 1 : 0;
    return 0;
}

int cp_set_lqr(cp_handle* h, const float* gains, int per_env, float* state8_out, float done_pos,
               float done_angle) {
    if (!h) return fail(h, "cp_set_lqr: null handle");
    if (!gains && state8_out) return fail(h, "cp_set_lqr: the 8-state readback needs the LQR policy on");
    if (gains && (h->cfg.phys.model_flags & CP_MODEL_SLEEPING))
        return fail(h, "cp_set_lqr: the LQR policy is not built for CP_MODEL_SLEEPING handles (oracle-only)");
    h->lqr.gains = gains;
    h->lqr.per_env = per_env ? 1 : 0;
    h->lqr.state8 = state8_out;
    h->lqr.done_pos = done_pos;
    h->lqr.done_angle = done_angle;
    choose_reset_shape(h);
    return 0;
}

// the forces copied (same type) or converted into the handle's bump buffer (its real type)
extern "C++" template <typename S>
static int set_bumps(cp_handle* h, const S* forces, void* stream, const char* what) {
    if (!h || !forces) return fail(h, std::string(what) + ": null argument");
    CP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    if (join_next_step(h, st)) return -1;  // an in-flight reset reads the bumps
    const size_t n = (size_t)h->cfg.num_envs * h->cfg.initial_force_steps * 4;
    if (n == 0) return 0;
    const bool same = h->f64 == std::is_same<S, double>::value;
    if (same) {
        CP_TRY(h, hipMemcpyAsync(h->b.bumps, forces, n * sizeof(S), hipMemcpyDeviceToDevice, st));
    } else if (h->f64) {
        hipLaunchKernelGGL((cp::cp_convert_kernel<S, double>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           forces, static_cast<double*>(h->b.bumps), n);
        CP_TRY(h, hipGetLastError());
    } else {
        hipLaunchKernelGGL((cp::cp_convert_kernel<S, float>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           forces, static_cast<float*>(h->b.bumps), n);
        CP_TRY(h, hipGetLastError());
    }
    return 0;
}

int cp_set_bump_forces(cp_handle* h, const float* forces, void* stream) {
    return set_bumps(h, forces, stream, "cp_set_bump_forces");
}

int cp_set_bump_forces64(cp_handle* h, const double* forces, void* stream) {
    return set_bumps(h, forces, stream, "cp_set_bump_forces64");
}

int64_t cp_state_bytes(const cp_handle* h) {
    if (!h) return fail(nullptr, "cp_state_bytes: null handle");
    return (int64_t)CP_STATE_FIELDS * h->cfg.num_envs * (h->f64 ? (int64_t)sizeof(double) : (int64_t)sizeof(float));
}

int cp_set_kernel_shape(cp_handle* h, int step_shape, int reset_shape) {
    if (!h) return fail(h, "cp_set_kernel_shape: null handle");
    auto ok = [](int v) {
        return v == CP_SHAPE_AUTO || v == CP_SHAPE_THROUGHPUT || v == CP_SHAPE_LATENCY || v == CP_SHAPE_WIDE ||
               v == CP_SHAPE_WIDE8 || v == CP_SHAPE_WIDE64 || v == CP_SHAPE_LIST;
    };
    if (!ok(step_shape) || !ok(reset_shape))
        return fail(h, "cp_set_kernel_shape: shapes must be CP_SHAPE_AUTO, CP_SHAPE_THROUGHPUT, CP_SHAPE_LATENCY, "
                       "CP_SHAPE_WIDE, CP_SHAPE_WIDE8, CP_SHAPE_WIDE64 or CP_SHAPE_LIST");
    auto fixed = [](int v) {
        return v == CP_SHAPE_THROUGHPUT || v == CP_SHAPE_WIDE || v == CP_SHAPE_WIDE8 || v == CP_SHAPE_WIDE64 ||
               v == CP_SHAPE_LIST;
    };
    if (step_shape == CP_SHAPE_WIDE64 || step_shape == CP_SHAPE_LIST)
        return fail(h, "cp_set_kernel_shape: CP_SHAPE_WIDE64 and CP_SHAPE_LIST are reset-kernel layouts");
    if ((h->f64 || (h->cfg.phys.model_flags & (CP_MODEL_PERSISTENT | CP_MODEL_SLEEPING))) &&
        (fixed(step_shape) || fixed(reset_shape)))
        return fail(h, "cp_set_kernel_shape: fp64, persistent-manifold and sleeping-model handles have the latency "
                       "shape only");
    h->step_req = step_shape;
    h->reset_req = reset_shape;
    choose_reset_shape(h);
    return 0;
}

int cp_get_kernel_shape(const cp_handle* h, int* step_shape, int* reset_shape) {
    if (!h) return fail(nullptr, "cp_get_kernel_shape: null handle");
    if (step_shape) *step_shape = h->step_lat;
    if (reset_shape) *reset_shape = h->reset_lat;
    return 0;
}

int cp_get_state(cp_handle* h, void* state_out, void* stream) {
    if (!h || !state_out) return fail(h, "cp_get_state: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    if (join_next_step(h, (hipStream_t)stream)) return -1;
    size_t n = (size_t)CP_STATE_FIELDS * h->cfg.num_envs;
    CP_TRY(h, hipMemcpyAsync(state_out, h->b.state, n * (h->f64 ? sizeof(double) : sizeof(float)), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    return 0;
}

int cp_set_state(cp_handle* h, const void* state_in, void* stream) {
    if (!h || !state_in) return fail(h, "cp_set_state: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    if (join_next_step(h, (hipStream_t)stream)) return -1;
    size_t n = (size_t)CP_STATE_FIELDS * h->cfg.num_envs;
    CP_TRY(h, hipMemcpyAsync(h->b.state, state_in, n * (h->f64 ? sizeof(double) : sizeof(float)), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    h->phase = -1;  // step counters of any value
    // the persistent manifolds are not part of the state SoA: no cached contact survives a teleport
    // (as in the reset kernel), so the next step rebuilds them from the new poses
    if (h->b.pman)
        CP_TRY(h, hipMemsetAsync(h->b.pman, 0, (size_t)CP_PM_FIELDS * 2 * h->cfg.num_envs *
                                                   (h->f64 ? sizeof(double) : sizeof(float)), (hipStream_t)stream));
    return 0;
}

int cp_episode_returns(cp_handle* h, float* returns_out, int32_t* lengths_out, void* stream) {
    if (!h) return fail(h, "cp_episode_returns: null handle");
    CP_TRY(h, hipSetDevice(h->device));
    if (join_next_step(h, (hipStream_t)stream)) return -1;
    size_t B = (size_t)h->cfg.num_envs;
    hipStream_t st = (hipStream_t)stream;
    if (returns_out) CP_TRY(h, hipMemcpyAsync(returns_out, h->b.last_ret, B * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (lengths_out)
        CP_TRY(h, hipMemcpyAsync(lengths_out, h->b.last_len, B * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return 0;
}

int cp_nonfinite_counts(cp_handle* h, int32_t* out, void* stream) {
    if (!h || !out) return fail(h, "cp_nonfinite_counts: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    if (join_next_step(h, (hipStream_t)stream)) return -1;
    CP_TRY(h, hipMemcpyAsync(out, h->b.nonfinite, (size_t)h->cfg.num_envs * sizeof(int32_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    return 0;
}

int cp_overflow_counts(cp_handle* h, int32_t* out, void* stream) {
    if (!h || !out) return fail(h, "cp_overflow_counts: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    if (join_next_step(h, (hipStream_t)stream)) return -1;
    CP_TRY(h, hipMemcpyAsync(out, h->b.overflow, (size_t)h->cfg.num_envs * sizeof(int32_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    return 0;
}

int cp_debug_stamps(cp_handle* h, uint64_t* out64, int reset) {
    if (!h || !out64) return fail(h, "cp_debug_stamps: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    CP_TRY(h, hipDeviceSynchronize());
    CP_TRY(h, hipMemcpy(out64, h->b.stamps, CP_STAMP_SLOTS * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) CP_TRY(h, hipMemset(h->b.stamps, 0, CP_STAMP_SLOTS * sizeof(uint64_t)));
#ifdef CP_STAMPS
    return 1;
#else
    return 0;
#endif
}

int cp_timing_begin(cp_handle* h, int max_launches) {
    if (!h || max_launches <= 0) return fail(h, "cp_timing_begin: bad argument");
    CP_TRY(h, hipSetDevice(h->device));
    timing_free(h->timing);
    h->timing.ev.resize((size_t)max_launches * 8);
    for (auto& e : h->timing.ev) CP_TRY(h, hipEventCreate(&e));
    h->timing.cap = max_launches;
    return 0;
}

int cp_timing_stride(cp_handle* h, int step_stride, int reset_stride) {
    if (!h || step_stride <= 0 || reset_stride <= 0) return fail(h, "cp_timing_stride: bad argument");
    h->timing.stride[0] = step_stride;
    h->timing.stride[1] = reset_stride;
    return 0;
}

int cp_timing_end(cp_handle* h, double* step_ms, int32_t* step_launches, double* reset_ms,
                  int32_t* reset_launches) {
    if (!h) return fail(h, "cp_timing_end: null handle");
    cp_timing& t = h->timing;
    double sums[3] = {0.0, 0.0, 0.0};
    int counts[3] = {t.nstep, t.nreset, t.nrender};
    for (int kind = 0; kind < 3; ++kind) {
        for (int n = 0; n < counts[kind]; ++n) {
            hipEvent_t a = t.ev[(size_t)(kind * t.cap + n) * 2], b = t.ev[(size_t)(kind * t.cap + n) * 2 + 1];
            CP_TRY(h, hipEventSynchronize(b));
            float ms = 0.0f;
            CP_TRY(h, hipEventElapsedTime(&ms, a, b));
            sums[kind] += ms;
        }
    }
    if (step_ms) *step_ms = sums[0];
    if (step_launches) *step_launches = counts[0];
    if (reset_ms) *reset_ms = sums[1];
    if (reset_launches) *reset_launches = counts[1];
    timing_free(t);
    t.render_ms = sums[2];
    t.render_launches = counts[2];
    return 0;
}

int cp_event_record_bytes(int action_kind, int repeats, int with_action) {
    if ((action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE) || repeats <= 0)
        return fail(nullptr, "cp_event_record_bytes: bad action kind or repeats");
    return cp::record_len(action_kind, repeats, with_action ? 1 : 0);
}

int cp_encode_events(cp_handle* h, int mode, const void* actions, int action_kind, const float* obs,
                     const float* terminal_obs, const float* reward, const uint8_t* done, const uint8_t* env_mask,
                     uint8_t* step_records, uint8_t* reset_records, uint8_t* flags, void* stream) {
    if (!h || !obs || !flags) return fail(h, "cp_encode_events: null argument");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(h, "cp_encode_events: bad action kind");
    if (mode == 0 && (!actions || !reward || !done || !step_records))
        return fail(h, "cp_encode_events: mode 0 needs actions, reward, done and step_records");
    if (mode == 1 && !reset_records) return fail(h, "cp_encode_events: mode 1 needs reset_records");
    if (mode != 0 && mode != 1) return fail(h, "cp_encode_events: mode must be 0 (step) or 1 (reset)");
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP)
        return fail(h, "cp_encode_events: not for CP_AUTORESET_NEXT_STEP handles");
    CP_TRY(h, hipSetDevice(h->device));
    const int B = h->cfg.num_envs;
    hipLaunchKernelGGL(cp::cp_event_kernel, dim3(grid_for(B, 256)), dim3(256), 0, (hipStream_t)stream, B,
                       h->cfg.action_repeats, mode, action_kind, h->cfg.autoreset, actions, obs, terminal_obs, reward,
                       done, env_mask, h->b.stepped, step_records, reset_records, flags);
    CP_TRY(h, hipGetLastError());
    return 0;
}

int cp_timing_render(cp_handle* h, double* render_ms, int32_t* render_launches) {
    if (!h) return fail(h, "cp_timing_render: null handle");
    if (render_ms) *render_ms = h->timing.render_ms;
    if (render_launches) *render_launches = h->timing.render_launches;
    return 0;
}

void cp_default_raster_config(cp_raster_config* rc) {
    std::memset(rc, 0, sizeof(*rc));
    rc->width = 50;        // --render-width, bullet_cartpole.py:35
    rc->height = 50;       // --render-height, :37
    rc->num_cameras = 1;   // --num-cameras, :27
    const float temp = 0.75f;  // :278-279
    rc->eye[0][0] = 0.0f; rc->eye[0][1] = temp; rc->eye[0][2] = temp;
    rc->eye[1][0] = temp; rc->eye[1][1] = 0.0f; rc->eye[1][2] = temp;
    rc->target[0] = 0.0f; rc->target[1] = 0.0f; rc->target[2] = 0.3f;  // :280
    rc->up[0] = 0.0f; rc->up[1] = 0.0f; rc->up[2] = 1.0f;              // :281
    rc->tan_half_fov = (float)std::tan(0.5 * 30.0 * 3.141592653589793 / 180.0);  // fov 30, :283
    rc->far_plane = 20.0f;                                             // :282
    // light from above and in front of camera 0 (unpinned: TinyRenderer's is not available)
    const double l[3] = {0.3, 0.5, 1.0};
    const double ln = std::sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
    for (int k = 0; k < 3; ++k) rc->light[k] = (float)(l[k] / ln);
    rc->ambient = 0.6f;
    rc->diffuse = 0.4f;
    rc->background[0] = 1.0f; rc->background[1] = 1.0f; rc->background[2] = 1.0f;
    static const float col[5][3] = {{0.3f, 0.3f, 0.0f},   // ground.urdf:15
                                    {0.9f, 0.2f, 0.1f},   // cart.urdf:25
                                    {0.2f, 0.7f, 0.1f},   // pole.urdf:30
                                    {0.2f, 0.9f, 0.1f},   // cart2.urdf:25
                                    {0.7f, 0.2f, 0.7f}};  // pole2.urdf:24
    std::memcpy(rc->color, col, sizeof(col));
}

int cp_set_raster(cp_handle* h, const cp_raster_config* rc, uint16_t* pixels_out) {
    if (!h) return fail(h, "cp_set_raster: null handle");
    CP_TRY(h, hipSetDevice(h->device));
    if (!pixels_out) {
        h->pixels = nullptr;
        (void)hipFree(h->b.rposes);
        (void)hipFree(h->b.rlist);
        (void)hipFree(h->b.rcount);
        (void)hipFree(h->b.rtable);
        h->b.rposes = nullptr;
        h->b.rlist = h->b.rcount = nullptr;
        h->b.rtable = nullptr;
        return 0;
    }
    if (!rc) return fail(h, "cp_set_raster: null config");
    if (h->cfg.autoreset == CP_AUTORESET_NEXT_STEP)
        return fail(h, "cp_set_raster: not for CP_AUTORESET_NEXT_STEP handles");
    const int R = h->cfg.action_repeats;
    if (rc->width <= 0 || rc->height <= 0 || rc->width > 4096 || rc->height > 4096)
        return fail(h, "cp_set_raster: width and height must be in 1..4096");
    if (rc->num_cameras != 1 && rc->num_cameras != 2) return fail(h, "--num-cameras must be 1 or 2");
    if (rc->num_cameras * R > cp::RMAX_FRAMES)
        return fail(h, "cp_set_raster: num_cameras * action_repeats must be <= 16");
    h->raster = *rc;
    h->pixels = pixels_out;
    if (!h->b.rposes) {
        const size_t B = (size_t)h->cfg.num_envs;
        hipError_t e = hipMalloc((void**)&h->b.rposes, B * R * CP_NUM_DYN * 7 * sizeof(float));
        if (e == hipSuccess) e = hipMalloc((void**)&h->b.rlist, B * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc((void**)&h->b.rcount, sizeof(int32_t));
        if (e != hipSuccess) {
            (void)hipFree(h->b.rposes);
            (void)hipFree(h->b.rlist);
            h->b.rposes = nullptr;
            h->b.rlist = nullptr;
            h->pixels = nullptr;
            return check(h, e, "cp_set_raster: hipMalloc");
        }
    }
    // per-camera ray table for this configuration (synchronous: a setup call)
    (void)hipFree(h->b.rtable);
    h->b.rtable = nullptr;
    const int npx = rc->width * rc->height;
    CP_TRY(h, hipMalloc((void**)&h->b.rtable, (size_t)rc->num_cameras * npx * 2 * sizeof(float4)));
    hipLaunchKernelGGL(cp::cp_raster_table_kernel, dim3(grid_for(npx, cp::RT), rc->num_cameras), dim3(cp::RT), 0, 0,
                       h->raster, h->cfg.phys, h->b.rtable,
                       reinterpret_cast<uint8_t*>(h->b.rtable + (size_t)rc->num_cameras * npx));
    CP_TRY(h, hipGetLastError());
    CP_TRY(h, hipDeviceSynchronize());
    return 0;
}

// ---------------------------------------------------------------- event log writer
}  // extern "C"

struct cp_eventlog {
    FILE* f = nullptr;
    std::vector<std::vector<uint8_t>> ep;  // open episode per env (encoded Episode body)
};

static int eventlog_flush(cp_eventlog* log, std::vector<uint8_t>& ep) {
    if (ep.empty()) return 0;
    const int32_t n = (int32_t)ep.size();  // struct.pack('=l', len(buff)), event_log.py:54
    if (std::fwrite(&n, sizeof(n), 1, log->f) != 1 || std::fwrite(ep.data(), 1, ep.size(), log->f) != ep.size())
        return fail(nullptr, "cp_eventlog: write failed");
    ep.clear();
    return 0;
}

extern "C" {

int cp_eventlog_open(const char* path, int num_envs, cp_eventlog** out) {
    if (!path || !out || num_envs <= 0) return fail(nullptr, "cp_eventlog_open: bad argument");
    cp_eventlog* log = new (std::nothrow) cp_eventlog();
    if (!log) return fail(nullptr, "cp_eventlog_open: out of memory");
    log->f = std::fopen(path, "ab");  // appends, as event_log.py:45
    if (!log->f) {
        delete log;
        return fail(nullptr, std::string("cp_eventlog_open: cannot open ") + path);
    }
    log->ep.resize((size_t)num_envs);
    *out = log;
    return 0;
}

int cp_eventlog_write(cp_eventlog* log, const uint8_t* flags, const uint8_t* step_records, int step_bytes,
                      const uint8_t* reset_records, int reset_bytes) {
    if (!log || !flags) return fail(nullptr, "cp_eventlog_write: null argument");
    for (size_t i = 0; i < log->ep.size(); ++i) {
        const uint8_t fl = flags[i];
        if ((fl & 1) && step_records) {
            const uint8_t* r = step_records + i * (size_t)step_bytes;
            log->ep[i].insert(log->ep[i].end(), r, r + step_bytes);
        }
        if ((fl & 2) && reset_records) {  // EventLog.reset + add_just_state (bullet_cartpole.py:342-344)
            if (eventlog_flush(log, log->ep[i])) return -1;
            const uint8_t* r = reset_records + i * (size_t)reset_bytes;
            log->ep[i].assign(r, r + reset_bytes);
        }
    }
    std::fflush(log->f);
    return 0;
}

int cp_eventlog_close(cp_eventlog* log) {
    if (!log) return fail(nullptr, "cp_eventlog_close: null handle");
    int rc = 0;
    for (auto& ep : log->ep)
        if (eventlog_flush(log, ep)) rc = -1;
    if (std::fclose(log->f) != 0) rc = fail(nullptr, "cp_eventlog_close: close failed");
    delete log;
    return rc;
}

int cp_get_stepped(cp_handle* h, uint8_t* out, void* stream) {
    if (!h || !out) return fail(h, "cp_get_stepped: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    CP_TRY(h, hipMemcpyAsync(out, h->b.stepped, h->cfg.num_envs, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

/* ---- replay memory (cp_replay.h) ---- */
static int replay_ok(const cp_replay* rm, const char* what) {
    if (!rm || !rm->state || !rm->state_1_idx || !rm->action || !rm->reward || !rm->terminal_mask ||
        !rm->state_2_idx || !rm->free_slots || !rm->ctrl || !rm->plan || !rm->scan)
        return fail(nullptr, std::string(what) + ": null replay buffer");
    if (rm->buffer_size < 1 || rm->state_dim < 1 || rm->action_dim < 1 ||
        rm->state_buffer_size < rm->buffer_size + rm->buffer_size / 2)
        return fail(nullptr, std::string(what) + ": bad sizes (state_buffer_size must be >= int(1.5 * buffer_size))");
    return 0;
}

int cp_replay_init(const cp_replay* rm, int32_t* cur, int rows, void* stream) {
    if (replay_ok(rm, "cp_replay_init")) return -1;
    if (rows < 0 || (rows > 0 && !cur)) return fail(nullptr, "cp_replay_init: bad rows / cur");
    const int64_t n = std::max<int64_t>(std::max<int64_t>(rm->state_buffer_size, rows), CP_RM_CTRL);
    hipLaunchKernelGGL(cprm::init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       *rm, cur, rows);
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

int cp_replay_add(const cp_replay* rm, int32_t* cur, int rows, const uint8_t* valid, const void* actions,
                  int action_kind, const float* reward, const uint8_t* done, const uint8_t* restart,
                  const void* next_states, const void* terminal_states, int state_kind, void* stream) {
    if (replay_ok(rm, "cp_replay_add")) return -1;
    if (rows < 0 || rows > rm->buffer_size) return fail(nullptr, "cp_replay_add: rows must be in [0, buffer_size]");
    if (rows == 0) return 0;
    if (!cur) return fail(nullptr, "cp_replay_add: null cur");
    if (valid && (!actions || !reward || !done || !next_states))
        return fail(nullptr, "cp_replay_add: events need actions, reward, done and next_states");
    if (restart && !next_states) return fail(nullptr, "cp_replay_add: restarts need next_states");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(nullptr, "cp_replay_add: bad action kind");
    if (state_kind != CP_STATES_F32 && state_kind != CP_STATES_F16)
        return fail(nullptr, "cp_replay_add: bad state kind");
    if (!valid && !restart) return 0;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 nb((unsigned)((rows + cprm::PLAN_THREADS - 1) / cprm::PLAN_THREADS)), nt(cprm::PLAN_THREADS);
    hipLaunchKernelGGL(cprm::count_kernel, nb, nt, 0, st, *rm, rows, valid);
    hipLaunchKernelGGL(cprm::free_count_kernel, nb, nt, 0, st, *rm, rows, valid, restart);
    hipLaunchKernelGGL(cprm::plan_kernel, nb, nt, 0, st, *rm, rows, valid, restart);
    switch (cprm::vec_for(rm->state_dim, state_kind)) {
        case 8: cprm::launch_write<8>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        case 4: cprm::launch_write<4>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        case 2: cprm::launch_write<2>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        default: cprm::launch_write<1>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                        terminal_states, state_kind, st);
    }
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

int cp_replay_sample(const cp_replay* rm, int n, const int32_t* idxs, uint64_t seed, uint64_t counter,
                     const cp_replay_batch* out, void* stream) {
    if (replay_ok(rm, "cp_replay_sample")) return -1;
    if (n < 0 || !out) return fail(nullptr, "cp_replay_sample: bad n / null out");
    if (n == 0) return 0;
    const int vec = cprm::vec_for(rm->state_dim, CP_STATES_F16);
    const int64_t threads = (int64_t)n * (rm->state_dim / vec);
    const dim3 grid((unsigned)((threads + 255) / 256));
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), c1 = (uint32_t)counter,
                   c2 = (uint32_t)(counter >> 32);
    const hipStream_t st = (hipStream_t)stream;
    switch (vec) {
        case 8: hipLaunchKernelGGL(cprm::sample_kernel<8>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        case 4: hipLaunchKernelGGL(cprm::sample_kernel<4>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        case 2: hipLaunchKernelGGL(cprm::sample_kernel<2>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        default: hipLaunchKernelGGL(cprm::sample_kernel<1>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out);
    }
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

}  // extern "C"
