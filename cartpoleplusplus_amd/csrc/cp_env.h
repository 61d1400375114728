// cp_env.h — the batched env's kernels over `real` (step, reset, init) and their host
// launchers; included once per real type after cp_math.h and cp_physics.h (cp_common.h):
// namespace cp (fp32, cp_kernels.hip) and cp64 (fp64, cp_kernels64.hip).
//
//   cp_step_kernel   R x S substeps fused in one launch; force applied after each
//                    substep (bullet_cartpole.py:199-207); obs at each repeat end
//                    (:237 -> :298-311); steps/done/reward (:239-260).  Finishing
//                    envs are appended to a reset list by wave ballot compaction.
//   cp_reset_kernel  spawn poses, 100 settle + 30 bump substeps (:313-346), over a
//                    compacted list of env ids (dense waves, no idle lanes).
//
// Memory: per-env state is SoA real [CP_STATE_FIELDS][B] in HBM (coalesced per field);
// inside a launch the env lives in VGPRs and its contact rows in a per-wave LDS pool
// (fp32: 20 KiB per wave, 8 waves per CU = 160 KiB).  Outputs (obs, terminal obs,
// readback, 8-states, raster poses) are float32 in both instantiations, as the reference's
// np.float32 state array (bullet_cartpole.py:148).  DESIGN.md §4-5.
#if !defined(CP_NS) || !defined(CP_REAL)
#error "define CP_NS and CP_REAL before including cp_env.h (see cp_kernels.hip)"
#endif

namespace CP_NS {

// occupancy target of the physics kernels (waves per SIMD); the register budget follows
#ifndef CP_WAVES_PER_EU
#define CP_WAVES_PER_EU 2
#endif

// fp64: only the 1-wave-per-SIMD (512 VGPR) kernel shape, with the slow-form rows (the fast
// form's precomputed rows do not fit twice the registers)
constexpr bool kF64 = sizeof(real) == 8;
// The throughput-shaped step / reset kernels rebuild the lane's SoA offsets (Mem) per substep and for the
// epilogue from an opaque env index instead of keeping the ones formed at the top live (round 5).  The
// step kernels take the all-inside face-contact exit (C3 kernel -0.6 %, C2 -2 %); the reset kernels' settle
// loops in the step kernel were measured slower and dropped.

using Bufs = cpc::Bufs;
using Lqr = cpc::Lqr;
using SoaF = SoaT<float>;

__constant__ float kDiscrete[CP_NUM_DISCRETE][2] = {{0.f, 0.f}, {-1.f, 0.f}, {1.f, 0.f}, {0.f, 1.f}, {0.f, -1.f}};

// raster obs: the repeat-end pose of the lane's own 2 bodies (xyz, quat xyzw) for the render kernel; dst is
// the env's [4][7] row, island p's lane writes bodies 2p, 2p + 1
CP_DEV void write_pose(const Body& B, float* o) {
    o[0] = (float)B.x.x; o[1] = (float)B.x.y; o[2] = (float)B.x.z;
    o[3] = (float)B.q[0]; o[4] = (float)B.q[1]; o[5] = (float)B.q[2]; o[6] = (float)B.q[3];
}
CP_DEV void write_rposes_own(const Own& O, int isl, float* dst) {
    float* o = dst + 2 * isl * 7;
    write_pose(O.c, o);
    write_pose(O.p, o + 7);
}

// per-wave stamp accumulation into b.stamps (lane 0 writes; CP_STAMPS builds only)
// Slots 11-15: the longest wave (cycles), and from the 100 MHz constant clock (s_memrealtime):
// the latest wave end, the complement of the earliest wave start, the sum and the max of the
// per-wave durations (the launch's wave-duration spread and the shader clock, tools/stamps.py).
CP_DEV void flush_stamps(const Stamps& ST, uint64_t* dst, uint64_t total, uint64_t rt0 = 0, uint64_t rt1 = 0,
                         const uint64_t* stamps_base = nullptr) {
#ifdef CP_STAMPS
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        atomicMax((unsigned long long*)&dst[11], (unsigned long long)total);
        atomicMax((unsigned long long*)&dst[12], (unsigned long long)rt1);
        atomicMax((unsigned long long*)&dst[13], (unsigned long long)~rt0);
        atomicAdd((unsigned long long*)&dst[14], (unsigned long long)(rt1 - rt0));
        atomicMax((unsigned long long*)&dst[15], (unsigned long long)(rt1 - rt0));
        if (dst == stamps_base) {  // the step kernel: wave count and duration per slow-path set
            // (slots 32-47) and a histogram of wave durations in 50 us bins (slots 48-63)
            atomicAdd((unsigned long long*)&dst[32 + 2 * ST.flags], 1ull);
            atomicAdd((unsigned long long*)&dst[33 + 2 * ST.flags], (unsigned long long)(rt1 - rt0));
            const uint64_t bin = (rt1 - rt0) / 5000u;
            atomicAdd((unsigned long long*)&dst[48 + (bin < 15u ? bin : 15u)], 1ull);
        }
        atomicAdd((unsigned long long*)&dst[0], (unsigned long long)ST.narrow);
        atomicAdd((unsigned long long*)&dst[1], (unsigned long long)ST.vel);
        atomicAdd((unsigned long long*)&dst[2], (unsigned long long)ST.solve);
        atomicAdd((unsigned long long*)&dst[3], (unsigned long long)ST.integ);
        atomicAdd((unsigned long long*)&dst[4], (unsigned long long)ST.sweeps);
        atomicAdd((unsigned long long*)&dst[5], (unsigned long long)ST.substeps);
        atomicAdd((unsigned long long*)&dst[6], (unsigned long long)total);
        atomicAdd((unsigned long long*)&dst[7], 1ull);
        if (ST.bb) {  // narrowphase split into the spare slots 8-10
            atomicAdd((unsigned long long*)&dst[8], (unsigned long long)ST.sel);
            atomicAdd((unsigned long long*)&dst[9], (unsigned long long)ST.bb);
            atomicAdd((unsigned long long*)&dst[10], (unsigned long long)ST.rows);
        }
    }
#else
    (void)ST; (void)dst; (void)total; (void)rt0; (void)rt1; (void)stamps_base;
#endif
}

// per-step outputs (obs rows, reward, done): written once, read by the caller after the launch.
template <typename T>
CP_DEV void put_out(T* p, T v) {
    *p = v;
}

// The lane's own island's fields of the state SoA: island p's bodies are dyn 2p, 2p + 1 (CP_SF_BODY(2p + k, c)),
// its cart's pending force CP_SF_PENDING(p, c), its sleep words CP_SF_SLEEP_*(2p + k).  The island part of
// the field index goes into the lane's buffer offset, so every field offset stays wave-uniform (SGPR soffset).
CP_DEV uint32_t isl_off(const Mem& G, int isl, int fields) { return G.off + (uint32_t)(isl * fields) * G.st.fstride; }
CP_DEV void load_body(Body& B, const Soa& st, int f0, uint32_t o) {
    B.x = mk(st.ld(f0 + 0, o), st.ld(f0 + 1, o), st.ld(f0 + 2, o));
#pragma unroll
    for (int k = 0; k < 4; ++k) B.q[k] = st.ld(f0 + 3 + k, o);
    B.v = mk(st.ld(f0 + 7, o), st.ld(f0 + 8, o), st.ld(f0 + 9, o));
    B.w = mk(st.ld(f0 + 10, o), st.ld(f0 + 11, o), st.ld(f0 + 12, o));
}
CP_DEV void store_body(const Body& B, const Soa& st, int f0, uint32_t o) {
    st.st(f0 + 0, o, B.x.x);
    st.st(f0 + 1, o, B.x.y);
    st.st(f0 + 2, o, B.x.z);
#pragma unroll
    for (int k = 0; k < 4; ++k) st.st(f0 + 3 + k, o, B.q[k]);
    st.st(f0 + 7, o, B.v.x);
    st.st(f0 + 8, o, B.v.y);
    st.st(f0 + 9, o, B.v.z);
    st.st(f0 + 10, o, B.w.x);
    st.st(f0 + 11, o, B.w.y);
    st.st(f0 + 12, o, B.w.z);
}
CP_DEV void load_own(Own& O, const Mem& G, int isl) {
    const uint32_t ob = isl_off(G, isl, 2 * CP_BODY_FIELDS), of = isl_off(G, isl, 3);
    load_body(O.c, G.st, CP_SF_BODY(0, 0), ob);
    load_body(O.p, G.st, CP_SF_BODY(1, 0), ob);
    O.f = mk(G.st.ld(CP_SF_PENDING(0, 0), of), G.st.ld(CP_SF_PENDING(0, 1), of), G.st.ld(CP_SF_PENDING(0, 2), of));
    O.wsm = 0u;  // the island's warm-start id words' point counts (pair_body)
#pragma unroll
    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) O.wsm |= ws_count(to_bits(G.lw(CP_SF_WS_ID(0, j)))) << (3 * j);
}
CP_DEV void store_own(const Own& O, const Mem& G, int isl) {
    const uint32_t ob = isl_off(G, isl, 2 * CP_BODY_FIELDS), of = isl_off(G, isl, 3);
    store_body(O.c, G.st, CP_SF_BODY(0, 0), ob);
    store_body(O.p, G.st, CP_SF_BODY(1, 0), ob);
    G.st.st(CP_SF_PENDING(0, 0), of, O.f.x);
    G.st.st(CP_SF_PENDING(0, 1), of, O.f.y);
    G.st.st(CP_SF_PENDING(0, 2), of, O.f.z);
}
// CP_MODEL_SLEEPING state of the lane's own bodies (SLP kernels only; the other models never touch these fields)
CP_DEV void load_sleep(Own& O, const Mem& G, int isl) {
    const uint32_t o = isl_off(G, isl, 2);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        O.sa[k] = to_bits(G.st.ld(CP_SF_SLEEP_ACT(k), o));
        O.st[k] = G.st.ld(CP_SF_SLEEP_TIMER(k), o);
    }
}
CP_DEV void store_sleep(const Own& O, const Mem& G, int isl) {
    const uint32_t o = isl_off(G, isl, 2);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        G.st.st(CP_SF_SLEEP_ACT(k), o, bits_to<real>(O.sa[k]));
        G.st.st(CP_SF_SLEEP_TIMER(k), o, O.st[k]);
    }
}
// the reset's pose of the lane's own bodies (resetBasePositionAndOrientation, bullet_cartpole.py:319-323)
template <int G0, int G1>
CP_DEV void spawn_body(Body& B, const cp_config& cfg, bool second) {
    B.x = mk(second ? real(cfg.phys.spawn_pos[G1][0]) : real(cfg.phys.spawn_pos[G0][0]),
             second ? real(cfg.phys.spawn_pos[G1][1]) : real(cfg.phys.spawn_pos[G0][1]),
             second ? real(cfg.phys.spawn_pos[G1][2]) : real(cfg.phys.spawn_pos[G0][2]));
    B.q[0] = real(0.0); B.q[1] = real(0.0); B.q[2] = real(0.0); B.q[3] = real(1.0);
    B.v = mk(real(0.0), real(0.0), real(0.0));
    B.w = mk(real(0.0), real(0.0), real(0.0));
}
CP_DEV void spawn_own(Own& O, const cp_config& cfg, bool second) {
    spawn_body<CP_BODY_CART, CP_BODY_CART2>(O.c, cfg, second);
    spawn_body<CP_BODY_POLE, CP_BODY_POLE2>(O.p, cfg, second);
}

CP_DEV int32_t ldi(const Soa& st, int f, uint32_t o) { return (int32_t)to_bits(st.ld(f, o)); }
CP_DEV void sti(const Soa& st, int f, uint32_t o, int32_t v) { st.st(f, o, bits_to<real>((uint32_t)v)); }

// true if every body value (pos, quat, v, w) of the lane's own bodies is finite: x * 0 is +-0 for a finite
// x and NaN for an inf or NaN, so the fma chain stays a zero exactly when all 26 values are finite
CP_DEV bool own_finite(const Own& O) {
    real acc = real(0.0);
    auto body = [&](const Body& y) {
        acc = fma_(y.x.x, real(0.0), acc); acc = fma_(y.x.y, real(0.0), acc); acc = fma_(y.x.z, real(0.0), acc);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = fma_(y.q[k], real(0.0), acc);
        acc = fma_(y.v.x, real(0.0), acc); acc = fma_(y.v.y, real(0.0), acc); acc = fma_(y.v.z, real(0.0), acc);
        acc = fma_(y.w.x, real(0.0), acc); acc = fma_(y.w.y, real(0.0), acc); acc = fma_(y.w.z, real(0.0), acc);
    };
    body(O.c);
    body(O.p);
    return acc == real(0.0);
}
// the whole env's finiteness on both lanes (DPP: both lanes of the pair active)
CP_DEV bool env_finite(const Own& O) {
    const uint32_t f = own_finite(O) ? 1u : 0u;
    return (f & partner_u(f)) != 0u;
}

// CP_RESET_CLEAR_NONFINITE_FORCE: a reset zeroes a cart's pending force with a non-finite component
CP_DEV V3 reset_force(const cp_config& cfg, V3 f) {
    if (!(cfg.reset_flags & CP_RESET_CLEAR_NONFINITE_FORCE)) return f;
    const real z = fma_(f.x, real(0.0), fma_(f.y, real(0.0), f.z * real(0.0)));
    return z == real(0.0) ? f : mk(real(0.0), real(0.0), real(0.0));
}

// obs row of a repeat (bullet_cartpole.py:298-311): cart and pole, island 0's own bodies (the lead lane's)
CP_DEV void write_obs_row(const Own& O, float* dst) {
    dst[0] = (float)O.c.x.x; dst[1] = (float)O.c.x.y; dst[2] = (float)O.c.x.z;
    dst[3] = (float)O.c.q[0]; dst[4] = (float)O.c.q[1]; dst[5] = (float)O.c.q[2]; dst[6] = (float)O.c.q[3];
    dst[7] = (float)O.p.x.x; dst[8] = (float)O.p.x.y; dst[9] = (float)O.p.x.z;
    dst[10] = (float)O.p.q[0]; dst[11] = (float)O.p.q[1]; dst[12] = (float)O.p.q[2];
    dst[13] = (float)O.p.q[3];
}

// 12-state pole readback (bullet_cartpole.py:212-229)
template <int POLE, int VEL>
CP_DEV void readback_pole(const Sim& S, float* dst) {
    const Body& p = S.b[POLE];
    const Body& vb = S.b[VEL];
    V3 rpy = quat_euler(p.q[0], p.q[1], p.q[2], p.q[3]);
    dst[0] = (float)p.x.x; dst[1] = (float)p.x.y; dst[2] = (float)p.x.z;
    dst[3] = (float)rpy.x; dst[4] = (float)rpy.y; dst[5] = (float)rpy.z;
    dst[6] = (float)vb.v.x; dst[7] = (float)vb.v.y; dst[8] = (float)vb.v.z;
    dst[9] = (float)vb.w.x; dst[10] = (float)vb.w.y; dst[11] = (float)vb.w.z;
}

// ---- closed-loop LQR policy (random_action_agent.py:60-135)
// pole 8-state of a pair (:121-135): x - x0, x', y, y', roll, roll', pitch, pitch'
CP_DEV void pole_state8(const Body& p, real x0, real s[8]) {
    const V3 rpy = quat_euler(p.q[0], p.q[1], p.q[2], p.q[3]);
    s[0] = p.x.x - x0; s[1] = p.v.x; s[2] = p.x.y; s[3] = p.v.y;
    s[4] = rpy.x; s[5] = p.w.x; s[6] = rpy.y; s[7] = p.w.y;
}

// u = -K s (:92-95, lqr zero point 0), accumulated k = 0..7 with fma
CP_DEV void lqr_u(const float* K, const real s[8], real& ux, real& uy) {
    real ax = real(0.0), ay = real(0.0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ax = fma_(real(K[k]), s[k], ax);
        ay = fma_(real(K[8 + k]), s[k], ay);
    }
    ux = -ax;
    uy = -ay;
}

CP_DEV bool lqr_out_of_bounds(const real s[8], real pos, real ang) {
    return abs_(s[0]) > pos || abs_(s[2]) > pos || abs_(s[4]) > ang || abs_(s[6]) > ang;
}

// the lane's own pair (island p's lane: pole p, cart p): its 8-state (written to s8_out[8 p ..] when given)
// -> the next control force u of its cart; true on both lanes if both pairs are out of bounds (:908).
// Both lanes of the env active (DPP).
CP_DEV bool lqr_observe(const Own& O, bool second, const cp_config& cfg, const Lqr& q, const float* K, real u[2],
                        float* s8_out) {
    real s[8];
    pole_state8(O.p, real(cfg.phys.spawn_pos[second ? CP_BODY_POLE2 : CP_BODY_POLE][0]), s);
    if (s8_out)
        for (int k = 0; k < 8; ++k) s8_out[(second ? 8 : 0) + k] = (float)s[k];
    lqr_u(K + (second ? 16 : 0), s, u[0], u[1]);
    const uint32_t out = lqr_out_of_bounds(s, real(q.done_pos), real(q.done_angle)) ? 1u : 0u;
    return q.done_pos > 0.0f && (out & partner_u(out)) != 0u;
}

// commented-out bounds check of the reference (:243-253), on the pole pose (island 0's lane's own pole)
CP_DEV bool bounds_exceeded_pole(const Body& p, const cp_config& cfg) {
    if (abs_(p.x.x) > real(cfg.pos_threshold) || abs_(p.x.y) > real(cfg.pos_threshold)) return true;
    real qx = p.q[0], qy = p.q[1], qz = p.q[2], qw = p.q[3];
    real Y = real(2.0) * fma_(qy, qz, qw * qx);
    real X = ((qw * qw - qx * qx) - qy * qy) + qz * qz;
    bool roll_out = (X > real(0.0)) ? (abs_(Y) > X * real(cfg.tan_angle_threshold)) : !(X == real(0.0) && Y == real(0.0));
    real sarg = real(-2.0) * fma_(qx, qz, -(qw * qy));
    bool pitch_out = abs_(sarg) > real(cfg.sin_angle_threshold);
    return roll_out || pitch_out;
}
// the env's bounds decision on both lanes: island 0's lane's pole (DPP broadcast; both lanes active)
CP_DEV bool bounds_exceeded(const Own& O, const cp_config& cfg) {
    return lane_of_u<0>(bounds_exceeded_pole(O.p, cfg) ? 1u : 0u) != 0u;
}

// Bump force k on cart C (LINK frame), bullet_cartpole.py:354-359
// (host mode: the forces in the handle's real type, so an fp64 handle gets the reference's doubles)
CP_DEV void bump_force(const cp_config& cfg, const void* bumps, int i, int episode, int k, int c, real& fx,
                       real& fy) {
    if (cfg.bump_mode == CP_BUMP_HOST) {
        const real* f = static_cast<const real*>(bumps) + (((size_t)i * cfg.initial_force_steps + k) * 2 + c) * 2;
        fx = f[0];
        fy = f[1];
        return;
    }
    const real F = cfg.initial_force;
    if (!cfg.random_theta) {
        fx = F;
        fy = F * real(0.0);
        return;
    }
    uint32_t idx = (uint32_t)(2 * k + c);
    uint64_t gid = (uint64_t)(cfg.env_id_offset + i);
    uint32_t w = philox_word(idx >> 2, (uint32_t)episode, (uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)cfg.seed,
                             (uint32_t)(cfg.seed >> 32), (int)(idx & 3u));
    real u = real(w >> 8) * real(5.9604644775390625e-08);
    real s, co;
    sincos_turns(u, s, co);
    fx = F * co;
    fy = F * s;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cp_init_kernel(cp_config cfg, Bufs b) {
    const int B = cfg.num_envs;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const Soa st = Soa::make(b.state, B, CP_STATE_FIELDS);
    const uint32_t o = Soa::eoff(i);
    for (int f = 0; f < CP_STATE_FIELDS; ++f) st.st(f, o, real(0.0));
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
#pragma unroll
        for (int k = 0; k < 3; ++k) st.st(CP_SF_BODY(d, k), o, real(cfg.phys.spawn_pos[d + 1][k]));
        st.st(CP_SF_BODY(d, 6), o, real(1.0));
    }
#pragma unroll
    for (int p = 0; p < CP_NUM_ISLANDS; ++p)
#pragma unroll
        for (int j = 0; j < CP_ISLAND_PAIRS; ++j) sti(st, CP_SF_WS_ID(p, j), o, -1);
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) sti(st, CP_SF_SLEEP_ACT(d), o, CP_ACT_ACTIVE | CP_ACT_AWAKE);
    sti(st, CP_SF_DONE, o, 1);  // not reset yet: reference raises, batched API reports done
    b.ret_acc[i] = 0.0f;
    b.last_ret[i] = 0.0f;
    b.last_len[i] = 0;
    b.overflow[i] = 0;
    b.nonfinite[i] = 0;
}

// LAT = false: the throughput shape of the step kernel (2 waves per SIMD), for reset bursts
// (fixed-length episodes end together).  LAT = true: one wave per SIMD with 512 registers and
// fast-form rows, for the short lists of desynchronised episodes (bounds termination), where
// the 130 serial substeps of one wave are the whole latency of the step.
// WIDE (latency shape only): 16 (or 8) lanes per env, 8 (4) replicas of the env's lane pair that divide the
// narrowphase (narrow_wide, cp_physics.h); lane 0 of the env's lanes is the lead, lanes 0-1 store the state.
template <bool LAT, bool PM = false, bool SLP = false, int WIDE = 0>
__global__ void __launch_bounds__(WAVE)
__attribute__((amdgpu_waves_per_eu(LAT ? 1 : CP_WAVES_PER_EU, LAT ? 1 : CP_WAVES_PER_EU)))
cp_reset_kernel(cp_config cfg, Bufs b, float* obs_out) {
    static_assert(!WIDE || (LAT && !PM && !SLP), "WIDE: latency shape, default contact model");
    constexpr int LW = WIDE ? WIDE : 2;  // lanes per env
    __shared__ real lds_pool[(PM ? POOL_FLOATS_PM : POOL_FLOATS) * WAVE];
    const int B = cfg.num_envs;
    const int t = blockIdx.x * WAVE + threadIdx.x;
    if (t == 0 && b.count_next) *b.count_next = 0;  // the next cp_step's list starts empty
    const int n = *b.count;
    if (n <= b.nlo || (b.nhi > 0 && n > b.nhi)) return;  // CP_SHAPE_LIST: another layout's range of list lengths
    if ((t / LW) >= n) return;  // envs past the compacted list
    const int isl = t & 1;
    const bool lead = (t & (LW - 1)) == 0;
    const bool owner = (t & (LW - 1)) < 2;  // the lane pair that stores the env's state (WIDE: replica 0)
    const int i = b.list[t / LW];
    // the env index through an opaque copy where the substeps and the epilogue address the state: the
    // lane's SoA offsets are rebuilt there instead of living through the 130 substeps (cp_step_kernel)
    auto late_i = [&]() {
        int x = i;
        asm volatile("" : "+v"(x));
        return x;
    };
    // WIDE: the replicas of an island share its pool column (the replica-0 lane's)
    real* pool0 = lds_pool + (threadIdx.x & ~(LW - 1u));
    real* pool = WIDE ? pool0 + isl : lds_pool + threadIdx.x;
    const Mem G = Mem::make(b.state, b.scratch, B, i, isl, b.pman);
    Lane L = Lane::make(isl, cfg.phys);
    L.pj = (int)((t & (LW - 1)) >> 1);
    Stamps ST;
    CP_STAMP(k0);
    CP_RT(r0);
    const bool second = isl != 0;
    Own O;
    load_own(O, G, isl);  // pending forces survive the reset (pybullet keeps them)
    O.f = reset_force(cfg, O.f);
    if constexpr (PM)  // resetBasePositionAndOrientation: no cached contact survives the teleport
        for (int j = 0; j < CP_ISLAND_PAIRS; ++j) G.sp(pmf(j, 0), bits_to<real>(0u));
    const int episode = ldi(G.st, CP_SF_EPISODE, G.off);
    spawn_own(O, cfg, second);
    if constexpr (SLP) sleep_wake_all(O);  // the teleported bodies are awake
#pragma unroll
    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {  // the lane's island's warm-start cache
        G.sw(CP_SF_WS_ID(0, j), bits_to<real>(0xFFFFFFFFu));
#pragma unroll
        for (int k = 0; k < 4; ++k) G.sl(CP_SF_WS_LAM(0, j, k), real(0.0));
    }
    O.wsm = 0u;
    int ov = 0;
    const int nsub = cfg.settle_steps + cfg.initial_force_steps;
    for (int s = 0; s < nsub; ++s) {
        const Mem Gs = (LAT && !kF64) ? G : Mem::make(b.state, b.scratch, B, late_i(), isl, b.pman);
        substep<LAT && !kF64, true, true, PM, SLP, WIDE>(O, cfg.phys, L, pool, pool0, ov, Gs, ST);
        const int k = s - cfg.settle_steps;
        if (k >= 0) {  // bump the lane's own cart (cart, then cart2 in the reference's draw order)
            real fx, fy;
            bump_force(cfg, b.bumps, i, episode, k, isl, fx, fy);
            apply_force_link(O, fx, fy);
        }
    }
    ov += (int)partner_u((uint32_t)ov);
#ifdef CP_STAMPS
    CP_STAMP(k1);
    CP_RT(r1);
    flush_stamps(ST, b.stamps + 16, k1 - k0, r0, r1);  // the reset kernel's counters: slots 16-26
#endif
    const Mem Ge = (LAT && !kF64) ? G : Mem::make(b.state, b.scratch, B, late_i(), isl, b.pman);
    const int il = late_i();
    if (owner) store_own(O, Ge, isl);  // each lane stores its own island
    if constexpr (SLP) store_sleep(O, Ge, isl);
    const bool fin = env_finite(O);
    const int R = cfg.action_repeats;
    if (b.rposes && owner)  // every repeat slot shows the reset pose (bullet_cartpole.py:342-345)
        for (int r = 0; r < R; ++r) write_rposes_own(O, isl, b.rposes + ((size_t)il * R + r) * CP_NUM_DYN * 7);
    if (!lead) return;
    b.overflow[il] += ov;
    if (!fin) b.nonfinite[il] += 1;
    float row[14];
    write_obs_row(O, row);
    float* o = obs_out + (size_t)il * R * 14;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int f = 0; f < 14; ++f) o[r * 14 + f] = row[f];
    sti(Ge.st, CP_SF_STEPS, Ge.off, 0);
    if (!b.keep_done) sti(Ge.st, CP_SF_DONE, Ge.off, 0);  // NEXT_STEP in flight: the fixup kernel clears it
    sti(Ge.st, CP_SF_EPISODE, Ge.off, episode + 1);
    b.ret_acc[il] = 0.0f;
}

// LAT: the latency shape of cp_reset_kernel<true> (1 wave per SIMD, 512 registers, fast-form
// rows) for batches whose waves all get a SIMD of their own (<= 32,768 envs).  WIDE: the latency shape on
// 16 lanes per env (cp_reset_kernel), for batches that leave most SIMDs idle.
template <int KIND, bool LQR, bool LAT, bool PM = false, bool SLP = false, int WIDE = 0>
__global__ void __launch_bounds__(WAVE)
__attribute__((amdgpu_waves_per_eu(LAT ? 1 : CP_WAVES_PER_EU, LAT ? 1 : CP_WAVES_PER_EU)))
cp_step_kernel(cp_config cfg, Bufs b, const void* actions, float* obs_out, float* reward_out, uint8_t* done_out,
               float* term_out, float* readback, int rb_bug, Lqr lq) {
    static_assert(!WIDE || (LAT && !PM && !SLP), "WIDE: latency shape, default contact model");
    constexpr int LW = WIDE ? WIDE : 2;  // lanes per env
    __shared__ real lds_pool[(PM ? POOL_FLOATS_PM : POOL_FLOATS) * WAVE];
    const int B = cfg.num_envs;
    const int t = blockIdx.x * WAVE + threadIdx.x;
    // the next call's reset-list counter (the reset kernel zeroes it too): cp_step launches no reset
    // kernel on calls where no episode can end (cp_kernels.hip may_finish)
    if (t == 0 && b.count_next) *b.count_next = 0;
    const int i = t / LW, isl = t & 1;
    const bool lead = (t & (LW - 1)) == 0;  // lane 0 of the env's lanes writes the env's outputs
    const bool owner = (t & (LW - 1)) < 2;  // the lane pair that stores the env's state (WIDE: replica 0)
    const bool inb = i < B;
    const int R = cfg.action_repeats, SR = cfg.steps_per_repeat;
    // WIDE: the replicas of an island share its pool column (the replica-0 lane's)
    real* pool0 = lds_pool + (threadIdx.x & ~(LW - 1u));
    real* pool = WIDE ? pool0 + isl : lds_pool + threadIdx.x;
    bool want_reset = false;
    bool render_me = false;  // simulated this step: its frames go to the render kernel
    Stamps ST;
    // the env index through an opaque register copy where the outputs are addressed after the substeps: the
    // 64-bit per-lane addresses formed once at the top otherwise live through the substep loop (spilled: the
    // step kernel's scratch frame, written at the top and read back at the end of every launch)
    auto late_i = [&]() {
        int x = i;
        asm volatile("" : "+v"(x));
        return x;
    };
    // the lane's island (lane parity) recomputed from the lane id where the late offsets need it (a kept copy
    // and the island offsets derived from it were spilled)
    auto late_isl = [&]() {
        return (int)(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 1u);
    };
    CP_STAMP(k0);
    CP_RT(r0);
    if (inb) {
        const Mem G = Mem::make(b.state, b.scratch, B, i, isl, b.pman);
        Lane L = Lane::make(isl, cfg.phys);
        L.pj = (int)((t & (LW - 1)) >> 1);
        const SoaF term = SoaF::make(b.term_obs, B, R * 14);
        const uint32_t toff = SoaF::eoff(i);
        float* obs = obs_out + (size_t)i * R * 14;
        const int done_field = ldi(G.st, CP_SF_DONE, G.off);
        const bool was_done = done_field != 0;
        if (lead) b.stepped[i] = was_done ? 0 : 1;
        if (cfg.autoreset == CP_AUTORESET_NEXT_STEP && done_field >= 2) {
            // finished in the previous call, reset on the library's second stream: this call's
            // outputs for it come from cp_nextstep_fixup_kernel, its action is ignored
        } else if (was_done) {  // step after done (bullet_cartpole.py:179-181)
            if (lead) {
                for (int f = 0; f < R * 14; ++f) obs[f] = term.ld(f, toff);
                reward_out[i] = 0.0f;
                done_out[i] = 1;
            }
        } else {
            real a00, a01, a10, a11;
            if constexpr (KIND == CP_ACTION_CONTINUOUS) {
                const float4 a = reinterpret_cast<const float4*>(actions)[i];
                a00 = a.x; a01 = a.y; a10 = a.z; a11 = a.w;
            } else {
                const char2 a = reinterpret_cast<const char2*>(actions)[i];
                int k0 = a.x, k1 = a.y;
                k0 = (k0 < 0 || k0 >= CP_NUM_DISCRETE) ? 0 : k0;
                k1 = (k1 < 0 || k1 >= CP_NUM_DISCRETE) ? 0 : k1;
                a00 = kDiscrete[k0][0]; a01 = kDiscrete[k0][1];
                a10 = kDiscrete[k1][0]; a11 = kDiscrete[k1][1];
            }
            const real F = cfg.action_force;
            const bool second = isl != 0;
            // the lane's own cart's action force (action[0] -> cart, action[1] -> cart2, :201-207)
            const real fa = (second ? a10 : a00) * F, fb = (second ? a11 : a01) * F;
            Own O;
            load_own(O, G, isl);
            if constexpr (SLP) load_sleep(O, G, isl);
            int ov = 0;
            real u[2] = {real(0.0), real(0.0)};  // LQR force of the own cart from the last observed state
            bool lqr_done = false;
            const float* K = nullptr;
            if constexpr (LQR) {
                K = lq.gains + (lq.per_env ? (size_t)i * 32 : 0);
                lqr_observe(O, second, cfg, lq, K, u, nullptr);
            }
            for (int r = 0; r < R; ++r) {
                for (int s = 0; s < SR; ++s) {
                    // the throughput shape: the lane's SoA offsets rebuilt per substep from the opaque index (not live
                    // through the loop; scratch 48 -> 24 B/lane); the 0-scratch latency kernels keep G (a lone wave
                    // pays the rebuild: latency reset list +2.6 %)
                    const Mem Gs = (LAT && !kF64) ? G : Mem::make(b.state, b.scratch, B, late_i(), late_isl(), b.pman);
                    substep<LAT && !kF64, false, true, PM, SLP, WIDE>(O, cfg.phys, L, pool, pool0, ov, Gs, ST);
                    if constexpr (LQR) {  // disturbance + control (:897-901), control from the pre-step state
                        apply_force_link(O, fa + u[0], fb + u[1]);
                        float* s8 = (lq.state8 && owner) ? lq.state8 + (((size_t)i * R + r) * SR + s) * 16 : nullptr;
                        lqr_done |= lqr_observe(O, second, cfg, lq, K, u, s8);
                    } else {
                        apply_force_link(O, fa, fb);
                    }
                    if (readback) {  // 12-states of both poles: the whole env on both lanes (DPP), the lead writes
                        const Sim V = env_view(O);
                        if (lead) {
                            float* rb = readback + (size_t)late_i() * 2 * R * SR * 12;
                            readback_pole<1, 1>(V, rb + ((size_t)(0 * R + r) * SR + s) * 12);
                            if (rb_bug) readback_pole<3, 1>(V, rb + ((size_t)(1 * R + r) * SR + s) * 12);
                            else readback_pole<3, 3>(V, rb + ((size_t)(1 * R + r) * SR + s) * 12);
                        }
                    }
                }
                if (lead) {
                    float row[14];
                    write_obs_row(O, row);
                    float* orow = obs_out + ((size_t)late_i() * R + r) * 14;
#pragma unroll
                    for (int f = 0; f < 14; ++f) put_out(&orow[f], row[f]);
                }
                if (b.rposes && owner) write_rposes_own(O, isl, b.rposes + ((size_t)late_i() * R + r) * CP_NUM_DYN * 7);
            }
            render_me = lead && b.rposes != nullptr;
            ov += (int)partner_u((uint32_t)ov);
            const int il = late_i();
            if (ov && lead) b.overflow[il] += ov;
            const int isle = (LAT && !kF64) ? isl : late_isl();
            const Mem Ge = (LAT && !kF64) ? G : Mem::make(b.state, b.scratch, B, il, isle, b.pman);
            const int steps = ldi(Ge.st, CP_SF_STEPS, Ge.off) + 1;
            bool done = steps >= cfg.max_episode_len;
            if (cfg.done_on_bounds && bounds_exceeded(O, cfg)) done = true;
            if (LQR && lqr_done) done = true;
            if (owner) store_own(O, Ge, isle);  // each lane stores its own island
            if constexpr (SLP) store_sleep(O, Ge, isle);
            const bool fin = env_finite(O);
            if (lead) {
                if (!fin) b.nonfinite[il] += 1;
                sti(Ge.st, CP_SF_STEPS, Ge.off, steps);
                put_out(&reward_out[il], 1.0f);  // bullet_cartpole.py:260
                put_out(&done_out[il], (uint8_t)(done ? 1 : 0));
                const float ret = b.ret_acc[il] + 1.0f;
                if (done) {
                    b.last_ret[il] = ret;
                    b.last_len[il] = steps;
                    b.ret_acc[il] = 0.0f;
                    const float* obs_l = obs_out + (size_t)il * R * 14;
                    const uint32_t toff_l = SoaF::eoff(il);
                    for (int f = 0; f < R * 14; ++f) term.st(f, toff_l, obs_l[f]);
                    if (term_out)
                        for (int f = 0; f < R * 14; ++f) term_out[(size_t)il * R * 14 + f] = obs_l[f];
                    sti(Ge.st, CP_SF_DONE, Ge.off, cfg.autoreset == CP_AUTORESET_NEXT_STEP ? 2 + b.npar : 1);
                    want_reset = cfg.autoreset != 0;
                } else {
                    b.ret_acc[il] = ret;
                }
            }
        }
    }
#ifdef CP_STAMPS
    CP_STAMP(k1);
    CP_RT(r1);
    flush_stamps(ST, b.stamps, k1 - k0, r0, r1, b.stamps);
#endif
    if (cfg.autoreset) {
        // wave ballot compaction of the finishing envs into the reset list
        const uint64_t bal = __ballot(want_reset);
        const int lane = threadIdx.x;  // want_reset is set on lead lanes only
        const int n = __popcll(bal);
        int base = 0;
        if (lane == 0 && n) base = atomicAdd(b.count, n);
        base = __shfl(base, 0);
        if (want_reset) b.list[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    }
    if (b.rposes) {
        const uint64_t bal = __ballot(render_me);
        const int lane = threadIdx.x & (WAVE - 1);
        const int n = __popcll(bal);
        int base = 0;
        if (lane == 0 && n) base = atomicAdd(b.rcount, n);
        base = __shfl(base, 0);
        if (render_me) b.rlist[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    }
}

// One env-step's action forces, action_force * action (bullet_cartpole.py:201-207): continuous
// float4 (a00 a01 a10 a11) or discrete int8 x 2 through kDiscrete (out-of-range index = 0).
template <int KIND>
CP_DEV void action_forces(const void* actions, size_t row, real F, real f[4]) {
    real a00, a01, a10, a11;
    if constexpr (KIND == CP_ACTION_CONTINUOUS) {
        const float4 a = reinterpret_cast<const float4*>(actions)[row];
        a00 = a.x; a01 = a.y; a10 = a.z; a11 = a.w;
    } else {
        const char2 a = reinterpret_cast<const char2*>(actions)[row];
        int k0 = a.x, k1 = a.y;
        k0 = (k0 < 0 || k0 >= CP_NUM_DISCRETE) ? 0 : k0;
        k1 = (k1 < 0 || k1 >= CP_NUM_DISCRETE) ? 0 : k1;
        a00 = kDiscrete[k0][0]; a01 = kDiscrete[k0][1];
        a10 = kDiscrete[k1][0]; a11 = kDiscrete[k1][1];
    }
    f[0] = a00 * F; f[1] = a01 * F; f[2] = a10 * F; f[3] = a11 * F;
}

// cp_rollout: K consecutive env-steps of every env in one launch, bit for bit the outputs and
// final state of K cp_step calls (bullet_cartpole.py:178-275 K times, each finishing episode
// reset in its step, :313-346).  Each lane pair runs a state machine over substeps:
//   STEP   the R x S substeps of step k, each followed by the step's action forces (+ LQR),
//          obs at each repeat end, reward / done at the end;
//   RESET  (autoreset of an episode that ended in step k) spawn poses, settle + bump substeps;
//          its obs are step k's obs, the finishing obs step k's terminal obs.
// Every lane with work runs ONE substep per loop trip whatever its phase, so an env that resets
// costs its own 130 substeps instead of stalling the wave's other envs at a step boundary, and a
// wave no longer waits for the slowest wave of the grid between steps.  The substep variant is
// the step kernel's (the reset kernel's C44 / ALLIN options compute the same numbers).  The
// episode counters live in registers for the whole launch (both lanes of a pair hold identical
// copies: no cross-lane memory traffic) and are written back once at the end.
// The state machine's cold per-lane values (step index, substep, counters, flags, LQR forces)
// are kept in the lane's column of the scratch SoA between substeps (Mem::lx / sx: coalesced,
// L2-resident, each lane reads only its own writes) rather than in registers across the
// substep, whose peak register pressure they would add to; the action forces are re-read
// from the action array after each substep.
enum : int { RC_K = CP_SCR_RC_BASE, RC_SUB, RC_STEPS, RC_EPISODE, RC_FLAGS, RC_RET, RC_U0, RC_U1, RC_U2, RC_U3, RC_END };
enum : uint32_t { RF_DONE = 1u, RF_RESETTING = 2u, RF_LAST_SIM = 4u, RF_LQR_DONE = 8u };
static_assert(RC_END - RC_K == CP_SCR_RC_FIELDS, "rollout state rows of the scratch SoA (cp_common.h)");
static_assert(RC_K >= CP_SCR_HDR_FIELDS, "rollout state must not overlap the CP_HDR_SCRATCH manifold headers");

template <int KIND, bool LQR, bool LAT, bool PM = false, bool SLP = false>
__global__ void __launch_bounds__(WAVE)
__attribute__((amdgpu_waves_per_eu(LAT ? 1 : CP_WAVES_PER_EU, LAT ? 1 : CP_WAVES_PER_EU)))
cp_rollout_kernel(cp_config cfg, Bufs b, int K, const void* actions, float* obs_out, float* reward_out,
                  uint8_t* done_out, float* term_out, Lqr lq) {
    __shared__ real lds_pool[(PM ? POOL_FLOATS_PM : POOL_FLOATS) * WAVE];
    const int B = cfg.num_envs;
    const int t = blockIdx.x * WAVE + threadIdx.x;
    const int i = t >> 1, isl = t & 1;
    if (i >= B) return;  // whole lane pairs (B envs = 2B lanes)
    const bool lead = isl == 0;
    const int R = cfg.action_repeats, SR = cfg.steps_per_repeat, RS = R * SR;
    const int nreset = cfg.settle_steps + cfg.initial_force_steps;
    real* pool = lds_pool + threadIdx.x;
    real* pool0 = lds_pool + (threadIdx.x & ~1u);
    const Mem G = Mem::make(b.state, b.scratch, B, i, isl, b.pman);
    const Lane L = Lane::make(isl, cfg.phys);
    const SoaF term = SoaF::make(b.term_obs, B, R * 14);
    const size_t obs_step = (size_t)B * R * 14;
    // the env index through an opaque register copy wherever the loop body forms an address: the
    // 64-bit per-lane addresses are otherwise hoisted out of the substep loop and spilled
    auto env = [&]() { uint32_t v = (uint32_t)i; asm volatile("" : "+v"(v)); return (size_t)v; };
    auto ldc = [&](int f) { return (int)to_bits(G.lx(f)); };
    auto stc = [&](int f, int v) { G.sx(f, bits_to<real>((uint32_t)v)); };
    auto ldu = [&](int f) { return G.lx(f); };
    Stamps ST;
    const bool second = isl != 0;
    Own O;
    load_own(O, G, isl);
    if constexpr (SLP) load_sleep(O, G, isl);
    int ov = 0;
    real u[2];  // the own cart's LQR force
    // the next simulated step from k on: steps of an env that is done before them only return its
    // last obs, reward 0, done 1 (:179-181); writes the cold state; false when the K steps are over
    auto begin_step = [&](int k, int steps, int episode, uint32_t flags, float ret_acc) -> bool {
        for (; k < K && (flags & RF_DONE); ++k) {
            flags &= ~RF_LAST_SIM;
            if (lead) {
                const size_t e = env();
                float* o = obs_out + (size_t)k * obs_step + e * R * 14;
                for (int q = 0; q < R * 14; ++q) o[q] = term.ld(q, SoaF::eoff((int)e));
                reward_out[(size_t)k * B + e] = 0.0f;
                done_out[(size_t)k * B + e] = 1;
            }
        }
        const bool more = k < K;
        if (more) {
            flags |= RF_LAST_SIM;
            if constexpr (LQR) {
                flags &= ~RF_LQR_DONE;
                lqr_observe(O, second, cfg, lq, lq.gains + (lq.per_env ? (size_t)i * 32 : 0), u, nullptr);
                G.sx(RC_U0, u[0]); G.sx(RC_U1, u[1]);
            }
        }
        stc(RC_K, k); stc(RC_SUB, 0); stc(RC_STEPS, steps); stc(RC_EPISODE, episode); stc(RC_FLAGS, (int)flags);
        G.sx(RC_RET, bits_to<real>(__float_as_uint(ret_acc)));
        return more;
    };
    bool work = begin_step(0, ldi(G.st, CP_SF_STEPS, G.off), ldi(G.st, CP_SF_EPISODE, G.off),
                           ldi(G.st, CP_SF_DONE, G.off) != 0 ? RF_DONE : 0u, b.ret_acc[i]);
    while (__ballot(work) != 0ull) {
        if (!work) continue;
        substep<LAT && !kF64, false, true, PM, SLP>(O, cfg.phys, L, pool, pool0, ov, G, ST);
        int k = ldc(RC_K), sub = ldc(RC_SUB);
        uint32_t flags = (uint32_t)ldc(RC_FLAGS);
        if (!(flags & RF_RESETTING)) {
            real f[4];
            const size_t e = env();
            action_forces<KIND>(actions, (size_t)k * B + e, real(cfg.action_force), f);
            const real fa = second ? f[2] : f[0], fb = second ? f[3] : f[1];  // the own cart's force
            if constexpr (LQR) {
                u[0] = ldu(RC_U0); u[1] = ldu(RC_U1);
                apply_force_link(O, fa + u[0], fb + u[1]);
                if (lqr_observe(O, second, cfg, lq, lq.gains + (lq.per_env ? (size_t)i * 32 : 0), u, nullptr))
                    flags |= RF_LQR_DONE;
                G.sx(RC_U0, u[0]); G.sx(RC_U1, u[1]);
            } else {
                apply_force_link(O, fa, fb);
            }
            ++sub;
            float* obs = obs_out + (size_t)k * obs_step + e * R * 14;
            if (lead && sub % SR == 0) {
                float row[14];
                write_obs_row(O, row);
                const int r = sub / SR - 1;
#pragma unroll
                for (int q = 0; q < 14; ++q) put_out(&obs[r * 14 + q], row[q]);
            }
            if (sub < RS) {
                stc(RC_SUB, sub);
                if (LQR) stc(RC_FLAGS, (int)flags);
                continue;
            }
            // step end (the step kernel's epilogue)
            const int steps = ldc(RC_STEPS) + 1;
            const int episode = ldc(RC_EPISODE);
            bool done = steps >= cfg.max_episode_len;
            if (cfg.done_on_bounds && bounds_exceeded(O, cfg)) done = true;
            if (LQR && (flags & RF_LQR_DONE)) done = true;
            const float ret = __uint_as_float(to_bits(G.lx(RC_RET))) + 1.0f;
            const bool fin = env_finite(O);
            if (lead) {
                if (!fin) b.nonfinite[e] += 1;
                put_out(&reward_out[(size_t)k * B + e], 1.0f);
                put_out(&done_out[(size_t)k * B + e], (uint8_t)(done ? 1 : 0));
            }
            if (done) {
                if (lead) {
                    b.last_ret[e] = ret;
                    b.last_len[e] = steps;
                    for (int q = 0; q < R * 14; ++q) term.st(q, SoaF::eoff((int)e), obs[q]);
                    if (term_out)
                        for (int q = 0; q < R * 14; ++q) term_out[(size_t)k * obs_step + e * R * 14 + q] = obs[q];
                }
                flags |= RF_DONE;
                if (cfg.autoreset) {  // the reset kernel's prologue: pending forces survive
                    O.f = reset_force(cfg, O.f);
                    spawn_own(O, cfg, second);
                    if constexpr (SLP) sleep_wake_all(O);
#pragma unroll
                    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {
                        G.sw(CP_SF_WS_ID(0, j), bits_to<real>(0xFFFFFFFFu));
#pragma unroll
                        for (int q = 0; q < 4; ++q) G.sl(CP_SF_WS_LAM(0, j, q), real(0.0));
                        if constexpr (PM) G.sp(pmf(j, 0), bits_to<real>(0u));
                    }
                    O.wsm = 0u;
                    stc(RC_SUB, 0);
                    stc(RC_STEPS, steps);
                    stc(RC_FLAGS, (int)(flags | RF_RESETTING));
                    G.sx(RC_RET, bits_to<real>(__float_as_uint(0.0f)));
                    continue;
                }
            }
            work = begin_step(k + 1, steps, episode, flags, done ? 0.0f : ret);
        } else {
            const int kb = sub - cfg.settle_steps;
            if (kb >= 0) {
                const int episode = ldc(RC_EPISODE);
                real fx, fy;
                const int e = (int)env();
                bump_force(cfg, b.bumps, e, episode, kb, isl, fx, fy);  // the own cart's bump
                apply_force_link(O, fx, fy);
            }
            if (++sub < nreset) {
                stc(RC_SUB, sub);
                continue;
            }
            // reset end (the reset kernel's epilogue): every repeat slot shows the new pose
            const bool fin = env_finite(O);
            if (lead) {
                if (!fin) b.nonfinite[env()] += 1;
                float row[14];
                write_obs_row(O, row);
                float* o = obs_out + (size_t)k * obs_step + env() * R * 14;
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int q = 0; q < 14; ++q) o[r * 14 + q] = row[q];
            }
            work = begin_step(k + 1, 0, ldc(RC_EPISODE) + 1, flags & ~(RF_DONE | RF_RESETTING), 0.0f);
        }
    }
    ov += (int)partner_u((uint32_t)ov);  // both lanes of every pair are here
    store_own(O, G, isl);  // each lane stores its own island
    if constexpr (SLP) store_sleep(O, G, isl);
    if (!lead) return;
    const uint32_t flags = (uint32_t)ldc(RC_FLAGS);
    sti(G.st, CP_SF_STEPS, G.off, ldc(RC_STEPS));
    sti(G.st, CP_SF_EPISODE, G.off, ldc(RC_EPISODE));
    sti(G.st, CP_SF_DONE, G.off, (flags & RF_DONE) ? 1 : 0);
    b.ret_acc[i] = __uint_as_float(to_bits(G.lx(RC_RET)));
    b.stepped[i] = (flags & RF_LAST_SIM) ? 1 : 0;  // step K-1's value, as after the K-th cp_step
    if (ov) b.overflow[i] += ov;
}

// CP_AUTORESET_NEXT_STEP, in the call after an env finished (list q = the previous call's reset
// list, whose reset kernel ran on the library's second stream and has completed): the new episode's
// first obs (written by that reset kernel into nobs), reward 0, done 0; the done field is cleared,
// so the env steps again from the next call.  An env whose done field is no longer 2 + q was
// resolved by a cp_reset in between and is skipped.
__global__ void __launch_bounds__(256) cp_nextstep_fixup_kernel(cp_config cfg, Bufs b, const int32_t* list,
                                                                 const int32_t* count, int q, const float* nobs,
                                                                 float* obs_out, float* reward_out, uint8_t* done_out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= *count) return;
    const int i = list[t];
    const Soa st = Soa::make(b.state, cfg.num_envs, CP_STATE_FIELDS);
    const uint32_t o = Soa::eoff(i);
    if (ldi(st, CP_SF_DONE, o) != 2 + q) return;
    const size_t n = (size_t)cfg.action_repeats * 14;
    for (size_t f = 0; f < n; ++f) obs_out[(size_t)i * n + f] = nobs[(size_t)i * n + f];
    reward_out[i] = 0.0f;
    done_out[i] = 0;
    sti(st, CP_SF_DONE, o, 0);
}

// cp_reset of a NEXT_STEP handle: a masked env whose reset is already done (done field >= 2)
// returns that reset's obs and is not reset again (one reset from its terminal state, as a lazy
// reset would give); the other masked envs go to the reset list (wave ballot compaction).
__global__ void __launch_bounds__(256) cp_nextstep_resolve_kernel(cp_config cfg, Bufs b, const uint8_t* mask,
                                                                   const float* nobs, float* obs_out) {
    const int B = cfg.num_envs;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool want = false;
    if (i < B && (mask == nullptr || mask[i] != 0)) {
        const Soa st = Soa::make(b.state, B, CP_STATE_FIELDS);
        const uint32_t o = Soa::eoff(i);
        if (ldi(st, CP_SF_DONE, o) >= 2) {
            const size_t n = (size_t)cfg.action_repeats * 14;
            for (size_t f = 0; f < n; ++f) obs_out[(size_t)i * n + f] = nobs[(size_t)i * n + f];
            sti(st, CP_SF_DONE, o, 0);
        } else {
            want = true;
        }
    }
    const uint64_t bal = __ballot(want);
    const int lane = threadIdx.x & (WAVE - 1);
    const int n = __popcll(bal);
    int base = 0;
    if (lane == 0 && n) base = atomicAdd(b.count, n);
    base = __shfl(base, 0);
    if (want) b.list[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
}

// ---------------------------------------------------------------- host launchers
#ifndef CP_KERNELS_ONLY  // tools/isa_one.sh: one kernel instantiated, no launchers
static inline unsigned env_grid(int n, int block) { return (unsigned)((n + block - 1) / block); }

void launch_init(const cp_config& cfg, const Bufs& b, hipStream_t st) {
    hipLaunchKernelGGL(cp_init_kernel, dim3(env_grid(cfg.num_envs, 256)), dim3(256), 0, st, cfg, b);
}

void launch_nextstep_fixup(const cp_config& cfg, const Bufs& b, const int32_t* list, const int32_t* count, int q,
                           const float* nobs, float* obs_out, float* reward_out, uint8_t* done_out, hipStream_t st) {
    hipLaunchKernelGGL(cp_nextstep_fixup_kernel, dim3(env_grid(cfg.num_envs, 256)), dim3(256), 0, st, cfg, b, list,
                       count, q, nobs, obs_out, reward_out, done_out);
}

void launch_nextstep_resolve(const cp_config& cfg, const Bufs& b, const uint8_t* mask, const float* nobs,
                             float* obs_out, hipStream_t st) {
    hipLaunchKernelGGL(cp_nextstep_resolve_kernel, dim3(env_grid(cfg.num_envs, 256)), dim3(256), 0, st, cfg, b, mask,
                       nobs, obs_out);
}

// shape: 0 throughput, 1 latency, 2 latency on the WIDE layout (cp_set_kernel_shape; fp32 default model only)
void launch_reset(int shape, const cp_config& cfg, const Bufs& b, float* obs_out, hipStream_t st) {
    const bool lat = shape != 0;
    const int wide = (kF64 || (cfg.phys.model_flags & (CP_MODEL_PERSISTENT | CP_MODEL_SLEEPING))) ? 0
                     : shape == CP_SHAPE_WIDE ? 16 : shape == CP_SHAPE_WIDE8 ? 8 : shape == CP_SHAPE_WIDE64 ? 64 : 0;
    const dim3 grid(env_grid((wide ? wide : 2) * cfg.num_envs, WAVE)), block(WAVE);  // lanes per env
    if (cfg.phys.model_flags & CP_MODEL_PERSISTENT) {  // the persistent-manifold model: latency shape only
        hipLaunchKernelGGL((cp_reset_kernel<true, true>), grid, block, 0, st, cfg, b, obs_out);
        return;
    }
    if (cfg.phys.model_flags & CP_MODEL_SLEEPING) {  // the sleeping model: latency shape only
        hipLaunchKernelGGL((cp_reset_kernel<true, false, true>), grid, block, 0, st, cfg, b, obs_out);
        return;
    }
    if constexpr (kF64) {
        (void)lat;
        hipLaunchKernelGGL(cp_reset_kernel<true>, grid, block, 0, st, cfg, b, obs_out);
    } else if (shape == CP_SHAPE_LIST) {
        // a launch per layout, each with the grid of its largest list and the range of list lengths it serves;
        // the others' waves read the length and exit (the tiers of wide_reset_shape_for by the list's length)
        const int B = cfg.num_envs;
        Bufs bt = b;
#define CP_LIST_TIER(KERN, LANES, LO, HI)                                                                \
        if (B > (LO)) {                                                                                   \
            bt.nlo = (LO);                                                                                \
            bt.nhi = (HI);                                                                                \
            const int cap = ((HI) > 0 && B > (HI)) ? (HI) : B;                                            \
            hipLaunchKernelGGL(KERN, dim3(env_grid((LANES) * cap, WAVE)), block, 0, st, cfg, bt, obs_out); \
        }
        CP_LIST_TIER((cp_reset_kernel<true, false, false, 64>), 64, 0, 1024)
        CP_LIST_TIER((cp_reset_kernel<true, false, false, 16>), 16, 1024, 4096)
        CP_LIST_TIER(cp_reset_kernel<true>, 2, 4096, 32768)
        CP_LIST_TIER(cp_reset_kernel<false>, 2, 32768, 0)
#undef CP_LIST_TIER
    } else {
        if (wide == 64) hipLaunchKernelGGL((cp_reset_kernel<true, false, false, 64>), grid, block, 0, st, cfg, b, obs_out);
        else if (wide == 16) hipLaunchKernelGGL((cp_reset_kernel<true, false, false, 16>), grid, block, 0, st, cfg, b, obs_out);
        else if (wide == 8) hipLaunchKernelGGL((cp_reset_kernel<true, false, false, 8>), grid, block, 0, st, cfg, b, obs_out);
        else if (lat) hipLaunchKernelGGL(cp_reset_kernel<true>, grid, block, 0, st, cfg, b, obs_out);
        else hipLaunchKernelGGL(cp_reset_kernel<false>, grid, block, 0, st, cfg, b, obs_out);
    }
}

template <int K, bool Q>
static void launch_step_t(int shape, const cp_config& cfg, const Bufs& b, const void* actions, float* obs_out,
                          float* reward_out, uint8_t* done_out, float* term_out, float* readback, int rb_bug,
                          const Lqr& lq, hipStream_t st) {
    const bool lat = shape != 0;
    const int wide = (kF64 || (cfg.phys.model_flags & (CP_MODEL_PERSISTENT | CP_MODEL_SLEEPING))) ? 0
                     : shape == CP_SHAPE_WIDE ? 16 : shape == CP_SHAPE_WIDE8 ? 8 : shape == CP_SHAPE_WIDE64 ? 16 : 0;  // (64 lanes: reset lists only)
    const dim3 grid(env_grid((wide ? wide : 2) * cfg.num_envs, WAVE)), block(WAVE);  // lanes per env
    if (cfg.phys.model_flags & CP_MODEL_PERSISTENT) {  // the persistent-manifold model: latency shape only
        hipLaunchKernelGGL((cp_step_kernel<K, Q, true, true>), grid, block, 0, st, cfg, b, actions, obs_out,
                           reward_out, done_out, term_out, readback, rb_bug, lq);
        return;
    }
    if constexpr (!Q) {  // the sleeping model: latency shape only, no LQR policy (cp_set_lqr rejects it)
        if (cfg.phys.model_flags & CP_MODEL_SLEEPING) {
            hipLaunchKernelGGL((cp_step_kernel<K, false, true, false, true>), grid, block, 0, st, cfg, b, actions,
                               obs_out, reward_out, done_out, term_out, readback, rb_bug, lq);
            return;
        }
    }
    if constexpr (kF64) {
        (void)lat;
        hipLaunchKernelGGL((cp_step_kernel<K, Q, true>), grid, block, 0, st, cfg, b, actions, obs_out, reward_out,
                           done_out, term_out, readback, rb_bug, lq);
    } else {
        if (wide == 16)
            hipLaunchKernelGGL((cp_step_kernel<K, Q, true, false, false, 16>), grid, block, 0, st, cfg, b, actions,
                               obs_out, reward_out, done_out, term_out, readback, rb_bug, lq);
        else if (wide == 8)
            hipLaunchKernelGGL((cp_step_kernel<K, Q, true, false, false, 8>), grid, block, 0, st, cfg, b, actions,
                               obs_out, reward_out, done_out, term_out, readback, rb_bug, lq);
        else if (lat)
            hipLaunchKernelGGL((cp_step_kernel<K, Q, true>), grid, block, 0, st, cfg, b, actions, obs_out, reward_out,
                               done_out, term_out, readback, rb_bug, lq);
        else
            hipLaunchKernelGGL((cp_step_kernel<K, Q, false>), grid, block, 0, st, cfg, b, actions, obs_out, reward_out,
                               done_out, term_out, readback, rb_bug, lq);
    }
}

template <int K, bool Q>
static void launch_rollout_t(bool lat, const cp_config& cfg, const Bufs& b, int steps, const void* actions,
                             float* obs_out, float* reward_out, uint8_t* done_out, float* term_out, const Lqr& lq,
                             hipStream_t st) {
    const dim3 grid(env_grid(2 * cfg.num_envs, WAVE)), block(WAVE);  // two lanes per env
    if constexpr (!Q) {
        if (cfg.phys.model_flags & CP_MODEL_SLEEPING) {
            hipLaunchKernelGGL((cp_rollout_kernel<K, false, true, false, true>), grid, block, 0, st, cfg, b, steps,
                               actions, obs_out, reward_out, done_out, term_out, lq);
            return;
        }
    }
    if (cfg.phys.model_flags & CP_MODEL_PERSISTENT)
        hipLaunchKernelGGL((cp_rollout_kernel<K, Q, true, true>), grid, block, 0, st, cfg, b, steps, actions, obs_out,
                           reward_out, done_out, term_out, lq);
    else if (lat || kF64)
        hipLaunchKernelGGL((cp_rollout_kernel<K, Q, true>), grid, block, 0, st, cfg, b, steps, actions, obs_out,
                           reward_out, done_out, term_out, lq);
    else
        hipLaunchKernelGGL((cp_rollout_kernel<K, Q, false>), grid, block, 0, st, cfg, b, steps, actions, obs_out,
                           reward_out, done_out, term_out, lq);
}

void launch_rollout(bool lat, int kind, const cp_config& cfg, const Bufs& b, int steps, const void* actions,
                    float* obs_out, float* reward_out, uint8_t* done_out, float* term_out, const Lqr& lq,
                    hipStream_t st) {
    const bool q = lq.gains != nullptr;
    if (kind == CP_ACTION_CONTINUOUS) {
        if (q) launch_rollout_t<CP_ACTION_CONTINUOUS, true>(lat, cfg, b, steps, actions, obs_out, reward_out, done_out,
                                                            term_out, lq, st);
        else launch_rollout_t<CP_ACTION_CONTINUOUS, false>(lat, cfg, b, steps, actions, obs_out, reward_out, done_out,
                                                           term_out, lq, st);
    } else {
        if (q) launch_rollout_t<CP_ACTION_DISCRETE, true>(lat, cfg, b, steps, actions, obs_out, reward_out, done_out,
                                                          term_out, lq, st);
        else launch_rollout_t<CP_ACTION_DISCRETE, false>(lat, cfg, b, steps, actions, obs_out, reward_out, done_out,
                                                         term_out, lq, st);
    }
}

void launch_step(int lat, int kind, const cp_config& cfg, const Bufs& b, const void* actions, float* obs_out,
                 float* reward_out, uint8_t* done_out, float* term_out, float* readback, int rb_bug, const Lqr& lq,
                 hipStream_t st) {
    const bool q = lq.gains != nullptr;
    if (kind == CP_ACTION_CONTINUOUS) {
        if (q) launch_step_t<CP_ACTION_CONTINUOUS, true>(lat, cfg, b, actions, obs_out, reward_out, done_out, term_out,
                                                         readback, rb_bug, lq, st);
        else launch_step_t<CP_ACTION_CONTINUOUS, false>(lat, cfg, b, actions, obs_out, reward_out, done_out, term_out,
                                                        readback, rb_bug, lq, st);
    } else {
        if (q) launch_step_t<CP_ACTION_DISCRETE, true>(lat, cfg, b, actions, obs_out, reward_out, done_out, term_out,
                                                       readback, rb_bug, lq, st);
        else launch_step_t<CP_ACTION_DISCRETE, false>(lat, cfg, b, actions, obs_out, reward_out, done_out, term_out,
                                                      readback, rb_bug, lq, st);
    }
}

#endif  // CP_KERNELS_ONLY
}  // namespace CP_NS
