// cp_physics.h — one fixed physics step of the 5-body cartpole scene, per lane pair.
//
// Two adjacent lanes simulate one environment (bullet_cartpole.py's whole pybullet
// world: ground, cart, pole, cart2, pole2 — :154-160); lane 2e+p owns contact
// island p.  Both lanes hold the env's body state in VGPRs with compile-time
// indices; each lane's contact rows live in its column of a per-wave LDS pool
// laid out [field][slot][lane] (conflict-free ds_read_b32).  A lane walks its
// island's 5 body pairs with a wave-uniform loop in the narrowphase and solves
// its island with statically unrolled per-pair code on a 2-body local view; an
// env with a cross-island contact is solved by both lanes redundantly in the
// global order.  The algorithm is DESIGN.md §Physics model; the CPU
// oracle (oracle/cp_oracle.c) states the same arithmetic, operation for operation.
// Written over `real`; included after cp_math.h once per real type (cp_common.h).
#if !defined(CP_NS) || !defined(CP_REAL)
#error "define CP_NS and CP_REAL before including cp_physics.h (see cp_kernels.hip)"
#endif
#include "cp_common.h"

#include <type_traits>

namespace CP_NS {

// Diagnostic phase stamps (built only with -DCP_STAMPS; see cp_debug_stamps).
// Wave-uniform cycle counters from s_memtime, accumulated per wave.
struct Stamps {
    uint64_t narrow = 0, vel = 0, solve = 0, integ = 0, sweeps = 0, substeps = 0;
    uint64_t sel = 0, bb = 0, rows = 0;  // narrowphase split: box/inertia selection, box_box, row setup
    uint32_t flags = 0;  // slow paths the wave took: 1 merged solve, 2 / 4 ground-cart / ground-pole rows not +z
};
#ifdef CP_STAMPS
#define CP_STAMP(var) uint64_t var = __builtin_amdgcn_s_memtime()
#define CP_RT(var) uint64_t var = __builtin_amdgcn_s_memrealtime()
#define CP_ACC(field, a, b) (ST.field += (b) - (a))
#else
#define CP_STAMP(var)
#define CP_RT(var) constexpr uint64_t var = 0
#define CP_ACC(field, a, b)
#endif

constexpr int WAVE = 64;
constexpr int MAXP = CP_ISLAND_POINTS;    // per island (= per lane)
constexpr int MAXF = CP_ISLAND_FRICTION;
// pool fields (per normal point): rb.xyz, inv_eff, target, lambda
constexpr int F_RBX = 0, F_RBY = 1, F_RBZ = 2, F_IE = 3, F_TG = 4, F_LAM = 5;
constexpr int NPF = 6;
// friction fields (per frictional point): lambda1, lambda2, inv_eff1, inv_eff2
constexpr int FF_L1 = 0, FF_L2 = 1, FF_IE1 = 2, FF_IE2 = 3;
constexpr int POOL_FLOATS = NPF * MAXP + 4 * MAXF;  // 80 floats per lane = 20 KiB per wave

CP_DEV real& pool_n(real* pool, int field, int slot) { return pool[(field * MAXP + slot) * WAVE]; }
CP_DEV real& pool_f(real* pool, int field, int slot) { return pool[(NPF * MAXP + field * MAXF + slot) * WAVE]; }
// CP_MODEL_PERSISTENT (PM) kernels: each normal row's own normal (a cached point keeps the normal it
// was added with), 3 more fields per row after the friction fields
constexpr int POOL_FLOATS_PM = POOL_FLOATS + 3 * MAXP;
CP_DEV real& pool_pn(real* pool, int c, int slot) { return pool[(POOL_FLOATS + c * MAXP + slot) * WAVE]; }
CP_DEV V3 pool_normal(real* pool, int slot) { return mk(pool_pn(pool, 0, slot), pool_pn(pool, 1, slot), pool_pn(pool, 2, slot)); }

// body pairs (a < b), Bullet-like order over the loadURDF ids
__host__ __device__ constexpr int pair_a(int p) {
    return p < 4 ? 0 : (p < 7 ? 1 : (p < 9 ? 2 : 3));
}
__host__ __device__ constexpr int pair_b(int p) {
    return p < 4 ? p + 1 : (p < 7 ? p - 2 : (p < 9 ? p - 4 : 4));
}

struct Body {
    V3 x, v, w;
    real q[4];
};

// Per-env simulation state held in registers for the duration of a kernel.
// A whole-env view (both lanes of the env hold the same values): assembled by DPP from the two lanes'
// Own states where a phase needs every body (the env's outputs, the cross rows of a merged solve).
struct Sim {
    Body b[CP_NUM_DYN];   // cart, pole, cart2, pole2
    V3 f0, f2;            // pending world force on cart / cart2 (pybullet force accumulator)
};

// Per-lane state across substeps: the lane's own island only (lane 2e: cart, pole; lane 2e+1: cart2,
// pole2).  The partner island's bodies come from the partner lane by DPP in the phases that need them
// (the narrowphase's cross pairs, a merged solve's cross rows, the sleeping islands, the outputs);
// holding the whole env in both lanes kept ~29 more values live through every substep (round 5,
// DESIGN.md §4).
struct Own {
    Body c, p;        // the island's cart and pole
    V3 f;             // pending world force on the island's cart (pybullet force accumulator)
    uint32_t wsm;     // 3 bits per local pair: the point count of the pair's warm-start id word (ws_count)
    uint32_t sa[2];   // CP_MODEL_SLEEPING (SLP kernels only): activation words of c, p (CP_ACT_* | CP_ACT_AWAKE)
    real st[2];       //   and their sleep timers
};

// The point count of a warm-start id word: its leading non-0xFF bytes when the word is a prefix (ids, then
// 0xFF padding: every word the kernels and cp_init write), 7 for any other word (a state set from outside),
// which makes the pair's cache rewritten like a changed one.
CP_DEV uint32_t ws_count(uint32_t id) {
    const uint32_t b0 = id & 0xFFu, b1 = (id >> 8) & 0xFFu, b2 = (id >> 16) & 0xFFu, b3 = id >> 24;
    const uint32_t n = b0 == 0xFFu ? 0u : b1 == 0xFFu ? 1u : b2 == 0xFFu ? 2u : b3 == 0xFFu ? 3u : 4u;
    const uint32_t pad = n >= 4u ? 0u : 0xFFFFFFFFu << (8u * n);  // the bytes past the prefix
    return (id & pad) == pad ? n : 7u;
}

// Per-env global memory touched once per substep (cold data kept out of VGPRs):
// the warm-start cache lives in the state SoA (SoaT: buffer-resource access, cp_common.h).
using Soa = SoaT<real>;
struct Mem {
    Soa st;           // state SoA [CP_STATE_FIELDS][B]
    Soa scr;          // scratch SoA [CP_SCR_FIELDS][2B], one column per lane (cp_common.h)
    Soa pm;           // CP_MODEL_PERSISTENT: the island's persistent manifolds [PM_FIELDS][2B], one column per lane
    uint32_t off;     // env index * sizeof(real)
    uint32_t woff;    // off + island * CP_ISLAND_PAIRS fields  (warm-start ids of the lane's island)
    uint32_t loff;    // off + island * 4*CP_ISLAND_PAIRS fields (warm-start impulses)
    uint32_t xoff;    // (2 * env + island) * sizeof(real)
    CP_DEV static Mem make(void* state, void* scratch, int B, int env, int isl, void* pman = nullptr) {
        Mem m;
        m.st = Soa::make(state, B, CP_STATE_FIELDS);
        m.scr = Soa::make(scratch, 2 * B, CP_SCR_FIELDS);
        m.pm = Soa::make(pman, pman ? 2 * B : 0, CP_PM_FIELDS);  // null: an empty resource (no PM kernel reads it)
        m.off = Soa::eoff(env);
        m.woff = m.off + (uint32_t)(isl * CP_ISLAND_PAIRS) * m.st.fstride;
        m.loff = m.off + (uint32_t)(isl * 4 * CP_ISLAND_PAIRS) * m.st.fstride;
        m.xoff = Soa::eoff(2 * env + isl);
        return m;
    }
    CP_DEV real ls(int f) const { return st.ld(f, off); }
    CP_DEV void ss(int f, real v) const { st.st(f, off, v); }
    CP_DEV real lw(int f) const { return st.ld(f, woff); }
    CP_DEV void sw(int f, real v) const { st.st(f, woff, v); }
    CP_DEV real ll(int f) const { return st.ld(f, loff); }
    CP_DEV void sl(int f, real v) const { st.st(f, loff, v); }
    CP_DEV real lx(int f) const { return scr.ld(f, xoff); }
    CP_DEV void sx(int f, real v) const { scr.st(f, xoff, v); }
    CP_DEV real lp(int f) const { return pm.ld(f, xoff); }
    CP_DEV void sp(int f, real v) const { pm.st(f, xoff, v); }
};

struct Box {
    V3 c;
    Axes ax;
    real h0, h1, h2;
};

// component-wise selects (a struct-valued ?: lets the compiler build the operands in scratch)
CP_DEV real sel3(real a, real b, real c, int i) { return i == 0 ? a : (i == 1 ? b : c); }
CP_DEV V3 sel3v(V3 a, V3 b, V3 c, int i) { return mk(sel3(a.x, b.x, c.x, i), sel3(a.y, b.y, c.y, i), sel3(a.z, b.z, c.z, i)); }
CP_DEV V3 selv(bool t, V3 a, V3 b) { return mk(t ? a.x : b.x, t ? a.y : b.y, t ? a.z : b.z); }
CP_DEV V3 axis_of(const Axes& A, int i) { return sel3v(A.a0, A.a1, A.a2, i); }
// (opaque register copies: a select chain over the fields would otherwise become one load through
// a computed address and keep the box in private memory)
CP_DEV real h_of(const Box& B, int i) {
    real h0 = B.h0, h1 = B.h1, h2 = B.h2;
    asm("" : "+v"(h0), "+v"(h1), "+v"(h2));
    return i == 0 ? h0 : (i == 1 ? h1 : h2);
}

// contact point candidate (reference-face coordinates u, v and separation n)
struct Out4 {
    real u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0}, n[4] = {0, 0, 0, 0};
    int id[4] = {0, 0, 0, 0};
    int m = 0;
};

// Face-contact geometry in reference-face coordinates (u, v along the face, n
// along its normal): incident-face centre c, half edges e1, e2, vertices P[4].
struct FaceGeom {
    real hu, hv, margin;
    real cu, cv, cn, e1u, e1v, e1n, e2u, e2v, e2n;
    real Pu[4], Pv[4], Pn[4];
    real idet;
    bool all_in;  // all four incident vertices inside the reference rectangle: C1 only
};

// Candidate K (compile-time slot in the canonical order: C1 0-3, C2 4-7, C3 8-23)
// and whether it is kept.  Same arithmetic as the oracle's candidate loops; the
// candidates are re-evaluated per pass instead of stored (72 registers saved).
template <int K>
CP_DEV bool cand(const FaceGeom& G, real& u, real& v, real& n) {
    if constexpr (K < 4) {
        u = G.Pu[K]; v = G.Pv[K]; n = G.Pn[K];
        return abs_(G.Pu[K]) <= G.hu && abs_(G.Pv[K]) <= G.hv && G.Pn[K] <= G.margin;
    } else if constexpr (K < 8) {
        constexpr int c = K - 4;
        const real X = (c == 0 || c == 3) ? G.hu : -G.hu;
        const real Y = (c < 2) ? G.hv : -G.hv;
        const real ru = X - G.cu, rv = Y - G.cv;
        const real al = fma_(ru, G.e2v, -(rv * G.e2u)) * G.idet;
        const real be = fma_(G.e1u, rv, -(G.e1v * ru)) * G.idet;
        const real dn = fma_(be, G.e2n, fma_(al, G.e1n, G.cn));
        u = X; v = Y; n = dn;
        return !G.all_in && abs_(al) < real(1.0) && abs_(be) < real(1.0) && dn <= G.margin;
    } else {
        constexpr int k = (K - 8) / 4, sd = (K - 8) % 4, k1 = (k + 1) & 3;
        const real lim = (sd & 1) ? ((sd < 2) ? -G.hu : -G.hv) : ((sd < 2) ? G.hu : G.hv);
        const real pc = (sd < 2) ? G.Pu[k] : G.Pv[k], qc = (sd < 2) ? G.Pu[k1] : G.Pv[k1];
        const real dp = pc - lim, dq = qc - lim;
        const bool cross_ = (dp < real(0.0) && dq > real(0.0)) || (dp > real(0.0) && dq < real(0.0));
        const real t = dp / (dp - dq);
        bool inr;
        if constexpr (sd < 2) {
            u = lim;
            v = fma_(G.Pv[k1] - G.Pv[k], t, G.Pv[k]);
            inr = abs_(v) <= G.hv;
        } else {
            v = lim;
            u = fma_(G.Pu[k1] - G.Pu[k], t, G.Pu[k]);
            inr = abs_(u) <= G.hu;
        }
        n = fma_(G.Pn[k1] - G.Pn[k], t, G.Pn[k]);
        return !G.all_in && cross_ && inr && n <= G.margin;
    }
}

// compile-time loop over the 24 candidate slots
template <int K = 0, typename Fn>
CP_DEV void for_cands(const FaceGeom& G, Fn&& fn) {
    if constexpr (K < 24) {
        real u, v, n;
        const bool ok = cand<K>(G, u, v, n);
        fn(K, ok, u, v, n);
        for_cands<K + 1>(G, fn);
    }
}

// Face contact (oracle: face_contact).  Fills up to 4 selected candidates.
// ALLIN: when every lane of the wave that reaches this has all four incident vertices inside
// the reference rectangle (the oracle's `inside == 4` exit: C1 candidates only, at most 4, so
// no reduction), emit those directly instead of evaluating the 24 candidate slots: the same
// points in the same order.  Every contact of a reset's settle substeps is of this kind.
template <bool ALLIN = false>
CP_DEV void face_contact(const Box& R, int ri, V3 nr, const Box& I, real margin, V3& fc, V3& u, V3& v,
                         Out4& out) {
    int r1 = ri == 2 ? 0 : ri + 1, r2 = ri == 0 ? 2 : ri - 1;
    fc = madd(R.c, nr, h_of(R, ri));
    u = axis_of(R.ax, r1);
    v = axis_of(R.ax, r2);
    FaceGeom G;
    G.margin = margin;
    G.hu = h_of(R, r1);
    G.hv = h_of(R, r2);
    real e0 = dot(nr, I.ax.a0), e1d = dot(nr, I.ax.a1), e2d = dot(nr, I.ax.a2);
    int j = 0;
    real best = abs_(e0);
    if (abs_(e1d) > best) { j = 1; best = abs_(e1d); }
    if (abs_(e2d) > best) { j = 2; }
    real ej = sel3(e0, e1d, e2d, j);
    real isg = (ej > real(0.0)) ? -real(1.0) : real(1.0);
    V3 ic = madd(I.c, axis_of(I.ax, j), isg * h_of(I, j));
    int j1 = j == 2 ? 0 : j + 1, j2 = j == 0 ? 2 : j - 1;
    V3 E1 = scl(axis_of(I.ax, j1), h_of(I, j1));
    V3 E2 = scl(axis_of(I.ax, j2), h_of(I, j2));
    V3 icr = sub(ic, fc);
    G.cu = dot(icr, u); G.cv = dot(icr, v); G.cn = dot(icr, nr);
    G.e1u = dot(E1, u); G.e1v = dot(E1, v); G.e1n = dot(E1, nr);
    G.e2u = dot(E2, u); G.e2v = dot(E2, v); G.e2n = dot(E2, nr);
    G.Pu[0] = (G.cu + G.e1u) + G.e2u; G.Pv[0] = (G.cv + G.e1v) + G.e2v; G.Pn[0] = (G.cn + G.e1n) + G.e2n;
    G.Pu[1] = (G.cu - G.e1u) + G.e2u; G.Pv[1] = (G.cv - G.e1v) + G.e2v; G.Pn[1] = (G.cn - G.e1n) + G.e2n;
    G.Pu[2] = (G.cu - G.e1u) - G.e2u; G.Pv[2] = (G.cv - G.e1v) - G.e2v; G.Pn[2] = (G.cn - G.e1n) - G.e2n;
    G.Pu[3] = (G.cu + G.e1u) - G.e2u; G.Pv[3] = (G.cv + G.e1v) - G.e2v; G.Pn[3] = (G.cn + G.e1n) - G.e2n;
    int inside = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) inside += (abs_(G.Pu[k]) <= G.hu && abs_(G.Pv[k]) <= G.hv) ? 1 : 0;
    G.all_in = inside == 4;
    if constexpr (ALLIN) {
        if (__ballot(!G.all_in) == 0ull) {
            out.m = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (G.Pn[k] <= margin) {
                    const int m = out.m;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (m == q) {
                            out.u[q] = G.Pu[k];
                            out.v[q] = G.Pv[k];
                            out.n[q] = G.Pn[k];
                            out.id[q] = k;
                        }
                    }
                    out.m = m + 1;
                }
            }
            return;
        }
    }
    G.idet = real(0.0);
    if (!G.all_in) {
        real det = fma_(G.e1u, G.e2v, -(G.e1v * G.e2u));
        G.idet = real(1.0) / det;
    }
    // pass 1: valid set and the deepest candidate (first minimum in canonical order)
    uint32_t valid = 0;
    int i0 = -1;
    real bn = real(0.0), u0 = real(0.0), v0 = real(0.0);
    for_cands(G, [&](int k, bool ok, real cu_, real cv_, real cn_) {
        if (ok) {
            valid |= 1u << k;
            if (i0 < 0 || cn_ < bn) { i0 = k; bn = cn_; u0 = cu_; v0 = cv_; }
        }
    });
    uint32_t sel = valid;
    if (__builtin_popcount(valid) > 4) {
        // deepest; farthest from it; max / min signed area  (oracle: same rule)
        int i1 = -1;
        real bd = real(0.0), u1 = real(0.0), v1 = real(0.0);
        for_cands(G, [&](int k, bool ok, real cu_, real cv_, real) {
            if (!ok || k == i0) return;
            real du = cu_ - u0, dv = cv_ - v0;
            real d2 = fma_(du, du, dv * dv);
            if (i1 < 0 || d2 > bd) { i1 = k; bd = d2; u1 = cu_; v1 = cv_; }
        });
        const real ex = u1 - u0, ey = v1 - v0;
        int i2 = -1;
        real ba = real(0.0);
        for_cands(G, [&](int k, bool ok, real cu_, real cv_, real) {
            if (!ok || k == i0 || k == i1) return;
            real ar = fma_(ex, cv_ - v0, -(ey * (cu_ - u0)));
            if (i2 < 0 || ar > ba) { i2 = k; ba = ar; }
        });
        int i3 = -1;
        real bb = real(0.0);
        for_cands(G, [&](int k, bool ok, real cu_, real cv_, real) {
            if (!ok || k == i0 || k == i1 || k == i2) return;
            real ar = fma_(ex, cv_ - v0, -(ey * (cu_ - u0)));
            if (i3 < 0 || ar < bb) { i3 = k; bb = ar; }
        });
        sel = (1u << i0) | (1u << i1) | (1u << i2) | (1u << i3);
    }
    // emit the selected candidates in canonical order
    out.m = 0;
    for_cands(G, [&](int k, bool, real cu_, real cv_, real cn_) {
        if ((sel >> k) & 1u) {
            const int m = out.m;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (m == q) {
                    out.u[q] = cu_;
                    out.v[q] = cv_;
                    out.n[q] = cn_;
                    out.id[q] = k;
                }
            }
            out.m = m + 1;
        }
    });
}

// Contact result of one box pair in world space.
struct Contact {
    V3 n;          // from A to B
    int m;         // points
    V3 p[4];       // world contact points (midway between the surfaces)
    real d[4];    // signed separation (negative = penetration)
    uint32_t ids;  // feature ids (warm-start keys), one byte per point (an int array here is
                   // written under path-dependent indices and lands in private memory)
};

// Box-box narrowphase (oracle: box_box).  Normal from A to B.
// ES: skip the edge axes' root where the separation tests cannot pass (below); the throughput-shaped kernels
// (C3 step kernel -1.1 %; in the latency step kernel it measured +2 %, so those keep the full path)
template <bool ALLIN = false, bool ES = false>
CP_DEV void box_box(const Box& A, const Box& B, real margin, real edge_bias, Contact& C, Stamps& ST) {
    (void)ST;
    C.m = 0;
    V3 d = sub(B.c, A.c);
    V3 Aax[3] = {A.ax.a0, A.ax.a1, A.ax.a2};
    V3 Bax[3] = {B.ax.a0, B.ax.a1, B.ax.a2};
    real Ah[3] = {A.h0, A.h1, A.h2}, Bh[3] = {B.h0, B.h1, B.h2};
    real Cm[3][3], AC[3][3], da[3], db[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Cm[i][j] = dot(Aax[i], Bax[j]);
            AC[i][j] = abs_(Cm[i][j]);
        }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        da[i] = dot(d, Aax[i]);
        db[i] = dot(d, Bax[i]);
    }
    real best = real(0.0);
    int kind = 0, bi = 0, bj = 0;
    V3 bax = mk(real(0.0), real(0.0), real(0.0));
    bool sep = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        real pr = fma_(Bh[0], AC[i][0], fma_(Bh[1], AC[i][1], Bh[2] * AC[i][2]));
        real s = abs_(da[i]) - (Ah[i] + pr);
        sep = sep || (s > margin);
        if (i == 0 || s > best) { best = s; kind = 0; bi = i; }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        real pr = fma_(Ah[0], AC[0][j], fma_(Ah[1], AC[1][j], Ah[2] * AC[2][j]));
        real s = abs_(db[j]) - (Bh[j] + pr);
        sep = sep || (s > margin);
        if (s > best) { best = s; kind = 1; bj = j; }
    }
    if (sep) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            V3 ax = cross(Aax[i], Bax[j]);
            real L2 = dot(ax, ax);
            if (L2 < real(1e-6)) continue;
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            real ra = fma_(Ah[i1], AC[i2][j], Ah[i2] * AC[i1][j]);
            real rb = fma_(Bh[j1], AC[i][j2], Bh[j2] * AC[i][j1]);
            real num = abs_(dot(d, ax)) - (ra + rb);   // separation * L
            if constexpr (ES) {
            // Both tests below compare num with (c * L) for c = margin and c = best + edge_bias, where
            // L = |a x b| <= 1 + 2^-11 (unit axes from normalised quaternions).  For num <= min(c, 0) (1 + 2^-10)
            // both are false for every such L, whatever the rounding of c * L (|round(c L)| < |c| (1 + 2^-10)
            // (1 - 2^-24) when c < 0; c L >= 0 when c >= 0), so the root and both products are skipped: the
            // same decisions as the oracle's (a NaN num or bound takes the full path).  Resting stacks: most
            // edge axes of the ground pairs (the ground's half extents dwarf num) and 4 of the cart-pole pair's 6.
            real lo = best + edge_bias;
            lo = lo < margin ? lo : margin;
            lo = lo < real(0.0) ? lo : real(0.0);
            if (num <= lo * real(1.0009765625)) continue;
            }
            real L = sqrt_(L2);
            sep = sep || (num > margin * L);
            if (num > (best + edge_bias) * L) { best = num / L; kind = 2; bi = i; bj = j; bax = ax; }
        }
    }
    if (sep) return;
    if (kind != 2) {
        // face of A (kind 0) or face of B (kind 1) is the reference face
        const bool fa = kind == 0;
        int ri = fa ? bi : bj;
        real sg = fa ? ((sel3(da[0], da[1], da[2], bi) >= real(0.0)) ? real(1.0) : -real(1.0))
                      : ((sel3(db[0], db[1], db[2], bj) >= real(0.0)) ? -real(1.0) : real(1.0));
        // the half extents as opaque register values: a select between two boxes' fields
        // otherwise becomes one load through a selected address, which puts both boxes
        // (and R, I) in private memory (scratch traffic every pair of every substep)
        real ah0 = A.h0, ah1 = A.h1, ah2 = A.h2, bh0 = B.h0, bh1 = B.h1, bh2 = B.h2;
        asm("" : "+v"(ah0), "+v"(ah1), "+v"(ah2), "+v"(bh0), "+v"(bh1), "+v"(bh2));
        Box R, I;
        R.c = selv(fa, A.c, B.c);
        R.ax.a0 = selv(fa, A.ax.a0, B.ax.a0);
        R.ax.a1 = selv(fa, A.ax.a1, B.ax.a1);
        R.ax.a2 = selv(fa, A.ax.a2, B.ax.a2);
        R.h0 = fa ? ah0 : bh0; R.h1 = fa ? ah1 : bh1; R.h2 = fa ? ah2 : bh2;
        I.c = selv(fa, B.c, A.c);
        I.ax.a0 = selv(fa, B.ax.a0, A.ax.a0);
        I.ax.a1 = selv(fa, B.ax.a1, A.ax.a1);
        I.ax.a2 = selv(fa, B.ax.a2, A.ax.a2);
        I.h0 = fa ? bh0 : ah0; I.h1 = fa ? bh1 : ah1; I.h2 = fa ? bh2 : ah2;
        V3 nr = scl(axis_of(R.ax, ri), sg);
        C.n = selv(fa, nr, neg(nr));
        V3 fc, u, v;
        Out4 o;
        face_contact<ALLIN>(R, ri, nr, I, margin, fc, u, v, o);
        int code = (fa ? ri : 3 + ri) * 32;
        C.m = o.m;
        C.ids = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            C.p[k] = madd(madd(madd(fc, u, o.u[k]), v, o.v[k]), nr, o.n[k] * real(0.5));
            C.d[k] = o.n[k];
            C.ids |= (uint32_t)(o.id[k] + code) << (8 * k);
        }
        return;
    }
    // edge-edge
    real L = sqrt_(dot(bax, bax));
    V3 w = mk(bax.x / L, bax.y / L, bax.z / L);
    w = selv(dot(w, d) < real(0.0), neg(w), w);
    C.n = w;
    V3 pa = A.c, pb = B.c;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        real sg = (dot(Aax[k], w) > real(0.0)) ? real(1.0) : -real(1.0);
        if (k != bi) pa = madd(pa, Aax[k], sg * Ah[k]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        real sg = (dot(Bax[k], w) > real(0.0)) ? -real(1.0) : real(1.0);
        if (k != bj) pb = madd(pb, Bax[k], sg * Bh[k]);
    }
    V3 ua = axis_of(A.ax, bi), ub = axis_of(B.ax, bj);
    V3 r = sub(pb, pa);
    real c = dot(ua, ub), ar = dot(ua, r), br = dot(ub, r);
    real den = fma_(-c, c, real(1.0));
    real s = fma_(-c, br, ar) / den;
    real t = fma_(c, ar, -br) / den;
    real ha = sel3(A.h0, A.h1, A.h2, bi), hb = sel3(B.h0, B.h1, B.h2, bj);
    s = s > ha ? ha : (s < -ha ? -ha : s);
    t = t > hb ? hb : (t < -hb ? -hb : t);
    V3 qa = madd(pa, ua, s), qb = madd(pb, ub, t);
    C.m = 1;
    C.p[0] = scl(add(qa, qb), real(0.5));
    C.d[0] = best;
    C.ids = (uint32_t)(6 * 32 + 3 * bi + bj);
}

CP_DEV void plane_space(V3 n, V3& t1, V3& t2) {
    if (abs_(n.z) > (real)0.7071067811865476) {
        real a = fma_(n.y, n.y, n.z * n.z);
        real k = real(1.0) / sqrt_(a);
        t1 = mk(real(0.0), -(n.z * k), n.y * k);
        t2 = mk(a * k, -(n.x * t1.z), n.x * t1.y);
    } else {
        real a = fma_(n.x, n.x, n.y * n.y);
        real k = real(1.0) / sqrt_(a);
        t1 = mk(-(n.y * k), n.x * k, real(0.0));
        t2 = mk(-(n.z * t1.y), n.z * t1.x, a * k);
    }
}

// ----------------------------------------------------------------------------
// Lane pairs.  Two adjacent lanes simulate one env: lane 2e+p owns contact island
// p: island 0 = ground, cart, pole (pairs 0 1 4) plus the
// cross pairs 5 6; island 1 = ground, cart2, pole2 (pairs 2 3 9) plus 7 8.  Both
// lanes keep the whole env state; they exchange results through DPP swaps.
CP_DEV V3 partner(V3 v) { return mk(partner(v.x), partner(v.y), partner(v.z)); }
template <int ISL>
CP_DEV V3 lane_of3(V3 v) { return mk(lane_of<ISL>(v.x), lane_of<ISL>(v.y), lane_of<ISL>(v.z)); }

// global pair of island `isl`'s local pair j (oracle: ISLAND_PAIR)
CP_DEV int island_pair(int isl, int j) { return (int)(((isl ? 0x87932u : 0x65410u) >> (4 * j)) & 15u); }
__host__ __device__ constexpr int island_of(int p) { return (p == 2 || p == 3 || p >= 7) ? 1 : 0; }
__host__ __device__ constexpr int local_of(int p) {
    return p < 2 ? p : (p < 4 ? p - 2 : (p == 4 ? 2 : (p == 9 ? 2 : (p == 5 || p == 7 ? 3 : 4))));
}

// Per-lane constants of the lane's island (lane-varying copies of cp_physics fields).
struct Lane {
    int isl;
    int pj;             // WIDE kernels: the local pair whose narrowphase this lane computes (>= 5: none)
    real im1, im2;      // inverse masses of the island's cart, pole
    real ii1[3], ii2[3];  // their body-frame inverse inertias
    real mu0, mu1, mu2; // friction products of local pairs 0..2
    CP_DEV static Lane make(int isl, const cp_physics& P) {
        Lane L;
        L.isl = isl;
        L.pj = 0;
        L.im1 = isl ? P.inv_mass[3] : P.inv_mass[1];
        L.im2 = isl ? P.inv_mass[4] : P.inv_mass[2];
        for (int k = 0; k < 3; ++k) {
            L.ii1[k] = isl ? P.inv_inertia[3][k] : P.inv_inertia[1][k];
            L.ii2[k] = isl ? P.inv_inertia[4][k] : P.inv_inertia[2][k];
        }
        const real fc = isl ? P.friction[3] : P.friction[1], fq = isl ? P.friction[4] : P.friction[2];
        L.mu0 = P.friction[0] * fc;
        L.mu1 = P.friction[0] * fq;
        L.mu2 = fc * fq;
        return L;
    }
};

// Per-substep context (registers).
struct Step {
    Sym M[CP_NUM_DYN];            // whole-env world inverse inertias (merged solve only)
    V3 n[CP_ISLAND_PAIRS];        // own island's manifold normals
    uint32_t pk[CP_ISLAND_PAIRS]; // cnt | base<<3 | fcnt<<8 | fbase<<11
};
CP_DEV int pk_cnt(uint32_t pk) { return (int)(pk & 7u); }
CP_DEV int pk_base(uint32_t pk) { return (int)((pk >> 3) & 31u); }
CP_DEV int pk_fcnt(uint32_t pk) { return (int)((pk >> 8) & 7u); }
CP_DEV int pk_fbase(uint32_t pk) { return (int)((pk >> 11) & 15u); }
// warm-start cache slots of the pair that may hold a nonzero impulse: max(new count, old
// count); the slots past it hold 0 before and after the refresh (substep_finish)
CP_DEV int pk_wcnt(uint32_t pk) { return (int)((pk >> 16) & 7u); }

// ---- independent island solve: the island's two dynamic bodies in local slots
// 1 (cart) and 2 (pole); slot 0 is the static ground.  Same arithmetic as the
// oracle's solve_row / apply_impulse on the global bodies.
struct Dyn {
    V3 x, v, w;
    Sym M;
};
struct Isl {
    Dyn d1, d2;
    real im1, im2;
};
template <int K>
CP_DEV Dyn& dyn(Isl& I) {
    if constexpr (K == 1) return I.d1;
    else return I.d2;
}
template <int K>
CP_DEV real dyn_im(const Isl& I) {
    if constexpr (K == 1) return I.im1;
    else return I.im2;
}

template <int A, int B>
CP_DEV void isl_impulse(Isl& I, V3 rb, V3 t, real lam) {
    Dyn& b = dyn<B>(I);
    V3 rbt = cross(rb, t);
    V3 ib = symv(b.M, rbt);
    b.v = madd(b.v, t, lam * dyn_im<B>(I));
    b.w = madd(b.w, ib, lam);
    if constexpr (A != 0) {
        Dyn& a = dyn<A>(I);
        V3 ra = add(rb, sub(b.x, a.x));
        V3 rat = cross(ra, t);
        V3 ia = symv(a.M, rat);
        a.v = madd(a.v, neg(t), lam * dyn_im<A>(I));
        a.w = madd(a.w, neg(ia), lam);
    }
}

template <int A, int B, bool FRICTION>
CP_DEV bool isl_row(Isl& I, V3 rb, V3 t, real inv_eff, real target, real& lam, real bound, real tol) {
    Dyn& b = dyn<B>(I);
    const real imb = dyn_im<B>(I);
    V3 rbt = cross(rb, t);
    V3 ib = symv(b.M, rbt);
    real vn;
    V3 ia = mk(real(0.0), real(0.0), real(0.0));
    if constexpr (A == 0) {
        vn = dot(t, b.v) + dot(b.w, rbt);
    } else {
        Dyn& a = dyn<A>(I);
        V3 ra = add(rb, sub(b.x, a.x));
        V3 rat = cross(ra, t);
        ia = symv(a.M, rat);
        vn = (dot(t, sub(b.v, a.v)) + dot(b.w, rbt)) - dot(a.w, rat);
    }
    real e = target - vn;
    real dl = e * inv_eff;
    real l0 = lam + dl;
    real ln;
    if constexpr (!FRICTION) ln = l0 > real(0.0) ? l0 : real(0.0);
    else ln = bound > real(0.0) ? clamp_sym(l0, bound) : lam;  // see isl_row_ez
    dl = ln - lam;
    lam = ln;
    real sb = dl * imb;
    b.v = madd(b.v, t, sb);
    b.w = madd(b.w, ib, dl);
    if constexpr (A != 0) {
        Dyn& a = dyn<A>(I);
        real sa = dl * dyn_im<A>(I);
        a.v = madd(a.v, neg(t), sa);
        a.w = madd(a.w, neg(ia), dl);
    }
    return abs_(dl) > tol * inv_eff;  // Bullet residual test (oracle: solve_row)
}

// isl_row<0, B> for a ground manifold whose normal is exactly +z (the static ground's top
// face is the reference face: every pole-ground manifold of the bench steady state,
// tools/row_classes.py).  Then plane_space gives t1 = (0, -1, 0), t2 = (1, -0, -0), and
// every term of isl_row that multiplies an exact 0 or +-1 drops out value-exactly:
// FMA(+-0, x, y) = y and FMA(+-1, x, y) = y +- x (finite operands; only the sign of an
// exact zero result can differ).  KIND 0: t = n, 1: t = t1, 2: t = t2.  Same values as
// isl_row, about 60 % of its VALU work (no r x t, 6 of the 9 products of M (r x t)).
template <int B, int KIND, bool FRICTION>
CP_DEV bool isl_row_ez(Isl& I, V3 rb, real inv_eff, real target, real& lam, real bound, real tol) {
    Dyn& b = dyn<B>(I);
    const real imb = dyn_im<B>(I);
    const Sym& M = b.M;
    V3 ib;
    real vn;
    if constexpr (KIND == 0) {         // r x n = (rb.y, -rb.x, 0)
        const real px = rb.y, py = -rb.x;
        ib = mk(fma_(M.m0, px, M.m1 * py), fma_(M.m1, px, M.m3 * py), fma_(M.m2, px, M.m4 * py));
        vn = b.v.z + fma_(b.w.x, px, b.w.y * py);
    } else if constexpr (KIND == 1) {  // r x t1 = (rb.z, 0, -rb.x)
        const real px = rb.z, pz = -rb.x;
        ib = mk(fma_(M.m0, px, M.m2 * pz), fma_(M.m1, px, M.m4 * pz), fma_(M.m2, px, M.m5 * pz));
        vn = -b.v.y + fma_(b.w.x, px, b.w.z * pz);
    } else {                           // r x t2 = (0, rb.z, -rb.y)
        const real py = rb.z, pz = -rb.y;
        ib = mk(fma_(M.m1, py, M.m2 * pz), fma_(M.m3, py, M.m4 * pz), fma_(M.m4, py, M.m5 * pz));
        vn = b.v.x + fma_(b.w.y, py, b.w.z * pz);
    }
    real e = target - vn;
    real dl = e * inv_eff;
    real l0 = lam + dl;
    real ln;
    // friction rows: Bullet skips the row while the normal impulse is not > 0 (lambda stays,
    // dl = 0, no residual); else the clamp as one v_med3_f32 (bound > 0): the same value as
    // the oracle's compare chain for every non-NaN l0, one dependent instruction instead of
    // three
    if constexpr (!FRICTION) ln = l0 > real(0.0) ? l0 : real(0.0);
    else ln = bound > real(0.0) ? clamp_sym(l0, bound) : lam;
    dl = ln - lam;
    lam = ln;
    real sb = dl * imb;
    if constexpr (KIND == 0) b.v.z = b.v.z + sb;
    else if constexpr (KIND == 1) b.v.y = b.v.y - sb;
    else b.v.x = b.v.x + sb;
    b.w = madd(b.w, ib, dl);
    return abs_(dl) > tol * inv_eff;  // Bullet residual test (oracle: solve_row)
}
CP_DEV bool is_plus_z(V3 n) { return n.x == real(0.0) && n.y == real(0.0) && n.z == real(1.0); }

// local pair j (0..2) of the island: (ground, cart), (ground, pole), (cart, pole)
template <int J> constexpr int loc_a() { return J == 2 ? 1 : 0; }
template <int J> constexpr int loc_b() { return J == 0 ? 1 : 2; }

template <int J, bool PM = false>
CP_DEV void isl_warmstart(Isl& I, const Step& T, real* pool) {
    const uint32_t pk = T.pk[J];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    for (int k = 0; k < cnt; ++k) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        isl_impulse<loc_a<J>(), loc_b<J>()>(I, rb, PM ? pool_normal(pool, s) : T.n[J], pool_n(pool, F_LAM, s));
    }
}

// the generic row loops are counted loops (unrolled to the 4-point bound they were measured slower)
#define CP_ROW_LOOP(k, n) for (int k = 0; k < (n); ++k)
template <int J, bool PM = false>
CP_DEV void isl_normal_rows(Isl& I, const Step& T, real* pool, real tol, bool& bad) {
    const uint32_t pk = T.pk[J];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    CP_ROW_LOOP(k, cnt) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real lam = pool_n(pool, F_LAM, s);
        bad |= isl_row<loc_a<J>(), loc_b<J>(), false>(I, rb, PM ? pool_normal(pool, s) : T.n[J], pool_n(pool, F_IE, s),
                                                      pool_n(pool, F_TG, s), lam, real(0.0), tol);
        pool_n(pool, F_LAM, s) = lam;
    }
}

template <int J, bool HOISTED = false, bool PM = false>
CP_DEV void isl_friction_rows(Isl& I, const Step& T, real mu, real* pool, real tol, bool& bad, V3 ht1 = V3{},
                              V3 ht2 = V3{}) {
    const uint32_t pk = T.pk[J];
    const int fcnt = pk_fcnt(pk);
    if (fcnt == 0) return;
    const int base = pk_base(pk), fbase = pk_fbase(pk);
    V3 t1, t2;
    if constexpr (HOISTED) {
        t1 = ht1;
        t2 = ht2;
    } else if constexpr (!PM) {
        // tangent basis inside the sweep (cross pairs: hoisted it would pin VGPRs for rare rows)
        V3 n = T.n[J];
        asm volatile("" : "+v"(n.x), "+v"(n.y), "+v"(n.z));
        plane_space(n, t1, t2);
    }
    CP_ROW_LOOP(k, fcnt) {
        const int s = base + k, fs = fbase + k;
        if constexpr (PM) plane_space(pool_normal(pool, s), t1, t2);  // the point's own normal
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real bound = mu * pool_n(pool, F_LAM, s);
        real l1 = pool_f(pool, FF_L1, fs), l2 = pool_f(pool, FF_L2, fs);
        bad |= isl_row<loc_a<J>(), loc_b<J>(), true>(I, rb, t1, pool_f(pool, FF_IE1, fs), real(0.0), l1, bound, tol);
        bad |= isl_row<loc_a<J>(), loc_b<J>(), true>(I, rb, t2, pool_f(pool, FF_IE2, fs), real(0.0), l2, bound, tol);
        pool_f(pool, FF_L1, fs) = l1;
        pool_f(pool, FF_L2, fs) = l2;
    }
}

// row loops unrolled to the 4-point manifold bound (a box pair makes at most 4 points):
// step kernel 0.709 -> 0.692 ms against the counted loop
#define CP_EZ_LOOP(k, n) _Pragma("unroll") for (int k = 0; k < 4; ++k) if (k < (n))
// The rows of ground pair J (0 or 1) when every lane of the wave with rows on it has a +z
// normal (wave-uniform choice in sweeps()): the same sweep with isl_row_ez.
template <int J>
CP_DEV void isl_normal_rows_ez(Isl& I, const Step& T, real* pool, real tol, bool& bad) {
    static_assert(loc_a<J>() == 0, "ground pairs only");
    const uint32_t pk = T.pk[J];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    CP_EZ_LOOP(k, cnt) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real lam = pool_n(pool, F_LAM, s);
        bad |= isl_row_ez<loc_b<J>(), 0, false>(I, rb, pool_n(pool, F_IE, s), pool_n(pool, F_TG, s), lam, real(0.0), tol);
        pool_n(pool, F_LAM, s) = lam;
    }
}
template <int J>
CP_DEV void isl_friction_rows_ez(Isl& I, const Step& T, real mu, real* pool, real tol, bool& bad) {
    static_assert(loc_a<J>() == 0, "ground pairs only");
    const uint32_t pk = T.pk[J];
    const int fcnt = pk_fcnt(pk);
    if (fcnt == 0) return;
    const int base = pk_base(pk), fbase = pk_fbase(pk);
    CP_EZ_LOOP(k, fcnt) {
        const int s = base + k, fs = fbase + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real bound = mu * pool_n(pool, F_LAM, s);
        real l1 = pool_f(pool, FF_L1, fs), l2 = pool_f(pool, FF_L2, fs);
        bad |= isl_row_ez<loc_b<J>(), 1, true>(I, rb, pool_f(pool, FF_IE1, fs), real(0.0), l1, bound, tol);
        bad |= isl_row_ez<loc_b<J>(), 2, true>(I, rb, pool_f(pool, FF_IE2, fs), real(0.0), l2, bound, tol);
        pool_f(pool, FF_L1, fs) = l1;
        pool_f(pool, FF_L2, fs) = l2;
    }
}

// ---- merged solve (an env with a cross-island contact): both lanes run the
// oracle's global-order solve redundantly on the whole env, reading each
// island's rows from that island's lane column of the LDS pool and its manifold
// header from that island's lane registers (DPP; both lanes of a merged env are
// active, so the partner read is defined).
struct Hdr {
    V3 n;
    uint32_t pk;
};
template <int PAIR>
CP_DEV Hdr pair_hdr(const Step& T, bool second) {
    (void)second;
    constexpr int j = local_of(PAIR), isl = island_of(PAIR) != 0 ? 1 : 0;
    const V3 tn = T.n[j];
    const uint32_t tpk = T.pk[j];
    Hdr h;  // the owning island's lane's header, on both lanes
    h.n = lane_of3<isl>(tn);
    h.pk = lane_of_u<isl>(tpk);
    return h;
}

// impulse lam along t at rb (oracle: apply_impulse); A == 0 is the static ground
template <int A, int B>
CP_DEV void apply_impulse(Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t, real lam) {
    V3 rbt = cross(rb, t);
    V3 ib = symv(T.M[B - 1], rbt);
    S.b[B - 1].v = madd(S.b[B - 1].v, t, lam * P.inv_mass[B]);
    S.b[B - 1].w = madd(S.b[B - 1].w, ib, lam);
    if constexpr (A != 0) {
        V3 ra = add(rb, sub(S.b[B - 1].x, S.b[A - 1].x));
        V3 rat = cross(ra, t);
        V3 ia = symv(T.M[A - 1], rat);
        S.b[A - 1].v = madd(S.b[A - 1].v, neg(t), lam * P.inv_mass[A]);
        S.b[A - 1].w = madd(S.b[A - 1].w, neg(ia), lam);
    }
}

// One PGS row (oracle: solve_row).  Returns |e * dlambda|.
template <int A, int B, bool FRICTION>
CP_DEV bool solve_row(Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t, real inv_eff, real target,
                      real& lam, real bound, real tol) {
    real imb = P.inv_mass[B];
    V3 rbt = cross(rb, t);
    V3 ib = symv(T.M[B - 1], rbt);
    real vn;
    V3 ia = mk(real(0.0), real(0.0), real(0.0));
    if constexpr (A == 0) {
        vn = dot(t, S.b[B - 1].v) + dot(S.b[B - 1].w, rbt);
    } else {
        V3 ra = add(rb, sub(S.b[B - 1].x, S.b[A - 1].x));
        V3 rat = cross(ra, t);
        ia = symv(T.M[A - 1], rat);
        vn = (dot(t, sub(S.b[B - 1].v, S.b[A - 1].v)) + dot(S.b[B - 1].w, rbt)) - dot(S.b[A - 1].w, rat);
    }
    real e = target - vn;
    real dl = e * inv_eff;
    real l0 = lam + dl;
    real ln;
    if constexpr (!FRICTION) ln = l0 > real(0.0) ? l0 : real(0.0);
    else ln = bound > real(0.0) ? clamp_sym(l0, bound) : lam;  // see isl_row_ez
    dl = ln - lam;
    lam = ln;
    real sb = dl * imb;
    S.b[B - 1].v = madd(S.b[B - 1].v, t, sb);
    S.b[B - 1].w = madd(S.b[B - 1].w, ib, dl);
    if constexpr (A != 0) {
        real sa = dl * P.inv_mass[A];
        S.b[A - 1].v = madd(S.b[A - 1].v, neg(t), sa);
        S.b[A - 1].w = madd(S.b[A - 1].w, neg(ia), dl);
    }
    return abs_(dl) > tol * inv_eff;  // Bullet residual test (oracle: solve_row)
}

template <int PAIR, bool PM = false>
CP_DEV void pair_warmstart(Sim& S, const Step& T, bool second, const cp_physics& P, real* pool0) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    real* pool = pool0 + island_of(PAIR);
    const Hdr H = pair_hdr<PAIR>(T, second);
    const uint32_t pk = H.pk;
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    for (int k = 0; k < cnt; ++k) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        apply_impulse<A, B>(S, T, P, rb, PM ? pool_normal(pool, s) : H.n, pool_n(pool, F_LAM, s));
    }
}

template <int PAIR, bool PM = false>
CP_DEV void pair_normal_rows(Sim& S, const Step& T, bool second, const cp_physics& P, real* pool0,
                             real tol, bool& bad) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    real* pool = pool0 + island_of(PAIR);
    const Hdr H = pair_hdr<PAIR>(T, second);
    const uint32_t pk = H.pk;
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    for (int k = 0; k < cnt; ++k) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real lam = pool_n(pool, F_LAM, s);
        bad |= solve_row<A, B, false>(S, T, P, rb, PM ? pool_normal(pool, s) : H.n, pool_n(pool, F_IE, s),
                                      pool_n(pool, F_TG, s), lam, real(0.0), tol);
        pool_n(pool, F_LAM, s) = lam;
    }
}

template <int PAIR, bool PM = false>
CP_DEV void pair_friction_rows(Sim& S, const Step& T, bool second, const cp_physics& P, real* pool0,
                               real tol, bool& bad) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    real* pool = pool0 + island_of(PAIR);
    const Hdr H = pair_hdr<PAIR>(T, second);
    const uint32_t pk = H.pk;
    const int fcnt = pk_fcnt(pk);
    if (fcnt == 0) return;
    const int base = pk_base(pk), fbase = pk_fbase(pk);
    const real mu = real(P.friction[A]) * real(P.friction[B]);  // oracle: (real) * (real)
    V3 t1, t2;
    if constexpr (!PM) {
        V3 n = H.n;
        asm volatile("" : "+v"(n.x), "+v"(n.y), "+v"(n.z));
        plane_space(n, t1, t2);
    }
    for (int k = 0; k < fcnt; ++k) {
        const int s = base + k, fs = fbase + k;
        if constexpr (PM) plane_space(pool_normal(pool, s), t1, t2);
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        real bound = mu * pool_n(pool, F_LAM, s);
        real l1 = pool_f(pool, FF_L1, fs), l2 = pool_f(pool, FF_L2, fs);
        bad |= solve_row<A, B, true>(S, T, P, rb, t1, pool_f(pool, FF_IE1, fs), real(0.0), l1, bound, tol);
        bad |= solve_row<A, B, true>(S, T, P, rb, t2, pool_f(pool, FF_IE2, fs), real(0.0), l2, bound, tol);
        pool_f(pool, FF_L1, fs) = l1;
        pool_f(pool, FF_L2, fs) = l2;
    }
}

// ---- body selection of the narrowphase pair loop.  The local pair j is wave-uniform and its
// bodies differ between the two islands only: with j dispatched through a uniform branch
// (pair_bodies), every selection is a 2-way select on the lane's island, one v_cndmask_b32 per
// value.  (A 5-way choice over the lane-varying body id compiles to an exec-mask branch tree:
// lone-wave narrowphase ~40k cycles per substep against ~30k for four opaque selects.)
__host__ __device__ constexpr int island_pair_c(int isl, int j) {
    return (int)(((isl ? 0x87932u : 0x65410u) >> (4 * j)) & 15u);
}
// Box of a body with the half extents of dynamic body G0 (island 0 lanes) or G1 (island 1 lanes): the
// axes are rebuilt from the quaternion here rather than kept live through the narrowphase (same
// arithmetic as the per-body quat_axes / world_inv_inertia).
template <int G0, int G1, bool AX = true>
CP_DEV Box box_of(bool second, const V3& x, const real q[4], const cp_physics& P) {
    static_assert(G0 >= 1 && G1 >= 1, "dynamic bodies only");
    Box b;
    b.h0 = second ? real(P.half_extents[G1][0]) : real(P.half_extents[G0][0]);
    b.h1 = second ? real(P.half_extents[G1][1]) : real(P.half_extents[G0][1]);
    b.h2 = second ? real(P.half_extents[G1][2]) : real(P.half_extents[G0][2]);
    b.c = x;
    if constexpr (AX) b.ax = quat_axes(q[0], q[1], q[2], q[3]);
    else b.ax = quat_axes(real(0.0), real(0.0), real(0.0), real(1.0));  // placeholder (pair_body: late B axes)
    return b;
}
template <int G0, int G1>
CP_DEV real pick_f(bool second, const float* v) { return second ? real(v[G1]) : real(v[G0]); }
template <int G0, int G1>
CP_DEV Sym inertia_pick(bool second, const Box& b, const cp_physics& P) {
    return world_inv_inertia(b.ax, second ? real(P.inv_inertia[G1][0]) : real(P.inv_inertia[G0][0]),
                             second ? real(P.inv_inertia[G1][1]) : real(P.inv_inertia[G0][1]),
                             second ? real(P.inv_inertia[G1][2]) : real(P.inv_inertia[G0][2]));
}
// f(std::integral_constant<int, J>) for the wave-uniform local pair j (GROUND: j is 0 or 1)
template <bool GROUND, typename F>
CP_DEV void pair_dispatch(int j, F&& f) {
    if constexpr (GROUND) {
        if (j == 0) f(std::integral_constant<int, 0>{});
        else f(std::integral_constant<int, 1>{});
    } else {
        if (j == 2) f(std::integral_constant<int, 2>{});
        else if (j == 3) f(std::integral_constant<int, 3>{});
        else f(std::integral_constant<int, 4>{});
    }
}

// Broadphase: true when a face axis of A already separates the pair by more than
// the margin (bounding radius of B as its projection, plus 1e-3 m of slack for
// rounding), i.e. when box_box would return no contact from its face-axis test.
CP_DEV bool face_separated(const Box& A, const Box& B, real margin) {
    const V3 d = sub(B.c, A.c);
    const real rb = sqrt_(fma_(B.h0, B.h0, fma_(B.h1, B.h1, B.h2 * B.h2)));
    const real lim = (margin + real(1e-3)) + rb;
    return (abs_(dot(d, A.ax.a0)) - A.h0 > lim) || (abs_(dot(d, A.ax.a1)) - A.h1 > lim) ||
           (abs_(dot(d, A.ax.a2)) - A.h2 > lim);
}
// row setup for direction t with pair bodies selected at run time (narrowphase)
CP_DEV real row_k_dyn(int a, real ima, real imb, V3 xa, V3 xb, const Sym& Ma, const Sym& Mb, V3 rb, V3 t) {
    V3 rbt = cross(rb, t);
    V3 ib = symv(Mb, rbt);
    if (a == 0) return imb + dot(rbt, ib);
    V3 ra = add(rb, sub(xb, xa));
    V3 rat = cross(ra, t);
    V3 ia = symv(Ma, rat);
    return ((ima + imb) + dot(rat, ia)) + dot(rbt, ib);
}

// btMultiBody::applyDeltaVeeMultiDof [ext]: every base velocity coordinate (world angular, then
// linear) clamped to +-m_maxCoordinateVelocity after each velocity change.  btClamp's
// compares, not v_med3 / v_min / v_max: a NaN passes through, as in the oracle (clamp_velocities)
// a select between two kernel-argument fields by value: the two loads go through an empty asm, so that
// the optimizer cannot fold them into one load through a selected address (which copies the whole
// cp_config argument into scratch memory)
CP_DEV real sel_arg(bool second, float a, float b) {
    real x = a, y = b;
    asm volatile("" : "+v"(x), "+v"(y));
    return second ? y : x;
}
CP_DEV real clamp_coord(real a, real lim) { return a < -lim ? -lim : (lim < a ? lim : a); }
CP_DEV void clamp_body(Body& b, real lim) {
    b.w = mk(clamp_coord(b.w.x, lim), clamp_coord(b.w.y, lim), clamp_coord(b.w.z, lim));
    b.v = mk(clamp_coord(b.v.x, lim), clamp_coord(b.v.y, lim), clamp_coord(b.v.z, lim));
}
CP_DEV void clamp_velocities(Own& O, const cp_physics& P) {
    const real lim = real(P.max_coord_velocity);
    if (!(lim > real(0.0))) return;  // uniform (a kernel argument)
    clamp_body(O.c, lim);
    clamp_body(O.p, lim);
}

// One body of island ISL (0: the even lane's, 1: the odd lane's) on both lanes of the pair (DPP).
template <int ISL>
CP_DEV Body body_of(const Body& b) {
    Body r;
    r.x = lane_of3<ISL>(b.x);
    r.v = lane_of3<ISL>(b.v);
    r.w = lane_of3<ISL>(b.w);
#pragma unroll
    for (int k = 0; k < 4; ++k) r.q[k] = lane_of<ISL>(b.q[k]);
    return r;
}
// The whole env on both lanes, from the two lanes' Own states (both lanes active).
CP_DEV Sim env_view(const Own& O) {
    Sim S;
    S.b[0] = body_of<0>(O.c);
    S.b[1] = body_of<0>(O.p);
    S.b[2] = body_of<1>(O.c);
    S.b[3] = body_of<1>(O.p);
    S.f0 = lane_of3<0>(O.f);
    S.f2 = lane_of3<1>(O.f);
    return S;
}

// ---- CP_MODEL_SLEEPING (the SLP kernels): Bullet's deactivation, operation for operation the oracle's
// body_aabb / sleep_islands / sleep_update (oracle/cp_oracle.c).  Each lane computes its
// own bodies' AABBs; the partner's come by DPP, so both lanes run the island pass on identical values.
// AABB of a body of half extents h: btTransformAabb of the box grown by the contact breaking threshold
CP_DEV void body_aabb(const Body& B, real h0, real h1, real h2, const cp_physics& P, V3& lo, V3& hi) {
    const Axes A = quat_axes(B.q[0], B.q[1], B.q[2], B.q[3]);
    const real thr = P.contact_margin;
    const real ex = (h0 * abs_(A.a0.x) + h1 * abs_(A.a1.x)) + h2 * abs_(A.a2.x);
    const real ey = (h0 * abs_(A.a0.y) + h1 * abs_(A.a1.y)) + h2 * abs_(A.a2.y);
    const real ez = (h0 * abs_(A.a0.z) + h1 * abs_(A.a1.z)) + h2 * abs_(A.a2.z);
    const V3 c = B.x;
    lo = mk((c.x - ex) - thr, (c.y - ey) - thr, (c.z - ez) - thr);
    hi = mk((c.x + ex) + thr, (c.y + ey) + thr, (c.z + ez) + thr);
}
CP_DEV bool aabb_overlap(const V3& la, const V3& ha, const V3& lb, const V3& hb) {
    return !(la.x > hb.x || ha.x < lb.x || la.y > hb.y || ha.y < lb.y || la.z > hb.z || ha.z < lb.z);
}
// the start of a step: islands of AABB-overlapping bodies and btSimulationIslandManager::buildIslands'
// activation pass; returns the mask of bodies that sleep this step (bit d = dynamic body d, env order)
CP_DEV uint32_t sleep_islands(Own& O, const cp_physics& P, bool second) {
    V3 lc, hc, lp, hp;
    body_aabb(O.c, sel_arg(second, P.half_extents[1][0], P.half_extents[3][0]),
              sel_arg(second, P.half_extents[1][1], P.half_extents[3][1]),
              sel_arg(second, P.half_extents[1][2], P.half_extents[3][2]), P, lc, hc);
    body_aabb(O.p, sel_arg(second, P.half_extents[2][0], P.half_extents[4][0]),
              sel_arg(second, P.half_extents[2][1], P.half_extents[4][1]),
              sel_arg(second, P.half_extents[2][2], P.half_extents[4][2]), P, lp, hp);
    V3 lo[CP_NUM_DYN], hi[CP_NUM_DYN];
    lo[0] = lane_of3<0>(lc); hi[0] = lane_of3<0>(hc);
    lo[1] = lane_of3<0>(lp); hi[1] = lane_of3<0>(hp);
    lo[2] = lane_of3<1>(lc); hi[2] = lane_of3<1>(hc);
    lo[3] = lane_of3<1>(lp); hi[3] = lane_of3<1>(hp);
    uint32_t act[CP_NUM_DYN];
    act[0] = lane_of_u<0>(O.sa[0]); act[1] = lane_of_u<0>(O.sa[1]);
    act[2] = lane_of_u<1>(O.sa[0]); act[3] = lane_of_u<1>(O.sa[1]);
    int root[CP_NUM_DYN] = {0, 1, 2, 3};
#pragma unroll
    for (int a = 0; a < CP_NUM_DYN; ++a)
#pragma unroll
        for (int b = a + 1; b < CP_NUM_DYN; ++b) {
            const bool ov = aabb_overlap(lo[a], hi[a], lo[b], hi[b]);
            const int ra = root[a], rb = root[b];
            const int lr = ra < rb ? ra : rb, hr = ra < rb ? rb : ra;
#pragma unroll
            for (int d = 0; d < CP_NUM_DYN; ++d) root[d] = (ov && root[d] == hr) ? lr : root[d];
        }
#pragma unroll
    for (int r = 0; r < CP_NUM_DYN; ++r) {
        bool any_active = false;
#pragma unroll
        for (int d = 0; d < CP_NUM_DYN; ++d) any_active |= root[d] == r && (act[d] & 15u) == CP_ACT_ACTIVE;
#pragma unroll
        for (int d = 0; d < CP_NUM_DYN; ++d) {
            const uint32_t aw = act[d] & (uint32_t)CP_ACT_AWAKE;
            const bool mine = root[d] == r;
            const uint32_t na = !any_active ? ((uint32_t)CP_ACT_SLEEPING | aw)
                              : ((act[d] & 15u) == CP_ACT_SLEEPING ? ((uint32_t)CP_ACT_WANTS | aw) : act[d]);
            act[d] = mine ? na : act[d];
        }
    }
    O.sa[0] = second ? act[2] : act[0];
    O.sa[1] = second ? act[3] : act[1];
    uint32_t mask = 0u;
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) mask |= ((act[d] & 15u) == CP_ACT_SLEEPING ? 1u : 0u) << d;
    return mask;
}
// the end of a step: btMultiBody::checkMotionAndSleepIfRequired + updateActivationState (own bodies)
CP_DEV void sleep_body(const Body& B, uint32_t& a, real& t, const cp_physics& P) {
    const real dt = P.dt, eps = P.sleep_epsilon, tmo = P.sleep_timeout;
    const V3 w = B.w, v = B.v;
    const real motion = ((((w.x * w.x + w.y * w.y) + w.z * w.z) + v.x * v.x) + v.y * v.y) + v.z * v.z;
    const bool still = motion < eps;
    t = still ? t + dt : real(0.0);
    a = still ? (t > tmo ? (a & ~(uint32_t)CP_ACT_AWAKE) : a) : (a | (uint32_t)CP_ACT_AWAKE);
    a = (a & (uint32_t)CP_ACT_AWAKE) ? ((uint32_t)CP_ACT_ACTIVE | (uint32_t)CP_ACT_AWAKE)
        : ((a & 15u) == CP_ACT_ACTIVE ? (uint32_t)CP_ACT_WANTS : a);
}
CP_DEV void sleep_update(Own& O, const cp_physics& P) {
    sleep_body(O.c, O.sa[0], O.st[0], P);
    sleep_body(O.p, O.sa[1], O.st[1], P);
}
CP_DEV void sleep_wake_all(Own& O) {  // resetBasePositionAndOrientation [ext, low confidence]
    O.sa[0] = O.sa[1] = (uint32_t)CP_ACT_ACTIVE | (uint32_t)CP_ACT_AWAKE;
    O.st[0] = O.st[1] = real(0.0);
}

// whole-env view for the cross rows: positions, velocities and inverse inertias of
// the own island's bodies from this lane, the other island's from the partner lane
// (both lanes of a merged env are active wherever this runs).
CP_DEV Sym partner_sym(const Sym& m) {
    Sym r;
    r.m0 = partner(m.m0); r.m1 = partner(m.m1); r.m2 = partner(m.m2);
    r.m3 = partner(m.m3); r.m4 = partner(m.m4); r.m5 = partner(m.m5);
    return r;
}
CP_DEV Sym sel_sym(bool t, const Sym& a, const Sym& b) {
    Sym r;
    r.m0 = t ? a.m0 : b.m0; r.m1 = t ? a.m1 : b.m1; r.m2 = t ? a.m2 : b.m2;
    r.m3 = t ? a.m3 : b.m3; r.m4 = t ? a.m4 : b.m4; r.m5 = t ? a.m5 : b.m5;
    return r;
}
template <int ISL>
CP_DEV Sym lane_of_sym(const Sym& m) {
    Sym r;
    r.m0 = lane_of<ISL>(m.m0); r.m1 = lane_of<ISL>(m.m1); r.m2 = lane_of<ISL>(m.m2);
    r.m3 = lane_of<ISL>(m.m3); r.m4 = lane_of<ISL>(m.m4); r.m5 = lane_of<ISL>(m.m5);
    return r;
}
CP_DEV void cross_view(Sim& S, Step& T, const Isl& I, bool second) {
    (void)second;
    // island 0's bodies (cart, pole) from the pair's even lane, island 1's (cart2, pole2) from the odd
    // lane, one DPP move per value on both lanes (S is scratch: each lane holds only its own island)
    S.b[0].x = lane_of3<0>(I.d1.x);
    S.b[1].x = lane_of3<0>(I.d2.x);
    S.b[2].x = lane_of3<1>(I.d1.x);
    S.b[3].x = lane_of3<1>(I.d2.x);
    S.b[0].v = lane_of3<0>(I.d1.v);
    S.b[0].w = lane_of3<0>(I.d1.w);
    S.b[1].v = lane_of3<0>(I.d2.v);
    S.b[1].w = lane_of3<0>(I.d2.w);
    S.b[2].v = lane_of3<1>(I.d1.v);
    S.b[2].w = lane_of3<1>(I.d1.w);
    S.b[3].v = lane_of3<1>(I.d2.v);
    S.b[3].w = lane_of3<1>(I.d2.w);
    const Sym oM1 = I.d1.M, oM2 = I.d2.M;
    T.M[0] = lane_of_sym<0>(oM1);
    T.M[1] = lane_of_sym<0>(oM2);
    T.M[2] = lane_of_sym<1>(oM1);
    T.M[3] = lane_of_sym<1>(oM2);
}
CP_DEV void cross_back(Isl& I, const Sim& S, bool second) {
    I.d1.v = selv(second, S.b[2].v, S.b[0].v);
    I.d1.w = selv(second, S.b[2].w, S.b[0].w);
    I.d2.v = selv(second, S.b[3].v, S.b[1].v);
    I.d2.w = selv(second, S.b[3].w, S.b[1].w);
}

// Per-lane solve state of one substep, between its phases (prep -> sweeps -> finish):
// everything a lane needs to run its island's PGS sweeps, plus its LDS pool column.
struct Ctx {
    Step T;          // own island's manifold headers (+ whole-env M for the cross rows)
    Isl I;           // own island's bodies
    real mu0, mu1, mu2;
    int used, tot;   // rows of the own island, of the env
    bool merged, active;
    bool xfric;      // merged, and a cross pair of the env has friction rows (only pole-pole contacts do:
                     // the carts' friction is 0); else the friction half of the cross block is a no-op
    uint32_t slp;    // CP_MODEL_SLEEPING: the bodies that sleep this step (bit d = dynamic body d); else 0
};

// One PGS sweep range [it0, it1) over the lane's island (+ the cross rows of a merged
// env).  S supplies positions for the cross rows and is scratch for their whole-env
// view.  Both lanes of an env stop together, after the first sweep in which no row of
// the env (island 0, island 1, cross) has a squared residual above the threshold:
// Bullet solves the two islands as one group (oracle: substep, step 4).
CP_DEV bool c44_ok(const Ctx& c);
// how often (in sweeps) the reset kernels' sweep loops re-test whether every active lane of the wave
// has the settle structure (the lanes without it usually converge first)
constexpr int kC44Check = 8;
CP_DEV bool c4k_ok(const Ctx& c);
CP_DEV void sweeps_c44_slow(Ctx& c, real* pool, real tol, int it0, int it1, Stamps& ST);
CP_DEV void sweeps_c4k_slow(Ctx& c, real* pool, real tol, int it0, int it1, Stamps& ST);
CP_DEV bool p1_ok(const Ctx& c);
// sweeps into a solve after which the throughput step kernels' wave raises its issue priority
constexpr int kPrioAfter = 16;
// HX = false: no env of the wave is merged (checked by the caller), so the cross-row blocks and the merge of
// their results into the island view are compiled out of the sweep
template <bool C44 = false, bool PM = false, bool HX = true>
CP_DEV void sweeps(Ctx& c, Sim& S, const cp_physics& P, real* pool, real* pool0, bool second, int it0, int it1,
                   Stamps& ST) {
    const real tol = sqrt_(real(P.residual_threshold));  // oracle: SQRT((real)threshold)
    // the ground-pole pair's tangent basis (with the URDF frictions the only island pair with
    // friction rows: the carts' friction is 0), once per substep instead of once per sweep:
    // step kernel 0.772 -> 0.753 ms
    V3 h1 = mk(real(0.0), real(0.0), real(0.0)), h2 = h1;
    if constexpr (!PM) plane_space(c.T.n[1], h1, h2);
    // ground pairs whose rows all have a +z normal in this wave run isl_row_ez (wave-uniform):
    // the ground-pole pair in every measured wave, the ground-cart pair in ~3 of 4 (PM: every row
    // has its own normal, the generic rows)
    const bool ez0 = !PM && __ballot(pk_cnt(c.T.pk[0]) > 0 && !is_plus_z(c.T.n[0])) == 0ull;
    const bool ez1 = !PM && __ballot(pk_cnt(c.T.pk[1]) > 0 && !is_plus_z(c.T.n[1])) == 0ull;
#ifdef CP_STAMPS
    ST.flags |= (ez0 ? 0u : 2u) | (ez1 ? 0u : 4u);
#endif
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
        // a wave deep into a long solve (a capped env: the launch's tail) takes its SIMD's issue
        // priority from its co-resident partner: C3 +1.2 % (threshold 8, 16 or 30 alike)
        if constexpr (!C44) {
            if (it == it0 + kPrioAfter) {
                __builtin_amdgcn_s_setprio(1);
            }
        }
        if constexpr (C44 && !PM) {  // every still-active lane in the settle structure (the reset kernels)
            if ((it - it0) % kC44Check == 0 && __ballot(c.active && !c44_ok(c)) == 0ull) {
                sweeps_c44_slow(c, pool, tol, it, it1, ST);
                return;
            }
            if (it == it0 && __ballot(c.active && !c4k_ok(c)) == 0ull) {  // the bump phase's structures
                sweeps_c4k_slow(c, pool, tol, it, it1, ST);
                return;
            }
        }
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false, badc = false;
        if (c.active) {
            if (ez0) isl_normal_rows_ez<0>(c.I, c.T, pool, tol, bad);
            else isl_normal_rows<0, PM>(c.I, c.T, pool, tol, bad);
            if (ez1) isl_normal_rows_ez<1>(c.I, c.T, pool, tol, bad);
            else isl_normal_rows<1, PM>(c.I, c.T, pool, tol, bad);
            isl_normal_rows<2, PM>(c.I, c.T, pool, tol, bad);
        }
        const bool cross = HX && c.active && c.merged;  // same on both lanes of an env
        if (HX && __ballot(cross) != 0ull && cross) {
            cross_view(S, c.T, c.I, second);
            pair_normal_rows<5, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<6, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<7, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<8, PM>(S, c.T, second, P, pool0, tol, badc);
            cross_back(c.I, S, second);
        }
        if (c.active) {
            if (ez0) isl_friction_rows_ez<0>(c.I, c.T, c.mu0, pool, tol, bad);
            else isl_friction_rows<0, false, PM>(c.I, c.T, c.mu0, pool, tol, bad);
            if (ez1) isl_friction_rows_ez<1>(c.I, c.T, c.mu1, pool, tol, bad);
            else if (PM) isl_friction_rows<1, false, PM>(c.I, c.T, c.mu1, pool, tol, bad);
            else isl_friction_rows<1, true>(c.I, c.T, c.mu1, pool, tol, bad, h1, h2);
            isl_friction_rows<2, false, PM>(c.I, c.T, c.mu2, pool, tol, bad);
        }
        // the friction half only where a cross pair has friction rows: cross_view + cross_back alone
        // change no value (the whole-env view and back), and a wave with a merged env pays them per sweep
        const bool crossf = cross && c.xfric;
        if (HX && __ballot(crossf) != 0ull && crossf) {
            cross_view(S, c.T, c.I, second);
            pair_friction_rows<5, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<6, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<7, PM>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<8, PM>(S, c.T, second, P, pool0, tol, badc);
            cross_back(c.I, S, second);
        }
        // every lane that entered the loop is here (pairs together): the env's joint decision
        const uint32_t pbad = partner_u(bad ? 1u : 0u);
        if (c.active && !bad && !badc && pbad == 0u) c.active = false;
    }
    if constexpr (!C44) __builtin_amdgcn_s_setprio(0);
}

// ---- fast-form island rows.  Bullet's sequential-impulse solver
// precomputes, per solver row, the lever-arm cross product r x t and the angular
// component M (r x t) once per step (btSequentialImpulseConstraintSolver::
// setupContactConstraint), so its sweeps only touch velocities.  fast_build does the
// same for the lane's island rows: the values are the ones isl_row computes inside
// the sweep loop (pure functions of loop-invariant operands: rb, n, the tangents,
// the positions and the world inverse inertias), so every sweep result is
// bit-identical to the slow form.  Rows live in registers, statically indexed by
// (local pair, point); used when no lane of the wave has friction rows on local
// pairs 0 or 2 (the default friction table: a cart's friction is 0).
struct GRow {
    V3 rbt, ib;
    real ie, tg, lam;
};
struct CRow {
    V3 rbt, ib, rat, ia;
    real ie, tg, lam;
};
struct FRow {
    V3 rbt1, ib1, rbt2, ib2;
    real ie1, ie2, l1, l2;
};
// pair_body: B's box axes built after the broadphase, for the lanes it passes (built early: measured slower)
constexpr bool kEarlyBax = false;
// HC2 = false: no lane of the wave has cart-pole rows (the pole off its cart: 72 % of a C3 episode's
// wave-sweeps), the 60 values of c2 are not built (the latency kernels' general loop then needs ~60 fewer
// registers, which were AGPR moves inside it)
template <bool HC2 = true>
struct FastIslT {
    GRow g0[4], g1[4];      // local pair 0 (ground, cart), 1 (ground, pole)
    CRow c2[HC2 ? 4 : 1];   // local pair 2 (cart, pole); unused when !HC2
    FRow f1[4];             // friction points of local pair 1
    V3 t1, t2;              // their tangents (plane_space of pair 1's normal)
};
using FastIsl = FastIslT<true>;

CP_DEV bool fast_ok(const Ctx& c) { return pk_fcnt(c.T.pk[0]) == 0 && pk_fcnt(c.T.pk[2]) == 0; }

template <int J>
CP_DEV void fast_ground_rows(GRow* R, const Ctx& c, real* pool) {
    const uint32_t pk = c.T.pk[J];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    const Sym& M = J == 0 ? c.I.d1.M : c.I.d2.M;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < cnt) {
            const int s = base + k;
            const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
            R[k].rbt = cross(rb, c.T.n[J]);
            R[k].ib = symv(M, R[k].rbt);
            R[k].ie = pool_n(pool, F_IE, s);
            R[k].tg = pool_n(pool, F_TG, s);
            R[k].lam = pool_n(pool, F_LAM, s);
        }
    }
}

CP_DEV void fast_cart_pole_rows(CRow* C, const Ctx& c, real* pool) {
    const uint32_t pk = c.T.pk[2];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    const V3 n = c.T.n[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < cnt) {
            const int s = base + k;
            const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
            CRow& R = C[k];
            R.rbt = cross(rb, n);
            R.ib = symv(c.I.d2.M, R.rbt);
            const V3 ra = add(rb, sub(c.I.d2.x, c.I.d1.x));
            R.rat = cross(ra, n);
            R.ia = symv(c.I.d1.M, R.rat);
            R.ie = pool_n(pool, F_IE, s);
            R.tg = pool_n(pool, F_TG, s);
            R.lam = pool_n(pool, F_LAM, s);
        }
    }
}

// The rows of the settle-loop structures alone (c4k_ok: local pair 0 in +z form, 0-4 cart-pole rows,
// nothing else): the latency reset kernels' common case.  Built apart from FastIsl so that only these
// ~100 values are live through sweeps_c44 / sweeps_c4k (with the whole FastIsl live, the register
// allocator parked a third of them in AGPRs: 50 v_accvgpr_read per settle sweep of 279 instructions)
struct FastC4 {
    GRow g0[4];
    CRow c2[4];
};
// the same for the pole lying on the ground (p1_ok, the step kernels' steady state): pair 0 (0 or 4 rows),
// pair 1's normal rows and friction points, +z forms (sweeps_p1_fast)
struct FastP1 {
    GRow g0[4], g1[4];
    FRow f1[4];
};

// local pair 1's friction points (the only island pair with friction rows under the URDF frictions)
CP_DEV void fast_friction_rows(FRow* Fr, V3& t1, V3& t2, const Ctx& c, real* pool) {
    const uint32_t pk = c.T.pk[1];
    const int fcnt = pk_fcnt(pk), base = pk_base(pk), fbase = pk_fbase(pk);
    plane_space(c.T.n[1], t1, t2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < fcnt) {
            const int s = base + k, fs = fbase + k;
            const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
            FRow& R = Fr[k];
            R.rbt1 = cross(rb, t1);
            R.ib1 = symv(c.I.d2.M, R.rbt1);
            R.rbt2 = cross(rb, t2);
            R.ib2 = symv(c.I.d2.M, R.rbt2);
            R.ie1 = pool_f(pool, FF_IE1, fs);
            R.ie2 = pool_f(pool, FF_IE2, fs);
            R.l1 = pool_f(pool, FF_L1, fs);
            R.l2 = pool_f(pool, FF_L2, fs);
        }
    }
}

template <bool HC2>
CP_DEV void fast_build(FastIslT<HC2>& F, const Ctx& c, real* pool) {
    fast_ground_rows<0>(F.g0, c, pool);
    fast_ground_rows<1>(F.g1, c, pool);
    if constexpr (HC2) fast_cart_pole_rows(F.c2, c, pool);
    fast_friction_rows(F.f1, F.t1, F.t2, c, pool);
}

// one ground row (A = static ground) on body b: isl_row<0, B, FRICTION> with r x t
// and M (r x t) precomputed
template <bool FRICTION>
CP_DEV bool fast_grow(Dyn& b, real imb, V3 t, V3 rbt, V3 ib, real inv_eff, real target, real& lam,
                      real bound, real tol) {
    const real vn = dot(t, b.v) + dot(b.w, rbt);
    const real e = target - vn;
    real dl = e * inv_eff;
    const real l0 = lam + dl;
    real ln;
    if constexpr (!FRICTION) ln = l0 > real(0.0) ? l0 : real(0.0);
    else ln = bound > real(0.0) ? clamp_sym(l0, bound) : lam;  // see isl_row_ez
    dl = ln - lam;
    lam = ln;
    const real sb = dl * imb;
    b.v = madd(b.v, t, sb);
    b.w = madd(b.w, ib, dl);
    return abs_(dl) > tol * inv_eff;  // Bullet residual test (oracle: solve_row)
}

// fast_grow for a ground manifold whose normal is exactly +z (wave-uniform choice, as
// isl_row_ez): KIND 0 the normal n = (0, 0, 1), 1 the tangent t1 = (0, -1, 0), 2 the tangent
// t2 = (1, -0, -0).  The precomputed r x t of such a row has one exact-zero component and
// M (r x t) equals isl_row_ez's reduced products (FMA(m, x, +-0) = m x), so these are
// isl_row_ez's operations with its r x t and M (r x t) precomputed.
template <int KIND, bool FRICTION>
CP_DEV bool fast_grow_ez(Dyn& b, real imb, const V3& rbt, const V3& ib, real inv_eff, real target, real& lam,
                         real bound, real tol) {
    real vn;
    if constexpr (KIND == 0) vn = b.v.z + fma_(b.w.x, rbt.x, b.w.y * rbt.y);        // r x n = (rb.y, -rb.x, 0)
    else if constexpr (KIND == 1) vn = -b.v.y + fma_(b.w.x, rbt.x, b.w.z * rbt.z);  // r x t1 = (rb.z, 0, -rb.x)
    else vn = b.v.x + fma_(b.w.y, rbt.y, b.w.z * rbt.z);                             // r x t2 = (0, rb.z, -rb.y)
    const real e = target - vn;
    real dl = e * inv_eff;
    const real l0 = lam + dl;
    real ln;
    if constexpr (!FRICTION) ln = l0 > real(0.0) ? l0 : real(0.0);
    else ln = bound > real(0.0) ? clamp_sym(l0, bound) : lam;
    dl = ln - lam;
    lam = ln;
    const real sb = dl * imb;
    if constexpr (KIND == 0) b.v.z = b.v.z + sb;
    else if constexpr (KIND == 1) b.v.y = b.v.y - sb;
    else b.v.x = b.v.x + sb;
    b.w = madd(b.w, ib, dl);
    return abs_(dl) > tol * inv_eff;  // Bullet residual test (oracle: solve_row)
}

// one cart-pole normal row: isl_row<1, 2, false> with both bodies' terms precomputed
CP_DEV bool fast_crow(Isl& I, V3 t, const CRow& R, real& lam, real tol) {
    const real vn = (dot(t, sub(I.d2.v, I.d1.v)) + dot(I.d2.w, R.rbt)) - dot(I.d1.w, R.rat);
    const real e = R.tg - vn;
    real dl = e * R.ie;
    const real l0 = lam + dl;
    const real ln = l0 > real(0.0) ? l0 : real(0.0);
    dl = ln - lam;
    lam = ln;
    const real sb = dl * I.im2;
    I.d2.v = madd(I.d2.v, t, sb);
    I.d2.w = madd(I.d2.w, R.ib, dl);
    const real sa = dl * I.im1;
    I.d1.v = madd(I.d1.v, neg(t), sa);
    I.d1.w = madd(I.d1.w, neg(R.ia), dl);
    return abs_(dl) > tol * R.ie;  // Bullet residual test (oracle: solve_row)
}

// The settle structure: the island's cart on the ground (4 rows of local pair 0, normal
// exactly +z) and its pole standing on the cart (4 rows of local pair 2), no other rows, no
// cross contact.  Every island of a reset's 100 settle substeps, and ~85 % of the islands
// that run to the sweep cap in the step.
CP_DEV bool c44_ok(const Ctx& c) {
    // no friction rows on pairs 0 and 2: the reference scene's cart has mu = 0 (cart.urdf), so its pairs have
    // none, but a configured cart friction gives them some, and the settle loops do not run them
    return pk_cnt(c.T.pk[0]) == 4 && pk_cnt(c.T.pk[2]) == 4 && pk_cnt(c.T.pk[1]) == 0 && !c.merged &&
           is_plus_z(c.T.n[0]) && pk_fcnt(c.T.pk[0]) == 0 && pk_fcnt(c.T.pk[2]) == 0;
}

// sweeps_fast when every active lane of the wave has the settle structure: the same rows in
// the same order (4 ground rows in +z form, then 4 cart-pole rows; no friction, no cross
// rows), straight-line, without the per-row lane guards of the general loop.
template <class FI>
CP_DEV void sweeps_c44(Ctx& c, FI& F, real tol, int it0, int it1, Stamps& ST) {
    const V3 n2 = c.T.n[2];
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false;
        if (c.active) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bad |= fast_grow_ez<0, false>(c.I.d1, c.I.im1, F.g0[k].rbt, F.g0[k].ib, F.g0[k].ie, F.g0[k].tg,
                                              F.g0[k].lam, real(0.0), tol);
#pragma unroll
            for (int k = 0; k < 4; ++k) bad |= fast_crow(c.I, n2, F.c2[k], F.c2[k].lam, tol);
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && pbad == 0u) c.active = false;
    }
}

// The bump phase's structures: the cart on the ground (4 rows of local pair 0, normal exactly +z) and
// 0-4 rows of its pole on the cart (a tilting or bouncing pole), no pole-ground rows, no cross contact.
// ~94 % of the island-substeps of a reset's 30 bump substeps that are not the settle structure
// (oracle ORC_STATS run of 256 resets).
CP_DEV bool c4k_ok(const Ctx& c) {
    return pk_cnt(c.T.pk[0]) == 4 && pk_cnt(c.T.pk[1]) == 0 && !c.merged && is_plus_z(c.T.n[0]) &&
           pk_fcnt(c.T.pk[0]) == 0 && pk_fcnt(c.T.pk[2]) == 0;
}

// sweeps_c44 with the cart-pole rows guarded by the lane's own count (the same rows in the same order
// as sweeps_fast runs them for this structure, without its other pairs' guards and checks)
template <class FI>
CP_DEV void sweeps_c4k(Ctx& c, FI& F, real tol, int it0, int it1, Stamps& ST) {
    const V3 n2 = c.T.n[2];
    const int cnt2 = pk_cnt(c.T.pk[2]);
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false;
        if (c.active) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bad |= fast_grow_ez<0, false>(c.I.d1, c.I.im1, F.g0[k].rbt, F.g0[k].ib, F.g0[k].ie, F.g0[k].tg,
                                              F.g0[k].lam, real(0.0), tol);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < cnt2) bad |= fast_crow(c.I, n2, F.c2[k], F.c2[k].lam, tol);
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && pbad == 0u) c.active = false;
    }
}

// the p1_ok island's rows (pole on the ground) in fast form, guard-free (the lean step loops)
template <class FI>
CP_DEV void sweeps_p1_fast(Ctx& c, FI& F, real tol, int it0, int it1, Stamps& ST) {
    const bool cart = pk_cnt(c.T.pk[0]) != 0;
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false;
        if (c.active) {
            if (cart) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    bad |= fast_grow_ez<0, false>(c.I.d1, c.I.im1, F.g0[k].rbt, F.g0[k].ib, F.g0[k].ie, F.g0[k].tg,
                                                  F.g0[k].lam, real(0.0), tol);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bad |= fast_grow_ez<0, false>(c.I.d2, c.I.im2, F.g1[k].rbt, F.g1[k].ib, F.g1[k].ie, F.g1[k].tg,
                                              F.g1[k].lam, real(0.0), tol);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const real bound = c.mu1 * F.g1[k].lam;
                bad |= fast_grow_ez<1, true>(c.I.d2, c.I.im2, F.f1[k].rbt1, F.f1[k].ib1, F.f1[k].ie1, real(0.0),
                                             F.f1[k].l1, bound, tol);
                bad |= fast_grow_ez<2, true>(c.I.d2, c.I.im2, F.f1[k].rbt2, F.f1[k].ib2, F.f1[k].ie2, real(0.0),
                                             F.f1[k].l2, bound, tol);
            }
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && pbad == 0u) c.active = false;
    }
}

// sweeps() when every active lane of the wave has the settle structure, rows from the LDS
// pool: then the ground-cart rows are pool slots 0-3 and the cart-pole rows slots 4-7 on every
// lane (the pool fills in pair order), so the loop is straight-line with compile-time slots.
CP_DEV void sweeps_c44_slow(Ctx& c, real* pool, real tol, int it0, int it1, Stamps& ST) {
    const V3 n2 = c.T.n[2];
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false;
        if (c.active) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
                real lam = pool_n(pool, F_LAM, s);
                bad |= isl_row_ez<1, 0, false>(c.I, rb, pool_n(pool, F_IE, s), pool_n(pool, F_TG, s), lam, real(0.0),
                                               tol);
                pool_n(pool, F_LAM, s) = lam;
            }
#pragma unroll
            for (int s = 4; s < 8; ++s) {
                const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
                real lam = pool_n(pool, F_LAM, s);
                bad |= isl_row<1, 2, false>(c.I, rb, n2, pool_n(pool, F_IE, s), pool_n(pool, F_TG, s), lam, real(0.0),
                                            tol);
                pool_n(pool, F_LAM, s) = lam;
            }
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && pbad == 0u) c.active = false;
    }
}

// sweeps_c44_slow for the bump phase's structures (c4k_ok): the cart-pole rows are pool slots 4 .. 4 +
// the lane's count - 1 (local pair 1 has no rows), guarded by that count
CP_DEV void sweeps_c4k_slow(Ctx& c, real* pool, real tol, int it0, int it1, Stamps& ST) {
    const V3 n2 = c.T.n[2];
    const int cnt2 = pk_cnt(c.T.pk[2]);
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false;
        if (c.active) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
                real lam = pool_n(pool, F_LAM, s);
                bad |= isl_row_ez<1, 0, false>(c.I, rb, pool_n(pool, F_IE, s), pool_n(pool, F_TG, s), lam, real(0.0),
                                               tol);
                pool_n(pool, F_LAM, s) = lam;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k < cnt2) {
                    const int s = 4 + k;
                    const V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
                    real lam = pool_n(pool, F_LAM, s);
                    bad |= isl_row<1, 2, false>(c.I, rb, n2, pool_n(pool, F_IE, s), pool_n(pool, F_TG, s), lam,
                                                real(0.0), tol);
                    pool_n(pool, F_LAM, s) = lam;
                }
            }
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && pbad == 0u) c.active = false;
    }
}

// The step kernels' dominant island (tools/row_classes.py: 94 % of the C3 steady state's island
// solves, and nearly all of the sweep-cap stragglers): the pole standing on the ground on its 1 cm
// base (local pair 1: 4 normal rows and 4 friction points, normal exactly +z), its cart either off
// the ground or standing on it (local pair 0: 0 or 4 rows, +z), nothing on the cart-pole pair, no
// friction rows on pairs 0 / 2, no cross contact.
CP_DEV bool p1_ok(const Ctx& c) {
    const int c0 = pk_cnt(c.T.pk[0]);
    return pk_cnt(c.T.pk[1]) == 4 && pk_fcnt(c.T.pk[1]) == 4 && is_plus_z(c.T.n[1]) && pk_cnt(c.T.pk[2]) == 0 &&
           pk_fcnt(c.T.pk[0]) == 0 && pk_fcnt(c.T.pk[2]) == 0 && !c.merged &&
           (c0 == 0 || (c0 == 4 && is_plus_z(c.T.n[0])));
}


// sweeps() with the island rows in fast form (same row order, same stopping rule)
template <bool C44, bool HC2, bool HX = true>
CP_DEV void sweeps_fast(Ctx& c, FastIslT<HC2>& F, Sim& S, const cp_physics& P, real* pool, real* pool0, bool second,
                        int it0, int it1, Stamps& ST) {
    const real tol = sqrt_(real(P.residual_threshold));  // oracle: SQRT((real)threshold)
    const int cnt0 = pk_cnt(c.T.pk[0]), cnt1 = pk_cnt(c.T.pk[1]), cnt2 = pk_cnt(c.T.pk[2]);
    const int fc1 = pk_fcnt(c.T.pk[1]);
    const V3 n0 = c.T.n[0], n1 = c.T.n[1], n2 = c.T.n[2];
    // ground pairs whose rows all have a +z normal in this wave run fast_grow_ez (wave-uniform)
    const bool ez0 = __ballot(cnt0 > 0 && !is_plus_z(n0)) == 0ull;
    const bool ez1 = __ballot(cnt1 > 0 && !is_plus_z(n1)) == 0ull;
    for (int it = it0; it < it1; ++it) {
        if (__ballot(c.active) == 0ull) break;
        // every still-active lane of the wave in the settle structure: the guard-free loop
        // (the reset kernel's option: there every settle substep is in it; in the step kernel
        // the periodic test cost more than it saved, 0.450 -> 0.480 ms at B = 4,096)
        if constexpr (C44 && HC2) {
            if ((it - it0) % kC44Check == 0 && __ballot(c.active && !c44_ok(c)) == 0ull) {
                CP_STAMP(q0);
                sweeps_c44(c, F, tol, it, it1, ST);
                return;
            }
            if (it == it0 && __ballot(c.active && !c4k_ok(c)) == 0ull) {  // the bump phase's structures
                sweeps_c4k(c, F, tol, it, it1, ST);
                return;
            }
        }
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        bool bad = false, badc = false;
        if (c.active) {
            if (ez0) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < cnt0) bad |= fast_grow_ez<0, false>(c.I.d1, c.I.im1, F.g0[k].rbt, F.g0[k].ib, F.g0[k].ie,
                                                                F.g0[k].tg, F.g0[k].lam, real(0.0), tol);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < cnt0) bad |= fast_grow<false>(c.I.d1, c.I.im1, n0, F.g0[k].rbt, F.g0[k].ib, F.g0[k].ie,
                                                          F.g0[k].tg, F.g0[k].lam, real(0.0), tol);
            }
            if (ez1) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < cnt1) bad |= fast_grow_ez<0, false>(c.I.d2, c.I.im2, F.g1[k].rbt, F.g1[k].ib, F.g1[k].ie,
                                                                F.g1[k].tg, F.g1[k].lam, real(0.0), tol);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < cnt1) bad |= fast_grow<false>(c.I.d2, c.I.im2, n1, F.g1[k].rbt, F.g1[k].ib, F.g1[k].ie,
                                                          F.g1[k].tg, F.g1[k].lam, real(0.0), tol);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if constexpr (HC2)
                    if (k < cnt2) bad |= fast_crow(c.I, n2, F.c2[k], F.c2[k].lam, tol);
        }
        const bool cross = HX && c.active && c.merged;  // same on both lanes of an env
        if (HX && __ballot(cross) != 0ull && cross) {
            cross_view(S, c.T, c.I, second);
            pair_normal_rows<5>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<6>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<7>(S, c.T, second, P, pool0, tol, badc);
            pair_normal_rows<8>(S, c.T, second, P, pool0, tol, badc);
            cross_back(c.I, S, second);
        }
        if (c.active) {
            if (ez1) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k < fc1) {
                        const real bound = c.mu1 * F.g1[k].lam;
                        bad |= fast_grow_ez<1, true>(c.I.d2, c.I.im2, F.f1[k].rbt1, F.f1[k].ib1, F.f1[k].ie1,
                                                     real(0.0), F.f1[k].l1, bound, tol);
                        bad |= fast_grow_ez<2, true>(c.I.d2, c.I.im2, F.f1[k].rbt2, F.f1[k].ib2, F.f1[k].ie2,
                                                     real(0.0), F.f1[k].l2, bound, tol);
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k < fc1) {
                        const real bound = c.mu1 * F.g1[k].lam;
                        bad |= fast_grow<true>(c.I.d2, c.I.im2, F.t1, F.f1[k].rbt1, F.f1[k].ib1, F.f1[k].ie1,
                                               real(0.0), F.f1[k].l1, bound, tol);
                        bad |= fast_grow<true>(c.I.d2, c.I.im2, F.t2, F.f1[k].rbt2, F.f1[k].ib2, F.f1[k].ie2,
                                               real(0.0), F.f1[k].l2, bound, tol);
                    }
                }
            }
        }
        const bool crossf = cross && c.xfric;  // see sweeps()
        if (HX && __ballot(crossf) != 0ull && crossf) {
            cross_view(S, c.T, c.I, second);
            pair_friction_rows<5>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<6>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<7>(S, c.T, second, P, pool0, tol, badc);
            pair_friction_rows<8>(S, c.T, second, P, pool0, tol, badc);
            cross_back(c.I, S, second);
        }
        const uint32_t pbad = partner_u(bad ? 1u : 0u);  // every lane that entered the loop is here
        if (c.active && !bad && !badc && pbad == 0u) c.active = false;
    }
}

// the island rows' impulses back into the pool (substep_finish refreshes the
// warm-start cache from it)
template <bool HC2>
CP_DEV void fast_store(const FastIslT<HC2>& F, const Ctx& c, real* pool) {
    const int cnt0 = pk_cnt(c.T.pk[0]), cnt1 = pk_cnt(c.T.pk[1]), cnt2 = pk_cnt(c.T.pk[2]);
    const int b0 = pk_base(c.T.pk[0]), b1 = pk_base(c.T.pk[1]), b2 = pk_base(c.T.pk[2]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < cnt0) pool_n(pool, F_LAM, b0 + k) = F.g0[k].lam;
        if (k < cnt1) pool_n(pool, F_LAM, b1 + k) = F.g1[k].lam;
        if constexpr (HC2)
            if (k < cnt2) pool_n(pool, F_LAM, b2 + k) = F.c2[k].lam;
    }
}

// The lean structure loops: every active lane of the wave in one of the common row structures at the first
// sweep -> only that structure's rows in fast form (FastC4, FastP1: ~100-120 values, no AGPR moves in the
// latency kernels) and its guard-free loop, the same rows in the same order as the general loops.
//   c4k_ok (FastC4, sweeps_c44 / sweeps_c4k): the cart on the ground and 0-4 rows of its pole standing on it:
//     every island of a reset's settle substeps, ~99 % of the bump substeps', a step's first substeps;
//   p1_ok (FastP1, sweeps_p1_fast, step kernels): the pole lying or standing on the ground (93-98 % of the
//     islands from step 26 of an episode on).
// PRIO (the throughput step kernels): the wave raises its issue priority after kPrioAfter sweeps, as sweeps().
// Returns false (nothing done) when the wave is not uniform.
template <bool C44, bool PRIO>
CP_DEV bool solve_lean(Ctx& c, const cp_physics& P, real* pool, int it0, int it1, Stamps& ST) {
    const real tol = sqrt_(real(P.residual_threshold));  // oracle: SQRT((real)threshold)
    // the sweeps in two segments around the priority raise (the loops stop at the first sweep with no
    // active lane, so the second segment continues exactly where the first left off)
    const int itp = (PRIO && it0 + kPrioAfter < it1) ? it0 + kPrioAfter : it1;
    auto run = [&](auto loop) {
        loop(it0, itp);
        if constexpr (PRIO) {
            if (itp < it1 && __ballot(c.active) != 0ull) {
                __builtin_amdgcn_s_setprio(1);
                loop(itp, it1);
                __builtin_amdgcn_s_setprio(0);
            }
        }
    };
    {
        if (__ballot(c.active && !c4k_ok(c)) == 0ull) {
            FastC4 F;
            fast_ground_rows<0>(F.g0, c, pool);
            fast_cart_pole_rows(F.c2, c, pool);
            if (__ballot(c.active && !c44_ok(c)) == 0ull)
                run([&](int a, int b) { sweeps_c44(c, F, tol, a, b, ST); });
            else
                run([&](int a, int b) { sweeps_c4k(c, F, tol, a, b, ST); });
            const int b0 = pk_base(c.T.pk[0]), cnt2 = pk_cnt(c.T.pk[2]), b2 = pk_base(c.T.pk[2]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // fast_store (c4k_ok: 4 rows on pair 0, none on pair 1)
                pool_n(pool, F_LAM, b0 + k) = F.g0[k].lam;
                if (k < cnt2) pool_n(pool, F_LAM, b2 + k) = F.c2[k].lam;
            }
            return true;
        }
    }
    if constexpr (!C44) {
        if (__ballot(c.active && !p1_ok(c)) == 0ull) {
            FastP1 F;
            V3 t1, t2;
            fast_ground_rows<0>(F.g0, c, pool);
            fast_ground_rows<1>(F.g1, c, pool);
            fast_friction_rows(F.f1, t1, t2, c, pool);
            run([&](int a, int b) { sweeps_p1_fast(c, F, tol, a, b, ST); });
            const int cnt0 = pk_cnt(c.T.pk[0]), b0 = pk_base(c.T.pk[0]), b1 = pk_base(c.T.pk[1]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // fast_store (p1_ok: pair 1 has 4 rows, pair 2 none)
                if (k < cnt0) pool_n(pool, F_LAM, b0 + k) = F.g0[k].lam;
                pool_n(pool, F_LAM, b1 + k) = F.g1[k].lam;
            }
            return true;
        }
    }
    (void)c; (void)P; (void)pool; (void)it0; (void)it1; (void)ST;
    return false;
}

// PGS sweeps [it0, it1) of the lane's island.  FAST: fast-form island rows when no
// lane of the wave has friction rows on local pairs 0 / 2 (wave-uniform choice; the
// fast form needs the register budget of the 1-wave-per-SIMD latency kernels).
template <bool FAST, bool C44 = false, bool PM = false>
CP_DEV void solve_range(Ctx& c, Sim& S, const cp_physics& P, real* pool, real* pool0, bool second, int it0, int it1,
                        Stamps& ST) {
    if constexpr (PM) {  // per-row normals: the generic rows (no fast form, no +z form, no settle loop)
        sweeps<false, true>(c, S, P, pool, pool0, second, it0, it1, ST);
        return;
    }
    if constexpr (FAST) {
        if (__ballot(!fast_ok(c)) == 0ull) {
            if (solve_lean<C44, false>(c, P, pool, it0, it1, ST)) return;
            // the step kernels: no merged env in the wave (61-96 % of a C3 episode's wave-sweeps from step 26 on)
            // -> the general loop without the cross-row block, and without the cart-pole rows when no lane has
            // any (the cross block's whole-env view and the 60 cart-pole row values were AGPR moves in it)
            if constexpr (!C44) {
                if (__ballot(c.active && c.merged) == 0ull) {
                    if (__ballot(c.active && pk_cnt(c.T.pk[2]) > 0) == 0ull) {
                        FastIslT<false> F;
                        fast_build(F, c, pool);
                        sweeps_fast<C44, false, false>(c, F, S, P, pool, pool0, second, it0, it1, ST);
                        fast_store(F, c, pool);
                    } else {
                        FastIsl F;
                        fast_build(F, c, pool);
                        sweeps_fast<C44, true, false>(c, F, S, P, pool, pool0, second, it0, it1, ST);
                        fast_store(F, c, pool);
                    }
                    return;
                }
            }
            FastIsl F;
            CP_STAMP(b0);
            fast_build(F, c, pool);
            CP_STAMP(b1);
            sweeps_fast<C44>(c, F, S, P, pool, pool0, second, it0, it1, ST);
            CP_STAMP(b2);
            fast_store(F, c, pool);
            return;
        }
    }
    // the throughput-shaped (burst) reset kernel: its settle and bump substeps are one structure in (nearly) every
    // wave, so the lean settle rows (FastC4, ~100 values) in registers instead of the LDS-row settle loop
    if constexpr (C44 && !FAST && !PM) {  // (fp64: the latency-shaped reset kernel, 512 registers)
        if (__ballot(!fast_ok(c)) == 0ull && solve_lean<true, false>(c, P, pool, it0, it1, ST)) return;
    }
    sweeps<C44>(c, S, P, pool, pool0, second, it0, it1, ST);
}

// the lane's island view: its two bodies (cart, pole or cart2, pole2) with their world
// inverse inertias, and the island's friction products
CP_DEV void island_view(const Own& O, const cp_physics& P, int isl_, Ctx& c) {
    // the island's constants are rebuilt here from the kernel arguments (a few selects) through
    // an opaque island flag: built once per kernel they stay live across the narrowphase and
    // are spilled there (scratch traffic every substep)
    uint32_t isl = (uint32_t)isl_;
    asm volatile("" : "+v"(isl));
    const Lane L = Lane::make((int)isl, P);
    Isl& I = c.I;
    I.d1.x = O.c.x;
    I.d1.v = O.c.v;
    I.d1.w = O.c.w;
    I.d2.x = O.p.x;
    I.d2.v = O.p.v;
    I.d2.w = O.p.w;
    I.d1.M = world_inv_inertia(quat_axes(O.c.q[0], O.c.q[1], O.c.q[2], O.c.q[3]), L.ii1[0], L.ii1[1], L.ii1[2]);
    I.d2.M = world_inv_inertia(quat_axes(O.p.q[0], O.p.q[1], O.p.q[2], O.p.q[3]), L.ii2[0], L.ii2[1], L.ii2[2]);
    I.im1 = L.im1;
    I.im2 = L.im2;
    c.mu0 = L.mu0;
    c.mu1 = L.mu1;
    c.mu2 = L.mu2;
}

// ---- CP_MODEL_PERSISTENT: Bullet's persistent contact manifold of one local pair (oracle:
// persistent_manifold, pm_sort_cached).  The cache slots are registers with compile-time indices
// (every slot choice is a select), loaded from and stored to the lane's column of Bufs::pman.
struct PMan {
    int cnt;
    V3 la[4], lb[4], n[4];
    real d[4], lam[4];
};
CP_DEV int pmf(int j, int off) { return j * CP_PM_PAIR_FIELDS + off; }
// field offsets in a pair's block: count 0, la 1 + 3c, lb 13 + 3c, n 25 + 3c, d 37 + c, lam 41 + c
CP_DEV void pm_load(const Mem& G, int j, PMan& M) {
    M.cnt = (int)to_bits(G.lp(pmf(j, 0)));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        M.la[c] = mk(G.lp(pmf(j, 1 + 3 * c)), G.lp(pmf(j, 2 + 3 * c)), G.lp(pmf(j, 3 + 3 * c)));
        M.lb[c] = mk(G.lp(pmf(j, 13 + 3 * c)), G.lp(pmf(j, 14 + 3 * c)), G.lp(pmf(j, 15 + 3 * c)));
        M.n[c] = mk(G.lp(pmf(j, 25 + 3 * c)), G.lp(pmf(j, 26 + 3 * c)), G.lp(pmf(j, 27 + 3 * c)));
        M.d[c] = G.lp(pmf(j, 37 + c));
        M.lam[c] = G.lp(pmf(j, 41 + c));
    }
}
CP_DEV void pm_store(const Mem& G, int j, const PMan& M) {
    G.sp(pmf(j, 0), bits_to<real>((uint32_t)M.cnt));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (c < M.cnt) {
            G.sp(pmf(j, 1 + 3 * c), M.la[c].x); G.sp(pmf(j, 2 + 3 * c), M.la[c].y); G.sp(pmf(j, 3 + 3 * c), M.la[c].z);
            G.sp(pmf(j, 13 + 3 * c), M.lb[c].x); G.sp(pmf(j, 14 + 3 * c), M.lb[c].y); G.sp(pmf(j, 15 + 3 * c), M.lb[c].z);
            G.sp(pmf(j, 25 + 3 * c), M.n[c].x); G.sp(pmf(j, 26 + 3 * c), M.n[c].y); G.sp(pmf(j, 27 + 3 * c), M.n[c].z);
            G.sp(pmf(j, 37 + c), M.d[c]);
            G.sp(pmf(j, 41 + c), M.lam[c]);
        }
    }
}
CP_DEV V3 box_local(const Box& B, V3 w) { return rot_t(B.ax, sub(w, B.c)); }
CP_DEV V3 box_world(const Box& B, V3 l) { return add(B.c, rot(B.ax, l)); }
CP_DEV real box_radius(const Box& B) { return sqrt_(dot(mk(B.h0, B.h1, B.h2), mk(B.h0, B.h1, B.h2))); }

// btPersistentManifold::sortCachedPoints (KEEP_DEEPEST_POINT, gContactCalcArea3Points): the slot a
// 5th point replaces (M.cnt == 4)
CP_DEV int pm_sort_cached(const PMan& M, V3 la, real d) {
    int deepest = -1;
    real maxpen = d;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (M.d[i] < maxpen) { deepest = i; maxpen = M.d[i]; }
    real res[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // a = new - [o0], b = [o1] - [o2]: (1,3,2) (0,3,2) (0,3,1) (0,2,1)
        const int o0 = i == 0 ? 1 : 0, o1 = i == 3 ? 2 : 3, o2 = i < 2 ? 2 : 1;
        const V3 cr = cross(sub(la, M.la[o0]), sub(M.la[o1], M.la[o2]));
        res[i] = i == deepest ? real(0.0) : dot(cr, cr);
    }
    int best = -1;
    real bv = real(-1e30);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (abs_(res[i]) > bv) { bv = abs_(res[i]); best = i; }
    return best;
}

// btManifoldResult::addContactPoint: the new point (world midpoint p, A->B normal n, separation d)
// replaces the nearest cached point in A's frame within thr (keeping its impulse), or is added
CP_DEV void pm_add(PMan& M, const Box& A, const Box& B, V3 p, V3 n, real d, real thr) {
    const V3 pa = madd(p, n, -(d * real(0.5))), pb = madd(p, n, d * real(0.5));
    const V3 la = box_local(A, pa), lb = box_local(B, pb);
    real best = thr * thr;
    int idx = -1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (c < M.cnt) {
            const V3 df = sub(M.la[c], la);
            const real d2 = dot(df, df);
            if (d2 < best) { best = d2; idx = c; }
        }
    }
    real lam = real(0.0);
    if (idx >= 0) {
        lam = idx == 0 ? M.lam[0] : idx == 1 ? M.lam[1] : idx == 2 ? M.lam[2] : M.lam[3];
        asm volatile("" : "+v"(lam));
    } else if (M.cnt == 4) {
        idx = pm_sort_cached(M, la, d);
    } else {
        idx = M.cnt;
        M.cnt += 1;
    }
    // slot writes as selects per compile-time slot (a guarded write is merged into one indexed store,
    // which puts the manifold in private memory)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool h = q == idx;
        M.la[q] = selv(h, la, M.la[q]);
        M.lb[q] = selv(h, lb, M.lb[q]);
        M.n[q] = selv(h, n, M.n[q]);
        M.d[q] = h ? d : M.d[q];
        M.lam[q] = h ? lam : M.lam[q];
    }
}

// btPersistentManifold::refreshContactPoints: separations from the current poses; a point separated
// by more than thr, or drifted sideways by more than thr, is removed (the last slot moved in)
CP_DEV void pm_refresh(PMan& M, const Box& A, const Box& B, real thr) {
#pragma unroll
    for (int c = 3; c >= 0; --c) {
        if (c < M.cnt) {
            const V3 pa = box_world(A, M.la[c]), pb = box_world(B, M.lb[c]);
            const real d = dot(sub(pb, pa), M.n[c]);
            bool keep = d <= thr;
            if (keep) {
                const V3 df = sub(pb, madd(pa, M.n[c], d));
                keep = dot(df, df) <= thr * thr;
            }
            const int last = M.cnt - 1;
            M.d[c] = keep ? d : M.d[c];
#pragma unroll
            for (int q = c + 1; q < 4; ++q) {  // removal: the last slot moves into slot c (selects)
                const bool h = !keep && q == last;
                M.la[c] = selv(h, M.la[q], M.la[c]);
                M.lb[c] = selv(h, M.lb[q], M.lb[c]);
                M.n[c] = selv(h, M.n[q], M.n[c]);
                M.d[c] = h ? M.d[q] : M.d[c];
                M.lam[c] = h ? M.lam[q] : M.lam[c];
            }
            M.cnt = keep ? M.cnt : last;
        }
    }
}

// Phase 1 of one p.stepSimulation() (DESIGN.md §Physics model 1-5a): narrowphase and
// row setup of the lane's island, unconstrained velocity update of the whole env,
// the island view and the warm start.  A lane with live == false (done env, padding)
// makes no contacts and writes nothing.
// ---- WIDE kernels (the latency-shaped step / reset kernels of small batches): an env
// runs on 16 lanes, 8 lane pairs, and every lane pair is a replica of the env (lane 2k + p holds island p, the
// same values on every pair k), so every DPP exchange between the two lanes of a pair and every wave-uniform
// decision stays what it is in the two-lane layout.  The replicas share one LDS pool column per island.  Only
// the narrowphase is divided: lane pair j (< 5) computes local pair j of both islands, so the 5 pairs of an
// island are found side by side instead of one after another; every replica then gathers the 5 pairs'
// point counts and normals (ds_bpermute), derives the same slots and caps the pair loop of the two-lane layout
// derives, and the pair's lane writes its rows into the island's pool column and its warm-start id word.
// A per-body field of a kernel argument (cp_physics) for a lane-varying body id: all five values through an
// empty asm, then selects (an indexed load would copy the argument struct into scratch memory).
CP_DEV real body_f(int id, const float v[CP_NUM_BODIES]) {
    real x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3], x4 = v[4];
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4));
    return id == 0 ? x0 : (id == 1 ? x1 : (id == 2 ? x2 : (id == 3 ? x3 : x4)));
}
CP_DEV real body_f3(int id, const float v[CP_NUM_BODIES][3], int k) {
    real x0 = v[0][k], x1 = v[1][k], x2 = v[2][k], x3 = v[3][k], x4 = v[4][k];
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4));
    return id == 0 ? x0 : (id == 1 ? x1 : (id == 2 ? x2 : (id == 3 ? x3 : x4)));
}
// One local pair's narrowphase on its lane of the WIDE layout: boxes, broadphase, warm-start cache, contact.
struct WPair {
    Box A, Bx;
    Contact C;
    bool near;
    uint32_t oid;
    real ol0, ol1, ol2, ol3;
    real mu;
    int a, bi;
};
template <bool ALLIN, bool ES>
CP_DEV void wide_contact(WPair& W, int j, bool plive, const Own& O, const V3& Pcx, const V3& Ppx, const real Pcq[4],
                         const real Ppq[4], const cp_physics& P, const Lane& L, const Mem& G, Stamps& ST) {
    const bool second = L.isl != 0;
    const int g = island_pair(L.isl, j);
    W.a = pair_a(g);
    W.bi = pair_b(g);
    // A: the ground (pairs 0, 1), the own cart (pair 2; island 0's cross pairs), the partner's pole (island 1's
    // cross pairs).  B: the own cart (pair 0; island 1's pair 3), the own pole (pairs 1, 2; island 1's pair 4),
    // the partner's cart / pole (island 0's pairs 3 / 4) -- substep_prep's pair_body per pair
    const bool a_ground = j < 2, a_ppole = j >= 3 && second;
    const bool b_partner = j >= 3 && !second, b_pole = j == 1 || j == 2 || j == 4;
    real bq[4];
    {
        const V3 zero = mk(real(0.0), real(0.0), real(0.0));
        W.A.c = a_ground ? zero : selv(a_ppole, Ppx, O.c.x);
        real aq[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) aq[k] = a_ground ? (k == 3 ? real(1.0) : real(0.0)) : (a_ppole ? Ppq[k] : O.c.q[k]);
        W.A.ax = quat_axes(aq[0], aq[1], aq[2], aq[3]);
        W.A.h0 = body_f3(W.a, P.half_extents, 0);
        W.A.h1 = body_f3(W.a, P.half_extents, 1);
        W.A.h2 = body_f3(W.a, P.half_extents, 2);
        W.Bx.c = b_partner ? selv(b_pole, Ppx, Pcx) : selv(b_pole, O.p.x, O.c.x);
#pragma unroll
        for (int k = 0; k < 4; ++k) bq[k] = b_partner ? (b_pole ? Ppq[k] : Pcq[k]) : (b_pole ? O.p.q[k] : O.c.q[k]);
        W.Bx.ax = quat_axes(real(0.0), real(0.0), real(0.0), real(1.0));  // placeholder: B's axes after the broadphase
        W.Bx.h0 = body_f3(W.bi, P.half_extents, 0);
        W.Bx.h1 = body_f3(W.bi, P.half_extents, 1);
        W.Bx.h2 = body_f3(W.bi, P.half_extents, 2);
    }
    W.C.m = 0;
    W.C.n = mk(real(0.0), real(0.0), real(1.0));
    const real newmargin = real(P.contact_margin);
    W.near = plive && !face_separated(W.A, W.Bx, newmargin);
    if (W.near) W.Bx.ax = quat_axes(bq[0], bq[1], bq[2], bq[3]);
    W.oid = 0xFFFFFFFFu;
    W.ol0 = W.ol1 = W.ol2 = W.ol3 = real(0.0);
    if (W.near) {  // the pair's warm-start cache (lane-varying field: into the lane's buffer offset)
        W.oid = to_bits(G.st.ld(CP_SF_WS_ID(0, 0), G.woff + (uint32_t)j * G.st.fstride));
        const uint32_t lo = G.loff + (uint32_t)(4 * j) * G.st.fstride;
        W.ol0 = G.st.ld(CP_SF_WS_LAM(0, 0, 0), lo); W.ol1 = G.st.ld(CP_SF_WS_LAM(0, 0, 1), lo);
        W.ol2 = G.st.ld(CP_SF_WS_LAM(0, 0, 2), lo); W.ol3 = G.st.ld(CP_SF_WS_LAM(0, 0, 3), lo);
    }
    CP_STAMP(w0);
    if (W.near) box_box<ALLIN, ES>(W.A, W.Bx, newmargin, P.edge_bias, W.C, ST);
    CP_STAMP(w1);
    CP_ACC(bb, w0, w1);
    W.mu = body_f(W.a, P.friction) * body_f(W.bi, P.friction);
}
// the pair's rows (its first mym points, the first myfm of them frictional) into the island's pool column from
// slot myb / friction slot myfb, as substep_prep's row setup; returns the pair's new warm-start id word
CP_DEV uint32_t wide_rows(const WPair& W, int myb, int myfb, int mym, int myfm, real* pool, const cp_physics& P) {
    const real inv_dt = P.inv_dt;
    uint32_t nid = 0xFFFFFFFFu;
    if (__ballot(mym > 0) == 0ull) return nid;
    const int a = W.a, bi = W.bi;
    const real ima = body_f(a, P.inv_mass), imb = body_f(bi, P.inv_mass);
    const Sym Ma = world_inv_inertia(W.A.ax, body_f3(a, P.inv_inertia, 0), body_f3(a, P.inv_inertia, 1),
                                     body_f3(a, P.inv_inertia, 2));
    const Sym Mb = world_inv_inertia(W.Bx.ax, body_f3(bi, P.inv_inertia, 0), body_f3(bi, P.inv_inertia, 1),
                                     body_f3(bi, P.inv_inertia, 2));
    const V3 xa = W.A.c, xb = W.Bx.c;
    V3 t1 = mk(real(0.0), real(0.0), real(0.0)), t2 = t1;
    if (W.mu > real(0.0)) plane_space(W.C.n, t1, t2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < mym) {
            const int s = myb + k;
            const V3 rb = sub(W.C.p[k], xb);
            const real K = row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, W.C.n);
            const real dist = W.C.d[k];
            const real tg = dist > real(0.0) ? -(dist * inv_dt) : -((P.erp * dist) * inv_dt);
            const int id = (int)((W.C.ids >> (8 * k)) & 0xFFu);
            real l0 = real(0.0);
            if ((int)(W.oid & 0xFFu) == id) l0 = W.ol0;
            else if ((int)((W.oid >> 8) & 0xFFu) == id) l0 = W.ol1;
            else if ((int)((W.oid >> 16) & 0xFFu) == id) l0 = W.ol2;
            else if ((int)((W.oid >> 24) & 0xFFu) == id) l0 = W.ol3;
            pool_n(pool, F_RBX, s) = rb.x;
            pool_n(pool, F_RBY, s) = rb.y;
            pool_n(pool, F_RBZ, s) = rb.z;
            pool_n(pool, F_IE, s) = real(1.0) / K;
            pool_n(pool, F_TG, s) = tg;
            pool_n(pool, F_LAM, s) = P.warmstart * l0;
            nid = (nid & ~(0xFFu << (8 * k))) | ((uint32_t)id << (8 * k));
            if (k < myfm) {
                const int fs = myfb + k;
                pool_f(pool, FF_IE1, fs) = real(1.0) / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t1);
                pool_f(pool, FF_IE2, fs) = real(1.0) / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t2);
                pool_f(pool, FF_L1, fs) = real(0.0);
                pool_f(pool, FF_L2, fs) = real(0.0);
            }
        }
    }
    return nid;
}
// the lane pair (of the env's LW / 2) that owns local pair j: LW >= 16 -> pair j on lane pair j (the lane pairs
// past 4 only replicate); LW 8 -> pairs 0-2 on lane pairs 0-2, both cross pairs (3, 4: mostly separated by the
// broadphase) on lane pair 3
template <int LW>
CP_DEV constexpr int wide_owner(int j) { return LW >= 16 ? j : (j < 3 ? j : 3); }
// the narrowphase + row setup of the substep on the WIDE layout: the same contacts, rows, slots, caps,
// warm-start reads and writes as substep_prep's pair loop over the lane's 5 pairs (bit for bit)
template <int LW, bool ALLIN, bool ES>
CP_DEV void narrow_wide(Own& O, const cp_physics& P, const Lane& L, real* pool, int& overflow, const Mem& G,
                        Stamps& ST, bool live, Step& T, int& used, int& fused) {
    static_assert(LW == 8 || LW == 16 || LW == 64, "WIDE: 8, 16 or 64 lanes per env");
    const int pj = L.pj;
    // the lane's pairs: j0 (LW 16: pj < 5; LW 8: pj < 4), and on LW 8's lane pair 3 also pair 4
    const bool has0 = LW >= 16 ? pj < CP_ISLAND_PAIRS : pj < 4;
    const bool has1 = LW == 8 && pj == 3;
    const int j0 = has0 ? pj : 0;
    // the partner island's bodies: the partner lane is the same pair's lane of the other island (a replica)
    const V3 Pcx = partner(O.c.x), Ppx = partner(O.p.x);
    real Pcq[4], Ppq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { Pcq[k] = partner(O.c.q[k]); Ppq[k] = partner(O.p.q[k]); }
    WPair W0, W1;
    CP_STAMP(s0);
    wide_contact<ALLIN, ES>(W0, j0, live && has0, O, Pcx, Ppx, Pcq, Ppq, P, L, G, ST);
    if constexpr (LW == 8) wide_contact<ALLIN, ES>(W1, 4, live && has1, O, Pcx, Ppx, Pcq, Ppq, P, L, G, ST);
    CP_STAMP(s1);
    CP_ACC(sel, s0, s1);  // (stamp builds: boxes, broadphase, cache loads and box_box; box_box alone in bb)
    // every replica gathers the island's 5 pairs: point count | friction bit, normal
    const int grp = (int)(threadIdx.x & ~(unsigned)(LW - 1)) + L.isl;
    const uint32_t word0 = (uint32_t)W0.C.m | (W0.mu > real(0.0) ? 8u : 0u);
    uint32_t word1 = 0u;
    if constexpr (LW == 8) word1 = (uint32_t)W1.C.m | (W1.mu > real(0.0) ? 8u : 0u);
    uint32_t cw[CP_ISLAND_PAIRS];
    V3 cn[CP_ISLAND_PAIRS];
#pragma unroll
    for (int k = 0; k < CP_ISLAND_PAIRS; ++k) {
        const int src = grp + 2 * wide_owner<LW>(k);
        const bool second_slot = LW == 8 && k == 4;
        const uint32_t w = second_slot ? word1 : word0;
        const V3 n = second_slot ? W1.C.n : W0.C.n;
        cw[k] = (uint32_t)__shfl((int)w, src, WAVE);
        cn[k] = mk(__shfl(n.x, src, WAVE), __shfl(n.y, src, WAVE), __shfl(n.z, src, WAVE));
    }
    // slots and caps in pair order (substep_prep: a point past MAXP rows, or a frictional point past MAXF, is
    // dropped and counted)
    int base = 0, fbase = 0, ov = 0;
    int b0 = 0, fb0 = 0, m0 = 0, fm0 = 0, b1 = 0, fb1 = 0, m1 = 0, fm1 = 0;
    int mk_[CP_ISLAND_PAIRS], bk_[CP_ISLAND_PAIRS], fmk_[CP_ISLAND_PAIRS], fbk_[CP_ISLAND_PAIRS];
#pragma unroll
    for (int k = 0; k < CP_ISLAND_PAIRS; ++k) {
        const int n = (int)(cw[k] & 7u);
        const bool fr = (cw[k] & 8u) != 0u;
        const int m = n < MAXP - base ? n : MAXP - base;
        const int fm = fr ? (m < MAXF - fbase ? m : MAXF - fbase) : 0;
        ov += (n - m) + (fr ? m - fm : 0);
        mk_[k] = m; bk_[k] = base; fmk_[k] = fm; fbk_[k] = fbase;
        if (has0 && k == j0) { b0 = base; fb0 = fbase; m0 = m; fm0 = fm; }
        if (LW == 8 && k == 4 && has1) { b1 = base; fb1 = fbase; m1 = m; fm1 = fm; }
        base += m;
        fbase += fm;
    }
    overflow += ov;
    used = base;
    fused = fbase;
    // the own pairs' rows into the island's pool column, and their warm-start id words (each pair's lane reads
    // it, and rewrites it, every substep)
    {
        const uint32_t nid = wide_rows(W0, b0, fb0, m0, fm0, pool, P);
        const int om = (int)((O.wsm >> (3 * j0)) & 7u);
        const bool idw = W0.near ? nid != W0.oid : om > 0;
        if (live && has0 && idw) G.st.st(CP_SF_WS_ID(0, 0), G.woff + (uint32_t)j0 * G.st.fstride, bits_to<real>(nid));
    }
    if constexpr (LW == 8) {
        const uint32_t nid = wide_rows(W1, b1, fb1, m1, fm1, pool, P);
        const int om = (int)((O.wsm >> 12) & 7u);
        const bool idw = W1.near ? nid != W1.oid : om > 0;
        if (live && has1 && idw) G.st.st(CP_SF_WS_ID(0, 0), G.woff + 4u * G.st.fstride, bits_to<real>(nid));
    }
    // every replica: the island's manifold headers and the warm-start point counts
#pragma unroll
    for (int k = 0; k < CP_ISLAND_PAIRS; ++k) {
        const uint32_t omk = (O.wsm >> (3 * k)) & 7u;
        const uint32_t m = (uint32_t)mk_[k];
        T.n[k] = cn[k];
        T.pk[k] = m | ((uint32_t)bk_[k] << 3) | ((uint32_t)fmk_[k] << 8) | ((uint32_t)fbk_[k] << 11) |
                  ((live ? (m > omk ? m : omk) : 0u) << 16);
        if (live) O.wsm = (O.wsm & ~(7u << (3 * k))) | (m << (3 * k));
    }
    CP_STAMP(s3);
    CP_ACC(rows, s1, s3);  // (stamp builds: the gather and slots, then the rows)
}

template <bool ALLIN = false, bool PM = false, bool SLP = false, bool ES = false, int WIDE = 0>
CP_DEV void substep_prep(Own& O, Sim& X, const cp_physics& P, const Lane& L, real* pool, real* pool0, int& overflow,
                         const Mem& G, Stamps& ST, bool live, Ctx& c) {
    const real dt = P.dt, inv_dt = P.inv_dt;
    CP_STAMP(t0);
    Step& T = c.T;
    // 2. narrowphase + row setup of the lane's island: wave-uniform loop over its 5
    //    local pairs (the global pair, hence the bodies, differ between the two lanes)
    int used = 0, fused = 0;
    static_assert(!(WIDE && (PM || SLP)), "the WIDE layout is built for the default contact model");
    if constexpr (WIDE != 0) {
        narrow_wide<WIDE, ALLIN, ES>(O, P, L, pool, overflow, G, ST, live, T, used, fused);
    } else {
    // one local pair; GROUND: j is 0 or 1, whose first body is the static ground on both
    // islands, so its box is compile-time (centre 0, identity axes)
    auto pair_body = [&](auto ground_tag, const int j) {
        constexpr bool GROUND = decltype(ground_tag)::value;
        const int g = island_pair(L.isl, j);
        const int a = GROUND ? 0 : pair_a(g);
        // CP_MODEL_SLEEPING: a pair with a sleeping body (a sleeping island) makes no contact and keeps its
        // warm-start cache (oracle: skip[p][j])
        bool plive = live;
        if constexpr (SLP) {
            const int bb = pair_b(g);
            plive = live && !(((c.slp >> (bb - 1)) & 1u) || (a > 0 && ((c.slp >> (a - 1)) & 1u)));
        }
        CP_STAMP(n0);
        // warm-start cache of the pair: loaded below for the pairs past the broadphase only, the old point
        // count from O.wsm (loading it first for every pair, to overlap the narrowphase, was measured slower)
        uint32_t oid = 0xFFFFFFFFu;
        real ol0 = real(0.0), ol1 = real(0.0), ol2 = real(0.0), ol3 = real(0.0);
        // the island flag through a volatile empty asm per pair: the box selections below are
        // otherwise loop-invariant per branch, and hoisting all of them out of the pair loop
        // keeps every body's axes live across the narrowphase (spills)
        uint32_t sec = (uint32_t)L.isl;
        asm volatile("" : "+v"(sec));
        const bool second = sec != 0u;
        Box A, Bx;
        real bqv[4];  // B's quaternion: its axes are built after the broadphase, for the pairs it passes only
        pair_dispatch<GROUND>(j, [&](auto jt) {
            constexpr int J = decltype(jt)::value;
            constexpr int a0 = pair_a(island_pair_c(0, J)), a1 = pair_a(island_pair_c(1, J));
            constexpr int b0 = pair_b(island_pair_c(0, J)), b1 = pair_b(island_pair_c(1, J));
            // the lane's own bodies through opaque copies (each pair rebuilds its boxes: see `sec`)
            V3 cx = O.c.x, px = O.p.x;
            real cq[4] = {O.c.q[0], O.c.q[1], O.c.q[2], O.c.q[3]}, pq[4] = {O.p.q[0], O.p.q[1], O.p.q[2], O.p.q[3]};
            if constexpr (J <= 2) {
                asm volatile("" : "+v"(cx.x), "+v"(cx.y), "+v"(cx.z), "+v"(cq[0]), "+v"(cq[1]), "+v"(cq[2]), "+v"(cq[3]));
                asm volatile("" : "+v"(px.x), "+v"(px.y), "+v"(px.z), "+v"(pq[0]), "+v"(pq[1]), "+v"(pq[2]), "+v"(pq[3]));
            }
            if constexpr (J == 0 || J == 1) {  // (ground, own cart) / (ground, own pole): the static ground,
                static_assert(a0 == 0 && a1 == 0, "ground pairs are ground pairs on both islands");  // centre 0,
                A.c = mk(real(0.0), real(0.0), real(0.0));                                          // identity axes
                A.ax = quat_axes(real(0.0), real(0.0), real(0.0), real(1.0));
                A.h0 = P.half_extents[0][0];
                A.h1 = P.half_extents[0][1];
                A.h2 = P.half_extents[0][2];
                if constexpr (J == 0) Bx = box_of<b0, b1, kEarlyBax || PM>(second, cx, cq, P);
                else Bx = box_of<b0, b1, kEarlyBax || PM>(second, px, pq, P);
#pragma unroll
                for (int k = 0; k < 4; ++k) bqv[k] = J == 0 ? cq[k] : pq[k];
            } else if constexpr (J == 2) {     // (own cart, own pole)
                A = box_of<a0, a1>(second, cx, cq, P);
                Bx = box_of<b0, b1, kEarlyBax || PM>(second, px, pq, P);
#pragma unroll
                for (int k = 0; k < 4; ++k) bqv[k] = pq[k];
            } else {
                // cross pairs: island 0 stores (cart, cart2) and (cart, pole2), island 1 (pole, cart2) and
                // (pole, pole2): A is island 0's own cart or the partner's pole, B the partner's or the own
                // body; the partner lane's pose by DPP (both lanes execute this uniform branch)
                V3 rx = J == 3 ? cx : px;
                real rq[4] = {J == 3 ? cq[0] : pq[0], J == 3 ? cq[1] : pq[1], J == 3 ? cq[2] : pq[2],
                              J == 3 ? cq[3] : pq[3]};
                const V3 Pcx = mk(partner(cx.x), partner(cx.y), partner(cx.z));          // partner's cart (J = 3)
                const V3 Ppx = mk(partner(px.x), partner(px.y), partner(px.z));          // partner's pole
                real Pcq[4], Ppq[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) { Pcq[k] = partner(cq[k]); Ppq[k] = partner(pq[k]); }
                // A: island 0 -> own cart, island 1 -> partner's pole
                real aq[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) aq[k] = second ? Ppq[k] : cq[k];
                A = box_of<a0, a1>(second, selv(second, Ppx, cx), aq, P);
                // B: island 0 -> partner's cart2 (J = 3) / pole2 (J = 4), island 1 -> own cart2 / pole2
                const V3 pbx = J == 3 ? Pcx : Ppx;
                real bq[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) bq[k] = second ? rq[k] : (J == 3 ? Pcq[k] : Ppq[k]);
                Bx = box_of<b0, b1, kEarlyBax || PM>(second, selv(second, rx, pbx), bq, P);
#pragma unroll
                for (int k = 0; k < 4; ++k) bqv[k] = bq[k];
            }
        });
        Contact C;
        C.m = 0;
        C.n = mk(real(0.0), real(0.0), real(1.0));
        CP_STAMP(n1);
        // PM: Bullet's box-box detector reports overlapping boxes only (margin 0); the manifold keeps
        // the points within the pair's relative breaking threshold
        const real newmargin = PM ? real(0.0) : real(P.contact_margin);
        const bool near = plive && !face_separated(A, Bx, newmargin);  // (B's centre and extents only)
        // (PM: the persistent manifold's refresh reads B's axes on every live lane: built early there)
        // B's axes for the pairs the broadphase passes (box_box, the row setup's inertias); the other lanes keep
        // the identity box_of<.., .., false> gave them, which nothing of theirs reads
        if constexpr (!PM)
            if (near) Bx.ax = quat_axes(bqv[0], bqv[1], bqv[2], bqv[3]);
        // a pair the broadphase separates makes no point: its cache is not read (m = 0, the id word's old count
        // from O.wsm decides the rewrite below); the others load it here, its latency overlapping box_box
        if constexpr (!PM) {
            if (near) {
                oid = to_bits(G.lw(CP_SF_WS_ID(0, j)));
                ol0 = G.ll(CP_SF_WS_LAM(0, j, 0)); ol1 = G.ll(CP_SF_WS_LAM(0, j, 1));
                ol2 = G.ll(CP_SF_WS_LAM(0, j, 2)); ol3 = G.ll(CP_SF_WS_LAM(0, j, 3));
            }
        }
        if (near) box_box<ALLIN, ES>(A, Bx, newmargin, P.edge_bias, C, ST);
        PMan M;
        M.cnt = 0;
        if constexpr (PM) {
            if (live) {
                pm_load(G, j, M);
                const real ra = box_radius(A), rb_ = box_radius(Bx);
                const real thr = real(P.contact_margin) * (ra < rb_ ? ra : rb_);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < C.m) pm_add(M, A, Bx, C.p[k], C.n, C.d[k], thr);
                pm_refresh(M, A, Bx, thr);
                pm_store(G, j, M);
            }
        }
        CP_STAMP(n2);
        CP_ACC(sel, n0, n1);
        CP_ACC(bb, n1, n2);
        const int base = used, fbase = fused;
        int m = 0, fm = 0;
        uint32_t nid = 0xFFFFFFFFu;
        const int npts = PM ? M.cnt : C.m;
        if (__ballot(npts > 0) != 0ull) {  // row setup, skipped when no lane of the wave has a contact
        real mu, ima, imb;
        Sym Ma, Mb;
        pair_dispatch<GROUND>(j, [&](auto jt) {
            constexpr int J = decltype(jt)::value;
            constexpr int a0 = pair_a(island_pair_c(0, J)), a1 = pair_a(island_pair_c(1, J));
            constexpr int b0 = pair_b(island_pair_c(0, J)), b1 = pair_b(island_pair_c(1, J));
            mu = pick_f<a0, a1>(second, P.friction) * pick_f<b0, b1>(second, P.friction);
            ima = pick_f<a0, a1>(second, P.inv_mass);
            imb = pick_f<b0, b1>(second, P.inv_mass);
            Ma = inertia_pick<a0, a1>(second, A, P);
            Mb = inertia_pick<b0, b1>(second, Bx, P);
        });
        const V3 xa = A.c, xb = Bx.c;
        V3 t1 = mk(real(0.0), real(0.0), real(0.0)), t2 = t1;
        if (!PM && mu > real(0.0)) plane_space(C.n, t1, t2);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < npts) {
                if (base + m >= MAXP) {
                    overflow += 1;  // dropped by the island pool cap (oracle: same count)
                } else {
                    const int s = base + m;
                    // PM: the cached point's own point on B, normal, separation and applied impulse
                    const V3 nk = PM ? M.n[k] : C.n;
                    V3 rb = sub(PM ? box_world(Bx, M.lb[k]) : C.p[k], xb);
                    real K = row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, nk);
                    real dist = PM ? M.d[k] : C.d[k];
                    real tg = dist > real(0.0) ? -(dist * inv_dt) : -((P.erp * dist) * inv_dt);
                    const int id = (int)((C.ids >> (8 * k)) & 0xFFu);
                    real l0 = real(0.0);
                    if constexpr (PM) {
                        l0 = M.lam[k];
                        pool_pn(pool, 0, s) = nk.x;
                        pool_pn(pool, 1, s) = nk.y;
                        pool_pn(pool, 2, s) = nk.z;
                        if (mu > real(0.0)) plane_space(nk, t1, t2);
                    } else {
                        if ((int)(oid & 0xFFu) == id) l0 = ol0;
                        else if ((int)((oid >> 8) & 0xFFu) == id) l0 = ol1;
                        else if ((int)((oid >> 16) & 0xFFu) == id) l0 = ol2;
                        else if ((int)((oid >> 24) & 0xFFu) == id) l0 = ol3;
                    }
                    pool_n(pool, F_RBX, s) = rb.x;
                    pool_n(pool, F_RBY, s) = rb.y;
                    pool_n(pool, F_RBZ, s) = rb.z;
                    pool_n(pool, F_IE, s) = real(1.0) / K;
                    pool_n(pool, F_TG, s) = tg;
                    pool_n(pool, F_LAM, s) = P.warmstart * l0;
                    nid = (nid & ~(0xFFu << (8 * m))) | ((uint32_t)id << (8 * m));
                    if (mu > real(0.0)) {
                        if (fbase + fm >= MAXF) {
                            overflow += 1;
                        } else {
                            const int fs = fbase + fm;
                            pool_f(pool, FF_IE1, fs) = real(1.0) / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t1);
                            pool_f(pool, FF_IE2, fs) = real(1.0) / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t2);
                            pool_f(pool, FF_L1, fs) = real(0.0);
                            pool_f(pool, FF_L2, fs) = real(0.0);
                            fm += 1;
                        }
                    }
                    m += 1;
                }
            }
        }
        }
        used = base + m;
        fused = fbase + fm;
        CP_STAMP(n3);
        CP_ACC(rows, n2, n3);
        // old point count = the leading non-0xFF bytes of the old id word (written as a prefix)
        const int om = (int)((O.wsm >> (3 * j)) & 7u);
        // the id word changes when the new prefix differs from the old word: loaded when near; a separated pair's
        // new word is all 0xFF, which differs from the old exactly when that held a point or was not a prefix
        const bool idw = near ? nid != oid : om > 0;
        if (!PM && plive) O.wsm = (O.wsm & ~(7u << (3 * j))) | ((uint32_t)m << (3 * j));
        const uint32_t pk = (uint32_t)m | ((uint32_t)base << 3) | ((uint32_t)fm << 8) | ((uint32_t)fbase << 11) |
                            ((uint32_t)(plive ? (m > om ? m : om) : 0) << 16);
        // the pair's manifold header into registers: a select per slot on the wave-uniform j
        // (a switch is merged back into one indexed store, which keeps T in private memory)
#pragma unroll
        for (int q = 0; q < CP_ISLAND_PAIRS; ++q) {
            const bool h = j == q;
            T.n[q] = selv(h, C.n, T.n[q]);
            T.pk[q] = h ? pk : T.pk[q];
        }
        if (!PM && plive && idw) G.sw(CP_SF_WS_ID(0, j), bits_to<real>(nid));  // unchanged: no write
    };
#pragma unroll 1
    for (int j = 0; j < 2; ++j) pair_body(std::true_type{}, j);
#pragma unroll 1
    for (int j = 2; j < CP_ISLAND_PAIRS; ++j) pair_body(std::false_type{}, j);
    }
    CP_STAMP(t1);
    CP_ACC(narrow, t0, t1);
    // 3. unconstrained velocity update of the lane's own bodies (island 0's lane: cart, pole)
    const real kl = P.lin_damping, ka = P.ang_damping;
    const bool second_l = L.isl != 0;
    auto vel_update = [&](Body& B, auto gsel, V3 F, int bit) {
        constexpr int G0 = decltype(gsel)::value, G1 = G0 + 2;  // cart 1 / 3, pole 2 / 4
        const real im = sel_arg(second_l, P.inv_mass[G0], P.inv_mass[G1]);
        const real I0 = sel_arg(second_l, P.inertia[G0][0], P.inertia[G1][0]);
        const real I1 = sel_arg(second_l, P.inertia[G0][1], P.inertia[G1][1]);
        const real I2 = sel_arg(second_l, P.inertia[G0][2], P.inertia[G1][2]);
        const real iI0 = sel_arg(second_l, P.inv_inertia[G0][0], P.inv_inertia[G1][0]);
        const real iI1 = sel_arg(second_l, P.inv_inertia[G0][1], P.inv_inertia[G1][1]);
        const real iI2 = sel_arg(second_l, P.inv_inertia[G0][2], P.inv_inertia[G1][2]);
        const Axes ax = quat_axes(B.q[0], B.q[1], B.q[2], B.q[3]);
        V3 v = B.v, w = B.w;
        real vlen = sqrt_(dot(v, v));
        real dv = fma_(kl, vlen, kl);
        V3 acc = mk(fma_(-v.x, dv, fma_(F.x, im, real(P.gravity[0]))), fma_(-v.y, dv, fma_(F.y, im, real(P.gravity[1]))),
                    fma_(-v.z, dv, fma_(F.z, im, real(P.gravity[2]))));
        V3 wl = rot_t(ax, w);
        V3 Iwl = mk(I0 * wl.x, I1 * wl.y, I2 * wl.z);
        V3 gl = cross(wl, Iwl);
        V3 al = mk(-(iI0 * gl.x), -(iI1 * gl.y), -(iI2 * gl.z));
        V3 aw = rot(ax, al);
        real wlen = sqrt_(dot(w, w));
        real dw = fma_(ka, wlen, ka);
        V3 accw = mk(fma_(-w.x, dw, aw.x), fma_(-w.y, dw, aw.y), fma_(-w.z, dw, aw.z));
        if constexpr (SLP) {  // CP_MODEL_SLEEPING: no gravity, forces or damping for a sleeping body
            const bool sd = ((c.slp >> bit) & 1u) != 0u;
            B.v = selv(sd, v, madd(v, acc, dt));
            B.w = selv(sd, w, madd(w, accw, dt));
        } else {
            (void)bit;
            B.v = madd(v, acc, dt);
            B.w = madd(w, accw, dt);
        }
    };
    const int bit0 = second_l ? 2 : 0;
    vel_update(O.c, std::integral_constant<int, 1>{}, O.f, bit0);
    vel_update(O.p, std::integral_constant<int, 2>{}, mk(real(0.0), real(0.0), real(0.0)), bit0 + 1);
    clamp_velocities(O, P);  // the unconstrained update goes through applyDeltaVeeMultiDof(output, dt)
    O.f = mk(real(0.0), real(0.0), real(0.0));  // 6. external forces are consumed by the step
    // 4. solve setup.  No cross-island contact: each lane solves its own island
    //    (oracle: independent islands); otherwise the env is "merged" and its cross
    //    rows run on both lanes.  (DPP reads the partner lane's register: evaluate it
    //    in converged code, never under a branch where the partner may be inactive.)
    const uint32_t own_cross = (pk_cnt(T.pk[3]) + pk_cnt(T.pk[4])) > 0 ? 1u : 0u;
    const uint32_t any_cross = own_cross | partner_u(own_cross);
    c.merged = any_cross != 0u;
    const uint32_t own_xf = (pk_fcnt(T.pk[3]) + pk_fcnt(T.pk[4])) > 0 ? 1u : 0u;
    const uint32_t any_xf = own_xf | partner_u(own_xf);  // unconditionally, like any_cross
    c.xfric = (any_cross & any_xf) != 0u;
#ifdef CP_STAMPS
    ST.flags |= __ballot(c.merged) != 0ull ? 1u : 0u;
#endif
    c.used = used;
    c.tot = used + (int)partner_u((uint32_t)used);
    const bool second = L.isl != 0;
    island_view(O, P, L.isl, c);
    Isl& I = c.I;
    CP_STAMP(t2);
    CP_ACC(vel, t1, t2);
    // Island rows run per lane; the rows of the two islands touch disjoint bodies,
    // so running them side by side equals the oracle's interleaved order.  Cross
    // rows (merged env) run on both lanes on the whole-env view after the island
    // rows of the same kind, as in the oracle.  Both lanes sweep until the env's joint
    // stopping test passes (one solver group, oracle: substep step 4).
    isl_warmstart<0, PM>(I, T, pool);
    isl_warmstart<1, PM>(I, T, pool);
    isl_warmstart<2, PM>(I, T, pool);
    if (__ballot(c.merged) != 0ull && c.merged) {
        cross_view(X, T, I, second);
        pair_warmstart<5, PM>(X, T, second, P, pool0); pair_warmstart<6, PM>(X, T, second, P, pool0);
        pair_warmstart<7, PM>(X, T, second, P, pool0); pair_warmstart<8, PM>(X, T, second, P, pool0);
        cross_back(I, X, second);
    }
    c.active = c.tot > 0;  // same on both lanes of the env
}

// Phase 3: whole-env velocities from the two lanes' islands (both lanes of every
// env active), the warm-start cache refresh and the integration (DESIGN.md
// §Physics model 5b-7).
template <bool PM = false, bool SLP = false, int WIDE = 0>
CP_DEV void substep_finish(Own& O, const cp_physics& P, const Lane& L, const Ctx& c, real* pool, const Mem& G,
                           Stamps& ST, bool live) {
    const real dt = P.dt, inv_dt = P.inv_dt;
    const bool second = L.isl != 0;
    CP_STAMP(t3);
    O.c.v = c.I.d1.v;  // the lane's own island's solved velocities
    O.c.w = c.I.d1.w;
    O.p.v = c.I.d2.v;
    O.p.w = c.I.d2.w;
    clamp_velocities(O, P);  // the solver's write-back goes through applyDeltaVeeMultiDof too
    // refresh the warm-start cache of the lane's island.  A pair with no point before or after
    // the substep holds 0 impulses and keeps them: it is not rewritten (the id word is a 0xFF-padded prefix,
    // the impulses past it 0, in every state the kernels and cp_init write; oracle: every slot
    // rewritten, same values)
    if (live && !PM) {
#pragma unroll
        for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {
            const int cnt = pk_cnt(c.T.pk[j]), base = pk_base(c.T.pk[j]);
            // (WIDE: the pair's own lane, which reads the entry in the next substep's narrowphase)
            if (pk_wcnt(c.T.pk[j]) > 0 && (WIDE == 0 || L.pj == wide_owner<WIDE == 0 ? 16 : WIDE>(j))) {  // one branch per pair: rewriting a zero slot with 0 is harmless
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    G.sl(CP_SF_WS_LAM(0, j, k), (k < cnt) ? pool_n(pool, F_LAM, base + k) : real(0.0));
            }
        }
    }
    if (live && PM) {  // the solved impulses of the cached points that got a row (oracle: q->pm)
#pragma unroll
        for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {
            const int cnt = pk_cnt(c.T.pk[j]), base = pk_base(c.T.pk[j]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < cnt) G.sp(pmf(j, 41 + k), pool_n(pool, F_LAM, base + k));
        }
    }
    // 5. integrate positions and orientations of the lane's own bodies
    const real hdt = real(0.5) * dt;
    const real c3 = ((dt * dt) * dt) * (real)0.020833333333;
    const real maxang = P.max_angular_step;
    auto integrate = [&](Body& B, int bit) {
        V3 v = B.v, w = B.w;
        const V3 x0 = B.x;
        const V3 x1 = madd(x0, v, dt);
        real ang = sqrt_(dot(w, w));
        if (ang * dt > maxang) ang = maxang * inv_dt;
        real half = hdt * ang;
        real sn, cs, s;
        sincos_small(half, sn, cs);
        if (ang < real(0.001)) s = fma_(-c3, ang * ang, hdt);
        else s = sn / ang;
        real dx = w.x * s, dy = w.y * s, dz = w.z * s, dw = cs;
        real qx = B.q[0], qy = B.q[1], qz = B.q[2], qw = B.q[3];
        real rw = fma_(dw, qw, -fma_(dx, qx, fma_(dy, qy, dz * qz)));
        real rx = fma_(dw, qx, fma_(dx, qw, fma_(dy, qz, -(dz * qy))));
        real ry = fma_(dw, qy, fma_(dy, qw, fma_(dz, qx, -(dx * qz))));
        real rz = fma_(dw, qz, fma_(dz, qw, fma_(dx, qy, -(dy * qx))));
        real n2 = fma_(rx, rx, fma_(ry, ry, fma_(rz, rz, rw * rw)));
        real inv = real(1.0) / sqrt_(n2);
        if constexpr (SLP) {  // btMultiBodyDynamicsWorld::integrateTransforms: a sleeping body keeps its pose,
            const bool sd = ((c.slp >> bit) & 1u) != 0u;  // its velocities are cleared
            const V3 z = mk(real(0.0), real(0.0), real(0.0));
            B.x = selv(sd, x0, x1);
            B.v = selv(sd, z, v);
            B.w = selv(sd, z, w);
            B.q[0] = sd ? qx : rx * inv;
            B.q[1] = sd ? qy : ry * inv;
            B.q[2] = sd ? qz : rz * inv;
            B.q[3] = sd ? qw : rw * inv;
        } else {
            (void)bit;
            B.x = x1;
            B.q[0] = rx * inv;
            B.q[1] = ry * inv;
            B.q[2] = rz * inv;
            B.q[3] = rw * inv;
        }
    };
    const int bit0 = second ? 2 : 0;
    integrate(O.c, bit0);
    integrate(O.p, bit0 + 1);
    if constexpr (SLP) sleep_update(O, P);  // updateActivationState, after the integration
    CP_STAMP(t4);
    CP_ACC(integ, t3, t4);
#ifdef CP_STAMPS
    ST.substeps += 1;
#endif
}

// The physics parameters through an opaque zero offset (an SGPR), once for the substep's narrowphase and once
// for its finish: the kernel-argument loads are then made where each phase needs them instead of hoisted out
// of the substep loop, whose uniform values (the per-body tables the WIDE narrowphase selects from) otherwise
// stay live through the sweep loops, spilled to VGPR lanes and reloaded in the sweep loop's header every sweep
// (the WIDE64 reset kernel's settle sweep: 16 v_readlane of ~240 instructions).  Used by the WIDE kernels and
// the fp64 reset kernel (its frame 280 -> 0 B per lane, reset 13.6 -> 13.1 ms); the fp32 two-lane kernels and
// the fp64 step kernel keep the hoisted loads (their register allocation spills more, or runs slower, with
// the fresh ones).
template <bool FRESH>
CP_DEV const cp_physics& fresh_phys(const cp_physics& P) {
    if constexpr (!FRESH) return P;
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    return *reinterpret_cast<const cp_physics*>(reinterpret_cast<const char*>(&P) + z);
}

// One p.stepSimulation() for this lane's env.
// FAST: fast-form island rows where the wave allows them (the 512-register kernels);
// C44: the latency-shaped reset kernel's options: the guard-free settle-structure loop
// (sweeps_c44) and the all-inside face-contact exit (face_contact<ALLIN>).
// PM: CP_MODEL_PERSISTENT (Bullet's persistent manifold, per-row normals in the pool).
// SLP: CP_MODEL_SLEEPING (Bullet's deactivation: sleeping islands are neither integrated nor solved).
template <bool FAST = false, bool C44 = false, bool ALLIN = C44, bool PM = false, bool SLP = false, int WIDE = 0>
CP_DEV void substep(Own& O, const cp_physics& P0, const Lane& L, real* pool, real* pool0, int& overflow,
                    const Mem& G, Stamps& ST, bool live = true) {
    constexpr bool kFresh = WIDE != 0 || (sizeof(real) == 8 && C44);
    const cp_physics& P = fresh_phys<kFresh>(P0);
    Ctx c;
    Sim X;  // scratch: the whole-env view of a merged env's cross rows (cross_view)
    c.slp = 0u;
    if constexpr (SLP) c.slp = sleep_islands(O, P, L.isl != 0);
    substep_prep<ALLIN, PM, SLP, !FAST, WIDE>(O, X, P, L, pool, pool0, overflow, G, ST, live, c);
    CP_STAMP(t2);
    solve_range<FAST, C44, PM>(c, X, P, pool, pool0, L.isl != 0, 0, P.solver_iterations, ST);
    CP_STAMP(t3);
    CP_ACC(solve, t2, t3);
    substep_finish<PM, SLP, WIDE>(O, fresh_phys<kFresh>(P0), L, c, pool, G, ST, live);
}

// LINK_FRAME force at the COM on the lane's own cart (cart on island 0's lane, cart2 on island 1's):
// world = R(q) f, accumulated until the next substep consumes it
CP_DEV void apply_force_link(Own& O, real fx, real fy) {
    Axes A = quat_axes(O.c.q[0], O.c.q[1], O.c.q[2], O.c.q[3]);
    V3 fw = rot(A, mk(fx, fy, real(0.0)));
    O.f = add(O.f, fw);
}

}  // namespace CP_NS
