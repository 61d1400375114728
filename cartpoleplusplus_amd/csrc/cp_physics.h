// cp_physics.h — one fixed physics step of the 5-body cartpole scene, per lane.
//
// One lane simulates one environment (bullet_cartpole.py's whole pybullet world:
// ground, cart, pole, cart2, pole2 — :154-160).  Per-env body state lives in
// VGPRs with compile-time indices; the contact rows of a substep live in a
// per-wave LDS pool laid out [field][slot][lane] (conflict-free ds_read_b32);
// the 10 body pairs are walked by a wave-uniform loop in the narrowphase and by
// statically unrolled per-pair code in the solver, so the solver never selects
// bodies at run time.  The algorithm is DESIGN.md §Physics model; the CPU
// oracle (oracle/cp_oracle.c) states the same arithmetic, operation for operation.
#pragma once
#include "../../include/cartpole_amd.h"
#include "cp_math.h"

namespace cp {

// Diagnostic phase stamps (built only with -DCP_STAMPS; see cp_debug_stamps).
// Wave-uniform cycle counters from s_memtime, accumulated per wave.
struct Stamps {
    uint64_t narrow = 0, vel = 0, solve = 0, integ = 0, sweeps = 0, substeps = 0;
};
#ifdef CP_STAMPS
#define CP_STAMP(var) uint64_t var = __builtin_amdgcn_s_memtime()
#define CP_ACC(field, a, b) (ST.field += (b) - (a))
#else
#define CP_STAMP(var)
#define CP_ACC(field, a, b)
#endif

constexpr int WAVE = 64;
constexpr int MAXP = CP_MAX_POINTS;
constexpr int MAXF = CP_MAX_FRICTION;
// pool fields (per normal point): rb.xyz, inv_eff, target, lambda
constexpr int F_RBX = 0, F_RBY = 1, F_RBZ = 2, F_IE = 3, F_TG = 4, F_LAM = 5;
constexpr int NPF = 6;
// friction fields (per frictional point): lambda1, lambda2, inv_eff1, inv_eff2
constexpr int FF_L1 = 0, FF_L2 = 1, FF_IE1 = 2, FF_IE2 = 3;
constexpr int POOL_FLOATS = NPF * MAXP + 4 * MAXF;  // 160 floats per env = 40 KiB per wave

CP_DEV float& pool_n(float* pool, int field, int slot) { return pool[(field * MAXP + slot) * WAVE]; }
CP_DEV float& pool_f(float* pool, int field, int slot) { return pool[(NPF * MAXP + field * MAXF + slot) * WAVE]; }

// body pairs (a < b), Bullet-like order over the loadURDF ids
__host__ __device__ constexpr int pair_a(int p) {
    return p < 4 ? 0 : (p < 7 ? 1 : (p < 9 ? 2 : 3));
}
__host__ __device__ constexpr int pair_b(int p) {
    return p < 4 ? p + 1 : (p < 7 ? p - 2 : (p < 9 ? p - 4 : 4));
}

struct Body {
    V3 x, v, w;
    float q[4];
};

// Per-env simulation state held in registers for the duration of a kernel.
struct Sim {
    Body b[CP_NUM_DYN];   // cart, pole, cart2, pole2
    V3 f0, f2;            // pending world force on cart / cart2 (pybullet force accumulator)
};

// Per-env global memory touched once per substep (cold data kept out of VGPRs):
// the warm-start cache lives in the state SoA, the manifold headers of the
// current substep are staged in a [4*CP_NUM_PAIRS][B] scratch.
// SoA field access through a buffer resource: the field base is a wave-uniform
// SGPR soffset (f * B * 4) and the env is a 32-bit VGPR voffset (i * 4), so each
// env keeps one offset register instead of a 64-bit address per field (the flat
// form made the compiler hoist and spill ~100 of them).  Limits one SoA array to
// 4 GiB: B * fields * 4 < 2^32 (checked at cp_create).
struct Soa {
    __amdgpu_buffer_rsrc_t r;
    uint32_t fstride;  // B * 4 bytes
    CP_DEV static Soa make(float* base, int B, int fields) {
        Soa s;
        s.r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)((uint32_t)B * 4u * (uint32_t)fields), 0x00020000);
        s.fstride = (uint32_t)B * 4u;
        return s;
    }
    CP_DEV float ld(int f, uint32_t off) const {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, (int)((uint32_t)f * fstride), 0));
    }
    CP_DEV void st(int f, uint32_t off, float v) const {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, (int)((uint32_t)f * fstride), 0);
    }
};
struct Mem {
    Soa st;           // state SoA [CP_STATE_FIELDS][B]
    Soa scr;          // scratch SoA [4*CP_NUM_PAIRS][B]
    uint32_t off;     // env index * 4
    CP_DEV float ls(int f) const { return st.ld(f, off); }
    CP_DEV void ss(int f, float v) const { st.st(f, off, v); }
    CP_DEV float lx(int f) const { return scr.ld(f, off); }
    CP_DEV void sx(int f, float v) const { scr.st(f, off, v); }
};

struct Box {
    V3 c;
    Axes ax;
    float h0, h1, h2;
};

// component-wise selects (a struct-valued ?: lets the compiler build the operands in scratch)
CP_DEV float sel3(float a, float b, float c, int i) { return i == 0 ? a : (i == 1 ? b : c); }
CP_DEV V3 sel3v(V3 a, V3 b, V3 c, int i) { return mk(sel3(a.x, b.x, c.x, i), sel3(a.y, b.y, c.y, i), sel3(a.z, b.z, c.z, i)); }
CP_DEV V3 selv(bool t, V3 a, V3 b) { return mk(t ? a.x : b.x, t ? a.y : b.y, t ? a.z : b.z); }
CP_DEV V3 axis_of(const Axes& A, int i) { return sel3v(A.a0, A.a1, A.a2, i); }
CP_DEV float h_of(const Box& B, int i) { return i == 0 ? B.h0 : (i == 1 ? B.h1 : B.h2); }

// contact point candidate (reference-face coordinates u, v and separation n)
struct Out4 {
    float u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0}, n[4] = {0, 0, 0, 0};
    int id[4] = {0, 0, 0, 0};
    int m = 0;
};

// Face contact (oracle: face_contact).  Fills up to 4 selected candidates.
CP_DEV void face_contact(const Box& R, int ri, V3 nr, const Box& I, float margin, V3& fc, V3& u, V3& v,
                         Out4& out) {
    int r1 = ri == 2 ? 0 : ri + 1, r2 = ri == 0 ? 2 : ri - 1;
    fc = madd(R.c, nr, h_of(R, ri));
    u = axis_of(R.ax, r1);
    v = axis_of(R.ax, r2);
    float hu = h_of(R, r1), hv = h_of(R, r2);
    float e0 = dot(nr, I.ax.a0), e1d = dot(nr, I.ax.a1), e2d = dot(nr, I.ax.a2);
    int j = 0;
    float best = fabsf(e0);
    if (fabsf(e1d) > best) { j = 1; best = fabsf(e1d); }
    if (fabsf(e2d) > best) { j = 2; }
    float ej = sel3(e0, e1d, e2d, j);
    float isg = (ej > 0.0f) ? -1.0f : 1.0f;
    V3 ic = madd(I.c, axis_of(I.ax, j), isg * h_of(I, j));
    int j1 = j == 2 ? 0 : j + 1, j2 = j == 0 ? 2 : j - 1;
    V3 E1 = scl(axis_of(I.ax, j1), h_of(I, j1));
    V3 E2 = scl(axis_of(I.ax, j2), h_of(I, j2));
    V3 icr = sub(ic, fc);
    float cu = dot(icr, u), cv = dot(icr, v), cn = dot(icr, nr);
    float e1u = dot(E1, u), e1v = dot(E1, v), e1n = dot(E1, nr);
    float e2u = dot(E2, u), e2v = dot(E2, v), e2n = dot(E2, nr);

    float Pu[4], Pv[4], Pn[4];
    Pu[0] = (cu + e1u) + e2u; Pv[0] = (cv + e1v) + e2v; Pn[0] = (cn + e1n) + e2n;
    Pu[1] = (cu - e1u) + e2u; Pv[1] = (cv - e1v) + e2v; Pn[1] = (cn - e1n) + e2n;
    Pu[2] = (cu - e1u) - e2u; Pv[2] = (cv - e1v) - e2v; Pn[2] = (cn - e1n) - e2n;
    Pu[3] = (cu + e1u) - e2u; Pv[3] = (cv + e1v) - e2v; Pn[3] = (cn + e1n) - e2n;

    // 24 candidate slots in canonical order: C1 0-3, C2 4-7, C3 8-23
    float Cu[24], Cv[24], Cn[24];
    uint32_t valid = 0;
    int inside = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        Cu[k] = Pu[k]; Cv[k] = Pv[k]; Cn[k] = Pn[k];
        const bool in = fabsf(Pu[k]) <= hu && fabsf(Pv[k]) <= hv;
        inside += in ? 1 : 0;
        if (in && Pn[k] <= margin) valid |= 1u << k;
    }
#pragma unroll
    for (int k = 4; k < 24; ++k) { Cu[k] = 0.0f; Cv[k] = 0.0f; Cn[k] = 0.0f; }
    // all four incident vertices inside the reference rectangle: C1 only (oracle: same rule)
    if (inside != 4) {
    float det = fmaf_(e1u, e2v, -(e1v * e2u));
    float idet = 1.0f / det;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float X = (c == 0 || c == 3) ? hu : -hu;
        float Y = (c < 2) ? hv : -hv;
        float ru = X - cu, rv = Y - cv;
        float al = fmaf_(ru, e2v, -(rv * e2u)) * idet;
        float be = fmaf_(e1u, rv, -(e1v * ru)) * idet;
        float dn = fmaf_(be, e2n, fmaf_(al, e1n, cn));
        Cu[4 + c] = X; Cv[4 + c] = Y; Cn[4 + c] = dn;
        if (fabsf(al) < 1.0f && fabsf(be) < 1.0f && dn <= margin) valid |= 1u << (4 + c);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int k1 = (k + 1) & 3;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int slot = 8 + 4 * k + s;
            float lim = (s & 1) ? ((s < 2) ? -hu : -hv) : ((s < 2) ? hu : hv);
            float pc = (s < 2) ? Pu[k] : Pv[k], qc = (s < 2) ? Pu[k1] : Pv[k1];
            float dp = pc - lim, dq = qc - lim;
            bool cross_ = (dp < 0.0f && dq > 0.0f) || (dp > 0.0f && dq < 0.0f);
            float t = dp / (dp - dq);
            float xu, xv;
            bool inr;
            if (s < 2) {
                xu = lim;
                xv = fmaf_(Pv[k1] - Pv[k], t, Pv[k]);
                inr = fabsf(xv) <= hv;
            } else {
                xv = lim;
                xu = fmaf_(Pu[k1] - Pu[k], t, Pu[k]);
                inr = fabsf(xu) <= hu;
            }
            float xn = fmaf_(Pn[k1] - Pn[k], t, Pn[k]);
            Cu[slot] = xu; Cv[slot] = xv; Cn[slot] = xn;
            if (cross_ && inr && xn <= margin) valid |= 1u << slot;
        }
    }
    }  // inside != 4
    uint32_t sel = valid;
    if (__builtin_popcount(valid) > 4) {
        // deepest; farthest from it; max / min signed area  (oracle: same rule)
        int i0 = -1;
        float bn = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k)
            if (((valid >> k) & 1u) && (i0 < 0 || Cn[k] < bn)) { i0 = k; bn = Cn[k]; }
        float u0 = 0.0f, v0 = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k)
            if (k == i0) { u0 = Cu[k]; v0 = Cv[k]; }
        int i1 = -1;
        float bd = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k) {
            if (!((valid >> k) & 1u) || k == i0) continue;
            float du = Cu[k] - u0, dv = Cv[k] - v0;
            float d2 = fmaf_(du, du, dv * dv);
            if (i1 < 0 || d2 > bd) { i1 = k; bd = d2; }
        }
        float u1 = 0.0f, v1 = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k)
            if (k == i1) { u1 = Cu[k]; v1 = Cv[k]; }
        float ex = u1 - u0, ey = v1 - v0;
        int i2 = -1;
        float ba = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k) {
            if (!((valid >> k) & 1u) || k == i0 || k == i1) continue;
            float ar = fmaf_(ex, Cv[k] - v0, -(ey * (Cu[k] - u0)));
            if (i2 < 0 || ar > ba) { i2 = k; ba = ar; }
        }
        int i3 = -1;
        float bb = 0.0f;
#pragma unroll
        for (int k = 0; k < 24; ++k) {
            if (!((valid >> k) & 1u) || k == i0 || k == i1 || k == i2) continue;
            float ar = fmaf_(ex, Cv[k] - v0, -(ey * (Cu[k] - u0)));
            if (i3 < 0 || ar < bb) { i3 = k; bb = ar; }
        }
        sel = (1u << i0) | (1u << i1) | (1u << i2) | (1u << i3);
    }
    // compact the selected candidates, canonical order
    out.m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if ((sel >> k) & 1u) {
            int m = out.m;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (m == j) {
                    out.u[j] = Cu[k];
                    out.v[j] = Cv[k];
                    out.n[j] = Cn[k];
                    out.id[j] = k;
                }
            }
            out.m = m + 1;
        }
    }
    if ((sel >> 4) == 0u) return;
#pragma unroll
    for (int k = 4; k < 24; ++k) {
        if ((sel >> k) & 1u) {
            int m = out.m;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (m == j) {
                    out.u[j] = Cu[k];
                    out.v[j] = Cv[k];
                    out.n[j] = Cn[k];
                    out.id[j] = k;
                }
            }
            out.m = m + 1;
        }
    }
}

// Contact result of one box pair in world space.
struct Contact {
    V3 n;          // from A to B
    int m;         // points
    V3 p[4];       // world contact points (midway between the surfaces)
    float d[4];    // signed separation (negative = penetration)
    int id[4];     // feature ids (warm-start keys)
};

// Box-box narrowphase (oracle: box_box).  Normal from A to B.
CP_DEV void box_box(const Box& A, const Box& B, float margin, float edge_bias, Contact& C) {
    C.m = 0;
    V3 d = sub(B.c, A.c);
    V3 Aax[3] = {A.ax.a0, A.ax.a1, A.ax.a2};
    V3 Bax[3] = {B.ax.a0, B.ax.a1, B.ax.a2};
    float Ah[3] = {A.h0, A.h1, A.h2}, Bh[3] = {B.h0, B.h1, B.h2};
    float Cm[3][3], AC[3][3], da[3], db[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Cm[i][j] = dot(Aax[i], Bax[j]);
            AC[i][j] = fabsf(Cm[i][j]);
        }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        da[i] = dot(d, Aax[i]);
        db[i] = dot(d, Bax[i]);
    }
    float best = 0.0f;
    int kind = 0, bi = 0, bj = 0;
    V3 bax = mk(0.0f, 0.0f, 0.0f);
    bool sep = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float pr = fmaf_(Bh[0], AC[i][0], fmaf_(Bh[1], AC[i][1], Bh[2] * AC[i][2]));
        float s = fabsf(da[i]) - (Ah[i] + pr);
        sep = sep || (s > margin);
        if (i == 0 || s > best) { best = s; kind = 0; bi = i; }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float pr = fmaf_(Ah[0], AC[0][j], fmaf_(Ah[1], AC[1][j], Ah[2] * AC[2][j]));
        float s = fabsf(db[j]) - (Bh[j] + pr);
        sep = sep || (s > margin);
        if (s > best) { best = s; kind = 1; bj = j; }
    }
    if (sep) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            V3 ax = cross(Aax[i], Bax[j]);
            float L2 = dot(ax, ax);
            if (L2 < 1e-6f) continue;
            float L = sqrtf(L2);
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            float ra = fmaf_(Ah[i1], AC[i2][j], Ah[i2] * AC[i1][j]);
            float rb = fmaf_(Bh[j1], AC[i][j2], Bh[j2] * AC[i][j1]);
            float num = fabsf(dot(d, ax)) - (ra + rb);   // separation * L
            sep = sep || (num > margin * L);
            if (num > (best + edge_bias) * L) { best = num / L; kind = 2; bi = i; bj = j; bax = ax; }
        }
    }
    if (sep) return;
    if (kind != 2) {
        // face of A (kind 0) or face of B (kind 1) is the reference face
        const bool fa = kind == 0;
        int ri = fa ? bi : bj;
        float sg = fa ? ((sel3(da[0], da[1], da[2], bi) >= 0.0f) ? 1.0f : -1.0f)
                      : ((sel3(db[0], db[1], db[2], bj) >= 0.0f) ? -1.0f : 1.0f);
        Box R, I;
        R.c = selv(fa, A.c, B.c);
        R.ax.a0 = selv(fa, A.ax.a0, B.ax.a0);
        R.ax.a1 = selv(fa, A.ax.a1, B.ax.a1);
        R.ax.a2 = selv(fa, A.ax.a2, B.ax.a2);
        R.h0 = fa ? A.h0 : B.h0; R.h1 = fa ? A.h1 : B.h1; R.h2 = fa ? A.h2 : B.h2;
        I.c = selv(fa, B.c, A.c);
        I.ax.a0 = selv(fa, B.ax.a0, A.ax.a0);
        I.ax.a1 = selv(fa, B.ax.a1, A.ax.a1);
        I.ax.a2 = selv(fa, B.ax.a2, A.ax.a2);
        I.h0 = fa ? B.h0 : A.h0; I.h1 = fa ? B.h1 : A.h1; I.h2 = fa ? B.h2 : A.h2;
        V3 nr = scl(axis_of(R.ax, ri), sg);
        C.n = selv(fa, nr, neg(nr));
        V3 fc, u, v;
        Out4 o;
        face_contact(R, ri, nr, I, margin, fc, u, v, o);
        int code = (fa ? ri : 3 + ri) * 32;
        C.m = o.m;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            C.p[k] = madd(madd(madd(fc, u, o.u[k]), v, o.v[k]), nr, o.n[k] * 0.5f);
            C.d[k] = o.n[k];
            C.id[k] = o.id[k] + code;
        }
        return;
    }
    // edge-edge
    float L = sqrtf(dot(bax, bax));
    V3 w = mk(bax.x / L, bax.y / L, bax.z / L);
    w = selv(dot(w, d) < 0.0f, neg(w), w);
    C.n = w;
    V3 pa = A.c, pb = B.c;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float sg = (dot(Aax[k], w) > 0.0f) ? 1.0f : -1.0f;
        if (k != bi) pa = madd(pa, Aax[k], sg * Ah[k]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float sg = (dot(Bax[k], w) > 0.0f) ? -1.0f : 1.0f;
        if (k != bj) pb = madd(pb, Bax[k], sg * Bh[k]);
    }
    V3 ua = axis_of(A.ax, bi), ub = axis_of(B.ax, bj);
    V3 r = sub(pb, pa);
    float c = dot(ua, ub), ar = dot(ua, r), br = dot(ub, r);
    float den = fmaf_(-c, c, 1.0f);
    float s = fmaf_(-c, br, ar) / den;
    float t = fmaf_(c, ar, -br) / den;
    float ha = sel3(A.h0, A.h1, A.h2, bi), hb = sel3(B.h0, B.h1, B.h2, bj);
    s = s > ha ? ha : (s < -ha ? -ha : s);
    t = t > hb ? hb : (t < -hb ? -hb : t);
    V3 qa = madd(pa, ua, s), qb = madd(pb, ub, t);
    C.m = 1;
    C.p[0] = scl(add(qa, qb), 0.5f);
    C.d[0] = best;
    C.id[0] = 6 * 32 + 3 * bi + bj;
}

CP_DEV void plane_space(V3 n, V3& t1, V3& t2) {
    if (fabsf(n.z) > (float)0.7071067811865476) {
        float a = fmaf_(n.y, n.y, n.z * n.z);
        float k = 1.0f / sqrtf(a);
        t1 = mk(0.0f, -(n.z * k), n.y * k);
        t2 = mk(a * k, -(n.x * t1.z), n.x * t1.y);
    } else {
        float a = fmaf_(n.x, n.x, n.y * n.y);
        float k = 1.0f / sqrtf(a);
        t1 = mk(-(n.y * k), n.x * k, 0.0f);
        t2 = mk(-(n.z * t1.y), n.z * t1.x, a * k);
    }
}

// ----------------------------------------------------------------------------
// Per-substep context (registers).
struct Step {
    Axes ax[CP_NUM_DYN];
    Sym M[CP_NUM_DYN];
    V3 n[CP_NUM_PAIRS];
    uint32_t pk[CP_NUM_PAIRS];  // cnt | base<<3 | fcnt<<8 | fbase<<11
};
CP_DEV int pk_cnt(uint32_t pk) { return (int)(pk & 7u); }
CP_DEV int pk_base(uint32_t pk) { return (int)((pk >> 3) & 31u); }
CP_DEV int pk_fcnt(uint32_t pk) { return (int)((pk >> 8) & 7u); }
CP_DEV int pk_fbase(uint32_t pk) { return (int)((pk >> 11) & 15u); }

// effective inverse mass along t (oracle: row_k); A == 0 is the static ground
template <int A, int B>
CP_DEV float row_k(const Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t) {
    float imb = P.inv_mass[B];
    V3 rbt = cross(rb, t);
    V3 ib = symv(T.M[B - 1], rbt);
    if constexpr (A == 0) {
        return imb + dot(rbt, ib);
    } else {
        float ima = P.inv_mass[A];
        V3 ra = add(rb, sub(S.b[B - 1].x, S.b[A - 1].x));
        V3 rat = cross(ra, t);
        V3 ia = symv(T.M[A - 1], rat);
        return ((ima + imb) + dot(rat, ia)) + dot(rbt, ib);
    }
}

template <int A, int B>
CP_DEV void apply_impulse(Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t, float lam) {
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
CP_DEV float solve_row(Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t, float inv_eff, float target,
                       float& lam, float bound) {
    float imb = P.inv_mass[B];
    V3 rbt = cross(rb, t);
    V3 ib = symv(T.M[B - 1], rbt);
    float vn;
    V3 ia = mk(0.0f, 0.0f, 0.0f);
    if constexpr (A == 0) {
        vn = dot(t, S.b[B - 1].v) + dot(S.b[B - 1].w, rbt);
    } else {
        V3 ra = add(rb, sub(S.b[B - 1].x, S.b[A - 1].x));
        V3 rat = cross(ra, t);
        ia = symv(T.M[A - 1], rat);
        vn = (dot(t, sub(S.b[B - 1].v, S.b[A - 1].v)) + dot(S.b[B - 1].w, rbt)) - dot(S.b[A - 1].w, rat);
    }
    float e = target - vn;
    float dl = e * inv_eff;
    float l0 = lam + dl;
    float ln;
    if constexpr (!FRICTION) ln = l0 > 0.0f ? l0 : 0.0f;
    else ln = l0 > bound ? bound : (l0 < -bound ? -bound : l0);
    dl = ln - lam;
    lam = ln;
    float sb = dl * imb;
    S.b[B - 1].v = madd(S.b[B - 1].v, t, sb);
    S.b[B - 1].w = madd(S.b[B - 1].w, ib, dl);
    if constexpr (A != 0) {
        float sa = dl * P.inv_mass[A];
        S.b[A - 1].v = madd(S.b[A - 1].v, neg(t), sa);
        S.b[A - 1].w = madd(S.b[A - 1].w, neg(ia), dl);
    }
    return fabsf(e * dl);
}

// One PGS row committed only where `act` (selects, not branches, so that two
// independent rows can share a basic block and interleave).  Same arithmetic as
// solve_row; returns |e * dlambda| or 0.
template <int A, int B, bool FRICTION>
CP_DEV float solve_row_sel(Sim& S, const Step& T, const cp_physics& P, V3 rb, V3 t, float inv_eff, float target,
                           float& lam, float bound, bool act) {
    float imb = P.inv_mass[B];
    V3 rbt = cross(rb, t);
    V3 ib = symv(T.M[B - 1], rbt);
    float vn;
    V3 ia = mk(0.0f, 0.0f, 0.0f);
    if constexpr (A == 0) {
        vn = dot(t, S.b[B - 1].v) + dot(S.b[B - 1].w, rbt);
    } else {
        V3 ra = add(rb, sub(S.b[B - 1].x, S.b[A - 1].x));
        V3 rat = cross(ra, t);
        ia = symv(T.M[A - 1], rat);
        vn = (dot(t, sub(S.b[B - 1].v, S.b[A - 1].v)) + dot(S.b[B - 1].w, rbt)) - dot(S.b[A - 1].w, rat);
    }
    float e = target - vn;
    float dl = e * inv_eff;
    float l0 = lam + dl;
    float ln;
    if constexpr (!FRICTION) ln = l0 > 0.0f ? l0 : 0.0f;
    else ln = l0 > bound ? bound : (l0 < -bound ? -bound : l0);
    dl = ln - lam;
    lam = act ? ln : lam;
    float sb = dl * imb;
    S.b[B - 1].v = selv(act, madd(S.b[B - 1].v, t, sb), S.b[B - 1].v);
    S.b[B - 1].w = selv(act, madd(S.b[B - 1].w, ib, dl), S.b[B - 1].w);
    if constexpr (A != 0) {
        float sa = dl * P.inv_mass[A];
        S.b[A - 1].v = selv(act, madd(S.b[A - 1].v, neg(t), sa), S.b[A - 1].v);
        S.b[A - 1].w = selv(act, madd(S.b[A - 1].w, neg(ia), dl), S.b[A - 1].w);
    }
    return act ? fabsf(e * dl) : 0.0f;
}

// Normal rows of two pairs from different islands, interleaved row by row.
template <int PA, int PB>
CP_DEV void pair2_normal_rows(Sim& S, const Step& T, const cp_physics& P, float* pool, float& resA, float& resB) {
    const uint32_t pkA = T.pk[PA], pkB = T.pk[PB];
    const int cA = pk_cnt(pkA), bA = pk_base(pkA), cB = pk_cnt(pkB), bB = pk_base(pkB);
    const int n = cA > cB ? cA : cB;
    for (int k = 0; k < n; ++k) {
        const bool actA = k < cA, actB = k < cB;
        const int sA = (bA + k) < MAXP ? bA + k : MAXP - 1;
        const int sB = (bB + k) < MAXP ? bB + k : MAXP - 1;
        V3 rbA = mk(pool_n(pool, F_RBX, sA), pool_n(pool, F_RBY, sA), pool_n(pool, F_RBZ, sA));
        V3 rbB = mk(pool_n(pool, F_RBX, sB), pool_n(pool, F_RBY, sB), pool_n(pool, F_RBZ, sB));
        float ieA = pool_n(pool, F_IE, sA), tgA = pool_n(pool, F_TG, sA), lamA = pool_n(pool, F_LAM, sA);
        float ieB = pool_n(pool, F_IE, sB), tgB = pool_n(pool, F_TG, sB), lamB = pool_n(pool, F_LAM, sB);
        float rA = solve_row_sel<pair_a(PA), pair_b(PA), false>(S, T, P, rbA, T.n[PA], ieA, tgA, lamA, 0.0f, actA);
        float rB = solve_row_sel<pair_a(PB), pair_b(PB), false>(S, T, P, rbB, T.n[PB], ieB, tgB, lamB, 0.0f, actB);
        resA = resA + rA;
        resB = resB + rB;
        if (actA) pool_n(pool, F_LAM, sA) = lamA;
        if (actB) pool_n(pool, F_LAM, sB) = lamB;
    }
}

// Friction rows (t1 then t2 per point) of two pairs from different islands, interleaved.
template <int PA, int PB>
CP_DEV void pair2_friction_rows(Sim& S, const Step& T, const cp_physics& P, float* pool, float& resA,
                                float& resB) {
    const uint32_t pkA = T.pk[PA], pkB = T.pk[PB];
    const int cA = pk_fcnt(pkA), cB = pk_fcnt(pkB);
    const int n = cA > cB ? cA : cB;
    if (n == 0) return;
    const int bA = pk_base(pkA), fA = pk_fbase(pkA), bB = pk_base(pkB), fB = pk_fbase(pkB);
    const float muA = P.friction[pair_a(PA)] * P.friction[pair_b(PA)];
    const float muB = P.friction[pair_a(PB)] * P.friction[pair_b(PB)];
    // tangent basis inside the sweep: hoisted out of the PGS loop for every pair it
    // would pin ~60 VGPRs for the whole solve
    V3 nA = T.n[PA], nB = T.n[PB];
    asm volatile("" : "+v"(nA.x), "+v"(nA.y), "+v"(nA.z), "+v"(nB.x), "+v"(nB.y), "+v"(nB.z));
    V3 a1, a2, b1, b2;
    plane_space(nA, a1, a2);
    plane_space(nB, b1, b2);
    for (int k = 0; k < n; ++k) {
        const bool actA = k < cA, actB = k < cB;
        const int sA = (bA + k) < MAXP ? bA + k : MAXP - 1, sB = (bB + k) < MAXP ? bB + k : MAXP - 1;
        const int gA = (fA + k) < MAXF ? fA + k : MAXF - 1, gB = (fB + k) < MAXF ? fB + k : MAXF - 1;
        V3 rbA = mk(pool_n(pool, F_RBX, sA), pool_n(pool, F_RBY, sA), pool_n(pool, F_RBZ, sA));
        V3 rbB = mk(pool_n(pool, F_RBX, sB), pool_n(pool, F_RBY, sB), pool_n(pool, F_RBZ, sB));
        const float boundA = muA * pool_n(pool, F_LAM, sA), boundB = muB * pool_n(pool, F_LAM, sB);
        float lA1 = pool_f(pool, FF_L1, gA), lA2 = pool_f(pool, FF_L2, gA);
        float lB1 = pool_f(pool, FF_L1, gB), lB2 = pool_f(pool, FF_L2, gB);
        const float ieA1 = pool_f(pool, FF_IE1, gA), ieA2 = pool_f(pool, FF_IE2, gA);
        const float ieB1 = pool_f(pool, FF_IE1, gB), ieB2 = pool_f(pool, FF_IE2, gB);
        constexpr int AA = pair_a(PA), AB = pair_b(PA), BA = pair_a(PB), BB = pair_b(PB);
        float rA1 = solve_row_sel<AA, AB, true>(S, T, P, rbA, a1, ieA1, 0.0f, lA1, boundA, actA);
        float rB1 = solve_row_sel<BA, BB, true>(S, T, P, rbB, b1, ieB1, 0.0f, lB1, boundB, actB);
        resA = resA + rA1;
        resB = resB + rB1;
        float rA2 = solve_row_sel<AA, AB, true>(S, T, P, rbA, a2, ieA2, 0.0f, lA2, boundA, actA);
        float rB2 = solve_row_sel<BA, BB, true>(S, T, P, rbB, b2, ieB2, 0.0f, lB2, boundB, actB);
        resA = resA + rA2;
        resB = resB + rB2;
        if (actA) { pool_f(pool, FF_L1, gA) = lA1; pool_f(pool, FF_L2, gA) = lA2; }
        if (actB) { pool_f(pool, FF_L1, gB) = lB1; pool_f(pool, FF_L2, gB) = lB2; }
    }
}

template <int PAIR>
CP_DEV void pair_warmstart(Sim& S, const Step& T, const cp_physics& P, float* pool) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    const uint32_t pk = T.pk[PAIR];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    for (int k = 0; k < cnt; ++k) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        apply_impulse<A, B>(S, T, P, rb, T.n[PAIR], pool_n(pool, F_LAM, s));
    }
}

template <int PAIR>
CP_DEV void pair_normal_rows(Sim& S, const Step& T, const cp_physics& P, float* pool, float& resid) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    const uint32_t pk = T.pk[PAIR];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
    for (int k = 0; k < cnt; ++k) {
        const int s = base + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        float lam = pool_n(pool, F_LAM, s);
        float r = solve_row<A, B, false>(S, T, P, rb, T.n[PAIR], pool_n(pool, F_IE, s), pool_n(pool, F_TG, s),
                                         lam, 0.0f);
        pool_n(pool, F_LAM, s) = lam;
        resid = resid + r;
    }
}

template <int PAIR>
CP_DEV void pair_friction_rows(Sim& S, const Step& T, const cp_physics& P, float* pool, float& resid) {
    constexpr int A = pair_a(PAIR), B = pair_b(PAIR);
    const uint32_t pk = T.pk[PAIR];
    const int fcnt = pk_fcnt(pk);
    if (fcnt == 0) return;
    const int base = pk_base(pk), fbase = pk_fbase(pk);
    const float mu = P.friction[A] * P.friction[B];
    // keep the tangent basis inside the sweep: hoisted out of the PGS loop for all
    // 10 pairs it would pin ~60 VGPRs for the whole solve
    V3 n = T.n[PAIR];
    asm volatile("" : "+v"(n.x), "+v"(n.y), "+v"(n.z));
    V3 t1, t2;
    plane_space(n, t1, t2);
    for (int k = 0; k < fcnt; ++k) {
        const int s = base + k, fs = fbase + k;
        V3 rb = mk(pool_n(pool, F_RBX, s), pool_n(pool, F_RBY, s), pool_n(pool, F_RBZ, s));
        float bound = mu * pool_n(pool, F_LAM, s);
        float l1 = pool_f(pool, FF_L1, fs), l2 = pool_f(pool, FF_L2, fs);
        float r1 = solve_row<A, B, true>(S, T, P, rb, t1, pool_f(pool, FF_IE1, fs), 0.0f, l1, bound);
        resid = resid + r1;
        float r2 = solve_row<A, B, true>(S, T, P, rb, t2, pool_f(pool, FF_IE2, fs), 0.0f, l2, bound);
        resid = resid + r2;
        pool_f(pool, FF_L1, fs) = l1;
        pool_f(pool, FF_L2, fs) = l2;
    }
}

template <int PAIR>
CP_DEV void pair_cache(const Step& T, float* pool, const Mem& G) {
    const uint32_t pk = T.pk[PAIR];
    const int cnt = pk_cnt(pk), base = pk_base(pk);
#pragma unroll
    for (int k = 0; k < 4; ++k) G.ss(CP_SF_WS_LAM(PAIR, k), (k < cnt) ? pool_n(pool, F_LAM, base + k) : 0.0f);
}

#define CP_FOR_PAIRS(F, ...) \
    F<0>(__VA_ARGS__); F<1>(__VA_ARGS__); F<2>(__VA_ARGS__); F<3>(__VA_ARGS__); F<4>(__VA_ARGS__); \
    F<5>(__VA_ARGS__); F<6>(__VA_ARGS__); F<7>(__VA_ARGS__); F<8>(__VA_ARGS__); F<9>(__VA_ARGS__)

// ---- uniform-index accessors for the wave-uniform narrowphase pair loop ----
CP_DEV V3 sel5v(int g, V3 z, V3 a, V3 b, V3 c, V3 d) {
    return mk(g == 1 ? a.x : g == 2 ? b.x : g == 3 ? c.x : g == 4 ? d.x : z.x,
              g == 1 ? a.y : g == 2 ? b.y : g == 3 ? c.y : g == 4 ? d.y : z.y,
              g == 1 ? a.z : g == 2 ? b.z : g == 3 ? c.z : g == 4 ? d.z : z.z);
}
CP_DEV float sel5(int g, float z, float a, float b, float c, float d) {
    return g == 1 ? a : g == 2 ? b : g == 3 ? c : g == 4 ? d : z;
}
CP_DEV Box box_of(int g, const Sim& S, const Step& T, const cp_physics& P) {
    Box b;
    b.h0 = P.half_extents[g][0];
    b.h1 = P.half_extents[g][1];
    b.h2 = P.half_extents[g][2];
    const V3 z = mk(0.0f, 0.0f, 0.0f);
    b.c = sel5v(g, z, S.b[0].x, S.b[1].x, S.b[2].x, S.b[3].x);
    b.ax.a0 = sel5v(g, mk(1.0f, 0.0f, 0.0f), T.ax[0].a0, T.ax[1].a0, T.ax[2].a0, T.ax[3].a0);
    b.ax.a1 = sel5v(g, mk(0.0f, 1.0f, 0.0f), T.ax[0].a1, T.ax[1].a1, T.ax[2].a1, T.ax[3].a1);
    b.ax.a2 = sel5v(g, mk(0.0f, 0.0f, 1.0f), T.ax[0].a2, T.ax[1].a2, T.ax[2].a2, T.ax[3].a2);
    return b;
}
CP_DEV Sym sym_of(int g, const Step& T) {
    Sym m;
    m.m0 = sel5(g, 0.0f, T.M[0].m0, T.M[1].m0, T.M[2].m0, T.M[3].m0);
    m.m1 = sel5(g, 0.0f, T.M[0].m1, T.M[1].m1, T.M[2].m1, T.M[3].m1);
    m.m2 = sel5(g, 0.0f, T.M[0].m2, T.M[1].m2, T.M[2].m2, T.M[3].m2);
    m.m3 = sel5(g, 0.0f, T.M[0].m3, T.M[1].m3, T.M[2].m3, T.M[3].m3);
    m.m4 = sel5(g, 0.0f, T.M[0].m4, T.M[1].m4, T.M[2].m4, T.M[3].m4);
    m.m5 = sel5(g, 0.0f, T.M[0].m5, T.M[1].m5, T.M[2].m5, T.M[3].m5);
    return m;
}
CP_DEV V3 pos_of(int g, const Sim& S) {
    return sel5v(g, mk(0.0f, 0.0f, 0.0f), S.b[0].x, S.b[1].x, S.b[2].x, S.b[3].x);
}

// row setup for direction t with pair bodies selected at run time (narrowphase)
CP_DEV float row_k_dyn(int a, float ima, float imb, V3 xa, V3 xb, const Sym& Ma, const Sym& Mb, V3 rb, V3 t) {
    V3 rbt = cross(rb, t);
    V3 ib = symv(Mb, rbt);
    if (a == 0) return imb + dot(rbt, ib);
    V3 ra = add(rb, sub(xb, xa));
    V3 rat = cross(ra, t);
    V3 ia = symv(Ma, rat);
    return ((ima + imb) + dot(rat, ia)) + dot(rbt, ib);
}

// One p.stepSimulation() for this lane's env (DESIGN.md §Physics model 1-6).
CP_DEV void substep(Sim& S, const cp_physics& P, float* pool, int& overflow, const Mem& G, Stamps& ST) {
    const float dt = P.dt, inv_dt = P.inv_dt;
    CP_STAMP(t0);
    Step T;
    // 1. orientation + world inverse inertia
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        T.ax[d] = quat_axes(S.b[d].q[0], S.b[d].q[1], S.b[d].q[2], S.b[d].q[3]);
        T.M[d] = world_inv_inertia(T.ax[d], P.inv_inertia[d + 1][0], P.inv_inertia[d + 1][1],
                                   P.inv_inertia[d + 1][2]);
    }
    // 2. narrowphase + row setup, wave-uniform loop over the 10 pairs
    int used = 0, fused = 0;
#pragma unroll 1
    for (int p = 0; p < CP_NUM_PAIRS; ++p) {
        const int a = pair_a(p), b = pair_b(p);
        Box A = box_of(a, S, T, P), Bx = box_of(b, S, T, P);
        Contact C;
        box_box(A, Bx, P.contact_margin, P.edge_bias, C);
        const float mu = P.friction[a] * P.friction[b];
        const float ima = P.inv_mass[a], imb = P.inv_mass[b];
        const V3 xa = pos_of(a, S), xb = pos_of(b, S);
        const Sym Ma = sym_of(a, T), Mb = sym_of(b, T);
        const uint32_t oid = __float_as_uint(G.ls(CP_SF_WS_ID(p)));
        const float ol0 = G.ls(CP_SF_WS_LAM(p, 0)), ol1 = G.ls(CP_SF_WS_LAM(p, 1));
        const float ol2 = G.ls(CP_SF_WS_LAM(p, 2)), ol3 = G.ls(CP_SF_WS_LAM(p, 3));
        const int base = used, fbase = fused;
        int m = 0, fm = 0;
        uint32_t nid = 0xFFFFFFFFu;
        V3 t1 = mk(0.0f, 0.0f, 0.0f), t2 = t1;
        if (mu > 0.0f) plane_space(C.n, t1, t2);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < C.m) {
                if (base + m >= MAXP) {
                    overflow += 1;  // dropped by the pool cap (oracle: same count)
                } else {
                    const int s = base + m;
                    V3 rb = sub(C.p[k], xb);
                    float K = row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, C.n);
                    float dist = C.d[k];
                    float tg = dist > 0.0f ? -(dist * inv_dt) : -((P.erp * dist) * inv_dt);
                    const int id = C.id[k];
                    float l0 = 0.0f;
                    if ((int)(oid & 0xFFu) == id) l0 = ol0;
                    else if ((int)((oid >> 8) & 0xFFu) == id) l0 = ol1;
                    else if ((int)((oid >> 16) & 0xFFu) == id) l0 = ol2;
                    else if ((int)((oid >> 24) & 0xFFu) == id) l0 = ol3;
                    pool_n(pool, F_RBX, s) = rb.x;
                    pool_n(pool, F_RBY, s) = rb.y;
                    pool_n(pool, F_RBZ, s) = rb.z;
                    pool_n(pool, F_IE, s) = 1.0f / K;
                    pool_n(pool, F_TG, s) = tg;
                    pool_n(pool, F_LAM, s) = P.warmstart * l0;
                    nid = (nid & ~(0xFFu << (8 * m))) | ((uint32_t)id << (8 * m));
                    if (mu > 0.0f) {
                        if (fbase + fm >= MAXF) {
                            overflow += 1;
                        } else {
                            const int fs = fbase + fm;
                            pool_f(pool, FF_IE1, fs) = 1.0f / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t1);
                            pool_f(pool, FF_IE2, fs) = 1.0f / row_k_dyn(a, ima, imb, xa, xb, Ma, Mb, rb, t2);
                            pool_f(pool, FF_L1, fs) = 0.0f;
                            pool_f(pool, FF_L2, fs) = 0.0f;
                            fm += 1;
                        }
                    }
                    m += 1;
                }
            }
        }
        used = base + m;
        fused = fbase + fm;
        const uint32_t pk = (uint32_t)m | ((uint32_t)base << 3) | ((uint32_t)fm << 8) | ((uint32_t)fbase << 11);
        G.sx(4 * p + 0, C.n.x);
        G.sx(4 * p + 1, C.n.y);
        G.sx(4 * p + 2, C.n.z);
        G.sx(4 * p + 3, __uint_as_float(pk));
        G.ss(CP_SF_WS_ID(p), __uint_as_float(nid));
    }
#pragma unroll
    for (int p = 0; p < CP_NUM_PAIRS; ++p) {
        T.n[p] = mk(G.lx(4 * p + 0), G.lx(4 * p + 1), G.lx(4 * p + 2));
        T.pk[p] = __float_as_uint(G.lx(4 * p + 3));
    }
    CP_STAMP(t1);
    CP_ACC(narrow, t0, t1);
    // 3. unconstrained velocity update
    const float kl = P.lin_damping, ka = P.ang_damping;
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        const int g = d + 1;
        const float im = P.inv_mass[g];
        V3 v = S.b[d].v, w = S.b[d].w;
        V3 F = (d == 0) ? S.f0 : ((d == 2) ? S.f2 : mk(0.0f, 0.0f, 0.0f));
        float vlen = sqrtf(dot(v, v));
        float dv = fmaf_(kl, vlen, kl);
        V3 acc = mk(fmaf_(-v.x, dv, fmaf_(F.x, im, P.gravity[0])), fmaf_(-v.y, dv, fmaf_(F.y, im, P.gravity[1])),
                    fmaf_(-v.z, dv, fmaf_(F.z, im, P.gravity[2])));
        V3 wl = rot_t(T.ax[d], w);
        V3 Iwl = mk(P.inertia[g][0] * wl.x, P.inertia[g][1] * wl.y, P.inertia[g][2] * wl.z);
        V3 gl = cross(wl, Iwl);
        V3 al = mk(-(P.inv_inertia[g][0] * gl.x), -(P.inv_inertia[g][1] * gl.y), -(P.inv_inertia[g][2] * gl.z));
        V3 aw = rot(T.ax[d], al);
        float wlen = sqrtf(dot(w, w));
        float dw = fmaf_(ka, wlen, ka);
        V3 accw = mk(fmaf_(-w.x, dw, aw.x), fmaf_(-w.y, dw, aw.y), fmaf_(-w.z, dw, aw.z));
        S.b[d].v = madd(v, acc, dt);
        S.b[d].w = madd(w, accw, dt);
    }
    // 4a. warm start, in solver pair order (oracle SOLVE_ORDER = 0 2 1 3 4 9 5 6 7 8)
    pair_warmstart<0>(S, T, P, pool); pair_warmstart<2>(S, T, P, pool);
    pair_warmstart<1>(S, T, P, pool); pair_warmstart<3>(S, T, P, pool);
    pair_warmstart<4>(S, T, P, pool); pair_warmstart<9>(S, T, P, pool);
    pair_warmstart<5>(S, T, P, pool); pair_warmstart<6>(S, T, P, pool);
    pair_warmstart<7>(S, T, P, pool); pair_warmstart<8>(S, T, P, pool);
    CP_STAMP(t2);
    CP_ACC(vel, t1, t2);
    // 4b. PGS sweeps; a lane stops after the sweep whose residual <= threshold
    bool active = used > 0;
    const float thr = P.residual_threshold;
    for (int it = 0; it < P.solver_iterations; ++it) {
        if (__ballot(active) == 0ull) break;
#ifdef CP_STAMPS
        ST.sweeps += 1;
#endif
        if (active) {
            // island 1 = pairs 0,1,4 ; island 2 = pairs 2,3,9 ; cross = 5..8 (oracle SOLVE_ORDER)
            float r1 = 0.0f, r2 = 0.0f, rc = 0.0f;
            pair_normal_rows<0>(S, T, P, pool, r1);
            pair_normal_rows<2>(S, T, P, pool, r2);
            pair_normal_rows<1>(S, T, P, pool, r1);
            pair_normal_rows<3>(S, T, P, pool, r2);
            pair_normal_rows<4>(S, T, P, pool, r1);
            pair_normal_rows<9>(S, T, P, pool, r2);
            pair_normal_rows<5>(S, T, P, pool, rc);
            pair_normal_rows<6>(S, T, P, pool, rc);
            pair_normal_rows<7>(S, T, P, pool, rc);
            pair_normal_rows<8>(S, T, P, pool, rc);
            pair_friction_rows<0>(S, T, P, pool, r1);
            pair_friction_rows<2>(S, T, P, pool, r2);
            pair_friction_rows<1>(S, T, P, pool, r1);
            pair_friction_rows<3>(S, T, P, pool, r2);
            pair_friction_rows<4>(S, T, P, pool, r1);
            pair_friction_rows<9>(S, T, P, pool, r2);
            pair_friction_rows<5>(S, T, P, pool, rc);
            pair_friction_rows<6>(S, T, P, pool, rc);
            pair_friction_rows<7>(S, T, P, pool, rc);
            pair_friction_rows<8>(S, T, P, pool, rc);
            const float resid = (r1 + r2) + rc;
            if (resid <= thr) active = false;
        }
    }
    CP_STAMP(t3);
    CP_ACC(solve, t2, t3);
    // 4c. refresh the warm-start cache
    CP_FOR_PAIRS(pair_cache, T, pool, G);
    // 5. integrate positions and orientations
    const float hdt = 0.5f * dt;
    const float c3 = ((dt * dt) * dt) * (float)0.020833333333;
    const float maxang = P.max_angular_step;
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        V3 v = S.b[d].v, w = S.b[d].w;
        S.b[d].x = madd(S.b[d].x, v, dt);
        float ang = sqrtf(dot(w, w));
        if (ang * dt > maxang) ang = maxang * inv_dt;
        float half = hdt * ang;
        float sn, cs, s;
        sincos_small(half, sn, cs);
        if (ang < 0.001f) s = fmaf_(-c3, ang * ang, hdt);
        else s = sn / ang;
        float dx = w.x * s, dy = w.y * s, dz = w.z * s, dw = cs;
        float qx = S.b[d].q[0], qy = S.b[d].q[1], qz = S.b[d].q[2], qw = S.b[d].q[3];
        float rw = fmaf_(dw, qw, -fmaf_(dx, qx, fmaf_(dy, qy, dz * qz)));
        float rx = fmaf_(dw, qx, fmaf_(dx, qw, fmaf_(dy, qz, -(dz * qy))));
        float ry = fmaf_(dw, qy, fmaf_(dy, qw, fmaf_(dz, qx, -(dx * qz))));
        float rz = fmaf_(dw, qz, fmaf_(dz, qw, fmaf_(dx, qy, -(dy * qx))));
        float n2 = fmaf_(rx, rx, fmaf_(ry, ry, fmaf_(rz, rz, rw * rw)));
        float inv = 1.0f / sqrtf(n2);
        S.b[d].q[0] = rx * inv;
        S.b[d].q[1] = ry * inv;
        S.b[d].q[2] = rz * inv;
        S.b[d].q[3] = rw * inv;
    }
    // 6. external forces are consumed by the step
    S.f0 = mk(0.0f, 0.0f, 0.0f);
    S.f2 = mk(0.0f, 0.0f, 0.0f);
    CP_STAMP(t4);
    CP_ACC(integ, t3, t4);
#ifdef CP_STAMPS
    ST.substeps += 1;
#endif
}

// LINK_FRAME force at the COM on cart (C = 0) or cart2 (C = 1): world = R(q) f
template <int C>
CP_DEV void apply_force_link(Sim& S, float fx, float fy) {
    const Body& B = S.b[C == 0 ? 0 : 2];
    Axes A = quat_axes(B.q[0], B.q[1], B.q[2], B.q[3]);
    V3 fw = rot(A, mk(fx, fy, 0.0f));
    if constexpr (C == 0) S.f0 = add(S.f0, fw);
    else S.f2 = add(S.f2, fw);
}

}  // namespace cp
