// cp_math.h — fp32 device math for the cartpole kernels (gfx950).
//
// Every fused multiply-add is explicit (__builtin_fmaf -> v_fma_f32) and the
// library is compiled with -ffp-contract=off, so each expression rounds exactly
// as written; division and sqrt are the IEEE-correct defaults.  The three
// transcendentals the step needs (small-angle sin/cos, bump direction, atan for
// Euler readback) are own polynomials, so results do not depend on the device
// math library.  DESIGN.md §Numerics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cp {

#define CP_DEV __device__ __forceinline__

CP_DEV float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

struct V3 {
    float x, y, z;
};

CP_DEV V3 mk(float x, float y, float z) { return V3{x, y, z}; }
CP_DEV V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
CP_DEV V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
CP_DEV V3 scl(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
CP_DEV V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
// a + b*s
CP_DEV V3 madd(V3 a, V3 b, float s) { return mk(fmaf_(b.x, s, a.x), fmaf_(b.y, s, a.y), fmaf_(b.z, s, a.z)); }
CP_DEV float dot(V3 a, V3 b) { return fmaf_(a.x, b.x, fmaf_(a.y, b.y, a.z * b.z)); }
CP_DEV V3 cross(V3 a, V3 b) {
    return mk(fmaf_(a.y, b.z, -(a.z * b.y)), fmaf_(a.z, b.x, -(a.x * b.z)), fmaf_(a.x, b.y, -(a.y * b.x)));
}

// Box axes (columns of R) from a unit quaternion xyzw.
struct Axes {
    V3 a0, a1, a2;
};
CP_DEV Axes quat_axes(float x, float y, float z, float w) {
    float x2 = x + x, y2 = y + y, z2 = z + z;
    float xx = x * x2, yy = y * y2, zz = z * z2;
    float xy = x * y2, xz = x * z2, yz = y * z2;
    float wx = w * x2, wy = w * y2, wz = w * z2;
    Axes r;
    r.a0 = mk(1.0f - (yy + zz), xy + wz, xz - wy);
    r.a1 = mk(xy - wz, 1.0f - (xx + zz), yz + wx);
    r.a2 = mk(xz + wy, yz - wx, 1.0f - (xx + yy));
    return r;
}
CP_DEV V3 rot(const Axes& A, V3 l) {
    return mk(fmaf_(A.a0.x, l.x, fmaf_(A.a1.x, l.y, A.a2.x * l.z)),
              fmaf_(A.a0.y, l.x, fmaf_(A.a1.y, l.y, A.a2.y * l.z)),
              fmaf_(A.a0.z, l.x, fmaf_(A.a1.z, l.y, A.a2.z * l.z)));
}
CP_DEV V3 rot_t(const Axes& A, V3 w) { return mk(dot(A.a0, w), dot(A.a1, w), dot(A.a2, w)); }

// symmetric 3x3 (xx xy xz yy yz zz)
struct Sym {
    float m0, m1, m2, m3, m4, m5;
};
CP_DEV Sym world_inv_inertia(const Axes& A, float i0, float i1, float i2) {
    V3 t0 = scl(A.a0, i0), t1 = scl(A.a1, i1), t2 = scl(A.a2, i2);
    Sym M;
    M.m0 = fmaf_(t0.x, A.a0.x, fmaf_(t1.x, A.a1.x, t2.x * A.a2.x));
    M.m1 = fmaf_(t0.x, A.a0.y, fmaf_(t1.x, A.a1.y, t2.x * A.a2.y));
    M.m2 = fmaf_(t0.x, A.a0.z, fmaf_(t1.x, A.a1.z, t2.x * A.a2.z));
    M.m3 = fmaf_(t0.y, A.a0.y, fmaf_(t1.y, A.a1.y, t2.y * A.a2.y));
    M.m4 = fmaf_(t0.y, A.a0.z, fmaf_(t1.y, A.a1.z, t2.y * A.a2.z));
    M.m5 = fmaf_(t0.z, A.a0.z, fmaf_(t1.z, A.a1.z, t2.z * A.a2.z));
    return M;
}
CP_DEV V3 symv(const Sym& M, V3 v) {
    return mk(fmaf_(M.m0, v.x, fmaf_(M.m1, v.y, M.m2 * v.z)),
              fmaf_(M.m1, v.x, fmaf_(M.m3, v.y, M.m4 * v.z)),
              fmaf_(M.m2, v.x, fmaf_(M.m4, v.y, M.m5 * v.z)));
}

// Taylor sin/cos for |x| <= pi/4 (constants rounded from double, as the oracle)
CP_DEV void sincos_small(float x, float& s, float& c) {
    float x2 = x * x;
    float p = fmaf_(x2, (float)2.7557319223985893e-6, (float)-1.9841269841269841e-4);
    p = fmaf_(x2, p, (float)8.3333333333333333e-3);
    p = fmaf_(x2, p, (float)-1.6666666666666667e-1);
    s = fmaf_(x * x2, p, x);
    float q = fmaf_(x2, (float)2.4801587301587302e-5, (float)-1.3888888888888889e-3);
    q = fmaf_(x2, q, (float)4.1666666666666667e-2);
    q = fmaf_(x2, q, -0.5f);
    c = fmaf_(x2, q, 1.0f);
}

// sin/cos(2*pi*u), u in [0,1): quadrant split + pi/4 rotation of a small angle
CP_DEV void sincos_turns(float u, float& so, float& co) {
    float y = u * 4.0f;
    int q = (int)y;
    q = q > 3 ? 3 : q;
    float f = y - (float)q;
    float x = (f - 0.5f) * (float)1.5707963267948966;
    float s, c;
    sincos_small(x, s, c);
    float S = (s + c) * (float)0.7071067811865476;
    float C = (c - s) * (float)0.7071067811865476;
    so = (q == 0) ? S : (q == 1) ? C : (q == 2) ? -S : -C;
    co = (q == 0) ? C : (q == 1) ? -S : (q == 2) ? -C : S;
}

CP_DEV float atan_pos(float z) {
    float base = 0.0f;
    if (z > (float)2.414213562373095) {
        base = (float)1.5707963267948966;
        z = -1.0f / z;
    } else if (z > (float)0.4142135623730950) {
        base = (float)0.7853981633974483;
        z = (z - 1.0f) / (z + 1.0f);
    }
    float z2 = z * z;
    float p = fmaf_(z2, (float)8.05374449538e-2, (float)-1.38776856032e-1);
    p = fmaf_(z2, p, (float)1.99777106478e-1);
    p = fmaf_(z2, p, (float)-3.33329491539e-1);
    return base + fmaf_(z * z2, p, z);
}
CP_DEV float atan2_own(float y, float x) {
    if (x == 0.0f && y == 0.0f) return 0.0f;
    float ax = fabsf(x), ay = fabsf(y);
    float r = (ay <= ax) ? atan_pos(ay / ax) : (float)1.5707963267948966 - atan_pos(ax / ay);
    if (x < 0.0f) r = (float)3.141592653589793 - r;
    if (y < 0.0f) r = -r;
    return r;
}
// roll, pitch, yaw as pybullet getEulerFromQuaternion
CP_DEV V3 quat_euler(float x, float y, float z, float w) {
    float sqw = w * w, sqx = x * x, sqy = y * y, sqz = z * z;
    float roll = atan2_own(2.0f * fmaf_(y, z, w * x), ((sqw - sqx) - sqy) + sqz);
    float sarg = -2.0f * fmaf_(x, z, -(w * y));
    float pitch;
    if (sarg <= -1.0f) pitch = (float)-1.5707963267948966;
    else if (sarg >= 1.0f) pitch = (float)1.5707963267948966;
    else pitch = atan2_own(sarg, sqrtf(fmaf_(-sarg, sarg, 1.0f)));
    float yaw = atan2_own(2.0f * fmaf_(x, y, w * z), ((sqw + sqx) - sqy) - sqz);
    return mk(roll, pitch, yaw);
}

// Philox4x32-10 (Salmon et al., SC'11), counter (c0..c3), key (k0,k1); returns word `lane`
CP_DEV uint32_t philox_word(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                            int lane) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    return lane == 0 ? c0 : lane == 1 ? c1 : lane == 2 ? c2 : c3;
}

}  // namespace cp
