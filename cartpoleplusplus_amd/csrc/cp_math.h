// cp_math.h — device math of the cartpole kernels (gfx950), over `real` (CP_REAL).
//
// Included once per real type by the translation unit that instantiates the physics
// (CP_NS / CP_REAL defined first: cp = float, cp64 = double; see cp_common.h).  Every
// fused multiply-add is explicit (fma_ -> v_fma_f32 / v_fma_f64) and the library is
// compiled with -ffp-contract=off, so each expression rounds exactly as written; division
// and sqrt are the IEEE-correct defaults.  The three transcendentals the step needs
// (small-angle sin/cos, bump direction, atan for Euler readback) are own polynomials, so
// results do not depend on the device math library.  Literals are real(<double literal>),
// the oracle's RC(x).  DESIGN.md §Numerics.
#if !defined(CP_NS) || !defined(CP_REAL)
#error "define CP_NS and CP_REAL before including cp_math.h (see cp_kernels.hip)"
#endif
#include "cp_common.h"

namespace CP_NS {
using namespace cpc;
// using-declarations: overloads added in this namespace (partner(V3), ...) must not hide cpc's
using cpc::abs_;
using cpc::bits_to;
using cpc::clamp_sym;
using cpc::fma_;
using cpc::partner;
using cpc::partner_u;
using cpc::lane_of;
using cpc::lane_of_u;
using cpc::sqrt_;
using cpc::to_bits;
using real = CP_REAL;

struct V3 {
    real x, y, z;
};

CP_DEV V3 mk(real x, real y, real z) { return V3{x, y, z}; }
CP_DEV V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
CP_DEV V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
CP_DEV V3 scl(V3 a, real s) { return mk(a.x * s, a.y * s, a.z * s); }
CP_DEV V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
// a + b*s
CP_DEV V3 madd(V3 a, V3 b, real s) { return mk(fma_(b.x, s, a.x), fma_(b.y, s, a.y), fma_(b.z, s, a.z)); }
CP_DEV real dot(V3 a, V3 b) { return fma_(a.x, b.x, fma_(a.y, b.y, a.z * b.z)); }
CP_DEV V3 cross(V3 a, V3 b) {
    return mk(fma_(a.y, b.z, -(a.z * b.y)), fma_(a.z, b.x, -(a.x * b.z)), fma_(a.x, b.y, -(a.y * b.x)));
}

// Box axes (columns of R) from a unit quaternion xyzw.
struct Axes {
    V3 a0, a1, a2;
};
CP_DEV Axes quat_axes(real x, real y, real z, real w) {
    real x2 = x + x, y2 = y + y, z2 = z + z;
    real xx = x * x2, yy = y * y2, zz = z * z2;
    real xy = x * y2, xz = x * z2, yz = y * z2;
    real wx = w * x2, wy = w * y2, wz = w * z2;
    Axes r;
    r.a0 = mk(real(1.0) - (yy + zz), xy + wz, xz - wy);
    r.a1 = mk(xy - wz, real(1.0) - (xx + zz), yz + wx);
    r.a2 = mk(xz + wy, yz - wx, real(1.0) - (xx + yy));
    return r;
}
CP_DEV V3 rot(const Axes& A, V3 l) {
    return mk(fma_(A.a0.x, l.x, fma_(A.a1.x, l.y, A.a2.x * l.z)),
              fma_(A.a0.y, l.x, fma_(A.a1.y, l.y, A.a2.y * l.z)),
              fma_(A.a0.z, l.x, fma_(A.a1.z, l.y, A.a2.z * l.z)));
}
CP_DEV V3 rot_t(const Axes& A, V3 w) { return mk(dot(A.a0, w), dot(A.a1, w), dot(A.a2, w)); }

// symmetric 3x3 (xx xy xz yy yz zz)
struct Sym {
    real m0, m1, m2, m3, m4, m5;
};
CP_DEV Sym world_inv_inertia(const Axes& A, real i0, real i1, real i2) {
    V3 t0 = scl(A.a0, i0), t1 = scl(A.a1, i1), t2 = scl(A.a2, i2);
    Sym M;
    M.m0 = fma_(t0.x, A.a0.x, fma_(t1.x, A.a1.x, t2.x * A.a2.x));
    M.m1 = fma_(t0.x, A.a0.y, fma_(t1.x, A.a1.y, t2.x * A.a2.y));
    M.m2 = fma_(t0.x, A.a0.z, fma_(t1.x, A.a1.z, t2.x * A.a2.z));
    M.m3 = fma_(t0.y, A.a0.y, fma_(t1.y, A.a1.y, t2.y * A.a2.y));
    M.m4 = fma_(t0.y, A.a0.z, fma_(t1.y, A.a1.z, t2.y * A.a2.z));
    M.m5 = fma_(t0.z, A.a0.z, fma_(t1.z, A.a1.z, t2.z * A.a2.z));
    return M;
}
CP_DEV V3 symv(const Sym& M, V3 v) {
    return mk(fma_(M.m0, v.x, fma_(M.m1, v.y, M.m2 * v.z)),
              fma_(M.m1, v.x, fma_(M.m3, v.y, M.m4 * v.z)),
              fma_(M.m2, v.x, fma_(M.m4, v.y, M.m5 * v.z)));
}

// fp64: the Taylor series through x^17 / x^18 (remainder < 1e-19 at pi/4: double-accurate), with the
// oracle's fp64 build's coefficients and Horner order (oracle/cp_oracle.c sincos_small)
__constant__ const double kSin64[8] = {-0.16666666666666666, 0.008333333333333333, -0.0001984126984126984,
                                       2.7557319223985893e-06, -2.505210838544172e-08, 1.6059043836821613e-10,
                                       -7.647163731819816e-13, 2.8114572543455206e-15};
__constant__ const double kCos64[9] = {-0.5, 0.041666666666666664, -0.001388888888888889, 2.48015873015873e-05,
                                       -2.755731922398589e-07, 2.08767569878681e-09, -1.1470745597729725e-11,
                                       4.779477332387385e-14, -1.5619206968586225e-16};

// Taylor sin/cos for |x| <= pi/4 (constants rounded from double, as the oracle)
CP_DEV void sincos_small(real x, real& s, real& c) {
    if constexpr (sizeof(real) == 8) {
        const real x2 = x * x;
        real p = (real)kSin64[7];
#pragma unroll
        for (int k = 6; k >= 0; --k) p = fma_(x2, p, (real)kSin64[k]);
        s = fma_(x * x2, p, x);
        real q = (real)kCos64[8];
#pragma unroll
        for (int k = 7; k >= 0; --k) q = fma_(x2, q, (real)kCos64[k]);
        c = fma_(x2, q, real(1.0));
        return;
    }
    real x2 = x * x;
    real p = fma_(x2, (real)2.7557319223985893e-6, (real)-1.9841269841269841e-4);
    p = fma_(x2, p, (real)8.3333333333333333e-3);
    p = fma_(x2, p, (real)-1.6666666666666667e-1);
    s = fma_(x * x2, p, x);
    real q = fma_(x2, (real)2.4801587301587302e-5, (real)-1.3888888888888889e-3);
    q = fma_(x2, q, (real)4.1666666666666667e-2);
    q = fma_(x2, q, -real(0.5));
    c = fma_(x2, q, real(1.0));
}

// sin/cos(2*pi*u), u in [0,1): quadrant split + pi/4 rotation of a small angle
CP_DEV void sincos_turns(real u, real& so, real& co) {
    real y = u * real(4.0);
    int q = (int)y;
    q = q > 3 ? 3 : q;
    real f = y - (real)q;
    real x = (f - real(0.5)) * (real)1.5707963267948966;
    real s, c;
    sincos_small(x, s, c);
    real S = (s + c) * (real)0.7071067811865476;
    real C = (c - s) * (real)0.7071067811865476;
    so = (q == 0) ? S : (q == 1) ? C : (q == 2) ? -S : -C;
    co = (q == 0) ? C : (q == 1) ? -S : (q == 2) ? -C : S;
}

CP_DEV real atan_pos(real z) {
    real base = real(0.0);
    if (z > (real)2.414213562373095) {
        base = (real)1.5707963267948966;
        z = -real(1.0) / z;
    } else if (z > (real)0.4142135623730950) {
        base = (real)0.7853981633974483;
        z = (z - real(1.0)) / (z + real(1.0));
    }
    real z2 = z * z;
    if constexpr (sizeof(real) == 8) {
        // fp64: the odd Taylor series of atan through z^47 on |z| <= tan(pi/8) (remainder < 1e-18:
        // double-accurate); coefficient k is (-1)^k / (2k + 1), folded at compile time (IEEE division,
        // the oracle's fp64 build computes the same doubles)
        real p = (real)(-1.0 / 47.0);
#pragma unroll
        for (int k = 22; k >= 1; --k) p = fma_(z2, p, (real)((k & 1 ? -1.0 : 1.0) / (double)(2 * k + 1)));
        return base + fma_(z * z2, p, z);
    }
    real p = fma_(z2, (real)8.05374449538e-2, (real)-1.38776856032e-1);
    p = fma_(z2, p, (real)1.99777106478e-1);
    p = fma_(z2, p, (real)-3.33329491539e-1);
    return base + fma_(z * z2, p, z);
}
CP_DEV real atan2_own(real y, real x) {
    if (x == real(0.0) && y == real(0.0)) return real(0.0);
    real ax = abs_(x), ay = abs_(y);
    real r = (ay <= ax) ? atan_pos(ay / ax) : (real)1.5707963267948966 - atan_pos(ax / ay);
    if (x < real(0.0)) r = (real)3.141592653589793 - r;
    if (y < real(0.0)) r = -r;
    return r;
}
// roll, pitch, yaw as pybullet getEulerFromQuaternion
CP_DEV V3 quat_euler(real x, real y, real z, real w) {
    real sqw = w * w, sqx = x * x, sqy = y * y, sqz = z * z;
    real roll = atan2_own(real(2.0) * fma_(y, z, w * x), ((sqw - sqx) - sqy) + sqz);
    real sarg = -real(2.0) * fma_(x, z, -(w * y));
    real pitch;
    if (sarg <= -real(1.0)) pitch = (real)-1.5707963267948966;
    else if (sarg >= real(1.0)) pitch = (real)1.5707963267948966;
    else pitch = atan2_own(sarg, sqrt_(fma_(-sarg, sarg, real(1.0))));
    real yaw = atan2_own(real(2.0) * fma_(x, y, w * z), ((sqw + sqx) - sqy) - sqz);
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

}  // namespace CP_NS
