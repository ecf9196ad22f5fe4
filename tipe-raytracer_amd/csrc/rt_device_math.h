// rt_device_math.h — device primitives of the RT_RNG_PHILOX stream spec:
// the Philox4x32-10 stream and the portable transcendentals (DESIGN.md
// "Portable math").  Built only from IEEE-754 +,-,*,/,sqrt, explicit fma,
// rint and bit casts, compiled with -ffp-contract=off, so results are
// bit-identical to the CPU restatement in oracle/pm_math.h.
//
// Register pressure: the ~60 FP64 coefficients live in a __constant__ table
// read through the scalar unit (s_load) at the point of use; the table index
// is laundered through an empty asm so LICM cannot hoist the loads out of the
// bounce/sample loops and pin 120 SGPRs (that pressure spilled into VGPR
// lanes and capped occupancy at 2 waves/SIMD in the first kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rt {

typedef const double __attribute__((address_space(4)))* cdptr;

// Opaque wave-uniform zero: defeats loop-invariant hoisting of what uses it.
__device__ __forceinline__ int opq0()
{
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

enum : int {
    // sin/cos (fdlibm minimax kernels, degree 13 / 14 on |r| <= pi/4)
    KC_TWO_OVER_PI = 0, KC_PIO2_1, KC_PIO2_1T,
    KC_S1, KC_S2, KC_S3, KC_S4, KC_S5, KC_S6,
    KC_C1, KC_C2, KC_C3, KC_C4, KC_C5, KC_C6,
    // acos (fdlibm)
    KC_PIO2_HI, KC_PIO2_LO, KC_PI,
    KC_PS0, KC_PS1, KC_PS2, KC_PS3, KC_PS4, KC_PS5, KC_QS1, KC_QS2, KC_QS3, KC_QS4,
    // log / exp
    KC_SQRT2, KC_L1, KC_L2, KC_L3, KC_L4, KC_L5, KC_L6, KC_L7, KC_L8, KC_L9, KC_L10, KC_L11,
    KC_LN2_HI, KC_LN2_LO, KC_INV_LN2, KC_LN2,
    KC_E2, KC_E3, KC_E4, KC_E5, KC_E6, KC_E7, KC_E8, KC_E9, KC_E10, KC_E11, KC_E12, KC_E13,
    // tri_uvmapping's per-material overrides (texture.h:71-87) and tracer's
    // literals: read at the point of use so they are never hoisted into
    // VGPRs (the compiler spilled them to scratch in every wave's prologue)
    KC_ES1, KC_A4, KC_IOR4, KC_RS4, KC_A3, KC_IOR3, KC_RS3, KC_THIRD, KC_TWO_THIRDS,
    // atan2 (fdlibm, sky mapping)
    KC_ATHI0, KC_ATHI1, KC_ATHI2, KC_ATHI3, KC_ATLO0, KC_ATLO1, KC_ATLO2, KC_ATLO3,
    KC_AT0, KC_AT1, KC_AT2, KC_AT3, KC_AT4, KC_AT5, KC_AT6, KC_AT7, KC_AT8, KC_AT9, KC_AT10, KC_PI_LO53,
    // acos(t)/sqrt(1-t) on [0, 1], degree 13 (Chebyshev interpolant, relative
    // error 2^-42.1 in FMA Horner): the sampler's fast phi path
    KC_AC0, KC_AC1, KC_AC2, KC_AC3, KC_AC4, KC_AC5, KC_AC6, KC_AC7, KC_AC8, KC_AC9, KC_AC10, KC_AC11,
    KC_AC12, KC_AC13,
    KC_COUNT
};

__constant__ const double kC[KC_COUNT] = {
    0x1.45f306dc9c883p-1, 0x1.921fb54400000p+0, 0x1.0b4611a626331p-34,
    -0x1.5555555555549p-3, 0x1.111111110f8a6p-7, -0x1.a01a019c161d5p-13, 0x1.71de357b1fe7dp-19,
    -0x1.ae5e68a2b9cebp-26, 0x1.5d93a5acfd57cp-33,
    0x1.555555555554cp-5, -0x1.6c16c16c15177p-10, 0x1.a01a019cb1590p-16, -0x1.27e4f809c52adp-22,
    0x1.1ee9ebdb4b1c4p-29, -0x1.8fae9be8838d4p-37,
    0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54, 0x1.921fb54442d18p+1,
    0x1.5555555555555p-3, -0x1.4d61203eb6f7dp-2, 0x1.9c1550e884455p-3, -0x1.48228b5688f3bp-5,
    0x1.9efe07501b288p-11, 0x1.23de10dfdf709p-15, -0x1.33a271c8a2d4bp+1, 0x1.02ae59c598ac8p+1,
    -0x1.6066c1b8d0159p-1, 0x1.3b8c5b12e9282p-4,
    0x1.6a09e667f3bcdp+0, 0x1.5555555555555p-2, 0x1.999999999999ap-3, 0x1.2492492492492p-3,
    0x1.c71c71c71c71cp-4, 0x1.745d1745d1746p-4, 0x1.3b13b13b13b14p-4, 0x1.1111111111111p-4,
    0x1.e1e1e1e1e1e1ep-5, 0x1.af286bca1af28p-5, 0x1.8618618618618p-5, 0x1.642c8590b2164p-5,
    0x1.62e42fee00000p-1, 0x1.a39ef35793c76p-33, 0x1.71547652b82fep+0, 0x1.62e42fefa39efp-1,
    0x1.0000000000000p-1, 0x1.5555555555555p-3, 0x1.5555555555555p-5, 0x1.1111111111111p-7,
    0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-16, 0x1.71de3a556c734p-19,
    0x1.27e4fb7789f5cp-22, 0x1.ae64567f544e4p-26, 0x1.1eed8eff8d898p-29, 0x1.6124613a86d09p-33,
    1.85, 0.6, 1.33, 0.93, 0.1, 1.50, 0.3, 1.0 / 3.0, 2.0 / 3.0,
    4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01, 1.57079632679489655800e+00,
    2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17, 6.12323399573676603587e-17,
    3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01, -1.11111104054623557880e-01,
    9.09088713343650656196e-02, -7.69187620504482999495e-02, 6.66107313738753120669e-02, -5.83357013379057348645e-02,
    4.97687799461593236017e-02, -3.65315727442169155270e-02, 1.62858201153657823623e-02, 0x1.1a62633145c07p-53,
    0x1.921fb54442754p+0, -0x1.b7812aea8849fp-3, 0x1.6cbe3d540e1c7p-4, -0x1.a017c9f170088p-5,
    0x1.13e462e97bdc4p-5, -0x1.8eee6d835d3f8p-6, 0x1.2fa02342d2e11p-6, -0x1.d62d02a699df8p-7,
    0x1.5fc3eaba82359p-7, -0x1.d837e1419ed96p-8, 0x1.03cccf4b0779fp-8, -0x1.a5fa2f9ab0735p-10,
    0x1.b5b26a8fad8b5p-12, -0x1.ac25f83fc9b71p-15,
};

// Opaque per-call base of the constant table: each function takes one
// (b = kcb()) and reads its coefficients at immediate offsets from it, so
// neither the loads nor per-constant addresses are hoisted into long-lived
// SGPRs (at most the table address itself stays live).
__device__ __forceinline__ cdptr kcb()
{
    cdptr p = (cdptr)kC;
    asm volatile("" : "+s"(p));
    return p;
}
// Scalar load of constant i from a base b = kcb().
#define KCV(b, i) ((b)[(i)])

// ---- Philox4x32-10 (Random123 / rocrand_philox4x32_10 engine) -------------
struct Philox {
    uint32_t w0, w1, w2, w3;
};

// a ^ b ^ k in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96
// (three-input xor; k a wave-uniform SGPR)
__device__ __forceinline__ uint32_t xor3_s(uint32_t a, uint32_t b, uint32_t k)
{
#if defined(__gfx950__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
#else
    return a ^ b ^ k;                  // other targets: the compiler's own xor chain
#endif
}

template <bool UNIFORM_KEY = true>
__device__ __forceinline__ Philox philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1)
{
    if (UNIFORM_KEY) asm volatile("" : "+s"(k0), "+s"(k1));   // key schedule in place (SALU), not hoisted
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 yields both halves of each 32x32 product; the
        // round's two xors with the key are one v_bitop3_b32 each
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0, n2;
        if (UNIFORM_KEY) {
            n0 = xor3_s((uint32_t)(p1 >> 32), c1, k0);
            n2 = xor3_s((uint32_t)(p0 >> 32), c3, k1);
        } else {
            n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
            n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        }
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return Philox{c0, c1, c2, c3};
}

// Draw stream of one (pixel, sample): draw n = word (n & 3) of
// philox(ctr = {n >> 2, 0, pixel, sample}, key = seed) >> 1   (rt.h)
struct Stream {
    uint32_t k0, k1, pixel, sample, n;
    uint32_t* cache;         // current Philox block: 4 words in LDS (stride 256)

    __device__ __forceinline__ void start(uint32_t px, uint32_t s, uint32_t key0, uint32_t key1, uint32_t* lds)
    {
        k0 = key0; k1 = key1; pixel = px; sample = s; n = 0; cache = lds;
    }
    __device__ __forceinline__ uint32_t next31()
    {
        const uint32_t slot = n & 3u;
        uint32_t w;
        if (slot == 0u) {
            const Philox blk = philox4x32_10(n >> 2, 0u, pixel, sample, k0, k1);
            cache[256] = blk.w1;
            cache[512] = blk.w2;
            cache[768] = blk.w3;
            w = blk.w0;
        } else {
            w = cache[slot * 256];
        }
        ++n;
        return w >> 1;
    }
    // next31 for a draw whose block the caller already put in the cache (slot 0
    // included)
    __device__ __forceinline__ uint32_t next31_cached()
    {
        const uint32_t w = cache[(n & 3u) * 256];
        ++n;
        return w >> 1;
    }
};

// rand()/(RAND_MAX + 1.0), rtutility.h:192
__device__ __forceinline__ double unit31(uint32_t r) { return (double)r / 2147483648.0; }

// ---- sin / cos of a float, evaluated in double, rounded to float ----------
__device__ __forceinline__ int pm_sincos(float x, double& s, double& c)
{
    const cdptr b = kcb();
    const double xd = (double)x;
    const double kd = rint(xd * KCV(b, KC_TWO_OVER_PI));
    const double r = fma(-kd, KCV(b, KC_PIO2_1T), fma(-kd, KCV(b, KC_PIO2_1), xd));
    const double z = r * r;
    // |z| == z (z >= +0): the abs modifier keeps each Horner step one VOP3
    // v_fma_f64 with the SGPR coefficient as addend; without it the compiler
    // picks v_fmac (tied VGPR addend) plus two v_mov of the coefficient.
    const double za = fabs(z);
    const double ps = fma(za, fma(za, fma(za, fma(za, fma(za, KCV(b, KC_S6), KCV(b, KC_S5)), KCV(b, KC_S4)),
                                          KCV(b, KC_S3)), KCV(b, KC_S2)), KCV(b, KC_S1));
    const double pc = fma(za, fma(za, fma(za, fma(za, fma(za, KCV(b, KC_C6), KCV(b, KC_C5)), KCV(b, KC_C4)),
                                          KCV(b, KC_C3)), KCV(b, KC_C2)), KCV(b, KC_C1));
    s = fma(r * z, ps, r);
    c = fma(z * z, pc, fma(-0.5, z, 1.0));
    // kd is an integer-valued double of small magnitude (|x| <= 2^27 here:
    // the sampler's x <= 2 pi), so the 32-bit conversion is exact
    return (int)kd & 3;
}

// Quadrant q of the reduced argument: sin x = (s, c, -s, -c)[q], cos x =
// (c, -s, -c, s)[q].  Rounding to float commutes with negation (round to
// nearest is symmetric), so the pair is rounded first and the quadrant is
// applied to the floats: one swap and two sign flips.
__device__ __forceinline__ void pm_sincosf(float x, float& sn, float& cs)
{
    double s, c;
    const int q = pm_sincos(x, s, c);
    const float fs = (float)s, fc = (float)c;
    const bool odd = (q & 1) != 0;
    const float a = odd ? fc : fs, b = odd ? fs : fc;
    const unsigned ns = (unsigned)(q & 2) << 30, nc = (unsigned)((q + 1) & 2) << 30;
    sn = __uint_as_float(__float_as_uint(a) ^ ns);
    cs = __uint_as_float(__float_as_uint(b) ^ nc);
}

// Exact f64 sqrt and division without their range fixups.  These are the
// compiler's own gfx950 lowerings of the IEEE operations -- sqrt: v_rsq +
// Goldschmidt/Newton (10 ops); x/d: v_div_scale, v_rcp, two Newton steps on
// the reciprocal, mul, fma, v_div_fmas, v_div_fixup -- with the scaling and
// special-value steps dropped.  Those steps are identities under the guards
// each call site checks (no zero/inf/NaN/denormal operand or intermediate,
// operand exponents well inside the range), so the results are bit-identical
// to `sqrt` and `/`; lanes outside the guards take the generic operations.
// The refined reciprocal depends only on the divisor, so one rcp_refined
// serves every quotient by the same d.  rt_selftest_math op 8 and the parity
// suite check them.
__device__ __forceinline__ double sqrt_core(double x)          // x in [2^-760, 2^760]
{
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    g = fma(fma(-g, g, x), h, g);
    return fma(fma(-g, g, x), h, g);
}
// sqrt_core(x) and a refined reciprocal of that root for div_core, without
// v_rcp_f64: the sqrt sequence's own h ~ 1/(2 sqrt x) (relative error
// ~1.5 e0^2 <= 2^-45 after its Goldschmidt step, e0 <= 2^-23.5 the error of
// v_rsq_f64) doubled is within 2^-45 of 1/L (L = the rounded root, itself
// within 2^-53 of sqrt x), and one Newton step on it, as rcp_refined's
// second step, leaves rc within 2^-89 + half an ulp of 1/L.  Same
// precondition for div_core as rcp_refined's result; rt_verify_normalize
// compares normalize() with IEEE a / sqrt(a.a) on 2^33 random vectors.
__device__ __forceinline__ void sqrt_rcp_core(double x, double& L, double& rc)   // x in [2^-760, 2^760]
{
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    g = fma(fma(-g, g, x), h, g);
    L = fma(fma(-g, g, x), h, g);
    const double r0 = h + h;
    rc = fma(r0, fma(-L, r0, 1.0), r0);
}
// sqrt_rcp_core for x within 2^-18 of 1 (the sampler's float-built unit
// vectors), without v_rsq_f64: e = x - 1 is exact (Sterbenz) and the series
// y = 1 - e/2 + 3e^2/8 is 1/sqrt(x) within 5|e|^3/16 (<= 2^-55.7) plus its
// rounding; then sqrt_core's shape: g = x y, h = y/2, and one Newton step
// L = g + (x - g^2) h.  L == sqrt(x) for EVERY double in [1 - 2^-18, 1 + 2^-18]
// (5.2e10 values, tools/check_near1.sh; tests/test_near1_sqrt.py checks a
// sample and the neighbourhood of 1).  rc: one Newton step on y (within
// 2^-51 of 1/L) leaves it within 2^-100 + half an ulp of 1/L, div_core's
// precondition.
__device__ __forceinline__ void sqrt_rcp_near1(double x, double& L, double& rc)   // |x - 1| <= 2^-18
{
    const double e = x - 1.0;
    const double y = fma(fma(e, 0.375, -0.5), e, 1.0);
    const double g = x * y, h = 0.5 * y;
    L = fma(fma(-g, g, x), h, g);
    rc = fma(y, fma(-L, y, 1.0), y);
}
// div_core that also keeps the sign of a zero x (x = -0: -0, as IEEE x / d
// for d > 0): the residual is formed as d q - x and subtracted, which gives
// the same rounded value as div_core for every x != 0.
__device__ __forceinline__ double div_core0(double x, double d, double rc)  // x = +-0 or |x| in [2^-900, 2^900]
{
    const double q = x * rc;
    return fma(-fma(d, q, -x), rc, q);
}
__device__ __forceinline__ double rcp_refined(double d)         // d in [2^-400, 2^400]
{
    double rc = __builtin_amdgcn_rcp(d);
    rc = fma(rc, fma(-d, rc, 1.0), rc);
    return fma(rc, fma(-d, rc, 1.0), rc);
}
__device__ __forceinline__ double div_core(double x, double d, double rc)   // |x| in [2^-900, 2^900]
{
    const double q = x * rc;
    return fma(fma(-d, q, x), rc, q);
}

// ---- acos (fdlibm scheme) --------------------------------------------------
__device__ __forceinline__ double pm_acos_R(cdptr b, double z)
{
    const double za = fabs(z);                    // z >= +0 (see pm_sincos)
    const double p = z * fma(za, fma(za, fma(za, fma(za, fma(za, KCV(b, KC_PS5), KCV(b, KC_PS4)), KCV(b, KC_PS3)),
                                            KCV(b, KC_PS2)), KCV(b, KC_PS1)), KCV(b, KC_PS0));
    const double q = fma(za, fma(za, fma(za, fma(za, KCV(b, KC_QS4), KCV(b, KC_QS3)), KCV(b, KC_QS2)), KCV(b, KC_QS1)), 1.0);
    return div_core(p, q, rcp_refined(q));   // q in [0.7, 1.1], p = +0 or >= 2^-70: exact
}

__device__ __forceinline__ double pm_acos(double x)
{
    // fdlibm's three cases evaluated branch-free: every lane performs exactly
    // the operations of its own case (same values as the branchy form in
    // oracle/pm_math.h), but the wave runs one rational R(z), one sqrt and
    // one extra division instead of three divergent copies of them.
    const cdptr b = kcb();
    const double PIO2_HI = KCV(b, KC_PIO2_HI), PIO2_LO = KCV(b, KC_PIO2_LO), PI = KCV(b, KC_PI);
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const uint32_t hx = (uint32_t)(u >> 32);
    const uint32_t ix = hx & 0x7fffffffu;
    const bool small = ix < 0x3fe00000u;          // |x| < 0.5
    const bool neg = (hx >> 31) != 0;
    const double z = small ? x * x : (neg ? (1.0 + x) * 0.5 : (1.0 - x) * 0.5);
    const double r = pm_acos_R(b, z);
    // The exact unscaled sqrt/division cores apply to every lane whose case
    // uses them: there z = (1 -+ x)/2 is in [2^-31, 0.25] (|x| < 1 on the
    // 2^-31 grid; x = -1 takes the override below), so s + df is in
    // [2^-15, 1] and the numerator is +0 or >= 2^-84 in magnitude.  Lanes of
    // the |x| < 0.5 case may feed them z = 0 (NaN, unused).
    const double s = sqrt_core(z);
    // x >= 0.5
    const double df = __longlong_as_double((long long)((unsigned long long)__double_as_longlong(s) & 0xffffffff00000000ull));
    const double sdf = s + df;
    const double c = div_core(fma(-df, df, z), sdf, rcp_refined(sdf));
    const double res_pos = 2.0 * (df + fma(r, s, c));
    // x <= -0.5
    const double res_neg = PI - 2.0 * (s + fma(r, s, -PIO2_LO));
    // |x| < 0.5
    const double res_small = (ix <= 0x3c600000u) ? PIO2_HI + PIO2_LO : PIO2_HI - (x - fma(-x, r, PIO2_LO));
    double res = small ? res_small : (neg ? res_neg : res_pos);
    if (ix >= 0x3ff00000u) {                       // |x| >= 1 or NaN (x == -1 only, in the sampler)
        if (((ix - 0x3ff00000u) | (uint32_t)u) == 0u) res = neg ? PI + 2.0 * PIO2_LO : 0.0;
        else res = (x - x) / (x - x);
    }
    return res;
}

// ---- sinf/cosf of (float)acos(x): the sampler's phi (rtutility.h:196-200) ---
// Fast path of pm_sincosf((float)pm_acos(x), sp, cp) for x = 2v - 1 on the
// 2^-30 grid.  Only the float phi reaches the image, and cos(phi) = x,
// sin(phi) = sqrt(1 - x^2) are known, so:
//   A  = sqrt(1 - |x|) * P(|x|)  (pi - that for x < 0)   |A - acos x| <= e1
//   f  = (float)A, certain when A -+ e1 round to the same float (then
//        pm_acos(x), within 1 ulp of acos x, rounds to f as well)
//   dl = f - A (exact); with the true offset f - phi = dl + (A - phi),
//   cos f = x cos dl - s sin dl,  sin f = s cos dl + x sin dl  (s = sin phi),
//   evaluated to second order (|dl| <= 2^-22.3, the cubic terms < 2^-66),
//   each certain when its value -+ its error bound rounds to one float.
// Error bounds: P 2^-42.1 and sqrt 2^-45 relative, so
// e1 = a0*2^-40 + 2^-49 (a0 = acos|x|; 2^-49 covers pi's rounding and the
// subtraction); cos: e1 + 2^-48; sin: e1 + s*2^-44 + 2^-48.  Returns false
// when any of the three roundings is not certain (about 1e-4 of the inputs;
// x = -1 gives NaN and false), and the caller runs the full path.  All 2^31
// inputs are checked against the full path on the GPU (rt_verify_sampler_phi).
__device__ __forceinline__ bool phi_sincosf_fast(double x, float& sp, float& cp)
{
    const cdptr b = kcb();
    const double ax = fabs(x);
    const double w = 1.0 - ax;                                 // exact on the grid
    const double r0 = __builtin_amdgcn_rsq(w);
    const double t0 = w * r0;
    const double sw = fma(t0 * 0.5, fma(-t0, r0, 1.0), t0);    // sqrt(w), 2^-45
    double p = KCV(b, KC_AC13);
#pragma unroll
    for (int j = 12; j >= 0; --j) p = fma(p, ax, KCV(b, KC_AC0 + j));
    const double a0 = sw * p;                                  // acos(|x|)
    const double A = x < 0.0 ? KCV(b, KC_PI) - a0 : a0;
    const double e1 = fma(a0, 0x1p-40, 0x1p-49);
    const float f = (float)(A - e1);
    const bool ok1 = __float_as_uint(f) == __float_as_uint((float)(A + e1));
    const double dl = (double)f - A;
    const double q = fma(-x, x, 1.0);                          // 1 - x^2
    const double r1 = __builtin_amdgcn_rsq(q);
    const double t1 = q * r1;
    const double s = fma(t1 * 0.5, fma(-t1, r1, 1.0), t1);     // sin(acos x), 2^-45
    const double d2 = dl * dl;
    const double C = fma(-s, dl, fma(-0.5 * x, d2, x));
    const double S = fma(x, dl, fma(-0.5 * s, d2, s));
    const double e2 = e1 + 0x1p-48;
    const double e3 = fma(s, 0x1p-44, e2);
    cp = (float)(C - e2);
    sp = (float)(S - e3);
    const bool ok2 = __float_as_uint(cp) == __float_as_uint((float)(C + e2));
    const bool ok3 = __float_as_uint(sp) == __float_as_uint((float)(S + e3));
    return ok1 && ok2 && ok3;
}

// ---- atan2 (oracle/pm_math.h pm_atan2; sky mapping only) -------------------
__device__ __forceinline__ double pm_atan_pos(cdptr b, double a)
{
    int id;
    double x = a;
    if (a >= 0x1p66) return KCV(b, KC_ATHI3) + KCV(b, KC_ATLO3);
    if (a < 0.4375) {
        if (a < 0x1p-29) return a;
        id = -1;
    } else if (a < 1.1875) {
        if (a < 0.6875) { id = 0; x = (2.0 * a - 1.0) / (2.0 + a); }
        else            { id = 1; x = (a - 1.0) / (a + 1.0); }
    } else if (a < 2.4375) { id = 2; x = (a - 1.5) / (1.0 + 1.5 * a); }
    else                   { id = 3; x = -1.0 / a; }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (KCV(b, KC_AT0) + w * (KCV(b, KC_AT2) + w * (KCV(b, KC_AT4) + w * (KCV(b, KC_AT6) +
                      w * (KCV(b, KC_AT8) + w * KCV(b, KC_AT10))))));
    const double s2 = w * (KCV(b, KC_AT1) + w * (KCV(b, KC_AT3) + w * (KCV(b, KC_AT5) + w * (KCV(b, KC_AT7) +
                      w * KCV(b, KC_AT9)))));
    if (id < 0) return x - x * (s1 + s2);
    return KCV(b, KC_ATHI0 + id) - ((x * (s1 + s2) - KCV(b, KC_ATLO0 + id)) - x);
}

__device__ __forceinline__ double pm_atan2(double y, double x)
{
    const cdptr b = kcb();
    const double pi = KCV(b, KC_PI), pi_lo = KCV(b, KC_PI_LO53), pio2 = KCV(b, KC_PIO2_HI);
    const double inf = __longlong_as_double(0x7ff0000000000000ll);
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (__signbit(x)) return __signbit(y) ? -pi : pi;
        return y;
    }
    if (x == 0.0) return y > 0 ? pio2 : -pio2;
    if (fabs(x) == inf) {
        const double q = fabs(y) == inf ? 0.5 * pio2 : 0.0;
        const double r = x > 0 ? q : pi - q;
        return y > 0 ? r : -r;
    }
    if (fabs(y) == inf) return y > 0 ? pio2 : -pio2;
    const double a = fabs(y / x);
    const double z = (fabs(y) > 0x1p60 * fabs(x)) ? pio2
                   : ((x < 0 && fabs(y) * 0x1p60 < fabs(x)) ? 0.0 : pm_atan_pos(b, a));
    if (x > 0) return y > 0 ? z : -z;
    return y > 0 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
}

// ---- pow ---------------------------------------------------------------------
__device__ __forceinline__ double pm_from_bits(unsigned long long b) { return __longlong_as_double((long long)b); }

// The log/exp kernels run once per AO cast (ambient_occlusion's pow,
// main.c:111).  Their coefficients are read one scalar load each from its own
// opaque base (KCV1): a Horner chain reading 11-12 of them from one base got
// its loads merged into s_load_dwordx16, whose 16 SGPRs the AO kernels then
// spilled to VGPR lanes and read back one by one (32 v_writelane/v_readlane
// per pow in the C4 kernel).
#define KCV1(i) (kcb()[(i)])

// pm_log for every x the pow path feeds it (special x give finite values that
// pm_pow discards): m in (0.70, 1.42], so 2 + f is in [1.7, 2.5] and f = m - 1
// is 0 or of magnitude >= 2^-53; the quotient is div_core0's exact IEEE one.
__device__ __forceinline__ double pm_log(cdptr b, double x)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = pm_from_bits((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > KCV(b, KC_SQRT2)) { m = m * 0.5; e = e + 1; }
    const double f = m - 1.0;
    const double d = 2.0 + f;
    const double s = div_core0(f, d, rcp_refined(d));
    const double z = s * s;
    const double t = KCV1(KC_L1) + z * (KCV1(KC_L2) + z * (KCV1(KC_L3) + z * (KCV1(KC_L4) +
                     z * (KCV1(KC_L5) + z * (KCV1(KC_L6) + z * (KCV1(KC_L7) + z * (KCV1(KC_L8) +
                     z * (KCV1(KC_L9) + z * (KCV1(KC_L10) + z * KCV1(KC_L11))))))))));
    const double lm = 2.0 * s + (2.0 * s) * (z * t);
    const double ed = (double)e;
    return ed * KCV1(KC_LN2_HI) + (lm + ed * KCV1(KC_LN2_LO));
}

// pm_exp without branches: the kernel runs on t clamped to [-708, 709] (the
// same t wherever it is used) and the out-of-range and NaN results are
// selected afterwards, as pm_math.h's early returns give them.
__device__ __forceinline__ double pm_exp(cdptr b, double t)
{
    const double tc = fmin(fmax(t, -708.0), 709.0);
    const double kd = rint(tc * KCV1(KC_INV_LN2));
    const double r = (tc - kd * KCV1(KC_LN2_HI)) - kd * KCV1(KC_LN2_LO);
    const double p = 1.0 + r * (1.0 + r * (KCV1(KC_E2) + r * (KCV1(KC_E3) + r * (KCV1(KC_E4) +
                     r * (KCV1(KC_E5) + r * (KCV1(KC_E6) + r * (KCV1(KC_E7) + r * (KCV1(KC_E8) +
                     r * (KCV1(KC_E9) + r * (KCV1(KC_E10) + r * (KCV1(KC_E11) + r * (KCV1(KC_E12) +
                     r * KCV1(KC_E13)))))))))))));
    const int k = (int)kd;
    const int k1 = k / 2, k2 = k - k1;
    const double s1 = pm_from_bits((unsigned long long)(k1 + 1023) << 52);
    const double s2 = pm_from_bits((unsigned long long)(k2 + 1023) << 52);
    double res = (p * s1) * s2;
    res = t > 709.0 ? __longlong_as_double(0x7ff0000000000000ll) : res;
    res = t < -708.0 ? 0.0 : res;
    return t != t ? t + t : res;               // NaN t: pm_math.h's arithmetic propagates it
}

// pm_pow (oracle/pm_math.h): a wave-uniform y (the AO intensity) keeps the
// first two cases uniform branches; the per-lane cases of x are selects over
// one log/exp evaluation (the subnormal scaling folded into its argument), so
// the AO kernels run one straight-line copy instead of five nested divergent
// branches around two inlined copies of log.
__device__ __forceinline__ double pm_pow(double x, double y)
{
    if (y == 0.0) return 1.0;
    if (y == (double)(int)y && y <= 64.0 && y >= -64.0) {
        const int n = (int)y;
        unsigned un = (unsigned)(n < 0 ? -n : n);
        double res = 1.0, base = x;
        while (un) {
            if (un & 1u) res = res * base;
            base = base * base;
            un >>= 1;
        }
        return n < 0 ? 1.0 / res : res;
    }
    const cdptr b = kcb();
    const double inf = __longlong_as_double(0x7ff0000000000000ll);
    const bool sub = x < 0x1p-1022;
    const double l = pm_log(b, sub ? x * 0x1p54 : x);
    double res = pm_exp(b, y * (sub ? l - 54.0 * KCV1(KC_LN2) : l));
    res = x == inf ? (y > 0.0 ? inf : 0.0) : res;
    res = x < 0.0 ? (x - x) / (x - x) : res;
    res = x == 0.0 ? (y > 0.0 ? 0.0 : inf) : res;
    return (x != x || y != y) ? x + y : res;
}

}  // namespace rt
