/*
 * oracle/pm_math.h — TEST INFRASTRUCTURE (CPU oracle only; never shipped).
 *
 * "Portable math": the transcendental functions of the RT_RNG_PHILOX stream
 * spec, written with IEEE-754 double +,-,*,/,sqrt, fma (one rounding: C99
 * fma() here, v_fma_f64 on the device) and exact conversions only (no libm
 * transcendentals), so that the oracle and the HIP kernel — two independent
 * restatements of DESIGN.md §"Portable math" — agree bit for bit.
 *
 * They stand in for the libm calls the reference makes on the sampling path:
 *   acos   rtutility.h:196   phi = acos(2v - 1)            (double)
 *   cosf   rtutility.h:198-200  cosf(theta), cosf(phi)      (float)
 *   sinf   rtutility.h:198-199  sinf(theta), sinf(phi)      (float)
 *   pow    main.c:109        pow(distance/dst, AO_intensity)
 * In RT_RNG_GLIBC mode the oracle calls libm itself (bit-exact to the
 * reference); tests measure how close these are to libm.
 */
#ifndef PM_MATH_H
#define PM_MATH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

static inline uint64_t pm_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double pm_from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* ---- sin/cos of a float argument, evaluated in double, rounded to float -- */
/* Cody-Waite reduction by pi/2 (33-bit head, exact with FMA, plus tail) and
 * the fdlibm minimax kernels (__kernel_sin degree 13, __kernel_cos degree 14)
 * in FMA Horner form on |r| <= pi/4.  The float results are the correctly
 * rounded sin/cos for every float in [0, 2*pi] (exhaustively checked against
 * sinl/cosl, DESIGN.md "Portable math"); the domain used is [0, 2*pi]. */
static const double PM_TWO_OVER_PI = 0x1.45f306dc9c883p-1;
static const double PM_PIO2_1 = 0x1.921fb54400000p+0;
static const double PM_PIO2_1T = 0x1.0b4611a626331p-34;
static const double PM_S1 = -0x1.5555555555549p-3, PM_S2 = 0x1.111111110f8a6p-7,
                    PM_S3 = -0x1.a01a019c161d5p-13, PM_S4 = 0x1.71de357b1fe7dp-19,
                    PM_S5 = -0x1.ae5e68a2b9cebp-26, PM_S6 = 0x1.5d93a5acfd57cp-33;
static const double PM_C1 = 0x1.555555555554cp-5, PM_C2 = -0x1.6c16c16c15177p-10,
                    PM_C3 = 0x1.a01a019cb1590p-16, PM_C4 = -0x1.27e4f809c52adp-22,
                    PM_C5 = 0x1.1ee9ebdb4b1c4p-29, PM_C6 = -0x1.8fae9be8838d4p-37;

/* returns quadrant q in [0,3]; *s = sin(r), *c = cos(r) */
static inline int pm_reduce_sincos(float x, double* s, double* c)
{
    double xd = (double)x;
    double kd = nearbyint(xd * PM_TWO_OVER_PI);          /* round half even */
    double r = fma(-kd, PM_PIO2_1T, fma(-kd, PM_PIO2_1, xd));
    double z = r * r;
    double ps = fma(z, fma(z, fma(z, fma(z, fma(z, PM_S6, PM_S5), PM_S4), PM_S3), PM_S2), PM_S1);
    double pc = fma(z, fma(z, fma(z, fma(z, fma(z, PM_C6, PM_C5), PM_C4), PM_C3), PM_C2), PM_C1);
    *s = fma(r * z, ps, r);
    *c = fma(z * z, pc, fma(-0.5, z, 1.0));
    return (int)((int64_t)kd & 3);
}

static inline float pm_sinf(float x)
{
    double s, c;
    int q = pm_reduce_sincos(x, &s, &c);
    double v = (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
    return (float)v;
}

static inline float pm_cosf(float x)
{
    double s, c;
    int q = pm_reduce_sincos(x, &s, &c);
    double v = (q == 0) ? c : (q == 1) ? -s : (q == 2) ? -c : s;
    return (float)v;
}

/* ---- acos: the classic fdlibm rational scheme (< 1 ulp), FMA Horner ------ */
static const double PM_PIO2_HI = 0x1.921fb54442d18p+0, PM_PIO2_LO = 0x1.1a62633145c07p-54,
                    PM_PI = 0x1.921fb54442d18p+1;
static const double PM_PS0 = 0x1.5555555555555p-3, PM_PS1 = -0x1.4d61203eb6f7dp-2,
                    PM_PS2 = 0x1.9c1550e884455p-3, PM_PS3 = -0x1.48228b5688f3bp-5,
                    PM_PS4 = 0x1.9efe07501b288p-11, PM_PS5 = 0x1.23de10dfdf709p-15;
static const double PM_QS1 = -0x1.33a271c8a2d4bp+1, PM_QS2 = 0x1.02ae59c598ac8p+1,
                    PM_QS3 = -0x1.6066c1b8d0159p-1, PM_QS4 = 0x1.3b8c5b12e9282p-4;

static inline double pm_acos_R(double z)
{
    double p = z * fma(z, fma(z, fma(z, fma(z, fma(z, PM_PS5, PM_PS4), PM_PS3), PM_PS2), PM_PS1), PM_PS0);
    double q = fma(z, fma(z, fma(z, fma(z, PM_QS4, PM_QS3), PM_QS2), PM_QS1), 1.0);
    return p / q;
}

static inline double pm_acos(double x)
{
    uint64_t u = pm_bits(x);
    uint32_t hx = (uint32_t)(u >> 32);
    uint32_t ix = hx & 0x7fffffffu;
    if (ix >= 0x3ff00000u) {                       /* |x| >= 1 or NaN */
        if (((ix - 0x3ff00000u) | (uint32_t)u) == 0u)
            return (hx >> 31) ? PM_PI + 2.0 * PM_PIO2_LO : 0.0;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000u) {                        /* |x| < 0.5 */
        if (ix <= 0x3c600000u) return PM_PIO2_HI + PM_PIO2_LO;
        double r = pm_acos_R(x * x);
        return PM_PIO2_HI - (x - fma(-x, r, PM_PIO2_LO));
    }
    if (hx >> 31) {                                /* x <= -0.5 */
        double z = (1.0 + x) * 0.5;
        double r = pm_acos_R(z);
        double s = sqrt(z);
        double w = fma(r, s, -PM_PIO2_LO);
        return PM_PI - 2.0 * (s + w);
    }
    {                                              /* x >= 0.5 */
        double z = (1.0 - x) * 0.5;
        double s = sqrt(z);
        double df = pm_from_bits(pm_bits(s) & 0xffffffff00000000ull);
        double c = fma(-df, df, z) / (s + df);
        double r = pm_acos_R(z);
        double w = fma(r, s, c);
        return 2.0 * (df + w);
    }
}

/* ---- pow --------------------------------------------------------------- */
/* Integer exponents |y| <= 64: square-and-multiply (pow(x,2) == x*x, the
 * correctly rounded value libm returns).  Otherwise exp(y*log(x)) with an
 * atanh-series log and a Taylor exp; deterministic, ~1e-15 relative. */
static const double PM_LN2_HI = 0x1.62e42fee00000p-1, PM_LN2_LO = 0x1.a39ef35793c76p-33;
static const double PM_INV_LN2 = 0x1.71547652b82fep+0;
static const double PM_SQRT2 = 0x1.6a09e667f3bcdp+0;

static inline double pm_log(double x)   /* x > 0, finite, normal */
{
    uint64_t u = pm_bits(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = pm_from_bits((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);  /* [1,2) */
    if (m > PM_SQRT2) { m = m * 0.5; e = e + 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double t = 0x1.5555555555555p-2 + z * (0x1.999999999999ap-3 + z * (0x1.2492492492492p-3 +
               z * (0x1.c71c71c71c71cp-4 + z * (0x1.745d1745d1746p-4 + z * (0x1.3b13b13b13b14p-4 +
               z * (0x1.1111111111111p-4 + z * (0x1.e1e1e1e1e1e1ep-5 + z * (0x1.af286bca1af28p-5 +
               z * (0x1.8618618618618p-5 + z * 0x1.642c8590b2164p-5)))))))));
    double lm = 2.0 * s + (2.0 * s) * (z * t);
    double ed = (double)e;
    return ed * PM_LN2_HI + (lm + ed * PM_LN2_LO);
}

static inline double pm_exp(double t)
{
    if (t > 709.0) return INFINITY;
    if (t < -708.0) return 0.0;
    double kd = nearbyint(t * PM_INV_LN2);
    double r = (t - kd * PM_LN2_HI) - kd * PM_LN2_LO;
    double p = 1.0 + r * (1.0 + r * (0x1.0000000000000p-1 + r * (0x1.5555555555555p-3 +
               r * (0x1.5555555555555p-5 + r * (0x1.1111111111111p-7 + r * (0x1.6c16c16c16c17p-10 +
               r * (0x1.a01a01a01a01ap-13 + r * (0x1.a01a01a01a01ap-16 + r * (0x1.71de3a556c734p-19 +
               r * (0x1.27e4fb7789f5cp-22 + r * (0x1.ae64567f544e4p-26 + r * (0x1.1eed8eff8d898p-29 +
               r * 0x1.6124613a86d09p-33))))))))))));
    int k = (int)kd;
    /* scale by 2^k in two steps so 2^k stays a normal number */
    int k1 = k / 2, k2 = k - k1;
    double s1 = pm_from_bits((uint64_t)(k1 + 1023) << 52);
    double s2 = pm_from_bits((uint64_t)(k2 + 1023) << 52);
    return (p * s1) * s2;
}

static inline double pm_pow(double x, double y)
{
    if (y == 0.0) return 1.0;
    if (y == (double)(int)y && y <= 64.0 && y >= -64.0) {
        int n = (int)y;
        unsigned un = (unsigned)(n < 0 ? -n : n);
        double res = 1.0, base = x;
        while (un) {
            if (un & 1u) res = res * base;
            base = base * base;
            un >>= 1;
        }
        return n < 0 ? 1.0 / res : res;
    }
    if (x != x || y != y) return x + y;
    if (x == 0.0) return y > 0.0 ? 0.0 : INFINITY;
    if (x < 0.0) return (x - x) / (x - x);   /* non-integer power of a negative */
    if (x == INFINITY) return y > 0.0 ? INFINITY : 0.0;
    if (x < 0x1p-1022) return pm_exp(y * (pm_log(x * 0x1p54) - 54.0 * 0x1.62e42fefa39efp-1));
    return pm_exp(y * pm_log(x));
}

/* ---- Philox4x32-10 (Random123; the rocrand/hiprand philox engine) ------- */
static inline void pm_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int round = 0; round < 10; ++round) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* ---- atan2 (fdlibm scheme: s_atan.c reduction to 4 anchors + odd series,
 * e_atan2.c quadrant logic), FMA-free as written here.  Used by the sky
 * mapping (sphere_uvmapping, texture.h:92-112).  < 1 ulp; checked against
 * libm in tests/test_oracle.py. */
static const double PM_ATANHI[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                    9.82793723247329054082e-01, 1.57079632679489655800e+00};
static const double PM_ATANLO[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                    1.39033110312309984516e-17, 6.12323399573676603587e-17};
static const double PM_AT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                                 1.42857142725034663711e-01, -1.11111104054623557880e-01,
                                 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                 6.66107313738753120669e-02, -5.83357013379057348645e-02,
                                 4.97687799461593236017e-02, -3.65315727442169155270e-02,
                                 1.62858201153657823623e-02};

/* atan(a) for a >= 0, finite */
static inline double pm_atan_pos(double a)
{
    int id;
    double x = a;
    if (a >= 0x1p66) return PM_ATANHI[3] + PM_ATANLO[3];
    if (a < 0.4375) {
        if (a < 0x1p-29) return a;
        id = -1;
    } else if (a < 1.1875) {
        if (a < 0.6875) { id = 0; x = (2.0 * a - 1.0) / (2.0 + a); }
        else            { id = 1; x = (a - 1.0) / (a + 1.0); }
    } else if (a < 2.4375) { id = 2; x = (a - 1.5) / (1.0 + 1.5 * a); }
    else                   { id = 3; x = -1.0 / a; }
    double z = x * x;
    double w = z * z;
    double s1 = z * (PM_AT[0] + w * (PM_AT[2] + w * (PM_AT[4] + w * (PM_AT[6] + w * (PM_AT[8] + w * PM_AT[10])))));
    double s2 = w * (PM_AT[1] + w * (PM_AT[3] + w * (PM_AT[5] + w * (PM_AT[7] + w * PM_AT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    return PM_ATANHI[id] - ((x * (s1 + s2) - PM_ATANLO[id]) - x);
}

static inline double pm_atan2(double y, double x)
{
    const double pi = 0x1.921fb54442d18p+1, pi_lo = 0x1.1a62633145c07p-53, pio2 = 0x1.921fb54442d18p+0;
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (signbit(x)) return signbit(y) ? -pi : pi;      /* atan2(+-0, x<=-0) */
        return y;                                           /* atan2(+-0, x>=+0) */
    }
    if (x == 0.0) return y > 0 ? pio2 : -pio2;
    if (isinf(x)) {                                         /* C99 F.10.1.4 */
        const double q = isinf(y) ? 0.5 * pio2 : 0.0;
        const double r = x > 0 ? q : pi - q;
        return y > 0 ? r : -r;
    }
    if (isinf(y)) return y > 0 ? pio2 : -pio2;
    const double a = fabs(y / x);
    double z = (fabs(y) > 0x1p60 * fabs(x)) ? pio2 : ((x < 0 && fabs(y) * 0x1p60 < fabs(x)) ? 0.0 : pm_atan_pos(a));
    if (x > 0) return y > 0 ? z : -z;
    return y > 0 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
}

#endif /* PM_MATH_H */
