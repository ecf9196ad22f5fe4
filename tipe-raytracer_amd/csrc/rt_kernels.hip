// rt_kernels.hip — the per-pixel path-tracing kernel for gfx950 (CDNA4).
//
// One thread renders one pixel (or one chunk of its samples): the sample
// loop, the nbRebondMax bounce loop, closest-hit scans, shading and AO all
// run in registers; HBM traffic is the final colors per pixel (plus, with
// sample chunking, one 72-byte partial sum per pixel and chunk).
//
// Semantics follow main.c (the authoritative CPU path), not main_cuda.cu:
//   fill_canva        main.c:245-284      -> render_kernel_q (task queue) /
//                                            render_kernel (fixed grid), combine_kernel
//   tracer            main.c:118-242      -> QPath (queue kernel), LanePath
//                                            (fixed grid)
//   closest_hit       main.c:52-92        -> closest_hit()
//   ambient_occlusion main.c:94-116       -> ao_factor()
//   hit_sphere        sphere.h:13-47      -> sphere_exact() (+ candidate pass)
//   hit_triangle      mesh.h:70-94, tri_uvmapping texture.h:44-90,
//   get_ray           camera.h:42-55, random_dir_no_norm / refracted_vec /
//   hsl               rtutility.h:81-231, write_color_canva rtutility.h:56-71
// Every floating-point value that reaches an output is produced by the
// reference's IEEE operations in its association order, one rounding each
// (-ffp-contract=off): results are bit-identical to the CPU restatement in
// RT_RNG_PHILOX mode.
//
// MI355X mapping (DESIGN.md "Kernel"):
//  * geometry is scanned in the same order by every lane of a wave: sphere
//    records come through the scalar unit (SMEM -> SGPRs, broadcast to the
//    64 lanes for free), two per s_load_dwordx16;
//  * closest hit = a cheap candidate pass (hardware rsq + one Newton step,
//    reciprocal multiply, rigorous error intervals) followed by the exact
//    reference arithmetic for the single winner; any interval overlap or
//    threshold ambiguity falls back to the exact scan for that ray, so the
//    result never depends on the approximation;
//  * per-lane divergent data (the winner's material, texels) is fetched once
//    per bounce from L1/L2;
//  * the IOR stack of pile.h reduces to one register (top n2), see QPath::finish_bounce;
//  * albedo/normal are final once the primary chain (camera ray through
//    alpha holes) ends, so they are added to the accumulators there instead
//    of being carried through the bounce loop;
//  * 256-thread blocks = four 8x8-pixel waves (ray coherence); grid.z splits
//    each pixel's samples into `chunks` fixed slices for load balance, summed
//    in chunk order by combine_kernel (a deterministic, GPU-count-independent
//    grouping that the oracle reproduces).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt/rt.h"
#include "rt_internal.h"
#include "rt_bvh.h"
#include "rt_device_math.h"

// Candidate-pass grazing threshold T1 = RT_CAND_T1 * Hs^2 and half-width
// M = RT_CAND_M * Hs (spheres_closest); M must exceed 2^-47.2 / sqrt(RT_CAND_T1)
// by a wide factor (static_assert below).
#ifndef RT_CAND_T1
#define RT_CAND_T1 0x1p-36
#endif
#ifndef RT_CAND_M
#define RT_CAND_M 0x1p-26
#endif
static_assert(RT_CAND_M * RT_CAND_M * RT_CAND_T1 >= 0x1.8p-89 && RT_CAND_M <= 0x1p-20,
              "candidate half-width M must be >= 8 x the sqrt error bound 2^-47.2/sqrt(T1)");
#ifndef RT_CAND_TAG                 // candidate pass: the running best carries its sphere slot in the low
#define RT_CAND_TAG 1               // 16 mantissa bits (spheres_closest), so no separate index select
#endif
#ifndef RT_CAND_MIN2                // candidate pass: min and second min of the tagged candidates, one
#define RT_CAND_MIN2 1              // ambiguity test after the scan (r04: C2 +4.3 %; 1: every instantiation but
#endif                              // CUDA semantics, 2: the sphere-scene queue kernel only)
#ifndef RT_CAND_GACC                // second-minimum pass: min |D| accumulated, one grazing test per ray (A/B)
#define RT_CAND_GACC 1              // (r04: C2 +0.3 % over RT_RAW_MIN alone)
#endif
#ifndef RT_QSPHERES                 // sphere-only scenes: a queue-kernel instantiation without triangle code
#define RT_QSPHERES 1               // (r04: 116 VGPRs, no spills; C2 +2.3 %)
#endif
#ifndef RT_QOPAQUE                  // sphere-only scenes whose materials are all opaque: an instantiation without
#define RT_QOPAQUE 1                // the alpha-hole and refraction code (r04: 109 VGPRs; C2 +1.0 %)
#endif
#ifndef RT_QOPAQUE_BVH              // deep-tree queue kernel for scenes whose every material (spheres, texels,
#define RT_QOPAQUE_BVH 1            // no material index 3 / 4) is opaque: no hole / refraction code (r04: C4 +2.9 %)
#endif
#ifndef RT_BOX_MM                   // slab test as one comparison max(tmin, -sabs) <= min(tmax, cull) (A/B knob)
#define RT_BOX_MM 1                 // (r04: C4 +0.3 %, sweep +0.6 %)
#endif
#ifndef RT_QLDS_IR                  // non-BVH queue kernels: incomingLight / rayColor in LDS (A/B knob)
#define RT_QLDS_IR 1                // (r04: C2 kernel 97 VGPRs; C2 +2.45 %, C3 +0.8 %)
#endif
#ifndef RT_QLDS_INC_BVH             // the opaque deep-tree kernel keeps incomingLight in LDS (A/B knob)
#define RT_QLDS_INC_BVH 1           // (r04: spills 4 -> 0, C4 +0.7 %)
#endif
#ifndef RT_TRI_BF                   // brute-force triangle scan without branches (r04: C3 +1.3 %, C5 +1.3 %)
#define RT_TRI_BF 1
#endif
#ifndef RT_WAVES_PER_SIMD_Q4        // occupancy bound of the shallow-tree queue kernel (A/B knob)
#define RT_WAVES_PER_SIMD_Q4 RT_WAVES_PER_SIMD_Q
#endif
#ifndef RT_WAVES_PER_SIMD_QS        // occupancy bound of the sphere-only queue kernel (A/B knob)
#define RT_WAVES_PER_SIMD_QS RT_WAVES_PER_SIMD_Q
#endif
#ifndef RT_RAW_MIN                  // normalize's range guard: min of |components| without canonicalizes
#define RT_RAW_MIN 1
#endif
#ifndef RT_AO_FIRST                 // AO scenes: the AO direction before the bounce direction (ROLE_AO)
#define RT_AO_FIRST 1
#endif
#ifndef RT_QTASK_TABLE              // sphere-scene queue kernel: tasks decoded per batch into LDS (A/B knob;
                                    // RT_QUEUE must then be 64, one task per lane of a batch)
#define RT_QTASK_TABLE 1
#endif
#ifndef RT_WAVES_PER_SIMD
#define RT_WAVES_PER_SIMD 4
#endif
#define RT_BVH_COOP 1               // fixed-grid BVH kernel: wave-cooperative deep traversal once this
                                    // many lanes wait for it (samples_coop)
#define RT_FLAT_FILL 2              // fixed-grid sphere kernel: camera rays start once this many eighths
                                    // of the live lanes wait (samples_flat)
#ifndef RT_TRI_UNORM                // triangle hits read the host-normalized normal (A/B knob)
#define RT_TRI_UNORM 1
#endif
#ifndef RT_MERGED_NRM               // AO queue kernels: one normal computation per round for hit lanes and
#define RT_MERGED_NRM 1             // pending bounces (A/B knob; C4 +2.4 %)
#endif
#ifndef RT_REFR_PREFETCH            // queue kernels: the refraction draw's Philox block made in the round's
#define RT_REFR_PREFETCH 1          // shared Philox step (A/B knob)
#endif
#ifndef RT_TEX_AFFINE               // texel lookups through the host's affine uv map when certain (A/B knob)
#define RT_TEX_AFFINE 1
#endif
#ifndef RT_TEX_CONST                // uv-less triangles take their constant texel (TriTex::tex0; A/B knob)
#define RT_TEX_CONST 1
#endif
#ifndef RT_WALK_PRIO                // BVH queue kernel: wave priority during its walk steps (0: off).  The walk
#define RT_WALK_PRIO 2              // is a chain of dependent node/record loads; ahead of the other waves'
#endif                              // VALU it issues sooner: C4 +2.0..2.4 %, sweep +1.7..2.6 % (levels 1-3
                                    // alike; the same priority while resolving hits: C3 -0.4 %)
#ifndef RT_QUEUE                    // sphere kernel, spp_chunks > 1: persistent lanes + (chunk, pixel) task queue
#define RT_QUEUE 64                 // (tasks per atomic grab of a wave; 0: off)
#endif
static_assert(RT_QUEUE == 0 || RT_QUEUE >= 64, "a wave's grab (up to 64 lanes) must fit one batch");
static_assert(!RT_QTASK_TABLE || RT_QUEUE == 64, "the task table holds one batch of 64 tasks per wave");
#ifndef RT_WAVES_PER_SIMD_Q         // queue kernel occupancy bound
#define RT_WAVES_PER_SIMD_Q RT_WAVES_PER_SIMD
#endif
#ifndef RT_PHASE_CLOCK              // diagnostic builds only (tools/phase_clock.py): render_kernel_q adds the
#define RT_PHASE_CLOCK 0            // wave's s_memtime cycles per round phase to its RT_QUEUE_TRACE record
#endif
// RT_QUEUE_TRACE words per lane: start, end, rounds, tasks (+ RT_PHASE_CLOCK:
// cycles in the sphere cast, the BVH walk, resolve, the task hand-out, and
// the next-ray step with finish_bounce)
#define RT_TRACE_WORDS (RT_PHASE_CLOCK ? 9 : 4)
#ifndef RT_WAVES_PER_SIMD_BVH       // the BVH variant (traversal state + LDS stack)
#define RT_WAVES_PER_SIMD_BVH 3
#endif

namespace rt {

struct V3 {
    double x, y, z;
};
__device__ __forceinline__ V3 v3(double a, double b, double c) { return V3{a, b, c}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 muls(V3 a, double t) { return v3(a.x * t, a.y * t, a.z * t); }
__device__ __forceinline__ V3 divs(V3 a, double t) { return v3(a.x / t, a.y / t, a.z / t); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

__device__ __forceinline__ V3 cross(V3 u, V3 v)
{
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

// normalize(a) = a / sqrt(dot(a, a)), vec3.h:137-139, bit-exact: fast lanes
// need dot(a,a) in [2^-760, 2^760] and every |component| >= 2^-900 (so zero
// components, NaN and extreme lengths take the generic path).
// min(|a|, |b|, |c|) as two v_min_f64 with abs source modifiers: fmin would
// first canonicalize each operand (one v_max_f64 x, x per component) under
// IEEE mode.  Only compared against a positive bound; a NaN component makes
// dot(a, a) NaN, which fails normalize's range test whatever this returns.
__device__ __forceinline__ double dmin_abs3(double a, double b, double c)
{
    double r;
    asm("v_min_f64 %0, |%1|, |%2|\n\tv_min_f64 %0, %0, |%3|" : "=&v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// max(|a|, |b|, |c|) (a NaN operand drops out: callers test the values it
// bounds for NaN themselves)
__device__ __forceinline__ double dmax_abs3(double a, double b, double c)
{
    double r;
    asm("v_max_f64 %0, |%1|, |%2|\n\tv_max_f64 %0, %0, |%3|" : "=&v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ V3 normalize(V3 a)
{
    const double n2 = dot(a, a);
    const double mn = RT_RAW_MIN ? dmin_abs3(a.x, a.y, a.z) : fmin(fmin(fabs(a.x), fabs(a.y)), fabs(a.z));
    if (n2 >= 0x1p-760 && n2 <= 0x1p760 && mn >= 0x1p-900) {
        double L, rc;                    // 1/L from the sqrt sequence's own rsq (rt_device_math.h)
        sqrt_rcp_core(n2, L, rc);
        return v3(div_core(a.x, L, rc), div_core(a.y, L, rc), div_core(a.z, L, rc));
    }
    return divs(a, sqrt(n2));
}

// normalize() of random_dir_no_norm's vector (rtutility.h:198-202): the
// components are float products, each nonzero (cos/sin of a float are never 0)
// or a signed zero (theta = 0: sin = +0), and |a|^2 is within 6 * 2^-24 of 1,
// so no range guard: sqrt_rcp_near1 and div_core0 on every lane.
__device__ __forceinline__ V3 normalize_unit(V3 a)
{
    double L, rc;
    sqrt_rcp_near1(dot(a, a), L, rc);
    return v3(div_core0(a.x, L, rc), div_core0(a.y, L, rc), div_core0(a.z, L, rc));
}

// The kernel's by-value parameters (kernarg segment) through an address the
// compiler cannot see through: fields read via it are loaded (s_load) where
// they are used instead of being held in SGPRs -- and spilled to VGPR lanes,
// one v_readlane per reload -- across a long loop.
// (KParams is the only argument of the kernels that use this: offset 0.)
typedef const __attribute__((address_space(4))) KParams* KParamsK;
__device__ __forceinline__ KParamsK kp_here()
{
    KParamsK p = (KParamsK)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}


// (int) of a double as the reference's x86-64 build executes it (cvttsd2si):
// NaN and out-of-range values give INT_MIN, the "integer indefinite".  C
// leaves this undefined; gfx950's v_cvt_i32_f64 saturates instead (NaN -> 0),
// so NaN radiance (e.g. AO_intensity truncated to 0, main.c:43/115) would
// otherwise resolve differently.
__device__ __forceinline__ int cvt_i32_x86(double x)
{
    return (x > -2147483649.0 && x < 2147483648.0) ? (int)x : (int)0x80000000u;
}

struct Mat {
    V3 diff, emis;
    double es, rs, alpha, ior;
};
__device__ __forceinline__ Mat load_mat(const DevMat* m)
{
    const DevMat r = *m;
    return Mat{v3(r.dr, r.dg, r.db), v3(r.er, r.eg, r.eb), r.es, r.rs, r.alpha, r.ior};
}

// Per-pixel sums (radiance, albedo, normal) live in LDS, one 9-double column
// per thread ([9][256], conflict-free), so they occupy no VGPRs across the
// bounce loop.  Only the owning thread touches its column: plain
// read-add-write, same IEEE adds in the same order as fill_canva's sums.
__device__ __forceinline__ void acc_add(double* acc, int base, V3 v)
{
    acc[(base + 0) * 256] = acc[(base + 0) * 256] + v.x;
    acc[(base + 1) * 256] = acc[(base + 1) * 256] + v.y;
    acc[(base + 2) * 256] = acc[(base + 2) * 256] + v.z;
}

enum : int { ACC_RAD = 0, ACC_ALB = 3, ACC_NRM = 6, ACC_SLOTS = 9 };

// Per-thread event counters (COUNT instantiation only).
struct Cnt {
    unsigned long long c[RT_NCOUNTERS];
};

// COUNT diagnostics: one lane per wave-level execution adds 64 lane slots.
__device__ __forceinline__ void wave_slots(Cnt& cnt, int k)
{
    if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) cnt.c[k] += 64;
}

enum : int { HIT_NONE = 0, HIT_SPHERE = 1, HIT_TRI = 2 };

__device__ __forceinline__ double dinf() { return __longlong_as_double(0x7ff0000000000000ll); }

// hit_sphere, sphere.h:13-47, exact reference arithmetic.  two_a = 2*a and
// four_a = 4*a with a = dot(d, d) (`4*a*c` == (4*a)*c).  A negative
// numerator decides t < 1e-4 without the division (2a > 0).
//
// With fast (two_a in [2^-100, 2^100], rc2a = rcp_refined(two_a)) the
// divisions run div_core: a hit needs n >= 1e-4*two_a >> 2^-900, and
// disc <= 2^760 bounds |n| by 2^512, so every quotient that can decide or
// become t is exact; smaller n give t < 1e-4 on both paths.
// CU: main_cuda.cu's hit_sphere (sphere.hu:27-45), t1 >= 0 then t2 >= 0.001;
// its t1 may be tiny, so the fast division also needs |n| >= 2^-900 there.
template <bool CU>
__device__ __forceinline__ bool sphere_exact(double cx, double cy, double cz, double r2, const V3 o, const V3 d,
                                             double two_a, double four_a, bool fast, double rc2a, double& t)
{
    const double e1 = CU ? 0.0 : 0.0001, e2 = CU ? 0.001 : 0.0001;
    const double ocx = o.x - cx, ocy = o.y - cy, ocz = o.z - cz;
    const double b = 2.0 * (ocx * d.x + ocy * d.y + ocz * d.z);
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - r2;
    const double disc = b * b - four_a * c;
    if (!(disc > 0)) return false;
    const bool f = fast && disc >= 0x1p-760 && disc <= 0x1p760;
    double sq;
    if (f) sq = sqrt_core(disc);
    else sq = sqrt(disc);
    const double n1 = -b - sq;
    if (!(n1 < 0.0)) {
        if (f && (!CU || n1 >= 0x1p-900)) t = div_core(n1, two_a, rc2a);
        else t = n1 / two_a;
        if (t >= e1) return true;
    }
    const double n2 = -b + sq;
    if (!(n2 < 0.0)) {
        if (f && (!CU || n2 >= 0x1p-900)) t = div_core(n2, two_a, rc2a);
        else t = n2 / two_a;
        if (t >= e2) return true;
    }
    return false;
}

// The reference's discriminant sign (sphere.h:24-25): COUNT statistics only.
__device__ __forceinline__ bool disc_positive(const SphGeo& s, const V3 o, const V3 d, double four_a)
{
    const double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
    const double b = 2.0 * (ocx * d.x + ocy * d.y + ocz * d.z);
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - s.r2;
    return b * b - four_a * c > 0;
}

// Exact reference scan over every sphere (main.c:59-78 with hit_sphere).
template <bool CU>
__device__ __forceinline__ int spheres_exact_scan(const KParams& kp, const V3 o, const V3 d, double two_a,
                                                  double four_a, bool fast, double rc2a, double& t_best)
{
    const cdptr sg = (cdptr)kp.sph;
    double t = dinf();
    int win = -1;
    for (int k = 0; k < kp.ns_pad; ++k) {
        double tk;
        if (sphere_exact<CU>(sg[4 * k], sg[4 * k + 1], sg[4 * k + 2], sg[4 * k + 3], o, d, two_a, four_a, fast,
                             rc2a, tk) &&
            tk < t) {
            t = tk;
            win = k;
        }
    }
    t_best = t;
    return win;
}

// Closest sphere (main.c:59-78): an FMA candidate pass with rigorous error
// intervals picks the winner, whose exact reference test then runs alone;
// any ambiguity reruns the exact scan for that ray (DESIGN.md "Exact closest
// hit").  Half-b form: h = (o-C).d, D = h^2 - a*c, roots n1,2 = -h -/+ sqrt(D)
// with t = n/a (the reference's t1,2 = (-b -/+ sqrt(disc))/(2a) scale
// exactly: b = 2h, disc = 4D).  Intervals are kept in n = a*t units, one
// per-ray half-width M for every sphere:
//   h  = od - C.d                       (3 fma; od = o.d per ray)
//   ca = a|o|^2 - 2a o.C + a*k          (4 fma; k = |C|^2 - r2 from the host)
//   D  = fma(h, h, -ca)
// Error bound: with Hs >= (|o| + L) sqrt(a), L >= |C_k| + R_k,
// |D - D_ref| <= 52.5u*Hs^2 <= 2^-47.3 Hs^2 (u = 2^-53), where D_ref =
// disc_ref/4.  Rays with D >= T1 = 2^-36 Hs^2 are resolved: the reference's
// disc > 0, and sa (v_rsq_f64 + one Newton step, <= 2^-45 relative) is within
// 2^-29.3 Hs of its rounded sqrt, so |n - n_ref| <= 2^-29.29 Hs; a*t_ref lies
// within u|n| of n_ref.  M = 2^-26 Hs (+ thr*2^-48 for the rounding of
// thr = a*1e-4) leaves a factor 9.8 of slack.  D < -T2 = -2^-44 Hs^2 is a sure
// miss; in between (grazing rays) the ray is ambiguous.  Root choice follows
// hit_sphere: n1 if it may reach 1e-4 (a straddle is ambiguous), else n2.
// Two winners closer than 2M are ambiguous, so a strictly smaller interval is
// a strictly smaller t_ref (the reference keeps the first of equal t).
// Non-finite o, d or Hs^2 > 2^1000 make the ray ambiguous up front.
// CU (main_cuda.cu's thresholds): t1 >= 0, t2 >= 0.001, one interval pair each.
// The candidate's n with its low 16 mantissa bits replaced by sphere slot k:
// one v_and_or_b32 with the mask in a VGPR (msk, loop-invariant; a literal
// would split it into v_and + v_or) and the wave-uniform slot as its one
// scalar operand.
__device__ __forceinline__ double cand_tag(double n, int k, uint32_t msk)
{
    uint32_t lo;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)__double2loint(n)), "v"(msk), "s"(k));
    return __hiloint2double(__double2hiint(n), (int)lo);
}

// min(a, |b|) with an abs source modifier (a >= 0; a NaN b drops out, which
// only happens for a NaN D: non-finite inputs are already ambiguous)
__device__ __forceinline__ double dmin_abs2(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// v_min_f64 / v_max_f64 of two finite, non-NaN operands (the candidate
// pass's tagged values): fmin/fmax would first canonicalize the bit-built
// operand (an extra v_max_f64 x, x each).
__device__ __forceinline__ double dmin_raw(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double dmax_raw(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// main.c:214's `r.x > 0.5 || r.y > 0.5 || r.z > 0.5` as max(x, y, z) > 0.5
// (a NaN component drops out of v_max_f64 exactly as it fails its own
// comparison; the throughputs are arithmetic results, never signalling
// NaNs).  The compiler makes the same fold itself, but through fmax, which
// canonicalizes all three operands first: 6 VALU instead of 3.
__device__ __forceinline__ bool any_above_half(V3 r)
{
    if (!RT_RAW_MIN) return r.x > 0.5 || r.y > 0.5 || r.z > 0.5;
    return dmax_raw(dmax_raw(r.x, r.y), r.z) > 0.5;
}

template <bool COUNT, bool CU, bool AMGM = false>
__device__ __forceinline__ int spheres_closest(const KParams& kp, const V3 o, const V3 d, double a, double two_a,
                                               double four_a, bool fast, double rc2a, double& t_best, Cnt& cnt)
{
    const cdptr sc = (cdptr)kp.sph_cand;
    const double INF = dinf();
    const double od = fma(o.z, d.z, fma(o.y, d.y, o.x * d.x));
    const double aoo = a * fma(o.z, o.z, fma(o.y, o.y, o.x * o.x));
    const double m2a = -2.0 * a;
    const double oax = m2a * o.x, oay = m2a * o.y, oaz = m2a * o.z;
    // Hs >= (|o| + L) sqrt(a): |o|_1 >= |o|_2.  AMGM (the sphere/brute-force
    // queue kernels without AO or sky): sqrt(a) <= (1 + a)/2, equal at a = 1 (the unit directions
    // of camera, bounce and AO rays; shorter lerped directions get a looser bound,
    // more rescans: 1.7e-4 per sample on C2), with 2^-50 for the fma's rounding
    // for every a >= 0 -- C2 +0.35 %; elsewhere v_rsq_f64 (within 2^-24), which
    // the BVH instantiations keep (their register allocation lost 1.9 % on C4
    // with the fma)
    const double sqa = AMGM ? fma(a, 0.5, 0.5 + 0x1p-50) : (a * __builtin_amdgcn_rsq(a)) * (1.0 + 0x1p-20);
    const double Hs = ((fabs(o.x) + fabs(o.y)) + fabs(o.z) + kp.cand_lmax) * sqa;
    const double Hs2 = Hs * Hs;
    const double T1 = Hs2 * RT_CAND_T1, nT2 = Hs2 * -0x1p-44;
    const double thr = a * 0.0001;
    const double thr1 = CU ? 0.0 : thr, thr2 = CU ? a * 0.001 : thr;
    const double M = fma(thr2, 0x1p-48, Hs * RT_CAND_M);
    const double thrP = thr1 + M, thrM = thr1 - M, M2 = 2.0 * M;
    const double thrP2 = thr2 + M, thrM2 = thr2 - M;
    double bn = INF;
    int bk = -1;
    // finite o, d, Hs^2 keep every D below finite; anything else takes the exact scan
    bool amb = !(fast && Hs2 <= 0x1p1000);
    uint32_t msk = 0xffff0000u;
    asm volatile("" : "+v"(msk));
    // RT_CAND_MIN2: the smallest and second-smallest tagged candidate (bn, bn2;
    // non-candidates enter as a finite sentinel above 2^1000 that keeps the
    // tag), ambiguity decided once after the scan (bn2 - bn <= 2M)
    constexpr bool MN = !CU && (RT_CAND_MIN2 == 1 || (RT_CAND_MIN2 == 2 && AMGM));
    double bn2 = __hiloint2double(0x7fefffff, -1);
    if (MN) bn = bn2;
    double gmin = bn2;                   // (RT_CAND_GACC) min |D| over the scan
    for (int k = 0; k < kp.ns_cand; k += 2) {
        double g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = sc[4 * k + j];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const double cx = g[4 * e], cy = g[4 * e + 1], cz = g[4 * e + 2], kk = g[4 * e + 3];
            const double h = fma(-cz, d.z, fma(-cy, d.y, fma(-cx, d.x, od)));
            const double ca = fma(cz, oaz, fma(cy, oay, fma(cx, oax, fma(a, kk, aoo))));
            const double D = fma(h, h, -ca);
            // D finite here.  The ambiguity tests use xor of nested conditions
            // (a implies b: b && !a == a ^ b) so each comparison is issued once.
            // MN: one |D| < T1 test (grazing band widened from [-T2, T1) to
            // (-T1, T1)); D <= -T1 gives a NaN root below, which no comparison
            // accepts, so `valid` is implied by the candidate test
            bool valid = true;
            if (MN && RT_CAND_GACC) {
                gmin = dmin_abs2(gmin, D);                  // grazing test once, after the scan
            } else if (MN) {
                amb = amb || fabs(D) < T1;
            } else {
                valid = D >= T1;
                amb = amb || (valid != (D >= nT2));         // -T2 <= D < T1: grazing
            }
            // sa ~ sqrt(D): v_rsq_f64 + one Newton step (sa = t + t*e/2)
            const double r0 = __builtin_amdgcn_rsq(D);
            const double tt = D * r0;
            const double sa = fma(tt * 0.5, fma(-tt, r0, 1.0), tt);
            const double n1 = -h - sa;
            const bool r1 = n1 >= thrM;                     // n1 may reach 1e-4: hit_sphere takes t1
            // the chosen root: n1 = -h - sa, or n2 = -h + sa; in the sphere-scene queue
            // kernel (AMGM) as one fma with a selected sign (s * sa is exact; C2
            // +0.7 %), elsewhere a select (the fma's constants cost the BVH
            // instantiations registers: sweep -1.4 %)
            const double n = AMGM ? fma(r1 ? -1.0 : 1.0, sa, -h) : (r1 ? n1 : sa - h);
            if (MN) {
                // candidates: every chosen root that may reach 1e-4 (n >= thr - M),
                // straddling ones included -- they are below any sure root, so
                // the winner's own test after the scan (bn < thrP) catches them
                const double nt = cand_tag(n, k + e, msk);
                const double nc = __hiloint2double(n >= thrM ? __double2hiint(nt) : 0x7fefffff, __double2loint(nt));
                bn2 = dmin_raw(bn2, dmax_raw(bn, nc));
                bn = dmin_raw(bn, nc);
                continue;
            }
            const double tP = CU ? (r1 ? thrP : thrP2) : thrP, tM = CU ? (r1 ? thrM : thrM2) : thrM;
            const bool sure = n >= tP;
            amb = amb || (valid && (sure != (n >= tM)));    // the chosen root straddles 1e-4
            const bool cand = valid && sure;
            // RT_CAND_TAG: n with its low 16 mantissa bits replaced by the slot
            // (one v_and_or_b32; host: ns_cand <= 65534); |nt - n| < 2^-36 |n|
            // <= 2^-34.4 Hs, inside M's slack
            const double nt = RT_CAND_TAG ? cand_tag(n, k + e, msk) : n;
            const double diff = nt - bn;
            const bool closer = cand && diff < -M2;
            amb = amb || (cand && fabs(diff) <= M2);        // (closer implies |diff| > M2)
            bn = closer ? nt : bn;
            if (!RT_CAND_TAG) bk = closer ? k + e : bk;
        }
    }
    if (MN) {
        // the winner is sure (its tagged value, within 2^-36 |n| of n, clears
        // thr + M with that margin) and every other candidate lies more than
        // 2M above it; no candidate: bn is the sentinel (> 2^1000)
        const bool any = bn < 0x1p600;
        if (RT_CAND_GACC) amb = amb || gmin < T1;
        amb = amb || (any && (bn < thrP * (1.0 + 0x1p-34) || !(bn2 - bn > M2)));
        bk = any ? (int)((uint32_t)__double2loint(bn) & 0xffffu) : -1;
    } else if (RT_CAND_TAG) {
        bk = bn < INF ? (int)((uint32_t)__double2loint(bn) & 0xffffu) : -1;
    }
    if (COUNT)
        for (int k = 0; k < kp.ns; ++k) cnt.c[RT_CNT_SPHERE_DISC] += disc_positive(kp.sph[k], o, d, four_a) ? 1 : 0;
    double t = INF;
    int win = -1;
    if (!amb && bk >= 0) {
        const SphGeo s = kp.sph[bk];
        if (sphere_exact<CU>(s.cx, s.cy, s.cz, s.r2, o, d, two_a, four_a, fast, rc2a, t)) win = bk;
        else amb = true;     // cannot happen within the bound; stay exact anyway
    }
    if (amb) {               // exact reference scan for this ray
        if (COUNT) cnt.c[RT_CNT_EXACT_RESCANS] += 1;
        win = spheres_exact_scan<CU>(kp, o, d, two_a, four_a, fast, rc2a, t);
    }
    t_best = t;
    return win;
}

// hit_triangle, mesh.h:70-94, exact reference arithmetic, folded into the
// running closest hit.  Acceptance is the reference's `dst >= 1e-7 && dst <
// best` plus its in-order tie-break: when the triangles are not scanned in
// the caller's order (BVH leaf order), an equal dst replaces a triangle
// winner with a larger caller index (orig).  det >= 1e-6 >= 2^-400 puts
// 1/det on the exact fast division (div_core).
// O32 (BVH leaves: a tree holds < 65535 nodes, so k * sizeof(TriGeo) < 2^32):
// the records are read at 32-bit byte offsets from the array's scalar base.
// UNI (the brute-force scan, k wave-uniform): the record through the scalar
// unit (s_load into SGPRs, read by the VALU as scalar operands), no vector
// memory instructions per triangle.
template <bool COUNT, bool CU = false, bool O32 = false, bool UNI = false>
__device__ __forceinline__ void tri_test(const KParams& kp, int k, const V3 o, const V3 d, double& best, int& kind,
                                         int& win, int& win_orig)
{
    const double eps = CU ? 0.00001 : 0.0000001;     // triangle.hu:262 / mesh.h:88
    TriGeo g;
    if (UNI) {
        const cdptr t = (cdptr)kp.tri + 12 * k;
        g.ax = t[0]; g.ay = t[1]; g.az = t[2];
        g.abx = t[3]; g.aby = t[4]; g.abz = t[5];
        g.acx = t[6]; g.acy = t[7]; g.acz = t[8];
        g.nx = t[9]; g.ny = t[10]; g.nz = t[11];
    } else if (O32) {
        // the whole record in six 16-byte loads and ONE wait: left to itself
        // the compiler sinks the A/AB/AC loads below the det test, a second
        // dependent round trip per leaf test
        g = *(const TriGeo*)((const char*)kp.tri + (uint32_t)k * (uint32_t)sizeof(TriGeo));
        asm volatile("" : "+v"(g.ax), "+v"(g.ay), "+v"(g.az), "+v"(g.abx), "+v"(g.aby), "+v"(g.abz), "+v"(g.acx),
                     "+v"(g.acy), "+v"(g.acz), "+v"(g.nx), "+v"(g.ny), "+v"(g.nz));
    } else {
        g = kp.tri[k];
    }
    const double det = -(d.x * g.nx + d.y * g.ny + d.z * g.nz);
    if (det >= 1E-6) {
        const V3 ao = v3(o.x - g.ax, o.y - g.ay, o.z - g.az);
        const V3 dao = cross(ao, d);
        double invDet;
        if (det <= 0x1p400) invDet = div_core(1.0, det, rcp_refined(det));
        else invDet = 1 / det;
        const double dst = (ao.x * g.nx + ao.y * g.ny + ao.z * g.nz) * invDet;
        if (dst >= eps && dst <= best) {
            const int orig = !kp.tri_orig ? k
                             : O32 ? *(const int*)((const char*)kp.tri_orig + (uint32_t)k * 4u) : kp.tri_orig[k];
            if (dst < best || (kind == HIT_TRI && orig < win_orig)) {
                const double u = (g.acx * dao.x + g.acy * dao.y + g.acz * dao.z) * invDet;
                const double v = -(g.abx * dao.x + g.aby * dao.y + g.abz * dao.z) * invDet;
                const double w = 1 - u - v;
                if (u >= eps && v >= eps && w >= eps) {
                    best = dst;
                    kind = HIT_TRI;
                    win = k;
                    win_orig = orig;
                }
            }
        }
    }
}

// tri_test for the brute-force scan in the caller's order (kp.tri_orig null:
// no tie rule, `dst < best` is mesh.h's and main.c:82's strict test), with
// no branches: every lane evaluates det, dst and the barycentrics with the
// reference operations and one combined condition picks the hit.  The
// branchy form ran these in nested divergent regions whose exec-mask
// bookkeeping cost more than the work they skipped: in a wave of
// incoherent rays some lane almost always passes the culling tests.  Lanes
// with det < 1e-6 compute a garbage 1/det (the fast reciprocal of a small,
// zero or negative value) that no condition lets through.
template <bool CU>
__device__ __forceinline__ void tri_test_bf(const KParams& kp, int k, const V3 o, const V3 d, double& best, int& kind,
                                            int& win)
{
    const double eps = CU ? 0.00001 : 0.0000001;     // triangle.hu:262 / mesh.h:88
    const cdptr t = (cdptr)kp.tri + 12 * k;
    const double ax = t[0], ay = t[1], az = t[2], abx = t[3], aby = t[4], abz = t[5];
    const double acx = t[6], acy = t[7], acz = t[8], nx = t[9], ny = t[10], nz = t[11];
    const double det = -(d.x * nx + d.y * ny + d.z * nz);
    const V3 ao = v3(o.x - ax, o.y - ay, o.z - az);
    const V3 dao = cross(ao, d);
    double invDet;
    if (det <= 0x1p400) invDet = div_core(1.0, det, rcp_refined(det));
    else invDet = 1 / det;
    const double dst = (ao.x * nx + ao.y * ny + ao.z * nz) * invDet;
    const double u = (acx * dao.x + acy * dao.y + acz * dao.z) * invDet;
    const double v = -(abx * dao.x + aby * dao.y + abz * dao.z) * invDet;
    const double w = 1 - u - v;
    // every lane evaluates the whole test: the empty asm keeps the compiler
    // from sinking the barycentrics under a branch on det and dst
    double uu = u, vv = v;
    asm volatile("" : "+v"(uu), "+v"(vv));
    const bool hit = (det >= 1E-6) & (dst >= eps) & (dst < best) & (uu >= eps) & (vv >= eps) & (w >= eps);
    if (hit) {
        best = dst;
        kind = HIT_TRI;
        win = k;
    }
}

// Triangle BVH traversal (rt_bvh.h: 4-wide nodes collapsed from the binary
// SAH tree, host build rt_bvh.cpp).  One 128-byte node holds four child
// boxes (float storage rounded outward; the slab math runs in double); leaf
// children are tested on the spot, the nearest hit internal child is entered
// next and the others are pushed on a per-lane LDS stack (uint16
// [kStack4][256], conflict-free).  A box is skipped only when no triangle in
// it can win or tie (rt_bvh.cpp): the ray misses the padded box, leaves it
// behind the origin (tmax < -sabs), or enters it beyond best*(1+srel)+sabs.
// Slab reciprocals use |d_i| >= 2^-200, which keeps the products finite
// without changing any decision for unit-length directions.
// The per-lane stack: one LDS allocation per kernel ([kStack4][256]).
__device__ __forceinline__ unsigned short* bvh_stack()
{
    __shared__ unsigned short stk_lds[kStack4 * 256];
    return stk_lds + threadIdx.x;
}
// The queue kernel's per-lane stack (BVH scenes): uint16 [entries][256].  The
// deep-tree instantiations (QB = 3) get kStackQ = 24 entries (12 KiB) when every
// material is opaque (OPQ: incomingLight also lives in LDS) and kStackQN = 32
// (16 KiB) otherwise, which keeps both at <= 40 KiB, i.e. 4 blocks (16 waves) per
// CU.  The QB = 4 instantiation (shallow trees: bvh_steps 4, i.e. depth4 <= 4) is
// admitted only when the tree's exact stack bound (rt_bvh.cpp stack4) is at most
// kStackQ4 = 14 entries, so its top-node cache and the task table fit the same
// 40 KiB.  An opaque tree whose bound lies in (24, 32] takes the non-OPQ QB = 3
// kernel; a bound above 32 the fixed grid (kStack4).  choose_render below is the
// one place that decides; the host stores its stack in KParams::stack_cap, which
// the COUNT runs check every push against (RT_CNT_BVH_STACK_OVER).
constexpr int kStackQ = 24, kStackQN = 32, kStackQ4 = 14;
template <int QB, bool OPQ>
__device__ __forceinline__ unsigned short* bvh_stack_q()
{
    __shared__ unsigned short stkq_lds[(QB == 4 ? kStackQ4 : OPQ ? kStackQ : kStackQN) * 256];
    return stkq_lds + threadIdx.x;
}
// ... and the block's copy of the tree's top nodes (RT_QB_TOP x 128 B, or
// twice as many 64-byte nodes; the block then needs <= 40 KiB of LDS, still
// 4 blocks per CU)
#ifndef RT_QB_TOP
#define RT_QB_TOP 40
#endif
// node visits per round of the deep-tree instantiations (QB 3): RT_QW_MIN,
// then more while >= RT_QW_LANES lanes still walk, at most RT_QW_MAX (r06,
// profiles/r06_walk: RTX_MAP/nature +17 %, C4 / mineways / a non-opaque tree
// +-0.5 %; a fixed 10 visits gave nature +16 % but the tree -13 %)
#ifndef RT_QW_MIN
#define RT_QW_MIN 3
#endif
#ifndef RT_QW_MAX
#define RT_QW_MAX 12
#endif
#ifndef RT_QW_LANES
#define RT_QW_LANES 32
#endif
// the queue kernel walks the 64-byte nodes (BvhNodeH) when the scene has them
#ifndef RT_QNODE_H
#define RT_QNODE_H 1
#endif
template <class NODE, int N>
__device__ __forceinline__ NODE* bvh_top_q()
{
    __shared__ NODE top_lds[N > 0 ? N : 1];
    return top_lds;
}
// Conservative single-precision slab test (the culling only has to be a
// superset of the double test on the padded boxes).  Per ray
// and axis: inv = rcp((float)d) (|d| clamped to >= 2^-60; <= 2 ulp of 1/d),
// and the offsets a = -(float)o * inv - E, b = -(float)o * inv + E with
//   E = 2^-19 (rbox + |(float)o|) |inv|,
// rbox >= every |bound| of the tree.  The entry plane of an axis is the lo
// bound when inv >= 0 and the hi bound when inv < 0 (the other is the exit
// plane), so with P the entry and Q the exit bound, fma(P, inv, a) and
// fma(Q, inv, b) lie below / above the exact (P - o) / d and (Q - o) / d:
// the rounding of d, o, inv, o*inv, the offsets and the fma together stay
// within 6 u (rbox + |o|) |inv| + 2 u E < E / 5 (u = 2^-24).  (These are the
// min and max of the two plane distances: lo <= hi and a < b order them.)
// The cull thresholds are rounded outward in the same way.
// Rays whose origin lies beyond the radius R_b the tree's padding assumed
// (kp.bvh_rb: the triangles' coordinate bound, raised over the spheres that
// cost the padding little, rt_bvh.cpp bvh_origin_radius) -- the camera, hit
// points on main.c:346's radius-1e5 sky sphere -- get the rest of the slack
// per ray: with R' = max(R_b, |o|_inf) every triangle's padding delta(R) grows
// by at most kdelta (R' - R_b) (delta is affine in R with slope 4 2^-44 1e6
// (e1+e2)^2 + 2^-48 <= kdelta, host), i.e. the ray's entry (exit) plane
// distances move down (up) by that over |d| per axis, and the distance slack
// S_abs = s_rel R grows by s_rel (R' - R_b), which lowers every entry distance
// and raises every exit distance by as much (the box test max(tmin, -S_abs)
// <= min(tmax, best (1 + s_rel) + S_abs) then holds for the larger S_abs).
// Both fold into the offsets a, b once per ray; the per-node test is unchanged.
struct Ray32 {
    float ix, iy, iz;            // ~1/d
    float ax, ay, az;            // offsets of the entry planes (lower bounds)
    float bx, by, bz;            // offsets of the exit planes (upper bounds)
};
__device__ __forceinline__ void ray32_axis(double oc, double dc, float rbox, float& inv, float& a, float& b)
{
    const double lim = 0x1p-60;
    const float df = (float)(fabs(dc) < lim ? copysign(lim, dc) : dc);
    inv = __builtin_amdgcn_rcpf(df);
    const float of = (float)oc;
    const float oi = of * inv;
    const float E = 0x1p-19f * ((rbox + fabsf(of)) * fabsf(inv));
    a = -oi - E;
    b = -oi + E;
}
// FAR: compiled into the kernels that may meet such origins (the non-opaque
// deep-tree queue kernel and the fixed-grid ones); launch_render gives the
// others (C4's OPQ kernel, QB 4) only launches with kp.bvh_far 0.
template <bool FAR = true>
__device__ __forceinline__ Ray32 ray32(const KParams& kp, const V3 o, const V3 d)
{
    Ray32 r;
    ray32_axis(o.x, d.x, kp.bvh_rbox, r.ix, r.ax, r.bx);
    ray32_axis(o.y, d.y, kp.bvh_rbox, r.iy, r.ay, r.by);
    ray32_axis(o.z, d.z, kp.bvh_rbox, r.iz, r.az, r.bz);
    // |(float)o| <= rb_f (host: rb_f (1 + 2^-23) <= R_b) puts o inside R_b;
    // the others take the exact excess (NaN origins miss every box anyway).
    // The float roundings of the widened offsets stay inside E's slack.
    // kp.bvh_far 0 (host: the camera and every sphere lie inside R_b, so every
    // ray origin does): one scalar branch per ray instead of the test.
    if (!FAR || !kp.bvh_far) return r;
    const float omf = fmaxf(fabsf((float)o.x), fmaxf(fabsf((float)o.y), fabsf((float)o.z)));
    if (!(omf <= kp.bvh_rb_f)) {
        const double ex = fmax(fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z))) - kp.bvh_rb, 0.0);
        const float dpad = (float)(kp.bvh_kdelta * ex) * (1.0f + 0x1p-20f);
        const float sx = (float)(kp.bvh_srel * ex) * (1.0f + 0x1p-20f);
        const float px = fmaf(dpad, fabsf(r.ix), sx), py = fmaf(dpad, fabsf(r.iy), sx),
                    pz = fmaf(dpad, fabsf(r.iz), sx);
        r.ax -= px; r.bx += px;
        r.ay -= py; r.by += py;
        r.az -= pz; r.bz += pz;
    }
    return r;
}
// float(best * srel + sabs) rounded up (the triangle test's distance cull)
__device__ __forceinline__ float cull32(const KParams& kp, double best)
{
    return (float)fma(best, 1.0 + kp.bvh_srel, kp.bvh_sabs) * (1.0f + 0x1p-22f);
}
// The four child boxes of a node: hit flags and near distances.  The entry
// and exit planes of each axis are picked by the sign of inv (one 16-byte
// row of lo or hi per axis: BvhNode4 stores lo[3][4] then hi[3][4]).
// Node rows of the HBM tree at 32-bit byte offsets from the tree's
// wave-uniform base: the loads take the scalar-base + 32-bit vector-offset
// form, one v_add_u32 per row instead of 64-bit address arithmetic.
__device__ __forceinline__ float4 bvh_row(const KParams& kp, uint32_t off)
{
    return *(const float4*)((const char*)kp.bvh + off);
}
// nd: the node (an LDS or generic pointer); or, with nd == nullptr, the HBM
// node at byte offset nb (C4 +2.3 %, sweep +1.2 % over 64-bit addresses)
__device__ __forceinline__ void box4(const KParams& kp, const BvhNode4* nd, const Ray32& r, float cull, bool h[4],
                                     float tn[4], int Ch[4], int Cn[4], uint32_t nb = 0)
{
    const float nsabs = (float)(-kp.bvh_sabs) * (1.0f + 0x1p-22f);
    const float4* rows = (const float4*)nd;             // rows 0-2: lo x/y/z, rows 3-5: hi x/y/z
    const int sx = (int)(__float_as_uint(r.ix) >> 31) * 3, sy = (int)(__float_as_uint(r.iy) >> 31) * 3,
              sz = (int)(__float_as_uint(r.iz) >> 31) * 3;
    float4 px, py, pz, qx, qy, qz;
    int4 cnt4;
    if (nd == nullptr) {
        px = bvh_row(kp, nb + (uint32_t)(sx * 16));
        py = bvh_row(kp, nb + (uint32_t)((1 + sy) * 16));
        pz = bvh_row(kp, nb + (uint32_t)((2 + sz) * 16));
        qx = bvh_row(kp, nb + (uint32_t)((3 - sx) * 16));
        qy = bvh_row(kp, nb + (uint32_t)((4 - sy) * 16));
        qz = bvh_row(kp, nb + (uint32_t)((5 - sz) * 16));
        const float4 c4 = bvh_row(kp, nb + (uint32_t)offsetof(BvhNode4, count));
        const float4 h4 = bvh_row(kp, nb + (uint32_t)offsetof(BvhNode4, child));
        cnt4 = make_int4(__float_as_int(c4.x), __float_as_int(c4.y), __float_as_int(c4.z), __float_as_int(c4.w));
        Ch[0] = __float_as_int(h4.x); Ch[1] = __float_as_int(h4.y); Ch[2] = __float_as_int(h4.z); Ch[3] = __float_as_int(h4.w);
    } else {
        px = rows[sx]; py = rows[1 + sy]; pz = rows[2 + sz];
        qx = rows[3 - sx]; qy = rows[4 - sy]; qz = rows[5 - sz];
        cnt4 = make_int4(nd->count[0], nd->count[1], nd->count[2], nd->count[3]);
        for (int c = 0; c < 4; ++c) Ch[c] = nd->child[c];
    }
    Cn[0] = cnt4.x; Cn[1] = cnt4.y; Cn[2] = cnt4.z; Cn[3] = cnt4.w;
    const float Px[4] = {px.x, px.y, px.z, px.w}, Py[4] = {py.x, py.y, py.z, py.w}, Pz[4] = {pz.x, pz.y, pz.z, pz.w};
    const float Qx[4] = {qx.x, qx.y, qx.z, qx.w}, Qy[4] = {qy.x, qy.y, qy.z, qy.w}, Qz[4] = {qz.x, qz.y, qz.z, qz.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float tmin = fmaxf(fmaxf(fmaf(Px[c], r.ix, r.ax), fmaf(Py[c], r.iy, r.ay)), fmaf(Pz[c], r.iz, r.az));
        const float tmax = fminf(fminf(fmaf(Qx[c], r.ix, r.bx), fmaf(Qy[c], r.iy, r.by)), fmaf(Qz[c], r.iz, r.bz));
        h[c] = Cn[c] >= 0 && (RT_BOX_MM ? fmaxf(tmin, nsabs) <= fminf(tmax, cull)
                                        : tmin <= tmax && tmax >= nsabs && tmin <= cull);
        tn[c] = tmin;
    }
}

// box4 on the 64-byte node (BvhNodeH, the queue kernel's): each plane is
// org + rel with binary16 org and rel (rt_bvh.h), so the entry distance is
// fma(rel, inv, A) with A = fma(org, inv, a) per axis and node, the halves
// read straight into v_fma_mix_f32.  Against box4's single fma the extra
// rounding of A adds at most u(|org| + |o|)|inv| + uE (u = 2^-24), and
// with rbox >= |org| + |rel| (host) the total stays below E / 3.
__device__ __forceinline__ float h16lo(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu)); }
__device__ __forceinline__ float h16hi(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16)); }
__device__ __forceinline__ void box4h(const KParams& kp, const BvhNodeH* nd, uint32_t nb, const Ray32& r, float cull,
                                      bool h[4], float tn[4], int Ch[4], int Cn[4])
{
    const float nsabs = (float)(-kp.bvh_sabs) * (1.0f + 0x1p-22f);
    const uint32_t sx = (__float_as_uint(r.ix) >> 31) * 3u, sy = (__float_as_uint(r.iy) >> 31) * 3u,
                   sz = (__float_as_uint(r.iz) >> 31) * 3u;
    uint2 px, py, pz, qx, qy, qz;
    uint4 t;
    {                                                    // the whole node in four 16-byte loads (HBM at
        const uint4* q = nd ? (const uint4*)nd                         // 32-bit offsets, or the LDS copy),
                            : (const uint4*)((const char*)kp.bvhh + nb);   // rows selected by sign
        const uint4 r0 = q[0], r1 = q[1], r2 = q[2];
        t = q[3];
        const uint2 lx = make_uint2(r0.x, r0.y), ly = make_uint2(r0.z, r0.w), lz = make_uint2(r1.x, r1.y);
        const uint2 hx = make_uint2(r1.z, r1.w), hy = make_uint2(r2.x, r2.y), hz = make_uint2(r2.z, r2.w);
        px = sx ? hx : lx; qx = sx ? lx : hx;
        py = sy ? hy : ly; qy = sy ? ly : hy;
        pz = sz ? hz : lz; qz = sz ? lz : hz;
    }
    const float Ax = fmaf(h16lo(t.x), r.ix, r.ax), Ay = fmaf(h16hi(t.x), r.iy, r.ay), Az = fmaf(h16lo(t.y), r.iz, r.az);
    const float Bx = fmaf(h16lo(t.x), r.ix, r.bx), By = fmaf(h16hi(t.x), r.iy, r.by), Bz = fmaf(h16lo(t.y), r.iz, r.bz);
    const uint32_t cn = t.y >> 16;
    Ch[0] = (int)(t.z & 0xffffu); Ch[1] = (int)(t.z >> 16); Ch[2] = (int)(t.w & 0xffffu); Ch[3] = (int)(t.w >> 16);
    const float Px[4] = {h16lo(px.x), h16hi(px.x), h16lo(px.y), h16hi(px.y)};
    const float Py[4] = {h16lo(py.x), h16hi(py.x), h16lo(py.y), h16hi(py.y)};
    const float Pz[4] = {h16lo(pz.x), h16hi(pz.x), h16lo(pz.y), h16hi(pz.y)};
    const float Qx[4] = {h16lo(qx.x), h16hi(qx.x), h16lo(qx.y), h16hi(qx.y)};
    const float Qy[4] = {h16lo(qy.x), h16hi(qy.x), h16lo(qy.y), h16hi(qy.y)};
    const float Qz[4] = {h16lo(qz.x), h16hi(qz.x), h16lo(qz.y), h16hi(qz.y)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int nib = (int)((cn >> (4 * c)) & 15u);
        Cn[c] = nib == 15 ? -1 : nib;
        const float tmin = fmaxf(fmaxf(fmaf(Px[c], r.ix, Ax), fmaf(Py[c], r.iy, Ay)), fmaf(Pz[c], r.iz, Az));
        const float tmax = fminf(fminf(fmaf(Qx[c], r.ix, Bx), fmaf(Qy[c], r.iy, By)), fmaf(Qz[c], r.iz, Bz));
        // RT_BOX_MM: max(tmin, -sabs) <= min(tmax, cull) is the same three
        // tests (-sabs < 0 <= cull) with one comparison instead of three
        h[c] = nib != 15 && (RT_BOX_MM ? fmaxf(tmin, nsabs) <= fminf(tmax, cull)
                                       : tmin <= tmax && tmax >= nsabs && tmin <= cull);
        tn[c] = tmin;
    }
}

// One node visit: the four child boxes, the triangles of the hit leaves, then
// the next node (nearest hit internal child, else the stack top).  Returns
// false when the traversal is over.  tris_bvh loops it to the end; the
// resumable trace (render_sm) runs a bounded number of visits per round.
#ifndef RT_DIAG_STALE                // diagnostic build: COUNT walks count visits to nodes whose entry
#define RT_DIAG_STALE 0              // distance already exceeds the cull distance (in the stack-over slot;
#endif                               // stack entries below depth 16 only)
__device__ __forceinline__ float* diag_lds()
{
    __shared__ float dg_lds[RT_DIAG_STALE ? 17 * 256 : 1];
    return dg_lds + threadIdx.x;
}
__device__ __forceinline__ unsigned* diag_cnt()
{
    __shared__ unsigned dc_lds[RT_DIAG_STALE == 2 ? 2 * 256 : 1];
    return dc_lds + threadIdx.x;
}
template <bool COUNT, bool CU, int NTOP = 0, bool H = false>
__device__ __forceinline__ bool bvh_step(const KParams& kp, const V3 o, const V3 d, const Ray32& r32,
                                         unsigned short* stk, int& node, int& sp, double& best, int& kind,
                                         int& win, int& win_orig, Cnt& cnt, const void* top = nullptr)
{
    if constexpr (RT_DIAG_STALE && (COUNT || RT_DIAG_STALE == 2)) {
        float* dg = diag_lds();
        if (node == 0) dg[16 * 256] = -__builtin_huge_valf();          // the root: a new walk
        const bool stale = dg[16 * 256] > cull32(kp, best);
        if (COUNT && stale) cnt.c[RT_CNT_BVH_STACK_OVER] += 1;
        if (!COUNT) {                                                  // queue kernel: per-lane sums
            unsigned* dc = diag_cnt();
            dc[0] += 1u;
            dc[256] += stale ? 1u : 0u;
        }
    }
    // NTOP > 0: the first NTOP nodes (breadth-first: the top levels) are read
    // from the block's LDS copy `top`, the rest from HBM/L2; H: 64-byte nodes
    if (COUNT) {
        cnt.c[RT_CNT_BVH_NODES] += 1;
        wave_slots(cnt, RT_CNT_BVH_LANE_SLOTS);
    }
    bool h[4];
    float tn[4];
    int Ch[4], Cn[4];
    const bool in_top = NTOP > 0 && node < NTOP;
    if (H)
        box4h(kp, in_top ? (const BvhNodeH*)top + node : nullptr, (uint32_t)node * (uint32_t)sizeof(BvhNodeH), r32,
              cull32(kp, best), h, tn, Ch, Cn);
    else
        box4(kp, in_top ? (const BvhNode4*)top + node : nullptr, r32, cull32(kp, best), h, tn, Ch, Cn,
             (uint32_t)node * (uint32_t)sizeof(BvhNode4));
    int next = -1;
    float tnext = 0.0f;
    unsigned lm = 0;                                     // hit leaf slots
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (!h[c]) continue;
        const int ch = Ch[c], n = Cn[c];
        if (n > 0) {
            lm |= 1u << c;
        } else if (next < 0) {
            next = ch;
            tnext = tn[c];
        } else {
            int push = ch;
            float tpush = tn[c];
            if (tn[c] < tnext) {                         // nearer: enter it, push the previous pick
                push = next;
                tpush = tnext;
                next = ch;
                tnext = tn[c];
            }
            if (!RT_DIAG_STALE && COUNT && sp >= kp.stack_cap) cnt.c[RT_CNT_BVH_STACK_OVER] += 1;
            if (!COUNT || sp < kStack4) {    // COUNT walks use the fixed grid's stack
                if (RT_DIAG_STALE && (COUNT || RT_DIAG_STALE == 2) && sp < 16) diag_lds()[sp * 256] = tpush;
                stk[sp * 256] = (unsigned short)push;
                ++sp;
            }
            (void)tpush;
        }
    }
    // The triangles of every hit leaf in one loop, one triangle per lane and
    // iteration: the wave runs max-over-lanes iterations instead of one
    // divergent loop per child slot.
    int k = 0, kend = 0;
    while (lm != 0u || k < kend) {
        if (COUNT) wave_slots(cnt, RT_CNT_LEAF_LANE_SLOTS);
        if (k >= kend) {
            const int c = __ffs(lm) - 1;
            lm &= lm - 1u;
            k = c == 0 ? Ch[0] : c == 1 ? Ch[1] : c == 2 ? Ch[2] : Ch[3];
            kend = k + (c == 0 ? Cn[0] : c == 1 ? Cn[1] : c == 2 ? Cn[2] : Cn[3]);
            if (COUNT) cnt.c[RT_CNT_BVH_TRI_TESTS] += (unsigned long long)(kend - k);
        }
        tri_test<COUNT, CU, true>(kp, k, o, d, best, kind, win, win_orig);
        ++k;
    }
    if (next >= 0) {
        node = next;
        if (RT_DIAG_STALE && (COUNT || RT_DIAG_STALE == 2)) diag_lds()[16 * 256] = tnext;
        return true;
    }
    if (sp == 0) return false;
    --sp;
    node = stk[sp * 256];
    if (RT_DIAG_STALE && (COUNT || RT_DIAG_STALE == 2))
        diag_lds()[16 * 256] = sp < 16 ? diag_lds()[sp * 256] : -__builtin_huge_valf();
    return true;
}

template <bool COUNT, bool CU>
__device__ __forceinline__ void tris_bvh(const KParams& kp, const V3 o, const V3 d, double& best, int& kind,
                                         int& win, int& win_orig, Cnt& cnt)
{
    unsigned short* stk = bvh_stack();
    const Ray32 r32 = ray32(kp, o, d);
    int node = 0, sp = 0;
    while (bvh_step<COUNT, CU>(kp, o, d, r32, stk, node, sp, best, kind, win, win_orig, cnt)) {
    }
}

// closest_hit, main.c:52-92: spheres, then triangles; a strictly closer hit
// replaces the record.  Returns the winner (kind, index, t).
// hit_BBox, triangle.hu:42-59 (CU mode): IEEE divisions, CUDA's double
// min/max = fmin/fmax; the triangles are skipped when it fails.
__device__ __forceinline__ bool cuda_bbox(const KParams& kp, const V3 o, const V3 d)
{
    const double t1x = (kp.cbb[0] - o.x) / d.x, t2x = (kp.cbb[3] - o.x) / d.x;
    const double t1y = (kp.cbb[1] - o.y) / d.y, t2y = (kp.cbb[4] - o.y) / d.y;
    const double t1z = (kp.cbb[2] - o.z) / d.z, t2z = (kp.cbb[5] - o.z) / d.z;
    const double tmax = fmin(fmin(fmax(t1x, t2x), fmax(t1y, t2y)), fmax(t1z, t2z));
    const double tmin = fmax(fmax(fmin(t1x, t2x), fmin(t1y, t2y)), fmin(t1z, t2z));
    return tmax - tmin > 0;
}

// The sphere half of closest_hit (and the cast counters): the winner index
// or -1, its t in best (+inf when none).
template <bool COUNT, bool CU, bool AMGM = false>
__device__ __forceinline__ int cast_spheres(const KParams& kp, const V3 o, const V3 d, double& best, Cnt& cnt)
{
    const double a = dot(d, d);          // sphere.h:20 (same for every sphere)
    const double two_a = 2 * a;          // sphere.h:27,36
    const double four_a = 4 * a;         // sphere.h:24
    const bool fast = two_a >= 0x1p-100 && two_a <= 0x1p100;
    const double rc2a = rcp_refined(two_a);
    if (COUNT) {
        cnt.c[RT_CNT_CASTS] += 1;
        cnt.c[RT_CNT_SPHERE_TESTS] += (unsigned long long)kp.ns;
        cnt.c[RT_CNT_TRI_TESTS] += (unsigned long long)kp.nt;
        wave_slots(cnt, RT_CNT_CAST_LANE_SLOTS);
    }
    int win = spheres_closest<COUNT, CU, AMGM>(kp, o, d, a, two_a, four_a, fast, rc2a, best, cnt);
    return win;
}

template <bool COUNT, bool BVH, bool CU = false, bool AMGM = false>
__device__ __forceinline__ int closest_hit(const KParams& kp, const V3 o, const V3 d, double& t_best, int& idx,
                                           Cnt& cnt)
{
    double best;
    int win = cast_spheres<COUNT, CU, AMGM>(kp, o, d, best, cnt);
    int kind = win >= 0 ? HIT_SPHERE : HIT_NONE;
    int win_orig = 0;
    if (CU && kp.nt > 0 && !cuda_bbox(kp, o, d)) {
        // main_cuda.cu:40-45: the ray misses the mesh box, no triangle tested
    } else if (BVH) {
        tris_bvh<COUNT, CU>(kp, o, d, best, kind, win, win_orig, cnt);
    } else if (RT_TRI_BF && !COUNT && !kp.tri_orig) {
        for (int k = 0; k < kp.nt; ++k) tri_test_bf<CU>(kp, k, o, d, best, kind, win);
    } else {
        for (int k = 0; k < kp.nt; ++k) tri_test<COUNT, CU, false, true>(kp, k, o, d, best, kind, win, win_orig);
    }
    t_best = best;
    idx = win;
    return kind;
}

// tri_uvmapping + get_barycentric_coord, texture.h:16-27,44-90, in two
// steps: the texel a hit picks (barycentrics, uv, fmod, the clamped index)
// and the material read from it (with the material-index overrides).  A
// refraction lane keeps the TexRef from resolve_hit to finish_bounce instead
// of recomputing the barycentrics (host: n_texels < 2^31).
struct TexRef {
    int index;                        // clamped texel index
    int m;                            // the triangle's material index (quelMatPourTri)
};
// hit_triangle's normal vec3_normalize(N) (mesh.h:91): RT_TRI_UNORM reads the
// host's copy (TriTex::un*, the same IEEE operations) instead of normalizing N
// per hit
__device__ __forceinline__ V3 tri_normal(const KParams& kp, int k)
{
    if (RT_TRI_UNORM) {
        const TriTex* t = kp.tri_tex + k;
        return v3(t->unx, t->uny, t->unz);
    }
    const TriGeo* g = kp.tri + k;
    return normalize(v3(g->nx, g->ny, g->nz));
}
// The texel through the host's affine uv map (rt_api.cpp tri_uv_affine): the
// reference's u, v are affine in P up to rounding, so with tw*u within eu of tu,
// x = floor(tw u_ref) - tw floor(u_ref) is certain when no integer lies in
// [tu - eu, tu + eu] (the wrap at integer u and the cells at multiples of 1/tw
// are all integers of tw*u); the same for v.  False: not certain (or P farther
// than diam from A, where the bound does not hold) -- the caller then takes the
// exact path.  rt_verify_texel_map checks it against tri_texel_exact.
__device__ __forceinline__ bool tri_texel_affine(const KParams& kp, int k, const V3 P, TexRef& t)
{
    const TriUV q = kp.tri_uv[k];
    const TriGeo* gp = kp.tri + k;
    const double dx = P.x - gp->ax, dy = P.y - gp->ay, dz = P.z - gp->az;
    const double uf = fma(q.gux, dx, fma(q.guy, dy, fma(q.guz, dz, q.u0)));
    const double vf = fma(q.gvx, dx, fma(q.gvy, dy, fma(q.gvz, dz, q.v0)));
    const double tw = (double)kp.tw, th = (double)kp.th;
    const double tu = uf * tw, tv = vf * th;
    const double lu = floor(tu - q.eu), lv = floor(tv - q.ev);
    if (!(dmax_abs3(dx, dy, dz) <= q.diam && lu == floor(tu + q.eu) && lv == floor(tv + q.ev))) return false;
    const int x = (int)fma(-tw, floor(uf), lu), y = (int)fma(-th, floor(vf), lv);
    const int m = kp.tri_tex[k].mat;
    long long index = ((long long)y * kp.tw + x) + ((long long)kp.th * kp.tw * m);
    index = index < 0 ? 0 : index;                       // reference UB -> clamp
    index = index >= kp.n_texels ? kp.n_texels - 1 : index;
    t = TexRef{(int)index, m};
    return true;
}
// tri_uvmapping + get_barycentric_coord with the reference's operations
__device__ __forceinline__ TexRef tri_texel_exact(const KParams& kp, int k, const V3 P, const V3 n)
{
    const TriGeo g = kp.tri[k];
    const TriTex tx = kp.tri_tex[k];
    const V3 A = v3(g.ax, g.ay, g.az), B = v3(tx.bx, tx.by, tx.bz), C = v3(tx.cx, tx.cy, tx.cz);
    // areaABC = dot(n, cross(B-A, C-A)) = dot(n, N): n is the triangle's own
    // unit normal (tri_normal), so the host's TriTex::area is the same value
    const double areaABC = RT_TRI_UNORM ? tx.area : dot(n, v3(g.nx, g.ny, g.nz));
    const double areaPBC = dot(n, cross(B - P, C - P));
    const double areaPCA = dot(n, cross(C - P, A - P));
    const double b0 = areaPBC / areaABC;
    const double b1 = areaPCA / areaABC;
    const double b2 = 1.0 - b0 - b1;
    double u = (b0 * tx.uau + b1 * tx.ubu + b2 * tx.ucu);
    double v = (b0 * tx.uav + b1 * tx.ubv + b2 * tx.ucv);
    u = u - trunc(u);                 // fmod(u, 1.0): exact
    v = v - trunc(v);
    if (u < 0) u += 1.0;
    if (v < 0) v += 1.0;
    const int x = cvt_i32_x86(u * (double)(kp.tw));
    const int y = cvt_i32_x86(v * (double)(kp.th));
    const int m = tx.mat;
    long long index = ((long long)y * kp.tw + x) + ((long long)kp.th * kp.tw * m);
    index = index < 0 ? 0 : index;                       // reference UB -> clamp
    index = index >= kp.n_texels ? kp.n_texels - 1 : index;
    return TexRef{(int)index, m};
}
__device__ __forceinline__ TexRef tri_texel(const KParams& kp, int k, const V3 P, const V3 n)
{
    if (RT_TEX_CONST && kp.tex_const)            // every uv 0: the texel does not depend on P
        return TexRef{kp.tri_tex[k].tex0, kp.tri_tex[k].mat};
    if (RT_TEX_AFFINE && kp.tri_uv) {
        TexRef t;
        if (tri_texel_affine(kp, k, P, t)) return t;
    }
    return tri_texel_exact(kp, k, P, n);
}
__device__ __forceinline__ Mat texel_material(const KParams& kp, TexRef t)
{
    const int m = t.m;
    Mat res = load_mat(kp.texels + t.index);
    const cdptr b = kcb();
    if (m == 1) {
        res.emis = v3(1, 1, 1);
        res.es = KCV(b, KC_ES1);          // 1.85
        res.alpha = 1.0;
    }
    if (m == 4) {
        res.alpha = KCV(b, KC_A4);        // 0.6
        res.ior = KCV(b, KC_IOR4);        // 1.33
        res.rs = KCV(b, KC_RS4);          // 0.93
    }
    if (m == 3) {
        res.alpha = KCV(b, KC_A3);        // 0.1
        res.ior = KCV(b, KC_IOR3);        // 1.50
        res.rs = KCV(b, KC_RS3);          // 0.3
    }
    return res;
}
__device__ __forceinline__ Mat tri_material(const KParams& kp, int k, const V3 P, const V3 n)
{
    return texel_material(kp, tri_texel(kp, k, P, n));
}

// Sky branch of closest_hit (main.c:64-71, commented out in the reference;
// RT_SKY_LAST_SPHERE): emissionColor = sphere_uvmapping's texel (texture.h:
// 92-112), alpha = 1.  The texel index is clamped into the table (the
// reference indexes unchecked).
__device__ __forceinline__ void sky_material(const KParams& kp, int idx, const SphGeo& s, V3 hp, Mat& mat)
{
    const double ri = kp.sph_rinv[idx];
    const double dx = (hp.x - s.cx) * ri, dy = (hp.y - s.cy) * ri, dz = (hp.z - s.cz) * ri;
    const cdptr b = kcb();
    const double PI = KCV(b, KC_PI);
    const double theta = pm_acos(-dy);
    const double phi = pm_atan2(-dz, dx) + PI;
    const double u = phi / (2 * PI), v = theta / PI;
    const int x = cvt_i32_x86(u * (double)kp.sky_w);
    const int y = cvt_i32_x86(v * (double)kp.sky_h);
    long long index = (long long)y * kp.sky_w + x;
    const long long n = (long long)kp.sky_w * kp.sky_h;
    index = index < 0 ? 0 : (index >= n ? n - 1 : index);
    const DevMat* t = kp.sky + index;
    mat.emis = v3(t->dr, t->dg, t->db);
    mat.alpha = 1.0;
}

// randomDouble(-0.5, 0.5) and randomDouble(0, 1) of one 31-bit draw r
// (rtutility.h:229-231: min + (max - min) * (r / 2^31)): r / 2^31 and the
// product by 1 are exact, so the result is ONE rounding of r 2^-31 - 0.5, i.e.
// fma(r, 2^-31, -0.5), and r 2^-31 itself for [0, 1) (0.0 + u == u for u >= 0)
__device__ __forceinline__ double rand_m05(uint32_t r) { return fma((double)r, 0x1p-31, -0.5); }
__device__ __forceinline__ double rand_01(uint32_t r) { return (double)r * 0x1p-31; }

// random_dir_no_norm's vector before its normalize, rtutility.h:192-200
// (float sinf/cosf of double args), from its two 31-bit draws ru, rv:
// u = ru / 2^31 and v = rv / 2^31 are exact, so 2 PI u = ru (2 PI 2^-31)
// (one rounding of the same product) and 2 v - 1 = fma(rv, 2^-30, -1) (2 v
// exact, one rounding of the difference): the reference's values in three
// VALU fewer
__device__ __forceinline__ V3 sampler_vec(uint32_t ru, uint32_t rv)
{
    const double theta = (double)ru * 0x1.921fb54442d18p-29;      // 2*PI*u
    const double xv = fma((double)rv, 0x1p-30, -1.0);              // phi = acos(2v - 1): only (float)phi is used
    float st_, ct_, sp_, cp_;
    if (!phi_sincosf_fast(xv, sp_, cp_)) {                // uncertain rounding (~1e-4): full path
        const double phi = pm_acos(xv);
        pm_sincosf((float)phi, sp_, cp_);
    }
    pm_sincosf((float)theta, st_, ct_);
    return v3((double)(ct_ * sp_), (double)(st_ * sp_), (double)cp_);
}

// random_dir_no_norm, rtutility.h:189-203
template <bool COUNT>
__device__ __forceinline__ V3 random_dir(Stream& st, Cnt& cnt)
{
    if (COUNT) cnt.c[RT_CNT_SHADE] += 1;
    const uint32_t ru = st.next31();
    const uint32_t rv = st.next31();
    const V3 dir = sampler_vec(ru, rv);
    return normalize_unit(dir);
}

// refracted_vec, rtutility.h:210-227 (indices squared: reference quirk)
__device__ __forceinline__ V3 refracted(V3 v, V3 nrm, double n1, double n2)
{
    n1 *= n1;
    n2 *= n2;
    const double cn = dot(nrm, v);
    const double radical = 1 - ((n1 / n2) * (n1 / n2)) * (1 - (cn * cn));
    if (radical > 0) {
        const V3 comp_tan = muls(v - muls(nrm, dot(v, nrm)), (n1 / n2));
        const V3 comp_normal = muls(v3(-nrm.x, -nrm.y, -nrm.z), sqrt(radical));
        return comp_tan + comp_normal;
    }
    return v - muls(nrm, 2 * dot(v, nrm));
}

// rgb_to_hsl / hsl_to_rgb round trip, rtutility.h:81-165 (main.c:155-158)
__device__ __forceinline__ double hue_to_rgb(double t1, double t2, double hue)
{
    if (hue < 0.0) hue += 1.0;
    if (hue > 1.0) hue -= 1.0;
    if (6.0 * hue < 1.0) return t1 + (t2 - t1) * 6.0 * hue;
    if (2.0 * hue < 1.0) return t2;
    if (3.0 * hue < 2.0) return t1 + (t2 - t1) * (KCV(kcb(), KC_TWO_THIRDS) - hue) * 6.0;
    return t1;
}
// CU: main_cuda.cu:92-93 raise L and S by 1.20 (main.c:156-157: x1.0)
template <bool CU = false>
__device__ __forceinline__ V3 hsl_roundtrip(V3 rgb)
{
    const double r = rgb.x, g = rgb.y, b = rgb.z;
    const double mx = (r > g) ? ((r > b) ? r : b) : ((g > b) ? g : b);
    const double mn = (r < g) ? ((r < b) ? r : b) : ((g < b) ? g : b);
    double h = 0.0, s, l = (mx + mn) / 2.0;
    if (mx == mn) {
        h = 0.0;
        s = 0.0;
    } else {
        const double d = mx - mn;
        s = (l < 0.5) ? (d / (mx + mn)) : (d / (2.0 - mx - mn));
        if (mx == r) h = (g - b) / d + ((g < b) ? 6.0 : 0.0);
        else if (mx == g) h = (b - r) / d + 2.0;
        else if (mx == b) h = (r - g) / d + 4.0;
        h /= 6.0;
    }
    l *= CU ? 1.20 : 1.0;
    s *= CU ? 1.20 : 1.0;
    if (s == 0.0) return v3(l, l, l);
    const double t2 = (l < 0.5) ? (l * (1.0 + s)) : (l + s - l * s);
    const double t1 = 2.0 * l - t2;
    const double third = KCV(kcb(), KC_THIRD);                 // 1.0 / 3.0
    return v3(hue_to_rgb(t1, t2, h + third), hue_to_rgb(t1, t2, h), hue_to_rgb(t1, t2, h - third));
}

// ambient_occlusion, main.c:94-116: one cast, only distance/dst matters.
template <bool COUNT, bool BVH, bool CU = false>
__device__ __forceinline__ double ao_factor(const KParams& kp, const V3 p, const V3 n, double AO, Stream& st,
                                            Cnt& cnt)
{
    const V3 rd = random_dir<COUNT>(st, cnt);
    const V3 dir = normalize(n + rd);
    double t;
    int idx;
    const int kind = closest_hit<COUNT, BVH, CU>(kp, p, dir, t, idx, cnt);
    double occ = 0.0;
    if (kind != HIT_NONE) {
        const V3 hp = p + muls(dir, t);
        const V3 df = hp - p;
        const double distance = sqrt(dot(df, df));
        double att = distance / t;
        att = pm_pow(att, AO);
        occ = occ + att;
    }
    return (occ / 1.0) / AO;
}

// tracer, main_cuda.cu:86-141 (rt.h RT_SEM_CUDA).  A pre-pass cast returns
// emitters (HSL round trip, L and S x1.20) and misses (zeros); the bounce
// loop starts again from the same ray, so its first cast reuses the pre-pass
// hit (the COUNT build recasts it, to count what main_cuda.cu casts); no
// alpha holes, refraction, textures or x1.3 brightening; a triangle's
// material is its own (kp.tri_mat); albedo/normal are the pre-pass hit's.
template <bool COUNT, bool BVH>
__device__ __forceinline__ bool cuda_hit(const KParams& kp, const V3 o, const V3 d, V3& hp, V3& hn, Mat& mat,
                                         Cnt& cnt)
{
    double t;
    int idx;
    const int kind = closest_hit<COUNT, BVH, true>(kp, o, d, t, idx, cnt);
    if (kind == HIT_NONE) return false;
    hp = o + muls(d, t);                                 // ray_at
    if (kind == HIT_SPHERE) {
        const SphGeo s = kp.sph[idx];
        hn = normalize(hp - v3(s.cx, s.cy, s.cz));   // sphere.hu:31,40
        mat = load_mat(kp.sph_mat + idx);
    } else {
        hn = tri_normal(kp, idx);                        // triangle.hu:266
        mat = load_mat(kp.tri_mat + idx);
    }
    return true;
}

template <bool COUNT, bool BVH>
__device__ __forceinline__ void trace_cuda(const KParams& kp, V3 o, V3 d, Stream& st, double* acc, Cnt& cnt)
{
    V3 hp, hn;
    Mat mat;
    if (!cuda_hit<COUNT, BVH>(kp, o, d, hp, hn, mat, cnt)) {    // return BLACK
        acc_add(acc, ACC_RAD, v3(0, 0, 0));
        acc_add(acc, ACC_ALB, v3(0, 0, 0));
        acc_add(acc, ACC_NRM, v3(0, 0, 0));
        return;
    }
    if (mat.es > 0) {
        const V3 col = hsl_roundtrip<true>(mat.emis);
        acc_add(acc, ACC_RAD, col);
        acc_add(acc, ACC_ALB, col);
        acc_add(acc, ACC_NRM, hn);
        return;
    }
    acc_add(acc, ACC_ALB, mat.diff);                     // the outer hitInfo, main_cuda.cu:140
    acc_add(acc, ACC_NRM, hn);
    V3 inc = v3(0, 0, 0), rc = v3(1, 1, 1);
    for (int i = 0; i < kp.B; i++) {
        if ((i > 0 || COUNT) && !cuda_hit<COUNT, BVH>(kp, o, d, hp, hn, mat, cnt)) break;
        o = hp;
        const V3 diffuse_dir = normalize(hn + random_dir<COUNT>(st, cnt));
        const V3 reflected_dir = d - muls(hn, 2 * dot(d, hn));
        d = diffuse_dir + muls(reflected_dir - diffuse_dir, mat.rs);   // vec3_lerp, rtutility.hu:31-35
        if (kp.useAO) {
            const double AO = ((cdptr)kp.uni)[opq0() + U_AO];
            const V3 em = muls(mat.emis, mat.es * 1.5 * AO);
            inc = inc + mulv(em, rc);
            rc = mulv(mat.diff, rc);
            const double occ = ao_factor<COUNT, BVH, true>(kp, hp, hn, AO, st, cnt);
            rc = mulv(rc, v3(occ, occ, occ));
        } else {
            const V3 em = muls(mat.emis, mat.es);
            inc = inc + mulv(em, rc);
            rc = mulv(mat.diff, rc);
        }
    }
    acc_add(acc, ACC_RAD, inc);
}

// write_color_canva, rtutility.h:56-71 (sqrtf of the float-rounded product)
__device__ __forceinline__ double resolve(double sum, double rapport)
{
    double r = (double)sqrtf((float)(rapport * sum));
    r = r < 0.0 ? 0.0 : (r > 0.999 ? 0.999 : r);
    return (double)cvt_i32_x86(256 * r);
}

__device__ __forceinline__ void store3(double* base, long long i, V3 v)
{
    base[3 * i + 0] = v.x;
    base[3 * i + 1] = v.y;
    base[3 * i + 2] = v.z;
}

__device__ __forceinline__ void write_pixel(const KParams& kp, long long li, V3 srad, V3 salb, V3 snrm)
{
    const double rapport = 1.0 / kp.S;
    store3(kp.canva, li, v3(resolve(srad.x, rapport), resolve(srad.y, rapport), resolve(srad.z, rapport)));
    const double S = (double)kp.S;
    if (kp.albedo) store3(kp.albedo, li, divs(salb, S));
    if (kp.normal) store3(kp.normal, li, divs(snrm, S));
    if (kp.radiance) store3(kp.radiance, li, divs(srad, S));
}

// Primary ray of sample st (main.c:258-270; camera.h:42-55 get_ray).
// The four camera draws of a sample (draws 0-3: word n of Philox block 0)
// from registers, for a camera ray computed ahead of its path
// (render_kernel_q): the lane's LDS block cache stays with the path in flight.
struct CamDraws {
    Philox b;
    int n;
    __device__ __forceinline__ uint32_t next31()
    {
        const uint32_t w = n == 0 ? b.w0 : n == 1 ? b.w1 : n == 2 ? b.w2 : b.w3;
        ++n;
        return w >> 1;
    }
};

template <bool CU, class ST>
__device__ __forceinline__ void camera_ray(const KParams& kp, int x, int g, ST& st, V3& no, V3& rd)
{
    const double ju = rand_m05(st.next31());     // randomDouble(-0.5, 0.5)
    const double jv = rand_m05(st.next31());
    const double jx = rand_m05(st.next31());
    const double jy = rand_m05(st.next31());
    const int b = opq0();
    const cdptr U = (cdptr)kp.uni;
    // main.c:265-266; main_cuda.cu:152-153 adds 0.5 first
    // (x + ju) / (W - 1): the numerators are 0 or of magnitude >= 2^-31 and
    // the divisors in [1, 2^31], inside div_core's exact range
    const double nu = CU ? (double)x + 0.5 + ju : (double)x + ju;
    const double nv = CU ? (double)g + 0.5 + jv : (double)g + jv;
    const double rcw = U[b + U_RC_WM1], rch = U[b + U_RC_HM1];
    const double u = rcw != 0.0 ? div_core(nu, U[b + U_WM1], rcw) : nu / U[b + U_WM1];
    const double v = rch != 0.0 ? div_core(nv, U[b + U_HM1], rch) : nv / U[b + U_HM1];
    const double dx = jx * U[b + U_OX], dy = jy * U[b + U_OY];
    // get_ray, camera.h:42-55
    const V3 co = v3(U[b + U_CAM_O], U[b + U_CAM_O + 1], U[b + U_CAM_O + 2]);
    const V3 ch = v3(U[b + U_CAM_H], U[b + U_CAM_H + 1], U[b + U_CAM_H + 2]);
    const V3 cv = v3(U[b + U_CAM_V], U[b + U_CAM_V + 1], U[b + U_CAM_V + 2]);
    const V3 cc = v3(U[b + U_CAM_C], U[b + U_CAM_C + 1], U[b + U_CAM_C + 2]);
    const V3 dir = cc + (muls(ch, u) + (muls(cv, v) - co));
    const V3 dest = co + muls(dir, U[b + U_FOCUS]);
    no = co + v3(dx, dy, 0);
    rd = normalize(dest - no);
}

// Resumable trace for the BVH kernel: the same tracer and
// ambient_occlusion arithmetic (main.c:94-242), as a per-lane state
// machine (LanePath).  A lane in
//   SM_RESOLVE shades the hit of its finished cast (a bounce or an AO cast),
//   SM_CAM     starts its next sample (or is done),
//   SM_CAST    runs the sphere half of the next cast and sets up traversal,
//   SM_TRAV    visits nodes of the triangle BVH,
// and a lane's casts, draws and sums happen in the same order as in tracer,
// so results are bit-identical.  samples_coop runs it (the fixed-grid BVH
// kernel: spp_chunks 1, trees too deep for the queue kernel's stacks); r01's
// samples_sm (each lane at most 4 node visits per round) is superseded by the
// queue kernel's resumable walks (render_kernel_q<.., QB>).
enum : int { SM_RESOLVE = 0, SM_CAM = 1, SM_CAST = 2, SM_TRAV = 3, SM_DONE = 4 };

// AOM: AO compiled out (0), always on (1), or read from kp.useAO (2); the
// queue kernel is instantiated per AO setting so a sphere scene without AO
// carries neither the AO cast's state nor its code.
enum : int { AO_OFF = 0, AO_ON = 1, AO_RUNTIME = 2 };

template <bool COUNT, bool SKY, int AOM = AO_RUNTIME>
struct LanePath {
    Stream st;
    V3 o, d, cd;                                 // ray, next bounce direction, current cast's direction
    V3 inc, rc;
    Ray32 r32;                                   // the cast's single-precision slab set-up (BVH)
    double top_n2, best;
    int i, kind, win, win_orig, node, sp, s, state;
    bool chain, ao_cast;

    // Zero-throughput exit (kp.zero_exit, set by the host only when it is
    // exact): once rayColor is (0, 0, 0) every later bounce adds em * 0 = +-0
    // to incomingLight (x + +-0 == x: incomingLight starts at +0 and is never
    // -0), multiplies rayColor by a finite diffuse colour or AO factor (still
    // 0), and chain (albedo/normal) is already off, since rayColor only
    // changes after it is cleared.  Draws are counter-based per sample, so
    // skipping the rest of the path changes no other sample.  The host
    // requires every emission, strength and diffuse value finite with
    // |x| <= 2^100 (no em overflow), and with AO 0 < AO_intensity <= 1000
    // and every coordinate within 2^20 (the AO factor pow(distance/dst, AO)/AO
    // then stays finite: distance/dst <= 1.02).
    __device__ __forceinline__ bool zero_rc(const KParams& kp) const
    {
        return kp.zero_exit && rc.x == 0.0 && rc.y == 0.0 && rc.z == 0.0;
    }

    __device__ __forceinline__ void init(int s0, int s1)
    {
        o = d = cd = inc = rc = v3(0, 0, 0);
        r32 = Ray32{0, 0, 0, 0, 0, 0, 0, 0, 0};
        top_n2 = 1.0;
        best = 0.0;
        i = 0; kind = HIT_NONE; win = -1; win_orig = 0; node = 0; sp = 0;
        chain = true;
        ao_cast = false;
        s = s0;
        state = s0 < s1 ? SM_CAM : SM_DONE;
    }

    // tracer's bounce body after the cast (main.c:127-241), or
    // ambient_occlusion's tail (main.c:104-115) for an AO cast
    __device__ __forceinline__ void resolve(const KParams& kp, double* acc, Cnt& cnt)
    {
        if (COUNT) wave_slots(cnt, RT_CNT_SHADE_LANE_SLOTS);
        bool more = true;                    // the path goes on to bounce i + 1
        bool add_inc = true;                 // false: direct view of a light (tracer returns early)
        st.k0 = kp.key0;                     // the key from the kernel argument (uniform), not
        st.k1 = kp.key1;                     // a loop-carried copy
        const bool use_ao = AOM == AO_RUNTIME ? kp.useAO != 0 : AOM == AO_ON;
        if (AOM != AO_OFF && ao_cast) {
            // ambient_occlusion's tail, main.c:104-115
            const double AO = ((cdptr)kp.uni)[opq0() + U_AO];
            double occ = 0.0;
            if (kind != HIT_NONE) {
                const V3 hp = o + muls(cd, best);
                const V3 df = hp - o;
                const double distance = sqrt(dot(df, df));
                double att = distance / best;
                att = pm_pow(att, AO);
                occ = occ + att;
            }
            occ = (occ / 1.0) / AO;
            rc = mulv(rc, v3(occ, occ, occ));
            ao_cast = false;
            if (zero_rc(kp)) more = false;   // an AO miss zeroes rayColor: nothing more to add
        } else if (kind == HIT_NONE) {       // miss: the path ends, main.c:236-238
            if (chain) {
                acc_add(acc, ACC_ALB, v3(0, 0, 0));
                acc_add(acc, ACC_NRM, v3(0, 0, 0));
            }
            more = false;
        } else {
            V3 hp, hn;
            Mat mat;
            if (kind == HIT_SPHERE) {
                const SphGeo sg = kp.sph[win];
                hp = o + muls(d, best);
                hn = normalize(hp - v3(sg.cx, sg.cy, sg.cz));
                mat = load_mat(kp.sph_mat + win);
                if (SKY && win == kp.ns - 1) sky_material(kp, win, sg, hp, mat);
            } else {
                if (COUNT) cnt.c[RT_CNT_TEX_HITS] += 1;
                hp = o + muls(d, best);
                hn = tri_normal(kp, win);
                mat = tri_material(kp, win, hp, hn);
            }
            bool lit = false;
            if (chain) {
                if (mat.es > 0) {
                    const V3 col = hsl_roundtrip(mat.emis);
                    acc_add(acc, ACC_RAD, col);
                    acc_add(acc, ACC_ALB, col);
                    acc_add(acc, ACC_NRM, hn);
                    lit = true;
                } else if (!(mat.alpha < 0.0001) || i == kp.B - 1) {
                    acc_add(acc, ACC_ALB, mat.diff);
                    acc_add(acc, ACC_NRM, hn);
                    chain = mat.alpha < 0.0001;
                }
            }
            if (lit) {
                more = false;
                add_inc = false;
            } else {
                o = hp;
                const V3 diffuse_dir = normalize(hn + random_dir<COUNT>(st, cnt));
                const V3 reflected_dir = d - muls(hn, 2 * dot(d, hn));
                const V3 dr = diffuse_dir + muls(reflected_dir - diffuse_dir, mat.rs);
                bool shade = !(mat.alpha < 0.0001);  // not an alpha hole (main.c:200-206)
                if (shade) {
                    chain = false;
                    if (mat.alpha <= 0.99) {
                        if (COUNT) cnt.c[RT_CNT_REFRACT] += 1;
                        V3 nn = hn;
                        double n1, n2;
                        if (dot(d, hn) > 0) {
                            nn = v3(-hn.x, -hn.y, -hn.z);
                            n1 = mat.ior;
                            n2 = top_n2;
                        } else {
                            n1 = top_n2;
                            n2 = mat.ior;
                            top_n2 = mat.ior;
                        }
                        const V3 refr = refracted(d, nn, n1, n2);
                        const double rnd = rand_01(st.next31());
                        if (rnd > mat.alpha) {
                            d = refr;
                            shade = false;
                        } else {
                            d = dr;
                        }
                    } else {
                        d = dr;
                    }
                }
                if (shade) {
                    V3 r = rc;
                    if (use_ao) {
                        const double AO = ((cdptr)kp.uni)[opq0() + U_AO];
                        const V3 em = muls(mat.emis, mat.es * 1.5 * AO);
                        inc = inc + mulv(em, r);
                        if (any_above_half(r)) r = mulv(mat.diff, muls(r, 1.3));
                        rc = mulv(mat.diff, r);
                        // ambient_occlusion's cast (main.c:96-103): from hp along n + random
                        cd = normalize(hn + random_dir<COUNT>(st, cnt));
                        ao_cast = true;
                    } else {
                        const V3 em = muls(mat.emis, mat.es);
                        inc = inc + mulv(em, r);
                        if (any_above_half(r)) r = mulv(mat.diff, muls(r, 1.3));
                        rc = mulv(mat.diff, r);
                    }
                    if (zero_rc(kp)) {           // black diffuse (a light, a green-then-red wall)
                        ao_cast = false;         // the AO cast could only scale 0
                        more = false;
                    }
                }
            }
        }
        if (AOM != AO_OFF && ao_cast) {
            state = SM_CAST;
        } else {
            if (more) {
                ++i;
                more = i < kp.B;
            }
            if (more) {
                cd = d;
                state = SM_CAST;
            } else {
                if (add_inc) acc_add(acc, ACC_RAD, inc);
                if (COUNT) {
                    cnt.c[RT_CNT_SAMPLES] += 1;
                    cnt.c[RT_CNT_RNG_DRAWS] += st.n;
                }
                ++s;
                state = SM_CAM;
            }
        }
    }

    // the next sample's primary ray (fill_canva's sample loop, main.c:258-270)
    __device__ __forceinline__ void start(const KParams& kp, int x, int g, uint32_t pixel, int s1, uint32_t* rng,
                                          double* acc, Cnt& cnt)
    {
        if (s >= s1) {
            state = SM_DONE;
        } else {
            st.start(pixel, (uint32_t)(kp.s_base + s), kp.key0, kp.key1, rng);
            camera_ray<false>(kp, x, g, st, o, d);
            cd = d;
            inc = v3(0, 0, 0);
            rc = v3(1, 1, 1);
            top_n2 = 1.0;
            i = 0;
            chain = true;
            ao_cast = false;
            if (kp.B <= 0) {                 // tracer returns (0, 0, 0) albedo/normal
                acc_add(acc, ACC_ALB, v3(0, 0, 0));
                acc_add(acc, ACC_NRM, v3(0, 0, 0));
                acc_add(acc, ACC_RAD, inc);
                if (COUNT) {
                    cnt.c[RT_CNT_SAMPLES] += 1;
                    cnt.c[RT_CNT_RNG_DRAWS] += st.n;
                }
                ++s;
            } else {
                state = SM_CAST;
            }
        }
    }

    // the whole cast in one go (spheres, then brute-force triangles or the
    // lane's own BVH walk)
    template <bool BVH = false>
    __device__ __forceinline__ void cast_flat(const KParams& kp, Cnt& cnt)
    {
        kind = closest_hit<COUNT, BVH>(kp, o, cd, best, win, cnt);
        state = SM_RESOLVE;
    }

    // start() for a camera ray computed ahead (draws 0-3 of sample s used):
    // the path's stream resumes at draw 4 (Philox block 1)
    __device__ __forceinline__ void begin(const KParams& kp, uint32_t pixel, V3 no, V3 rd, uint32_t* rng, double* acc,
                                          Cnt& cnt)
    {
        st.start(pixel, (uint32_t)(kp.s_base + s), kp.key0, kp.key1, rng);
        st.n = 4;
        o = no;
        d = rd;
        cd = rd;
        inc = v3(0, 0, 0);
        rc = v3(1, 1, 1);
        top_n2 = 1.0;
        i = 0;
        chain = true;
        ao_cast = false;
        state = SM_CAST;                 // kp.B > 0 (the queue kernel's prefetch is off otherwise)
    }

    // closest_hit's sphere half and the traversal set-up
    __device__ __forceinline__ void cast(const KParams& kp, Cnt& cnt)
    {
        win = cast_spheres<COUNT, false>(kp, o, cd, best, cnt);
        kind = win >= 0 ? HIT_SPHERE : HIT_NONE;
        win_orig = 0;
        if (kp.bvh) r32 = ray32(kp, o, cd);
        node = 0;
        sp = 0;
        state = SM_TRAV;
    }

    // up to k node visits; RESOLVE when the traversal is over
    __device__ __forceinline__ void trav(const KParams& kp, unsigned short* stk, int k, Cnt& cnt)
    {
#pragma unroll 1
        for (int j = 0; j < k; ++j) {
            if (!bvh_step<COUNT, false>(kp, o, cd, r32, stk, node, sp, best, kind, win, win_orig, cnt)) {
                state = SM_RESOLVE;
                break;
            }
        }
    }
};



// The fixed-grid sphere kernel's sample loop as LanePath rounds: each
// round every lane with a path casts and shades one bounce; a lane whose path
// ended (a miss, a light seen directly, the bounce budget, or zero
// throughput) waits for its next sample's camera ray, which starts once
// RT_FLAT_FILL eighths of the wave's live lanes wait (the camera ray then
// costs the wave one pass for many lanes).  Same casts, draws and sums per
// sample as tracer, so bit-identical; it lets the zero-throughput exit
// save the cast instead of idling the lane until the wave's longest path.
template <bool COUNT, bool SKY>
__device__ __forceinline__ void samples_flat(const KParams& kp, int x, int g, uint32_t pixel, int s0, int s1,
                                             uint32_t* rng, double* acc, Cnt& cnt)
{
    LanePath<COUNT, SKY> L;
    L.init(s0, s1);
    while (L.state != SM_DONE) {
        const unsigned long long live = __ballot(1), wait = __ballot(L.state == SM_CAM);
        const bool go = wait == live || __popcll(wait) * 8 >= __popcll(live) * RT_FLAT_FILL;
        if (go && L.state == SM_CAM) L.start(kp, x, g, pixel, s1, rng, acc, cnt);
        if (L.state == SM_CAST) {
            L.cast_flat(kp, cnt);
            L.resolve(kp, acc, cnt);
        }
    }
}

// Wave-cooperative traversal of the deep casts (fixed-grid BVH kernel).  About 5 %
// of C4's casts go below the tree's root; walked by their own lanes they
// keep a wave at a few active lanes for ~25 node visits and ~12 triangle
// tests (leaf loop 2.6 % lane efficiency).  Here a lane runs its cast's root
// node itself; a deeper cast parks (SM_TRAV) and once RT_BVH_COOP lanes of
// the wave are parked (or nothing else can move) every live lane of the wave
// works on their subtrees: a task is (ray, node); a lane walks its task
// depth-first with its own LDS stack and hands siblings to a per-wave LIFO
// (so idle lanes pick them up) while that holds fewer than 64 entries.  The
// ray is read from its owner lane (ds_bpermute); triangle hits are merged
// into the owner's record in a wave-uniform loop with the same rule as
// tri_test (strictly closer, or an equal-dst triangle with a smaller caller
// index; a sphere keeps an equal-dst hit).  That rule is a total order, so
// the winner is the one tracer finds, whatever order the triangles are
// tested in; culling against an older `best` only tests more boxes.
__device__ __forceinline__ double rl_d(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double shfl_d(double v, int src)
{
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)b, src, 64), hi = __shfl((int)(b >> 32), src, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long lanes_below() { return (1ull << (threadIdx.x & 63)) - 1ull; }

// Append each lane's n (0..4) items to the wave's LIFO (cnt: wave-uniform).
__device__ __forceinline__ void lifo_push(volatile unsigned* q, int& cnt, int n, const unsigned* it)
{
    unsigned long long b[4];
    int base = cnt, tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = __ballot(n > j);
    int off = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        off += __popcll(b[j] & lanes_below());
        tot += __popcll(b[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < n) q[base + off + j] = it[j];
    cnt = base + tot;
    __builtin_amdgcn_wave_barrier();
}

// One node visit of a cooperative task: as bvh_step, but hit internal
// children other than the next one go to push[] (for the LIFO) when
// to_lifo, else on the lane's own stack.  hit: a triangle beat the record.
template <bool COUNT>
__device__ __forceinline__ bool coop_step(const KParams& kp, const V3 o, const V3 d, const Ray32& r32,
                                          unsigned short* stk, int& node, int& sp, double& best, int& kind,
                                          int& win, int& win_orig, bool& hit, bool to_lifo, unsigned* push,
                                          int& npush, Cnt& cnt)
{
    const BvhNode4* nd = kp.bvh + node;
    if (COUNT) {
        cnt.c[RT_CNT_BVH_NODES] += 1;
        wave_slots(cnt, RT_CNT_BVH_LANE_SLOTS);
    }
    bool h[4];
    float tn[4];
    int Ch[4], Cn[4];
    box4(kp, nd, r32, cull32(kp, best), h, tn, Ch, Cn);
    int next = -1;
    float tnext = 0.0f;
    unsigned lm = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (!h[c]) continue;
        const int ch = nd->child[c], n = nd->count[c];
        if (n > 0) {
            lm |= 1u << c;
        } else if (next < 0) {
            next = ch;
            tnext = tn[c];
        } else {
            int pu = ch;
            if (tn[c] < tnext) {
                pu = next;
                next = ch;
                tnext = tn[c];
            }
            if (to_lifo) {
                push[npush] = (unsigned)pu;
                ++npush;
            } else {
                if (COUNT && sp >= kp.stack_cap) cnt.c[RT_CNT_BVH_STACK_OVER] += 1;
                if (!COUNT || sp < kStack4) {
                    stk[sp * 256] = (unsigned short)pu;
                    ++sp;
                }
            }
        }
    }
    int k = 0, kend = 0;
    while (lm != 0u || k < kend) {
        if (COUNT) wave_slots(cnt, RT_CNT_LEAF_LANE_SLOTS);
        if (k >= kend) {
            const int c = __ffs(lm) - 1;
            lm &= lm - 1u;
            k = nd->child[c];
            kend = k + nd->count[c];
            if (COUNT) cnt.c[RT_CNT_BVH_TRI_TESTS] += (unsigned long long)(kend - k);
        }
        const int w0 = win, k0 = kind;
        tri_test<COUNT, false>(kp, k, o, d, best, kind, win, win_orig);
        hit = hit || win != w0 || kind != k0;
        ++k;
    }
    if (next >= 0) {
        node = next;
        return true;
    }
    if (sp == 0) return false;
    --sp;
    node = stk[sp * 256];
    return true;
}

template <bool COUNT, bool SKY>
__device__ __forceinline__ void samples_coop(const KParams& kp, int x, int g, uint32_t pixel, int s0, int s1,
                                             uint32_t* rng, double* acc, Cnt& cnt)
{
    constexpr int QW = 256;                      // < 64 entries + 3 pushes x 64 lanes
    __shared__ unsigned lifo_lds[4][QW];
    volatile unsigned* q = lifo_lds[threadIdx.x >> 6];
    unsigned short* stk = bvh_stack();
    const int lane = threadIdx.x & 63;
    LanePath<COUNT, SKY> L;
    L.init(s0, s1);
    while (L.state != SM_DONE) {
        if (L.state == SM_RESOLVE) L.resolve(kp, acc, cnt);
        if (L.state == SM_CAM) L.start(kp, x, g, pixel, s1, rng, acc, cnt);
        if (L.state == SM_CAST) {
            L.cast(kp, cnt);
            L.trav(kp, stk, 1, cnt);             // the root node; SM_TRAV: parked
        }
        const unsigned long long parked = __ballot(L.state == SM_TRAV);
        const unsigned long long movable = __ballot(L.state == SM_RESOLVE || L.state == SM_CAM);
        if (parked == 0ull || (__popcll(parked) < RT_BVH_COOP && movable != 0ull)) continue;

        // ---- cooperative phase (wave-uniform) ----
        int qn = 0;
        {
            unsigned it[4];
            int n = 0;
            if (L.state == SM_TRAV) {            // next node + the root's pushes (sp <= 3)
                it[0] = (unsigned)lane | ((unsigned)L.node << 6);
                for (int j = 0; j < L.sp; ++j) it[1 + j] = (unsigned)lane | ((unsigned)stk[j * 256] << 6);
                n = 1 + L.sp;
            }
            lifo_push(q, qn, n, it);
        }
        bool has = false;
        int tr = 0, tnode = 0, tsp = 0;
        V3 to = v3(0, 0, 0), td = to;
        Ray32 tr32 = Ray32{0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (;;) {
            const unsigned long long idle = __ballot(!has);
            const int take = min(__popcll(idle), qn);
            bool fresh = false;
            if (!has) {
                const int rank = __popcll(idle & lanes_below());
                if (rank < take) {
                    const unsigned item = q[qn - 1 - rank];
                    tr = (int)(item & 63u);
                    tnode = (int)(item >> 6);
                    tsp = 0;
                    has = true;
                    fresh = true;
                }
            }
            qn -= take;
            __builtin_amdgcn_wave_barrier();
            if (__ballot(has) == 0ull) break;
            // the owner's ray for new tasks, its current record for every task
            // (all live lanes run the permutes; owners are live)
            if (__ballot(fresh) != 0ull) {
                const V3 ro = v3(shfl_d(L.o.x, tr), shfl_d(L.o.y, tr), shfl_d(L.o.z, tr));
                const V3 rd = v3(shfl_d(L.cd.x, tr), shfl_d(L.cd.y, tr), shfl_d(L.cd.z, tr));
                if (fresh) {
                    to = ro;
                    td = rd;
                    tr32 = ray32(kp, ro, rd);
                }
            }
            double best = shfl_d(L.best, tr);
            int kind = __shfl(L.kind, tr, 64), win = __shfl(L.win, tr, 64), win_orig = __shfl(L.win_orig, tr, 64);
            bool hit = false;
            unsigned push[3];
            int npush = 0;
            const bool to_lifo = qn < 64;
            if (has) {
                if (!coop_step<COUNT>(kp, to, td, tr32, stk, tnode, tsp, best, kind, win, win_orig, hit, to_lifo,
                                      push, npush, cnt))
                    has = false;
#pragma unroll
                for (int j = 0; j < 3; ++j) push[j] = (unsigned)tr | (push[j] << 6);
            }
            lifo_push(q, qn, npush, push);
            // merge the lanes' better triangles into their owners' records
            unsigned long long m = __ballot(hit);
            while (m != 0ull) {
                const int l = __ffsll(m) - 1;
                m &= m - 1ull;
                const int r = __builtin_amdgcn_readlane(tr, l);
                const double db = rl_d(best, l);
                const int dw = __builtin_amdgcn_readlane(win, l), dorig = __builtin_amdgcn_readlane(win_orig, l);
                if (lane == r && (db < L.best || (db == L.best && L.kind == HIT_TRI && dorig < L.win_orig))) {
                    L.best = db;
                    L.kind = HIT_TRI;
                    L.win = dw;
                    L.win_orig = dorig;
                }
            }
        }
        if (L.state == SM_TRAV) L.state = SM_RESOLVE;
    }
}

// n / d and n % d for 32-bit n by a launch-constant d with m = kp's
// floor((2^32 - 1) / d) (host, qdiv_magic): the high product is q or q - 1,
// one remainder check fixes it (5 integer ops instead of a division).
__device__ __forceinline__ unsigned udiv_q(unsigned n, unsigned d, unsigned m, unsigned& r)
{
    unsigned q = __umulhi(n, m);
    const unsigned rr = n - q * d;
    const bool up = rr >= d;
    r = up ? rr - d : rr;
    return up ? q + 1u : q;
}

// First sample of chunk c, rt.h rt_chunk_bound: w(c)*S/den with w(c) = c
// (den = P) or the tapered weights (den = (P - L) 2^L + 2^L - 1); 32-bit magic
// division when (den + 1) * S < 2^32 (qm_chunks != 0), else 64-bit.
__device__ __forceinline__ int chunk_start(int S, int chunks, int taper, unsigned den, unsigned qm_chunks, unsigned c)
{
    unsigned w = c;
    if (taper) {                     // L = taper levels: weights 2^L x E, then 2^(L-1) .. 1
        const unsigned E = (unsigned)chunks - (unsigned)taper, one = 1u << taper;
        w = c <= E ? c << taper : (E << taper) + one - (one >> (c - E));
    }
    if (qm_chunks != 0u) {
        unsigned r;
        return (int)udiv_q(w * (unsigned)S, den, qm_chunks, r);
    }
    return (int)(((long long)w * S) / den);
}

// Body of render_kernel (main.c semantics) and render_kernel_cuda
// (main_cuda.cu's): one thread = (pixel, chunk of its samples).
template <bool COUNT, bool BVH, bool SKY, bool CU>
__device__ __forceinline__ void render_body(const KParams& kp)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = kp.band_y0 + blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int chunk = blockIdx.z;
    Cnt cnt;
    if (COUNT)
        for (int k = 0; k < RT_NCOUNTERS; ++k) cnt.c[k] = 0;
    bool valid = x < kp.W && ly < kp.local_rows && ly < kp.band_y0 + kp.band_rows;
    int g = 0;
    if (valid) {
        const int lt = ly / kp.tile_rows, yy = ly - lt * kp.tile_rows;
        g = kp.row_base + (kp.tile_first + lt * kp.tile_step) * kp.tile_rows + yy;
        valid = g < kp.row_end;
    }
    if (valid) {
        const uint32_t pixel = (uint32_t)g * (uint32_t)kp.W + (uint32_t)x;
        const int s0 = chunk_start(kp.S, kp.chunks, kp.chunk_taper, kp.chunk_den, 0u, (unsigned)chunk);
        const int s1 = chunk_start(kp.S, kp.chunks, kp.chunk_taper, kp.chunk_den, 0u, (unsigned)chunk + 1u);
        __shared__ double acc_lds[ACC_SLOTS * 256];
        __shared__ uint32_t rng_lds[4 * 256];
        double* acc = acc_lds + threadIdx.x;
        const long long li = (long long)ly * kp.W + x;
        // accumulate mode with one chunk continues the running sums in sample
        // order (fill_canva's fold, carried across launches); otherwise 0
        const bool carry = !COUNT && kp.sums && kp.chunks == 1;
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[j * 256] = carry ? kp.sums[li * 9 + j] : 0.0;
        if constexpr (BVH && !CU) {
            samples_coop<COUNT, SKY>(kp, x, g, pixel, s0, s1, rng_lds + threadIdx.x, acc, cnt);
        } else if constexpr (!BVH && !CU) {
            samples_flat<COUNT, SKY>(kp, x, g, pixel, s0, s1, rng_lds + threadIdx.x, acc, cnt);
        } else {                             // CU: main_cuda.cu's nested sample loop (main_cuda.cu:150-165)
            for (int s = s0; s < s1; ++s) {
                Stream st;
                st.start(pixel, (uint32_t)(kp.s_base + s), kp.key0, kp.key1, rng_lds + threadIdx.x);
                V3 no, rd;
                camera_ray<CU>(kp, x, g, st, no, rd);
                trace_cuda<COUNT, BVH>(kp, no, rd, st, acc, cnt);
                if (COUNT) {
                    cnt.c[RT_CNT_SAMPLES] += 1;
                    cnt.c[RT_CNT_RNG_DRAWS] += st.n;
                }
            }
        }
        if (!COUNT) {
            const V3 srad = v3(acc[0], acc[256], acc[512]);
            const V3 salb = v3(acc[768], acc[1024], acc[1280]);
            const V3 snrm = v3(acc[1536], acc[1792], acc[2048]);
            if (carry) {
#pragma unroll
                for (int j = 0; j < 9; ++j) kp.sums[li * 9 + j] = acc[j * 256];
            } else if (kp.chunks == 1) {
                write_pixel(kp, li, srad, salb, snrm);
            } else {
                double* p = kp.partial + ((long long)chunk * kp.band_rows * kp.W +
                                          ((long long)(ly - kp.band_y0) * kp.W + x)) * 9;
                p[0] = srad.x; p[1] = srad.y; p[2] = srad.z;
                p[3] = salb.x; p[4] = salb.y; p[5] = salb.z;
                p[6] = snrm.x; p[7] = snrm.y; p[8] = snrm.z;
            }
        }
    }
    if (COUNT) {
        for (int k = 0; k < RT_NCOUNTERS; ++k) {
            unsigned long long v = cnt.c[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (lane == 0 && v) atomicAdd(kp.counters + k, v);
        }
    }
}

// fill_canva, main.c:245-284: thread = (pixel, chunk of its samples).
template <bool COUNT, bool BVH, bool SKY>
__global__ __launch_bounds__(256, BVH ? RT_WAVES_PER_SIMD_BVH : RT_WAVES_PER_SIMD) void render_kernel(const KParams kp)
{
    render_body<COUNT, BVH, SKY, false>(kp);
}

// render_canva, main_cuda.cu:143-171 semantics (rt.h RT_SEM_CUDA).
template <bool COUNT, bool BVH>
__global__ __launch_bounds__(256, BVH ? RT_WAVES_PER_SIMD_BVH : RT_WAVES_PER_SIMD) void render_kernel_cuda(
    const KParams kp)
{
    render_body<COUNT, BVH, false, true>(kp);
}

#if RT_QUEUE > 0
// Persistent sphere kernel over (chunk, pixel) tasks (RT_QUEUE > 0;
// spp_chunks > 1, no BVH, main.c semantics).  A task is one pixel's samples
// [c*S/P, (c+1)*S/P) in order, summed in the lane's LDS column and written to
// the chunk partials, which combine_kernel sums in chunk order: the result is
// the fixed-grid kernel's bit for bit whichever lane runs the task.  Paths
// run as LanePath rounds (samples_flat); a lane whose task is done starts its
// next one, so lanes with short paths (misses, lights, zero throughput) do
// not idle until the wave's longest slice ends.
// Tasks come from a per-launch counter, RT_QUEUE tasks per atomic: a wave
// takes a batch and hands its tasks to its lanes as they need them.  Static
// task lists were 1.3x slower: the dispatcher places waves unevenly over the
// SIMDs (per-lane clocks: waves with the same work ended between 21 and
// 45 ms), so only a dynamic queue keeps every SIMD busy to the end; one
// atomic per lane grab was 1.8x slower (same-address atomics).  The grid is
// the resident capacity; every lane leaves once the counter passes the
// task count.

// One lane's path in render_kernel_q: tracer's state (main.c:118-242) for
// the sample in flight.  Rounds run in three steps so that a lane whose path
// ends starts its next sample's camera ray in the SAME instructions that
// continuing lanes use for their bounce direction (one Philox block and one
// normalize serve both):
//   resolve_hit   everything of tracer's bounce body that does not need the
//                 next direction: hit point, material, albedo/normal chain,
//                 the light seen directly, alpha holes, and -- when the
//                 surface is opaque -- the shading, the zero-throughput exit
//                 and the bounce budget; it leaves the lane a role
//   next_ray      BOUNCE: random_dir_no_norm and normalize(n + dir)
//                 CAMERA: the 4 camera draws and get_ray, normalize
//                 (both: draws from one Philox block, one normalize)
//   finish_bounce reflect/lerp, the refraction branch (whose draw follows
//                 the direction draws), AO set-up
// The draws keep the reference's per-sample order (counter-based stream:
// direction n, n+1, refraction n+2, AO next), so results are bit-identical
// to tracer; work whose result cannot reach the output is skipped: the
// direction after the last bounce, and the AO cast of the last bounce
// (tracer multiplies rayColor by it and then returns incomingLight).
enum : int { ROLE_NONE = 0, ROLE_BOUNCE = 1, ROLE_CAMERA = 2, ROLE_AO = 3, ROLE_PBOUNCE = 4 };
// AO scenes (AOM == AO_ON), an opaque bounce whose draws start a Philox block
// (draw n = 4k: the camera takes draws 0-3 and a shaded bounce with its AO
// ray 4 more, so every such bounce in scenes without translucent surfaces or
// alpha holes): the lane makes ONE direction per round.  ROLE_AO makes the AO
// direction from draws n+2, n+3 right after the shading (ambient_occlusion,
// main.c:96-103), keeping draws n, n+1 of the same block in the LDS cache;
// after the AO cast, ROLE_PBOUNCE makes the bounce direction from them
// (main.c:161-166) and the lerp.  The draws, and so the results, are the
// reference's; each round's shared next-ray step then serves every lane that
// needs a direction, instead of a second sampling pass for the AO ray in
// finish_bounce, and the bounce direction is skipped when the AO factor
// ends the path.

// What resolve_hit leaves for next_ray / finish_bounce in the same round (not
// live across rounds, so not in QPath: the cast and the BVH walk do not carry
// these registers).
struct QHit {
    V3 hn;                           // the hit's normal
    double rs;                       // its reflectionStrength
    bool refr, hole;                 // refraction decided after the direction draws; alpha hole
    TexRef tex;                      // (triangle hits) the texel resolve_hit read: the refraction branch
                                     // re-reads the material from it instead of redoing the barycentrics
};

// NT: the scene has no triangles (every hit is a sphere); OP: every material
// is opaque (host: !(alpha < 0.0001) && !(alpha <= 0.99), so no alpha hole
// and no refraction branch is ever taken and neither is compiled in)
// IR: incomingLight / rayColor live in the lane's LDS column (slots
// ACC_SLOTS..+5 of the sums array) instead of twelve VGPRs
// KT: a refraction lane keeps its triangle hit's texel (QHit::tex) from
// resolve_hit to finish_bounce instead of redoing the barycentrics (the
// brute-force kernel, QB 0: C3 +7.0 %, C5 +6.7 %; the BVH kernels recompute,
// their registers are tighter: sweep -1.9 % with KT)
template <bool SKY, int AOM, bool NT = false, bool OP = false, int IR = 0, bool KT = false>   // IR 1: incomingLight only
struct QPath {
    V3 o, d, cd, inc, rc;            // cd: the cast's direction (AO casts; else d)
    double* accp;                    // (IR) the lane's LDS column
    double top_n2, best;
    int i, kind, win, s, state;
    bool chain, ao_cast;
    bool pend;                       // (AO_ON) the bounce direction waits for the AO cast (ROLE_PBOUNCE)
    int pkw;                         // ... the bounce hit: win | kind << 30 (its normal is recomputed at o)
    double prs;                      // ... and its reflectionStrength

    __device__ __forceinline__ V3 cast_dir() const { return AOM == AO_ON ? cd : d; }
    __device__ __forceinline__ V3 inc_get() const
    {
        if (IR) return v3(accp[(ACC_SLOTS + 0) * 256], accp[(ACC_SLOTS + 1) * 256], accp[(ACC_SLOTS + 2) * 256]);
        return inc;
    }
    __device__ __forceinline__ V3 rc_get() const
    {
        if (IR == 2) return v3(accp[(ACC_SLOTS + 3) * 256], accp[(ACC_SLOTS + 4) * 256], accp[(ACC_SLOTS + 5) * 256]);
        return rc;
    }
    __device__ __forceinline__ void inc_set(V3 v)
    {
        if (IR) {
            accp[(ACC_SLOTS + 0) * 256] = v.x;
            accp[(ACC_SLOTS + 1) * 256] = v.y;
            accp[(ACC_SLOTS + 2) * 256] = v.z;
        } else {
            inc = v;
        }
    }
    __device__ __forceinline__ void rc_set(V3 v)
    {
        if (IR == 2) {
            accp[(ACC_SLOTS + 3) * 256] = v.x;
            accp[(ACC_SLOTS + 4) * 256] = v.y;
            accp[(ACC_SLOTS + 5) * 256] = v.z;
        } else {
            rc = v;
        }
    }

    // The hit's material (sky_material / texel_material are pure functions of
    // the hit, so a refraction lane re-reads it instead of keeping it live;
    // for a triangle it keeps only the texel, H.tex).
    __device__ __forceinline__ Mat hit_material(const KParams& kp, V3 hp, QHit& H) const
    {
        if (NT || kind == HIT_SPHERE) {
            Mat mat = load_mat(kp.sph_mat + win);
            if (SKY && win == kp.ns - 1) sky_material(kp, win, kp.sph[win], hp, mat);
            return mat;
        }
        if (!KT) return tri_material(kp, win, hp, H.hn);
        H.tex = tri_texel(kp, win, hp, H.hn);
        return texel_material(kp, H.tex);
    }
    __device__ __forceinline__ Mat hit_material_again(const KParams& kp, V3 hp, const QHit& H) const
    {
        if (NT || kind == HIT_SPHERE) {
            Mat mat = load_mat(kp.sph_mat + win);
            if (SKY && win == kp.ns - 1) sky_material(kp, win, kp.sph[win], hp, mat);
            return mat;
        }
        if (!KT) return tri_material(kp, win, hp, H.hn);
        return texel_material(kp, H.tex);
    }

    __device__ __forceinline__ static bool zero_rc_of(const KParams& kp, V3 r)
    {
        return kp.zero_exit && r.x == 0.0 && r.y == 0.0 && r.z == 0.0;
    }
    __device__ __forceinline__ bool zero_rc(const KParams& kp) const { return zero_rc_of(kp, rc_get()); }

    // After a cast (state SM_RESOLVE).  Returns the role for next_ray, or
    // ROLE_NONE; a lane whose path is over gets state SM_CAM (sum added).
    // the normal of a hit at point p: sphere (hit_sphere's normalize(p - C),
    // sphere.h:33) or triangle (tri_normal)
    __device__ __forceinline__ static V3 hit_normal(const KParams& kp, V3 p, int k, int w)
    {
        if (NT || k == HIT_SPHERE) {
            const SphGeo sg = kp.sph[w];
            return normalize(p - v3(sg.cx, sg.cy, sg.cz));
        }
        return tri_normal(kp, w);
    }

    __device__ __forceinline__ int resolve_hit(const KParams& kp, double* acc, QHit& H, uint32_t sn)
    {
        // (AO kernels only: without AO there is no second normal; C2 -0.7 % there)
        constexpr bool MN = RT_MERGED_NRM && AOM == AO_ON;
        bool ended = false, add_inc = true, hit = false, nrm = false;
        V3 np = v3(0, 0, 0);
        int nk = HIT_NONE, nw = 0;
        int role = ROLE_NONE;
        // a hit's material, chain sums, emitter / hole / refraction / shading and
        // the next role (main.c:137-234), H.hn set
        auto hit_rest = [&](const V3 hp) __attribute__((always_inline)) {
            const Mat mat = hit_material(kp, hp, H);
            bool lit = false;
            if (chain) {
                if (mat.es > 0) {                        // direct view of a light, main.c:154-160
                    V3 col;
                    if ((NT || kind == HIT_SPHERE) && !(SKY && win == kp.ns - 1)) {
                        const double* sd = kp_here()->sph_disp + 3 * win;   // (host: the same round trip)
                        col = v3(sd[0], sd[1], sd[2]);
                    } else {
                        col = hsl_roundtrip(mat.emis);
                    }
                    acc_add(acc, ACC_RAD, col);
                    acc_add(acc, ACC_ALB, col);
                    acc_add(acc, ACC_NRM, H.hn);
                    lit = true;
                } else if (OP || !(mat.alpha < 0.0001) || i == kp.B - 1) {
                    acc_add(acc, ACC_ALB, mat.diff);
                    acc_add(acc, ACC_NRM, H.hn);
                    chain = !OP && mat.alpha < 0.0001;
                }
            }
            if (lit) {
                ended = true;
                add_inc = false;
            } else {
                o = hp;
                H.rs = mat.rs;
                H.refr = false;
                H.hole = !OP && mat.alpha < 0.0001;
                if (H.hole) {                              // alpha H.hole: straight on, main.c:200-206;
                    if (i + 1 >= kp.B) ended = true;     // its direction draws are made (and unused)
                    else role = ROLE_BOUNCE;             // so the stream's block cache stays in order
                } else {
                    chain = false;
                    if (!OP && mat.alpha <= 0.99) {      // refraction: decided after the direction draws
                        H.refr = true;
                        role = ROLE_BOUNCE;
                    } else {
                        const V3 nrc = shade(kp, mat);
                        if (zero_rc_of(kp, nrc) || i + 1 >= kp.B) {
                            ended = true;                // nothing more reaches the sum
                        } else if (AOM == AO_ON && RT_AO_FIRST && (sn & 3u) == 0u) {
                            role = ROLE_AO;              // AO direction first (ROLE_AO above)
                            pend = true;
                            pkw = win | (kind << 30);
                            prs = mat.rs;
                        } else {
                            role = ROLE_BOUNCE;
                        }
                    }
                }
            }
        };
        if (AOM == AO_ON && ao_cast) {
            // ambient_occlusion's tail, main.c:104-115
            const double AO = ((cdptr)kp.uni)[opq0() + U_AO];
            double occ = 0.0;
            if (kind != HIT_NONE) {
                const V3 hp = o + muls(cast_dir(), best);
                const V3 df = hp - o;
                const double distance = sqrt(dot(df, df));
                double att = distance / best;
                att = pm_pow(att, AO);
                occ = occ + att;
            }
            occ = (occ / 1.0) / AO;
            const V3 r2 = mulv(rc_get(), v3(occ, occ, occ));
            rc_set(r2);
            ao_cast = false;
            ++i;                                         // the bounce after the AO cast
            ended = zero_rc_of(kp, r2) || i >= kp.B;
            if (!ended) {
                if (pend) {                              // its direction is still to be made
                    role = ROLE_PBOUNCE;
                    const int pw = pkw & 0x3fffffff;     // the bounce hit's normal (o is its hit point)
                    if (MN) {                            // below, with the hit lanes' normals
                        np = o;
                        nw = pw;
                        nk = pkw >> 30;
                        nrm = true;
                    } else if (NT || (pkw >> 30) == HIT_SPHERE) {
                        const SphGeo sg = kp.sph[pw];
                        H.hn = normalize(o - v3(sg.cx, sg.cy, sg.cz));
                    } else {
                        H.hn = tri_normal(kp, pw);
                    }
                    H.rs = prs;
                    H.refr = H.hole = false;
                } else {
                    cd = d;
                    state = SM_CAST;
                }
            }
            pend = false;
        } else if (kind == HIT_NONE) {                   // miss: the path ends, main.c:236-238
            if (chain) {
                acc_add(acc, ACC_ALB, v3(0, 0, 0));
                acc_add(acc, ACC_NRM, v3(0, 0, 0));
            }
            ended = true;
        } else {
            if (MN) {                                    // the rest after the merged normal below
                hit = true;
                np = o + muls(d, best);                  // ray_at
                nw = win;
                nk = kind;
                nrm = true;
            } else {
                const V3 hp = o + muls(d, best);         // ray_at
                H.hn = hit_normal(kp, hp, kind, win);
                hit_rest(hp);
            }
        }
        // RT_MERGED_NRM: the normal of the hit each lane goes on from -- this cast's,
        // or the bounce hit waiting for the AO cast -- in ONE normalize for the
        // wave instead of one per branch
        if (MN && nrm) H.hn = hit_normal(kp, np, nk, nw);
        if (MN && hit) hit_rest(np);
        if (ended) {
            if (add_inc) acc_add(acc, ACC_RAD, inc_get());
            ++s;
            state = SM_CAM;
            role = ROLE_NONE;
        }
        return role;
    }

    // shading of an opaque surface (main.c:208-234 without the AO cast)
    __device__ __forceinline__ V3 shade_with(const KParams& kp, V3 emis, double es, V3 diff)
    {
        V3 r = rc_get();
        if (AOM == AO_ON) {
            const double AO = ((cdptr)kp.uni)[opq0() + U_AO];
            const V3 em = muls(emis, es * 1.5 * AO);
            inc_set(inc_get() + mulv(em, r));
        } else {
            const V3 em = muls(emis, es);
            inc_set(inc_get() + mulv(em, r));
        }
        if (any_above_half(r)) r = mulv(diff, muls(r, 1.3));
        const V3 nrc = mulv(diff, r);
        rc_set(nrc);
        return nrc;
    }
    __device__ __forceinline__ V3 shade(const KParams& kp, const Mat& mat) { return shade_with(kp, mat.emis, mat.es, mat.diff); }

    // After next_ray gave a bounce lane its diffuse direction dn.
    __device__ __forceinline__ void finish_bounce(const KParams& kp, V3 dn, Stream& st, double* acc, const QHit& H)
    {
        if (!OP && H.hole) {                               // the ray goes on unchanged from the hit point
            ++i;
            cd = d;
            state = SM_CAST;
            return;
        }
        const V3 reflected_dir = d - muls(H.hn, 2 * dot(d, H.hn));
        const V3 dr = dn + muls(reflected_dir - dn, H.rs);
        bool shaded = true;
        if (!OP && H.refr) {                               // main.c:167-193
            const Mat mat = hit_material_again(kp, o, H);
            V3 nn = H.hn;
            double n1, n2;
            if (dot(d, H.hn) > 0) {                        // leaving: pop restores the stack
                nn = v3(-H.hn.x, -H.hn.y, -H.hn.z);
                n1 = mat.ior;
                n2 = top_n2;
            } else {                                     // entering: push (top.n2, ior)
                n1 = top_n2;
                n2 = mat.ior;
                top_n2 = mat.ior;
            }
            const V3 rf = refracted(d, nn, n1, n2);
            // (RT_REFR_PREFETCH) the draw is in the block cache whatever its slot
            const double rnd = rand_01(RT_REFR_PREFETCH ? st.next31_cached() : st.next31());
            if (rnd > mat.alpha) {
                d = rf;
                shaded = false;
            } else {
                d = dr;
                shade(kp, mat);
            }
        } else {
            d = dr;
        }
        bool ended = false;
        if (!OP && H.refr && shaded) ended = zero_rc(kp);
        if (AOM == AO_ON && shaded && !ended && i + 1 < kp.B) {
            // ambient_occlusion's cast (main.c:96-103): from the hit along n + random
            Cnt cnt;
            cd = normalize(H.hn + random_dir<false>(st, cnt));
            ao_cast = true;
            state = SM_CAST;
            return;
        }
        ++i;
        ended = ended || i >= kp.B;
        if (ended) {                                     // (refraction lanes only) the sample is over
            acc_add(acc, ACC_RAD, inc_get());
            ++s;
            state = SM_CAM;
        } else {
            cd = d;
            state = SM_CAST;
        }
    }
};

// Task t of a queue launch as render_kernel_q's LDS table entry: e[0] its
// chunk-partial index chunk * band_rows * W + p (~0: past the last task),
// e[1] the pixel g * W + x (~0: a padding row of the tiling, no work), e[2]
// the row g, e[3], e[4] its first and end sample (rt.h rt_chunk_bound).
constexpr int kTaskWords = 5;
__device__ __forceinline__ void decode_task(KParamsK K, unsigned t, uint32_t e[kTaskWords])
{
    for (int j = 0; j < kTaskWords; ++j) e[j] = 0xffffffffu;
    if (t >= K->npx_here * (unsigned)K->chunks) return;
    unsigned p;
    const unsigned chunk = udiv_q(t, K->npx_here, K->qm_npx, p);
    e[0] = chunk * ((unsigned)K->band_rows * (unsigned)K->W) + p;
    unsigned xr;
    const unsigned row = udiv_q(p, (unsigned)K->W, K->qm_w, xr);
    const int ly = K->band_y0 + (int)row;
    if (ly >= K->local_rows) return;
    unsigned yy;
    const int lt = (int)udiv_q((unsigned)ly, (unsigned)K->tile_rows, K->qm_tile, yy);
    const int g = K->row_base + (K->tile_first + lt * K->tile_step) * K->tile_rows + (int)yy;
    if (g >= K->row_end) return;
    e[1] = (uint32_t)g * (uint32_t)K->W + xr;
    e[2] = (uint32_t)g;
    e[3] = (uint32_t)chunk_start(K->S, K->chunks, K->chunk_taper, K->chunk_den, K->qm_chunks, chunk);
    e[4] = (uint32_t)chunk_start(K->S, K->chunks, K->chunk_taper, K->chunk_den, K->qm_chunks, chunk + 1u);
}

template <bool SKY, int AOM, int QB, bool OPQ = false>   // OPQ: (BVH scenes) every material opaque
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(QB < 0 ? RT_WAVES_PER_SIMD_QS
                                                                     : QB == 4 ? RT_WAVES_PER_SIMD_Q4
                                                                               : RT_WAVES_PER_SIMD_Q)))
void render_kernel_q(const KParams kp)
{
    // incomingLight / rayColor in LDS: both for the non-BVH kernels, incomingLight
    // alone for the opaque deep-tree kernel (its stack leaves room for 3 doubles)
    constexpr int QIR = RT_QLDS_IR && QB <= 0 ? 2 : (RT_QLDS_INC_BVH && QB == 3 && OPQ) ? 1 : 0;
    __shared__ double acc_lds[(ACC_SLOTS + 3 * QIR) * 256];
    __shared__ uint32_t rng_lds[4 * 256];
    double* acc = acc_lds + threadIdx.x;
    uint32_t* rng = rng_lds + threadIdx.x;
    const int lane = threadIdx.x & 63;
    unsigned qb = 0, qe = 0;         // the wave's batch of tasks [qb, qe) (wave-uniform)
    QPath<SKY, AOM, QB < 0, QB == -2 || OPQ, QIR, QB == 0> L;
    L.accp = acc;
    L.o = L.d = L.cd = L.inc = L.rc = v3(0, 0, 0);
    L.inc_set(v3(0, 0, 0));
    L.rc_set(v3(0, 0, 0));
    L.top_n2 = 1.0;
    L.best = 0.0;
    L.i = 0; L.kind = HIT_NONE; L.win = -1; L.s = 0;
    L.chain = true; L.ao_cast = false;
    L.pend = false;
    L.pkw = 0;
    L.prs = 0.0;
    L.state = SM_CAM;                // s = 0 >= s1 = 0: takes a task first
#if RT_DIAG_STALE == 2
    diag_cnt()[0] = 0u;
    diag_cnt()[256] = 0u;
#endif
    int x = 0, g = 0, s1 = 0;
    int node = 0, sp = 0, win_orig = 0;      // BVH walk in flight (state SM_TRAV)
    unsigned chunk = 0, p = 0, pixel = 0;
    bool owns = false;               // the lane's LDS sums belong to task (chunk, p)
    // sphere / brute-force scenes (QB 0): each wave decodes its batches of tasks into LDS
    // (not for QB 3, the deep-tree instantiation: there the table's registers
    // cost spills, C4 -0.6 %; C2 +3.5 %, C3 +1.0 %, sweep +2.3 %)
    constexpr bool TTAB = RT_QTASK_TABLE && QB != 3;
    __shared__ uint32_t ttab_lds[TTAB ? 4 * kTaskWords * 64 : 1];
    unsigned qidx = 0;               // (TTAB) partial index of the lane's task
    Stream st;                       // draw stream of the sample in flight (next31 for refraction / AO)
    st.start(0u, 0u, kp.key0, kp.key1, rng);
    // shallow trees (QB 4: depth4 <= 4, e.g. the 50-node sweep tree) keep
    // their top nodes in LDS: sweep +5.7 %; deep ones gain nothing (C4 -0.5 %)
    // deep trees (QB 3) walk the 64-byte nodes (host: kp.bvhh set); the shallow
    // ones keep their LDS copy in 128-byte nodes (64-byte: sweep -0.8 %)
    constexpr bool HN = RT_QNODE_H != 0 && QB == 3;
    using QNode = std::conditional_t<HN, BvhNodeH, BvhNode4>;
    constexpr int NTOP = QB == 4 ? RT_QB_TOP * (int)(sizeof(BvhNode4) / sizeof(QNode)) : 0;
    if (NTOP > 0) {                          // the tree's top nodes into LDS, once per block
        float4* dst = (float4*)bvh_top_q<QNode, NTOP>();
        const float4* src = HN ? (const float4*)kp.bvhh : (const float4*)kp.bvh;
        const int n = min(NTOP, kp.bvh_nodes) * (int)(sizeof(QNode) / sizeof(float4));
        for (int i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
        __syncthreads();
    }
    const long long t_start = kp.trace ? wall_clock64() : 0;
    unsigned rounds = 0, ntasks = 0;
#if RT_PHASE_CLOCK
    // wave-uniform clock reads at the round's uniform points (SGPR sums)
    unsigned long long ph[5] = {0, 0, 0, 0, 0}, tc = __builtin_amdgcn_s_memtime();
    auto phase = [&](int k) __attribute__((always_inline)) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        ph[k] += t - tc;
        tc = t;
    };
#define RT_PHASE(k) phase(k)
#else
#define RT_PHASE(k) ((void)0)
#endif
    while (true) {
        ++rounds;
        RT_PHASE(4);                 // the previous round's next-ray step and finish_bounce
        // ---- 1. closest hit (main.c:52-92) for every lane with a ray ------
        if (QB > 0) {
            // spheres, then the triangle BVH: up to QB node visits
            // per round; a deeper walk resumes next round (its lane skips
            // the path work meanwhile), so a wave never waits for its
            // deepest lane's whole walk
            if (L.state == SM_CAST) {
                Cnt cnt;
                L.win = cast_spheres<false, false>(kp, L.o, L.cast_dir(), L.best, cnt);
                L.kind = L.win >= 0 ? HIT_SPHERE : HIT_NONE;
                win_orig = 0;
                node = 0;
                sp = 0;
                L.state = SM_TRAV;
            }
            RT_PHASE(0);
            if (__ballot(L.state == SM_TRAV) != 0ull) {
#if RT_WALK_PRIO
                __builtin_amdgcn_s_setprio(RT_WALK_PRIO);
#endif
                const V3 dd = L.cast_dir();
                const Ray32 r32 = ray32<QB == 3 && !OPQ>(kp, L.o, dd);
                unsigned short* stk = bvh_stack_q<QB, OPQ>();
                const QNode* top = NTOP > 0 ? bvh_top_q<QNode, NTOP>() : nullptr;
                // deep trees (QB 3): at least RT_QW_MIN visits, then more while at
                // least RT_QW_LANES lanes of the wave are still walking, up to
                // RT_QW_MAX (long walks -- e.g. rays skimming RTX_MAP/nature's
                // terrain -- finish in fewer rounds, short ones hand the wave back
                // to the path work as before)
                constexpr int JMIN = QB == 3 ? RT_QW_MIN : QB, JMAX = QB == 3 ? RT_QW_MAX : QB;
#pragma unroll 1
                for (int j = 0; j < JMAX; ++j) {
                    if (L.state == SM_TRAV) {
                        Cnt cnt;
                        if (!bvh_step<false, false, NTOP, HN>(kp, L.o, dd, r32, stk, node, sp, L.best, L.kind, L.win,
                                                           win_orig, cnt, top))
                            L.state = SM_RESOLVE;
                    }
                    const unsigned long long wm = __ballot(L.state == SM_TRAV);
                    if (wm == 0ull || (j + 1 >= JMIN && __popcll(wm) < RT_QW_LANES)) break;
                }
#if RT_WALK_PRIO
                __builtin_amdgcn_s_setprio(0);
#endif
            }
        } else if (QB < 0 && L.state == SM_CAST) {          // sphere-only scenes: no triangle scan
            Cnt cnt;
            L.win = cast_spheres<false, false, !SKY && AOM != AO_ON>(kp, L.o, L.cast_dir(), L.best, cnt);
            L.kind = L.win >= 0 ? HIT_SPHERE : HIT_NONE;
            L.state = SM_RESOLVE;
        } else if (L.state == SM_CAST) {
            Cnt cnt;
            L.kind = closest_hit<false, false, false, !SKY && AOM != AO_ON>(kp, L.o, L.cast_dir(), L.best, L.win, cnt);
            L.state = SM_RESOLVE;
        }
        RT_PHASE(QB > 0 ? 1 : 0);
        // ---- 2. the hit, up to the next direction --------------------------
        int role = ROLE_NONE;
        QHit H;
        H.hn = v3(0, 0, 0);
        H.rs = 0.0;
        H.refr = H.hole = false;
        if (L.state == SM_RESOLVE) role = L.resolve_hit(kp, acc, H, st.n);
        RT_PHASE(2);
        // ---- 3. lanes whose task is done take the next one -----------------
        const bool need = L.state == SM_CAM && L.s >= s1;
        const unsigned long long nm = __ballot(need);
        if (nm) {                    // wave-uniform: tasks for the lanes that need one
            // launch constants re-read here (SMEM) instead of living in SGPRs
            // spilled to VGPR lanes across the whole round
            const KParamsK K = kp_here();
            unsigned t = 0;
            const unsigned nn = (unsigned)__popcll(nm), avail = qe - qb;
            const unsigned rank = (unsigned)__popcll(nm & ((1ull << lane) - 1ull));
            if constexpr (TTAB) {
                // a batch's 64 tasks are decoded once, by the whole wave, into the
                // wave's LDS table when the batch is grabbed; a lane taking a task
                // reads its entry: lanes taking the rest of the current batch
                // before the new batch overwrites the table, the others after
                uint32_t* tw = ttab_lds + (threadIdx.x >> 6) * (kTaskWords * 64);
                const bool old = rank < avail;
                uint32_t e[kTaskWords];
                if (need && old) {
                    const unsigned slot = (qb - (qe - RT_QUEUE)) + rank;
#pragma unroll
                    for (int j = 0; j < kTaskWords; ++j) e[j] = tw[j * 64 + slot];
                }
                if (avail < nn) {
                    unsigned nb = 0;
                    if (lane == __ffsll((long long)nm) - 1) nb = atomicAdd(K->task_ctr, (unsigned)RT_QUEUE);
                    nb = __shfl(nb, __ffsll((long long)nm) - 1, 64);
                    uint32_t d[kTaskWords];
                    decode_task(K, nb + (unsigned)lane, d);
#pragma unroll
                    for (int j = 0; j < kTaskWords; ++j) tw[j * 64 + lane] = d[j];
                    if (need && !old) {
#pragma unroll
                        for (int j = 0; j < kTaskWords; ++j) e[j] = tw[j * 64 + (rank - avail)];
                    }
                    qb = nb + (nn - avail);
                    qe = nb + RT_QUEUE;
                } else {
                    qb += nn;
                }
                if (need) {
                    ++ntasks;
                    if (owns) {      // task done: its sums to the chunk partials
                        double* q = K->partial + (size_t)qidx * 9;
#pragma unroll
                        for (int j = 0; j < 9; ++j) q[j] = acc[j * 256];
                        owns = false;
                    }
                    if (e[0] == 0xffffffffu) {
                        L.state = SM_DONE;
                    } else if (e[1] != 0xffffffffu) {  // otherwise the lane takes its next task next round
                        qidx = e[0];
                        pixel = e[1];
                        g = (int)e[2];
                        x = (int)(pixel - e[2] * (unsigned)K->W);
                        L.s = (int)e[3];
                        s1 = (int)e[4];
#pragma unroll
                        for (int j = 0; j < 9; ++j) acc[j * 256] = 0.0;
                        owns = true;
                    }
                }
            } else {
            if (avail < nn) {        // a new batch (nn <= 64 <= RT_QUEUE): old tasks first
                unsigned nb = 0;
                if (lane == __ffsll((long long)nm) - 1) nb = atomicAdd(K->task_ctr, (unsigned)RT_QUEUE);
                nb = __shfl(nb, __ffsll((long long)nm) - 1, 64);
                t = rank < avail ? qb + rank : nb + (rank - avail);
                qb = nb + (nn - avail);
                qe = nb + RT_QUEUE;
            } else {
                t = qb + rank;
                qb += nn;
            }
            if (need) {
                ++ntasks;
                if (owns) {          // task done: its sums to the chunk partials
                    double* q = K->partial + ((size_t)chunk * ((unsigned)K->band_rows * (unsigned)K->W) + p) * 9;
#pragma unroll
                    for (int j = 0; j < 9; ++j) q[j] = acc[j * 256];
                    owns = false;
                }
                if (t >= K->npx_here * (unsigned)K->chunks) {
                    L.state = SM_DONE;
                } else {
                    // task t = (chunk, pixel p of the band): launch-constant divisors
                    chunk = udiv_q(t, K->npx_here, K->qm_npx, p);
                    unsigned xr;
                    const unsigned row = udiv_q(p, (unsigned)K->W, K->qm_w, xr);
                    const int ly = K->band_y0 + (int)row;
                    x = (int)xr;
                    bool valid = ly < K->local_rows;
                    if (valid) {
                        unsigned yy;
                        const int lt = (int)udiv_q((unsigned)ly, (unsigned)K->tile_rows, K->qm_tile, yy);
                        g = K->row_base + (K->tile_first + lt * K->tile_step) * K->tile_rows + (int)yy;
                        valid = g < K->row_end;
                    }
                    if (valid) {     // otherwise the lane takes its next task next round
                        pixel = (uint32_t)g * (uint32_t)K->W + (uint32_t)x;
                        L.s = chunk_start(K->S, K->chunks, K->chunk_taper, K->chunk_den, K->qm_chunks, chunk);
                        s1 = chunk_start(K->S, K->chunks, K->chunk_taper, K->chunk_den, K->qm_chunks, chunk + 1u);
#pragma unroll
                        for (int j = 0; j < 9; ++j) acc[j * 256] = 0.0;
                        owns = true;
                    }
                }
            }
            }
        }
        if (__ballot(L.state != SM_DONE) == 0ull) break;     // every lane of the wave is done
        RT_PHASE(3);
        // tracer with nbRebondMax <= 0 returns (0, 0, 0) albedo/normal/colour
        if (kp.B <= 0 && L.state == SM_CAM && L.s < s1) {
            acc_add(acc, ACC_ALB, v3(0, 0, 0));
            acc_add(acc, ACC_NRM, v3(0, 0, 0));
            acc_add(acc, ACC_RAD, v3(0, 0, 0));
            ++L.s;
            continue;
        }
        if (L.state == SM_CAM && L.s < s1) role = ROLE_CAMERA;
        // ---- 4. next ray: bounce direction or camera ray (shared work) ----
        if (role != ROLE_NONE) {
            const bool cam = role == ROLE_CAMERA;
            const bool aor = AOM == AO_ON && role == ROLE_AO, pbr = AOM == AO_ON && role == ROLE_PBOUNCE;
            // draws: a bounce uses draws n, n+1 of its sample (rtutility.h:
            // 189-203); a camera ray draws 0-3 of sample s (main.c:265-269);
            // ROLE_AO draws n+2, n+3 of block n/4 and keeps n, n+1 in the
            // cache's words 0-1 for ROLE_PBOUNCE
            const uint32_t nd = cam ? 0u : st.n;
            const uint32_t sa = nd & 3u, sb = (nd + 1u) & 3u;
            uint32_t wa = 0, wb = 0;
            Philox blk{0, 0, 0, 0};
            if (pbr) {
                wa = rng[0];
                wb = rng[256];
            } else {
                if (!cam && !aor && sa != 0u) wa = rng[sa * 256];          // cached word of the current block
                if (!cam && !aor && sb != 0u && sa != 0u) wb = rng[sb * 256];
                // RT_REFR_PREFETCH: a refraction lane whose direction draws are
                // both cached (n = 2 mod 4) but whose refraction draw n+2 opens
                // the next block makes that block here, in the round's one Philox,
                // instead of in finish_bounce's own (a second Philox per round)
                const bool rpre = RT_REFR_PREFETCH && !cam && !aor && !pbr && H.refr && sa == 2u;
                if (cam || aor || sa == 0u || sb == 0u || rpre) {         // a new block: one Philox for every role
                    const uint32_t bi = cam ? 0u : ((nd + (sa == 0u ? 0u : rpre ? 2u : 1u)) >> 2);
                    blk = philox4x32_10(bi, 0u, pixel, (uint32_t)(kp.s_base + L.s), kp.key0, kp.key1);
                    if (aor) {                                      // the bounce's draws, for ROLE_PBOUNCE
                        rng[0] = blk.w0;
                        rng[256] = blk.w1;
                    } else if (!cam) {                              // keep the rest of the block
                        if (rpre) rng[0] = blk.w0;
                        rng[256] = blk.w1;
                        rng[512] = blk.w2;
                        rng[768] = blk.w3;
                    }
                }
                if (aor) {
                    wa = blk.w2;
                    wb = blk.w3;
                } else if (!cam) {
                    if (sa == 0u) wa = blk.w0;
                    if (sb == 0u) wb = blk.w0;
                    else if (sa == 0u) wb = blk.w1;
                }
            }
            V3 X;
            V3 no = v3(0, 0, 0);
            if (cam) {
                CamDraws w{blk, 0};
                const double ju = rand_m05(w.next31());     // randomDouble(-0.5, 0.5)
                const double jv = rand_m05(w.next31());
                const int b = opq0();
                const cdptr U = (cdptr)kp.uni;
                const double nu = (double)x + ju, nv = (double)g + jv;
                const double rcw = U[b + U_RC_WM1], rch = U[b + U_RC_HM1];
                const double u = rcw != 0.0 ? div_core(nu, U[b + U_WM1], rcw) : nu / U[b + U_WM1];
                const double v = rch != 0.0 ? div_core(nv, U[b + U_HM1], rch) : nv / U[b + U_HM1];
                const V3 co = v3(U[b + U_CAM_O], U[b + U_CAM_O + 1], U[b + U_CAM_O + 2]);
                const V3 ch = v3(U[b + U_CAM_H], U[b + U_CAM_H + 1], U[b + U_CAM_H + 2]);
                const V3 cv = v3(U[b + U_CAM_V], U[b + U_CAM_V + 1], U[b + U_CAM_V + 2]);
                const V3 cc = v3(U[b + U_CAM_C], U[b + U_CAM_C + 1], U[b + U_CAM_C + 2]);
                const V3 dir = cc + (muls(ch, u) + (muls(cv, v) - co));     // get_ray, camera.h:42-55
                const V3 dest = co + muls(dir, U[b + U_FOCUS]);
                if (kp.cam_pin) {                              // zero aperture: the origin itself (host-checked)
                    no = co;
                } else {
                    const double jx = rand_m05(w.next31());
                    const double jy = rand_m05(w.next31());
                    const double dx = jx * U[b + U_OX], dy = jy * U[b + U_OY];
                    no = co + v3(dx, dy, 0);
                }
                X = dest - no;
            } else {
                // random_dir_no_norm (rtutility.h:189-203), then n + dir (main.c:163)
                X = H.hn + normalize_unit(sampler_vec(wa >> 1, wb >> 1));
                st.n += aor ? 0u : pbr ? 4u : 2u;
            }
            const V3 dn = normalize(X);
            if (cam) {                                         // the new sample's primary ray
                L.o = no;
                L.d = dn;
                if (AOM == AO_ON) L.cd = dn;
                L.inc_set(v3(0, 0, 0));
                L.rc_set(v3(1, 1, 1));
                L.top_n2 = 1.0;
                L.i = 0;
                L.chain = true;
                L.ao_cast = false;
                L.state = SM_CAST;
                st.start(pixel, (uint32_t)(kp.s_base + L.s), kp.key0, kp.key1, rng);
                st.n = 4;                                      // draws 0-3 were the camera's
            } else if (aor) {                                  // ambient_occlusion's cast (main.c:96-103)
                L.cd = dn;
                L.ao_cast = true;
                L.state = SM_CAST;
            } else if (pbr) {                                  // main.c:161-166 after the AO cast
                const V3 reflected_dir = L.d - muls(H.hn, 2 * dot(L.d, H.hn));
                L.d = dn + muls(reflected_dir - dn, H.rs);
                L.cd = L.d;
                L.state = SM_CAST;
            } else {
                L.finish_bounce(kp, dn, st, acc, H);
            }
        }
    }
    if (kp.trace) {                  // diagnostics (RT_QUEUE_TRACE): per lane start, end, rounds, tasks
        unsigned long long* q = kp.trace + ((size_t)blockIdx.x * 256 + threadIdx.x) * RT_TRACE_WORDS;
        q[0] = (unsigned long long)t_start;
        q[1] = (unsigned long long)wall_clock64();
        q[2] = rounds;
        q[3] = ntasks;
#if RT_DIAG_STALE == 2
        q[2] = diag_cnt()[0];        // diagnostic: node visits and stale visits of the lane
        q[3] = diag_cnt()[256];
#endif
#if RT_PHASE_CLOCK
        for (int k = 0; k < 5; ++k) q[4 + k] = ph[k];
#endif
    }
}
#endif

// Sum the chunk partials of each pixel in chunk order, then resolve.
__global__ __launch_bounds__(256) void combine_kernel(const KParams kp)
{
    const int rows = min(kp.band_rows, kp.local_rows - kp.band_y0);
    const long long npx = (long long)kp.band_rows * kp.W;      // partial plane stride
    const long long nb = (long long)rows * kp.W;
    for (long long bi = (long long)blockIdx.x * blockDim.x + threadIdx.x; bi < nb;
         bi += (long long)gridDim.x * blockDim.x) {
        const int ly = kp.band_y0 + (int)(bi / kp.W);
        const long long li = (long long)kp.band_y0 * kp.W + bi;
        const int lt = ly / kp.tile_rows, yy = ly - lt * kp.tile_rows;
        const int g = kp.row_base + (kp.tile_first + lt * kp.tile_step) * kp.tile_rows + yy;
        if (g >= kp.row_end) continue;
        double a[9];
        int c0 = 0;
        if (kp.sums) {                                   // accumulate: running sums + slices in order
#pragma unroll
            for (int j = 0; j < 9; ++j) a[j] = kp.sums[li * 9 + j];
        } else {
            const double* p = kp.partial + bi * 9;
#pragma unroll
            for (int j = 0; j < 9; ++j) a[j] = p[j];
            c0 = 1;
        }
        for (int c = c0; c < kp.chunks; ++c) {
            const double* q = kp.partial + ((long long)c * npx + bi) * 9;
#pragma unroll
            for (int j = 0; j < 9; ++j) a[j] = a[j] + q[j];
        }
        if (kp.sums) {
#pragma unroll
            for (int j = 0; j < 9; ++j) kp.sums[li * 9 + j] = a[j];
        } else {
            write_pixel(kp, li, v3(a[0], a[1], a[2]), v3(a[3], a[4], a[5]), v3(a[6], a[7], a[8]));
        }
    }
}

// Un-permute a rank-major gather of cyclic row tiles into the full frame.
__global__ __launch_bounds__(256) void assemble_kernel(const double* __restrict__ gathered, long long rank_stride,
                                                       int world, int tile_rows, int rows_per_rank, int W, int H,
                                                       double* __restrict__ out)
{
    const long long n = (long long)W * H * 3;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const long long px = e / 3;
        const int c = (int)(e - px * 3);
        const int g = (int)(px / W), i = (int)(px - (long long)g * W);
        const int t = g / tile_rows, y = g - t * tile_rows;
        const int r = t % world, lt = t / world;
        const long long src = (long long)r * rank_stride + ((long long)lt * tile_rows + y) * W + i;
        out[e] = gathered[src * 3 + c];
    }
}

// Per-launch uniform block: the values travel as this kernel's by-value
// argument (captured at enqueue), so the copy is stream-ordered without a
// pageable host staging buffer.
// The camera's (W-1) and (H-1) reciprocals are refined here on the device
// (rcp_refined is the device's own sequence) so camera_ray divides with
// div_core; 0 (W or H of 1, a zero divisor) selects the plain division.
__global__ void set_uniforms_kernel(const UniBlock u, double* __restrict__ dst)
{
    const int i = threadIdx.x;
    if (i < U_COUNT) {
        double v = u.v[i];
        if (i == U_RC_WM1 || i == U_RC_HM1) {
            const double d = u.v[i == U_RC_WM1 ? U_WM1 : U_HM1];
            v = (d >= 1.0 && d <= 0x1p400) ? rcp_refined(d) : 0.0;
        }
        dst[i] = v;
    }
}

int launch_set_uniforms(const UniBlock& u, double* d_uni, void* stream)
{
    hipLaunchKernelGGL(set_uniforms_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, u, d_uni);
    return (int)hipGetLastError();
}

// Device-math self test (rt_selftest_math).
__global__ void selftest_kernel(int op, const double* __restrict__ in, double* __restrict__ out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (op) {
    case 0: out[i] = pm_acos(in[i]); break;
    case 1: {
        float s, c;
        pm_sincosf((float)in[i], s, c);
        out[i] = (double)s;
        break;
    }
    case 2: {
        float s, c;
        pm_sincosf((float)in[i], s, c);
        out[i] = (double)c;
        break;
    }
    case 3: out[i] = pm_pow(in[2 * i], in[2 * i + 1]); break;
    case 4: out[i] = sqrt(in[i]); break;
    case 5: out[i] = in[2 * i] / in[2 * i + 1]; break;
    case 6: out[i] = (double)sqrtf((float)in[i]); break;
    case 7: {
        const double* q = in + 6 * i;
        const Philox p = philox4x32_10<false>((uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3],
                                       (uint32_t)q[4], (uint32_t)q[5]);
        out[4 * i + 0] = p.w0;
        out[4 * i + 1] = p.w1;
        out[4 * i + 2] = p.w2;
        out[4 * i + 3] = p.w3;
        break;
    }
    case 9: out[i] = pm_atan2(in[2 * i], in[2 * i + 1]); break;
    case 8: {                                   // normalize (fast lanes and generic lanes)
        const V3 v = normalize(v3(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
        out[3 * i + 0] = v.x;
        out[3 * i + 1] = v.y;
        out[3 * i + 2] = v.z;
        break;
    }
    default: out[i] = 0.0;
    }
}

// OIDN input planes from a device frame, denoiser.h:44-60 (IEEE f32 ops).
__global__ __launch_bounds__(256) void denoise_pack_kernel(long long n, const double* __restrict__ canva,
                                                           const double* __restrict__ albedo,
                                                           const double* __restrict__ normal, float* __restrict__ c3,
                                                           float* __restrict__ a3, float* __restrict__ n3)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        c3[i] = (float)canva[i] / 255.0f;
        if (a3) a3[i] = (float)albedo[i];
        if (n3) n3[i] = (float)normal[i];
    }
}

int launch_denoise_pack(long long npx, const double* canva, const double* albedo, const double* normal, float* color3,
                        float* albedo3, float* normal3, void* stream)
{
    const long long n = npx * 3;
    long long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(denoise_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, canva,
                       albedo ? albedo : nullptr, normal, color3, albedo ? albedo3 : nullptr,
                       normal ? normal3 : nullptr);
    return (int)hipGetLastError();
}

// rt_resolve_async: running sums -> frame planes for kp.S total samples
// (write_color_canva / divide_scalar, main.c:275-279).
__global__ __launch_bounds__(256) void resolve_kernel(const KParams kp)
{
    const long long npx = (long long)kp.local_rows * kp.W;
    for (long long li = (long long)blockIdx.x * blockDim.x + threadIdx.x; li < npx;
         li += (long long)gridDim.x * blockDim.x) {
        const int ly = (int)(li / kp.W);
        const int lt = ly / kp.tile_rows, yy = ly - lt * kp.tile_rows;
        const int g = kp.row_base + (kp.tile_first + lt * kp.tile_step) * kp.tile_rows + yy;
        if (g >= kp.row_end) continue;
        const double* a = kp.sums + li * 9;
        write_pixel(kp, li, v3(a[0], a[1], a[2]), v3(a[3], a[4], a[5]), v3(a[6], a[7], a[8]));
    }
}

int launch_resolve(const KParams& kp, void* stream)
{
    const long long npx = (long long)kp.local_rows * kp.W;
    long long blocks = (npx + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(resolve_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, kp);
    return (int)hipGetLastError();
}

static dim3 grid_for(const KParams& kp)
{
    return dim3((unsigned)((kp.W + 15) / 16), (unsigned)((kp.band_rows + 15) / 16), (unsigned)kp.chunks);
}

// Kernel instantiation per scene features: BVH traversal and the sky branch
// are compiled only into the variants that use them, so a sphere-only scene
// runs a kernel without their registers.
template <bool COUNT>
static void launch_variant(const KParams& kp_in, void* stream)
{
    const dim3 g = grid_for(kp_in);
    const hipStream_t st = (hipStream_t)stream;
    KParams kp = kp_in;
    if (kp.cuda && kp.bvh) hipLaunchKernelGGL((render_kernel_cuda<COUNT, true>), g, dim3(256), 0, st, kp);
    else if (kp.cuda) hipLaunchKernelGGL((render_kernel_cuda<COUNT, false>), g, dim3(256), 0, st, kp);
    else if (kp.bvh && kp.sky) hipLaunchKernelGGL((render_kernel<COUNT, true, true>), g, dim3(256), 0, st, kp);
    else if (kp.bvh) hipLaunchKernelGGL((render_kernel<COUNT, true, false>), g, dim3(256), 0, st, kp);
    else if (kp.sky) hipLaunchKernelGGL((render_kernel<COUNT, false, true>), g, dim3(256), 0, st, kp);
    else hipLaunchKernelGGL((render_kernel<COUNT, false, false>), g, dim3(256), 0, st, kp);
}

#if RT_QUEUE > 0
template <bool SKY, int AOM, int QB, bool OPQ = false>
static void queue_occupancy(int& nb)
{
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, render_kernel_q<SKY, AOM, QB, OPQ>, 256, 0);
}

// Resident blocks of the queue kernel on this device (grid of render_kernel_q).
// Cached per device and variant; rt_fill_canva may run on several host
// threads at once (main.c's pthreads), so the cache is atomic (every thread
// computes the same value).
template <int QB, bool OPQ = false>
static void queue_occupancy_v(bool sky, bool ao, int& nb)
{
    if (sky && ao) queue_occupancy<true, AO_ON, QB, OPQ>(nb);
    else if (sky) queue_occupancy<true, AO_OFF, QB, OPQ>(nb);
    else if (ao) queue_occupancy<false, AO_ON, QB, OPQ>(nb);
    else queue_occupancy<false, AO_OFF, QB, OPQ>(nb);
}
static unsigned queue_grid(bool sky, bool ao, int qb, bool opq)
{
    static std::atomic<int> cached[24][64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::atomic<int>& slot = cached[(sky ? 1 : 0) + (ao ? 2 : 0) + 4 * (qb == 0 ? 0 : qb == 3 ? (opq ? 5 : 1) : qb == 4 ? 2 : qb == -1 ? 3 : 4)][dev & 63];
    int c = slot.load(std::memory_order_relaxed);
    if (c <= 0) {
        int nb = 0, ncu = 0;
        if (qb == -2) queue_occupancy_v<-2>(sky, ao, nb);
        else if (qb == -1) queue_occupancy_v<-1>(sky, ao, nb);
        else if (qb == 0) queue_occupancy_v<0>(sky, ao, nb);
        else if (qb == 3 && opq) queue_occupancy_v<3, true>(sky, ao, nb);
        else if (qb == 3) queue_occupancy_v<3>(sky, ao, nb);
        else queue_occupancy_v<4>(sky, ao, nb);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        c = std::max(1, nb) * std::max(1, ncu);
        if (std::getenv("RT_QUEUE_VERBOSE")) std::fprintf(stderr, "render_kernel_q: %d blocks/CU x %d CUs -> %d\n", nb, ncu, c);
        slot.store(c, std::memory_order_relaxed);
    }
    // RT_QUEUE_BLOCKS (tests, experiments) is read on every launch, so a test
    // can shrink the grid to a few blocks and give every lane hundreds of tasks.
    if (const char* e = std::getenv("RT_QUEUE_BLOCKS")) c = std::max(1, std::atoi(e));
    return (unsigned)c;
}

template <int QB, bool OPQ = false>
static void queue_launch(bool sky, bool ao, unsigned nb, hipStream_t st, const KParams& k2)
{
    if (sky && ao) hipLaunchKernelGGL((render_kernel_q<true, AO_ON, QB, OPQ>), dim3(nb), dim3(256), 0, st, k2);
    else if (sky) hipLaunchKernelGGL((render_kernel_q<true, AO_OFF, QB, OPQ>), dim3(nb), dim3(256), 0, st, k2);
    else if (ao) hipLaunchKernelGGL((render_kernel_q<false, AO_ON, QB, OPQ>), dim3(nb), dim3(256), 0, st, k2);
    else hipLaunchKernelGGL((render_kernel_q<false, AO_OFF, QB, OPQ>), dim3(nb), dim3(256), 0, st, k2);
}

// floor((2^32 - 1) / d) for udiv_q
static unsigned qdiv_magic(unsigned d) { return d ? (unsigned)(0xffffffffull / d) : 0u; }
#endif

static thread_local const char* t_last_kernel = "none";
const char* last_render_kernel() { return t_last_kernel; }

// Which render kernel a launch takes (launch_render) and the LDS stack entries
// that kernel gives a BVH walk.  task_ok: the launch has render_kernel_q's task
// counter (spp_chunks > 1 and the band's tasks fit 32 bits, launch_on_stream).
// Node visits per lane and round: 4 for shallow trees (128-byte nodes, kp.bvh),
// 3 for deep ones (kp.bvh_steps, host; compile-time per instantiation).  The
// deep-tree instantiation walks the 64-byte nodes kp.bvhh: a deep tree that
// pack_bvh_h refused (a coordinate beyond binary16's range, a leaf index above
// 65535, an oversized leaf) renders with QB 4's walk when its stack fits there,
// else with the fixed-grid kernel; a shallow one keeps the queue kernel.
RenderChoice choose_render(const KParams& kp, bool task_ok)
{
    RenderChoice c;
    c.queue = false;
    c.qb = 0;
    c.opq = false;
    c.stack_cap = kp.bvh ? kStack4 : 0;
#if RT_QUEUE > 0
    bool qbvh = false;
    if (kp.bvh != nullptr && kp.bvh_stack <= kStackQN) {
        c.qb = kp.bvh_steps <= 3 || kp.bvh_stack > kStackQ4 ? 3 : 4;
        // a deep tree without 64-byte nodes whose stack fits QB 4's walks the
        // 128-byte nodes there (e.g. main()'s pyramide_eau mesh: triangles of
        // ~4000 units pad their boxes beyond binary16's range)
        if (c.qb == 3 && RT_QNODE_H && kp.bvhh == nullptr && kp.bvh_stack <= kStackQ4 && !kp.bvh_far) c.qb = 4;
        if (c.qb == 4 && kp.bvh_far) c.qb = 3;           // QB 4 has no far-origin margins (ray32<false>)
        qbvh = c.qb == 4 || !RT_QNODE_H || kp.bvhh != nullptr;
    }
    if (task_ok && kp.chunks > 1 && (!kp.bvh || qbvh) && !kp.cuda && !kp.sums) {
        c.queue = true;
        if (!qbvh) c.qb = RT_QSPHERES && kp.nt == 0 ? (RT_QOPAQUE && kp.opaque ? -2 : -1) : 0;
        c.opq = RT_QOPAQUE_BVH && c.qb == 3 && kp.opaque_all && kp.bvh_stack <= kStackQ && !kp.bvh_far;
        if (kp.bvh) c.stack_cap = c.qb == 4 ? kStackQ4 : c.opq ? kStackQ : kStackQN;
    }
#endif
    return c;
}

int launch_render(const KParams& kp, void* stream)
{
    const RenderChoice rc = choose_render(kp, kp.task_ctr != nullptr);
#if RT_QUEUE > 0
    if (rc.queue) {
        const hipStream_t st = (hipStream_t)stream;
        const bool sky = kp.sky != nullptr, ao = kp.useAO != 0;
        (void)hipMemsetAsync(kp.task_ctr, 0, sizeof(unsigned), st);
        const int qb = rc.qb;
        const bool opq = rc.opq;
        t_last_kernel = qb == 3   ? (opq ? "render_kernel_q<QB=3,OP>" : "render_kernel_q<QB=3>")
                        : qb == 4 ? "render_kernel_q<QB=4>"
                        : qb == -2 ? "render_kernel_q<QB=-2>"
                        : qb < 0  ? "render_kernel_q<QB=-1>"
                                  : "render_kernel_q<QB=0>";
        const unsigned nb = queue_grid(sky, ao, qb, opq);
        unsigned long long* tr = nullptr;
        const char* tf = std::getenv("RT_QUEUE_TRACE");
        if (tf) (void)hipMalloc((void**)&tr, (size_t)nb * 256 * RT_TRACE_WORDS * sizeof(unsigned long long));
        KParams k2 = kp;
        k2.trace = tr;
        const int rows_here = std::max(0, std::min(kp.band_rows, kp.local_rows - kp.band_y0));
        k2.npx_here = (unsigned)rows_here * (unsigned)kp.W;
        k2.qm_npx = qdiv_magic(k2.npx_here);
        k2.qm_w = qdiv_magic((unsigned)kp.W);
        k2.qm_tile = qdiv_magic((unsigned)kp.tile_rows);
        // chunk starts c*S/P in 32 bits when (P + 1) * S fits
        k2.qm_chunks = (unsigned long long)(kp.chunk_den + 1) * (unsigned long long)kp.S < (1ull << 32)
                           ? qdiv_magic(kp.chunk_den) : 0u;
        if (qb == 3 && opq) queue_launch<3, true>(sky, ao, nb, st, k2);
        else if (qb == 3) queue_launch<3>(sky, ao, nb, st, k2);
        else if (qb == 4) queue_launch<4>(sky, ao, nb, st, k2);
        else if (qb == -2) queue_launch<-2>(sky, ao, nb, st, k2);
        else if (qb < 0) queue_launch<-1>(sky, ao, nb, st, k2);
        else queue_launch<0>(sky, ao, nb, st, k2);
        if (tr) {
            std::vector<unsigned long long> h((size_t)nb * 256 * RT_TRACE_WORDS);
            (void)hipStreamSynchronize(st);
            (void)hipMemcpy(h.data(), tr, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            (void)hipFree(tr);
            if (FILE* f = std::fopen(tf, "ab")) {
                std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                std::fclose(f);
            }
        }
    } else
#endif
    {
        launch_variant<false>(kp, stream);
        t_last_kernel = kp.cuda ? "render_kernel_cuda" : kp.bvh ? "render_kernel<BVH>"
                                                                                                 : "render_kernel";
    }
    if (kp.chunks > 1) {
        const long long npx = (long long)kp.band_rows * kp.W;
        long long blocks = (npx + 255) / 256;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL(combine_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, kp);
    }
    return (int)hipGetLastError();
}

int launch_count(const KParams& kp, void* stream)
{
    launch_variant<true>(kp, stream);
    return (int)hipGetLastError();
}

int launch_assemble(const double* gathered, long long rank_stride, int world, int tile_rows, int rows_per_rank, int W,
                    int H, double* out, void* stream)
{
    const long long n = (long long)W * H * 3;
    long long blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, gathered,
                       rank_stride, world, tile_rows, rows_per_rank, W, H, out);
    return (int)hipGetLastError();
}

// Every sampler input r in [r0, r0 + n): phi_sincosf_fast against the full
// path pm_sincosf((float)pm_acos(2 r/2^31 - 1)).  counts[0] += inputs that
// fall back, counts[1] += inputs whose fast result differs (must stay 0).
__global__ __launch_bounds__(256) void verify_phi_kernel(unsigned long long r0, unsigned long long n,
                                                        unsigned long long* counts)
{
    const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    bool fb = false, bad = false;
    if (i < n) {
        const double xv = 2 * unit31((uint32_t)(r0 + i)) - 1;
        float sp, cp, s2, c2;
        const bool ok = phi_sincosf_fast(xv, sp, cp);
        pm_sincosf((float)pm_acos(xv), s2, c2);
        fb = !ok;
        bad = ok && (__float_as_uint(sp) != __float_as_uint(s2) || __float_as_uint(cp) != __float_as_uint(c2));
    }
    const unsigned long long nf = __popcll(__ballot(fb)), nb = __popcll(__ballot(bad));
    if ((threadIdx.x & 63) == 0) {
        if (nf) atomicAdd(counts, nf);
        if (nb) atomicAdd(counts + 1, nb);
    }
}

// Sphere closest hit of arbitrary rays (o, d: 6 doubles each): the candidate
// pass (spheres_closest, with its own exact fallback) against the plain exact
// scan.  counts[0] += rays the candidate pass sent to the exact scan,
// counts[1] += rays whose winner or t differs (must stay 0).
__global__ __launch_bounds__(256) void verify_spheres_kernel(const KParams kp, const double* __restrict__ rays,
                                                            long long n, unsigned long long* counts)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    bool fb = false, bad = false;
    if (i < n) {
        const V3 o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const V3 d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        const double a = dot(d, d), two_a = 2 * a, four_a = 4 * a;
        const bool fast = two_a >= 0x1p-100 && two_a <= 0x1p100;
        const double rc2a = rcp_refined(two_a);
        Cnt cnt;
        cnt.c[RT_CNT_EXACT_RESCANS] = 0;
        double t1, t2;
        const int w1 = spheres_closest<true, false>(kp, o, d, a, two_a, four_a, fast, rc2a, t1, cnt);
        const int w2 = spheres_exact_scan<false>(kp, o, d, two_a, four_a, fast, rc2a, t2);
        fb = cnt.c[RT_CNT_EXACT_RESCANS] != 0;
        bad = w1 != w2 || (w1 >= 0 && __double_as_longlong(t1) != __double_as_longlong(t2));
    }
    const unsigned long long nf = __popcll(__ballot(fb)), nb = __popcll(__ballot(bad));
    if ((threadIdx.x & 63) == 0) {
        if (nf) atomicAdd(counts, nf);
        if (nb) atomicAdd(counts + 1, nb);
    }
}

// normalize() (fast lanes: sqrt_rcp_core / rcp_refined + div_core) and its
// seeded forms against IEEE a / sqrt(a.a) on n pseudo-random vectors (Philox,
// key = seed), by q.w2 & 7:
//   0-3  normalize(): unit-scale vectors, n + dir sums, one common scale 2^e
//        (e in [-400, 400)), a scale per component
//   4-5  normalize_unit() on the sampler's vectors (sampler_vec of two 31-bit
//        draws, as random_dir makes them)
//   6-7  normalize() on hit-point offsets hp - C: C with components
//        scaled by 2^[-8, 12), |r| = 2^[-10, 10) times [1, 2), hp = C + r u for a
//        random unit u (rounded, as a hit point is), seeded as the host does
// counts[0] += vectors on a fast path, counts[1] += results that differ.
__device__ __forceinline__ double vn_comp(uint32_t hi, uint32_t lo)
{
    const unsigned long long m = ((unsigned long long)hi << 21) ^ (unsigned long long)(lo >> 11);
    const double u = (double)(m & ((1ull << 53) - 1)) * 0x1p-53;             // [0, 1)
    return (hi & 0x80000000u) ? -u : u;
}
__global__ __launch_bounds__(256) void verify_normalize_kernel(unsigned long long seed, unsigned long long i0,
                                                               unsigned long long n, unsigned long long* counts)
{
    const unsigned long long i = i0 + (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    bool fp = false, bad = false;
    if (i < i0 + n) {
        const Philox p = philox4x32_10<false>((uint32_t)i, (uint32_t)(i >> 32), 0x6e6f726du, 0u, (uint32_t)seed,
                                              (uint32_t)(seed >> 32));
        const Philox q = philox4x32_10<false>((uint32_t)i, (uint32_t)(i >> 32), 0x6e6f726du, 1u, (uint32_t)seed,
                                              (uint32_t)(seed >> 32));
        V3 a = v3(vn_comp(p.w0, p.w1), vn_comp(p.w2, p.w3), vn_comp(q.w0, q.w1));
        const uint32_t cls = q.w2 & 7u;
        V3 got;
        if (cls >= 4u) {                            // the sampler's unit vectors
            a = sampler_vec(p.w0 >> 1, p.w1 >> 1);
            fp = true;
            got = normalize_unit(a);
        } else {
            if (cls == 1u) {                               // n + dir: unit normal plus a unit vector
                const V3 nn = divs(a, sqrt(dot(a, a)));
                a = nn + v3(vn_comp(q.w3, p.w0), vn_comp(p.w1 ^ q.w3, p.w2), vn_comp(p.w3, q.w0 ^ p.w1));
            } else if (cls == 2u) {                        // one scale for the vector
                const int e = (int)(q.w3 % 800u) - 400;
                a = v3(ldexp(a.x, e), ldexp(a.y, e), ldexp(a.z, e));
            } else if (cls == 3u) {                        // a scale per component
                a = v3(ldexp(a.x, (int)(q.w3 % 900u) - 450), ldexp(a.y, (int)((q.w3 >> 10) % 900u) - 450),
                       ldexp(a.z, (int)((q.w3 >> 20) % 900u) - 450));
            }
            const double n2 = dot(a, a);
            const double mn = fmin(fmin(fabs(a.x), fabs(a.y)), fabs(a.z));
            fp = n2 >= 0x1p-760 && n2 <= 0x1p760 && mn >= 0x1p-900;
            got = normalize(a);
        }
        const V3 want = divs(a, sqrt(dot(a, a)));
        bad = __double_as_longlong(got.x) != __double_as_longlong(want.x) ||
              __double_as_longlong(got.y) != __double_as_longlong(want.y) ||
              __double_as_longlong(got.z) != __double_as_longlong(want.z);
        bad = bad && !(got.x != got.x && want.x != want.x);   // NaN == NaN
    }
    const unsigned long long nf = __popcll(__ballot(fp)), nb = __popcll(__ballot(bad));
    if ((threadIdx.x & 63) == 0) {
        if (nf) atomicAdd(counts, nf);
        if (nb) atomicAdd(counts + 1, nb);
    }
}

int launch_verify_normalize(unsigned long long seed, unsigned long long n, unsigned long long* d_counts)
{
    const unsigned long long per = 1ull << 30;          // launches of at most 2^30 vectors
    for (unsigned long long i0 = 0; i0 < n; i0 += per) {
        const unsigned long long m = std::min(per, n - i0);
        hipLaunchKernelGGL(verify_normalize_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, nullptr, seed,
                           i0, m, d_counts);
    }
    return hipGetLastError();
}

// rt_verify_texel_map: point i (3 doubles) on triangle tri[i] through the
// affine texel map and through the exact path; counts[0] += certain,
// counts[1] += certain but a different texel
__global__ __launch_bounds__(256) void verify_texel_kernel(const KParams kp, const double* __restrict__ pts,
                                                           const int* __restrict__ tri, long long n,
                                                           unsigned long long* counts)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    bool fast = false, bad = false;
    if (i < n) {
        const int k = tri[i];
        const V3 P = v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        const TexRef e = tri_texel_exact(kp, k, P, tri_normal(kp, k));
        TexRef f{0, 0};
        fast = tri_texel_affine(kp, k, P, f);
        bad = fast && (f.index != e.index || f.m != e.m);
    }
    const unsigned long long nf = __popcll(__ballot(fast)), nb = __popcll(__ballot(bad));
    if ((threadIdx.x & 63) == 0) {
        if (nf) atomicAdd(counts, nf);
        if (nb) atomicAdd(counts + 1, nb);
    }
}

int launch_verify_texel(const KParams& kp, const double* d_pts, const int* d_tri, long long n,
                        unsigned long long* d_counts)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(verify_texel_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, kp, d_pts,
                       d_tri, n, d_counts);
    return hipGetLastError();
}

int launch_verify_spheres(const KParams& kp, const double* d_rays, long long n, unsigned long long* d_counts)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(verify_spheres_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, kp, d_rays,
                       n, d_counts);
    return hipGetLastError();
}

int launch_verify_phi(unsigned long long r0, unsigned long long n, unsigned long long* d_counts)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(verify_phi_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, r0, n, d_counts);
    return hipGetLastError();
}

int launch_selftest(int op, const double* d_in, double* d_out, int n, void* stream)
{
    hipLaunchKernelGGL(selftest_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, op,
                       d_in, d_out, n);
    return (int)hipGetLastError();
}

}  // namespace rt
