/*
 * oracle/rt_oracle.h — TEST INFRASTRUCTURE: CPU restatement of the
 * reference render path (xelema/tipe-raytracer main.c + headers).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so.  The product (librt_hip.so) never links or calls it.
 *
 * Pinning: RT_RNG_GLIBC mode (libm + the process' glibc rand()) reproduces
 * the reference's own composition — main.c:22-284 + denoiser.h:11-29
 * compiled verbatim in oracle/_ref/libref_tracer.so — bit for bit on every
 * plane (tests/golden/composition.json: config 1 in full, AO, refraction,
 * textures, alpha holes, the C4 tree, random scenes); leaf functions are
 * compared with the reference headers compiled in oracle/_ref/libref_leaf.so
 * and with tests/golden/kat_leaf.json (see oracle/Makefile).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include "../include/rt/rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_hit {          /* HitInfo, hitinfo.h:15-21 */
    int didHit;
    double dst;
    rt_point3 hitPoint;
    rt_vec3 normal;
    rt_material mat;
} oracle_hit;

/* Full render of rows row_hi..row_lo (descending, main.c:248) using
 * nthreads pthreads over contiguous row bands (main.c:407-449).  Any of
 * albedo/normal/radiance may be NULL; radiance receives sum/S (pre-gamma).
 * counters: RT_NCOUNTERS totals, may be NULL.  In RT_RNG_GLIBC mode the
 * libc generator is reseeded with srand(1) first when reseed != 0. */
int oracle_render_rows(const rt_scene* scene, const rt_params* params,
                       int row_hi, int row_lo, int nthreads, int reseed,
                       rt_color* canva, rt_color* albedo, rt_color* normal,
                       rt_color* radiance, unsigned long long* counters);

/* Force the math library: -1 auto (libm for GLIBC, portable for PHILOX),
 * 0 libm, 1 portable.  Global; for experiments only. */
void oracle_set_math(int mode);
/* Speed only: skip the triangle scan of rays that cannot meet the mesh's
 * padded box (main.c mode; default on, identical frames either way). */
void oracle_set_mesh_cull(int on);

/* Leaf functions (for parity against the compiled reference headers). */
oracle_hit oracle_hit_sphere(rt_point3 center, double radius, rt_ray r);
oracle_hit oracle_hit_triangle(const rt_triangle* tri, rt_ray r);
oracle_hit oracle_hit_sphere_cuda(rt_point3 center, double radius, rt_ray r);   /* sphere.hu:13-47 */
rt_material oracle_tri_uvmapping(const rt_triangle* tri, const oracle_hit* h,
                                 const rt_material* mat_list, int tw, int th,
                                 int tri_index, const int* quelMatPourTri);
rt_vec3 oracle_refracted_vec(rt_vec3 v, rt_vec3 n, double n1, double n2);
rt_vec3 oracle_reflected_vec(rt_vec3 v, rt_vec3 n);
rt_color oracle_write_color_canva(rt_color c, int spp);
rt_color oracle_rgb_to_hsl(rt_color c);
rt_color oracle_hsl_to_rgb(rt_color c);
rt_camera oracle_init_camera(rt_point3 origin, rt_point3 target, rt_vec3 up,
                             double vfov, double ratio);
rt_ray oracle_get_ray(double u, double v, const rt_camera* cam, double focus,
                      double dx, double dy);

/* One sample through tracer() (main.c:118-242) with the given stream:
 * rng = RT_RNG_GLIBC uses libc rand() as-is; RT_RNG_PHILOX uses
 * (seed, pixel, sample).  out[0..2] = radiance, albedo, normal. */
void oracle_trace_sample(const rt_scene* scene, const rt_params* params,
                         rt_ray r, unsigned pixel, unsigned sample, rt_color out[3]);

/* IOR stack (pile.h) ops on an opaque stack, for semantic tests:
 * ops[i] = materialIndex to enter via index_suivant_pile + info_pile_actuelle,
 * exit[i] != 0 additionally pops (main.c:169-181).  Writes n1,n2 per op. */
void oracle_pile_sequence(const double* ops, const int* exit_flags, int n,
                          double* n1_out, double* n2_out);

/* Portable math + Philox (oracle/pm_math.h) exported for tests. */
double oracle_pm_acos(double x);
float  oracle_pm_sinf(float x);
float  oracle_pm_cosf(float x);
double oracle_pm_pow(double x, double y);
double oracle_pm_atan2(double y, double x);
long long oracle_sky_index(rt_vec3 center, double radius, rt_vec3 hitPoint, int w, int h, int portable);
void   oracle_philox(const unsigned* ctr4, const unsigned* key2, unsigned* out4);
/* Exhaustive scan: counts floats x in [lo, hi] (as float bit ranges) where
 * pm_sinf/pm_cosf differ from libm sinf/cosf.  Uses nthreads. */
void oracle_scan_sincosf(float lo, float hi, int nthreads,
                         unsigned long long* n_total, unsigned long long* n_sin_diff,
                         unsigned long long* n_cos_diff);
/* Strided scan of the floats in [lo, hi]: counts where pm_sinf/pm_cosf
 * differ from the correctly rounded float sin/cos (via sinl/cosl). */
void oracle_scan_sincosf_cr(float lo, float hi, long long step, int nthreads,
                            unsigned long long* n_total, unsigned long long* n_sin_diff,
                            unsigned long long* n_cos_diff);
/* acos over the 2^31 grid inputs 2*(k/2^31)-1, k = k0..k1-1 (step): counts
 * results differing from libm acos, and those whose float rounding differs. */
void oracle_scan_acos(long long k0, long long k1, long long step, int nthreads,
                      unsigned long long* n_total, unsigned long long* n_diff,
                      unsigned long long* n_float_diff);

#ifdef __cplusplus
}
#endif
#endif
