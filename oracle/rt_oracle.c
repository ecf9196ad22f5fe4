/*
 * oracle/rt_oracle.c — TEST INFRASTRUCTURE: plain-C restatement of the
 * reference render path, written from its semantics (not copied).
 *
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg.  Every function cites the reference file:line it restates.
 *
 * Two stream modes (rt.h RT_RNG_*):
 *  - GLIBC : the process' glibc rand() and libm, exactly as the reference;
 *            single-threaded output reproduces main.c bit for bit.
 *  - PHILOX: per-(pixel, sample) Philox4x32-10 stream + portable math
 *            (pm_math.h); the spec the HIP kernel implements.
 *
 * Compile with -ffp-contract=off: every + - * / is one IEEE rounding, in
 * the reference's association order.
 *
 * Pinning (both parts against the reference's own code compiled here):
 *  - leaf functions (hit_sphere, hit_triangle, tri_uvmapping, camera,
 *    optics, pile, HSL, write_color_canva) against the reference headers
 *    (oracle/_ref/libref_leaf.so, tests/golden/kat_leaf.json);
 *  - the composition — closest_hit / ambient_occlusion / tracer / fill_canva
 *    (main.c:52-284) and add_col_alb_norm (denoiser.h:23-29) — against those
 *    line ranges compiled VERBATIM (oracle/build_ref_tracer.sh, sha256-pinned,
 *    no stub header; oracle/_ref/libref_tracer.so).  GLIBC mode reproduces
 *    them bit for bit on every plane: config 1 in full (P3 md5
 *    930550ea86f4b2de4ac3a92726beb976), AO at int 2 and 2.5, translucent and
 *    alpha-hole spheres, the C3 pyramid, mineways' alpha texels, the C4 tree
 *    + AO and random scenes (tests/golden/composition.json,
 *    tests/test_oracle_composition.py).  PHILOX mode runs the same
 *    composition code with the other stream and the portable math.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"
#include "pm_math.h"

#define REF_PI 3.1415926535897932385          /* rtutility.h:14 */

static int g_math_mode = -1;
void oracle_set_math(int mode) { g_math_mode = mode; }

/* ------------------------------------------------------------------------ */
/* vec3 helpers — vec3.h:57-139, ray.h:26-29                                 */
/* ------------------------------------------------------------------------ */
static inline rt_vec3 v3(double a, double b, double c) { rt_vec3 r = {{a, b, c}}; return r; }
static inline rt_vec3 add(rt_vec3 a, rt_vec3 b) { return v3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
static inline rt_vec3 sub(rt_vec3 a, rt_vec3 b) { return v3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
static inline rt_vec3 mul(rt_vec3 a, rt_vec3 b) { return v3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
static inline rt_vec3 mul_s(rt_vec3 a, double t) { return v3(a.e[0] * t, a.e[1] * t, a.e[2] * t); }
static inline rt_vec3 div_s(rt_vec3 a, double t) { return v3(a.e[0] / t, a.e[1] / t, a.e[2] / t); }
static inline rt_vec3 neg(rt_vec3 a) { return v3(-a.e[0], -a.e[1], -a.e[2]); }
static inline double dot(rt_vec3 a, rt_vec3 b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
static inline rt_vec3 cross(rt_vec3 u, rt_vec3 v)
{
    return v3(u.e[1] * v.e[2] - u.e[2] * v.e[1],
              u.e[2] * v.e[0] - u.e[0] * v.e[2],
              u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
static inline double length(rt_vec3 a) { return sqrt(dot(a, a)); }
static inline rt_vec3 normalize(rt_vec3 a) { return div_s(a, length(a)); }
static inline rt_vec3 ray_at(rt_ray r, double t) { return add(r.origin, mul_s(r.dir, t)); }
static inline rt_vec3 lerp(rt_vec3 x, rt_vec3 y, double t) { return add(x, mul_s(sub(y, x), t)); }  /* rtutility.h:32-34 */

/* ------------------------------------------------------------------------ */
/* per-thread render context                                                 */
/* ------------------------------------------------------------------------ */
typedef struct ctx {
    const rt_scene* sc;
    int B, useAO;
    double AO;
    int rng, portable;
    int sky;                 /* rt.h RT_SKY_LAST_SPHERE with a sky table */
    int cuda;                /* rt.h RT_SEM_CUDA: main_cuda.cu's integrator */
    rt_point3 bb_lo, bb_hi;  /* CUDA mode: the triangles' bounding box */
    int mesh_cull;           /* main.c mode: skip the triangle scan for rays that miss mb_lo..mb_hi */
    rt_point3 mb_lo, mb_hi;  /* the triangles' box padded by 2^-16 (1 + max |coordinate|) */
    uint64_t seed;
    uint32_t pixel, sample, n;
    uint32_t block[4];
    unsigned long long cnt[RT_NCOUNTERS];
} ctx;

/* rand() replacement point: rtutility.h:171-172,192-193,230 */
static inline unsigned rnd31(ctx* c)
{
    c->cnt[RT_CNT_RNG_DRAWS]++;
    if (c->rng == RT_RNG_GLIBC) return (unsigned)rand();
    if ((c->n & 3u) == 0u) {
        uint32_t ctr[4] = {c->n >> 2, 0u, c->pixel, c->sample};
        uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
        pm_philox4x32_10(ctr, key, c->block);
    }
    uint32_t w = c->block[c->n & 3u];
    c->n++;
    return w >> 1;
}

/* randomDouble, rtutility.h:229-231 */
static inline double random_double(ctx* c, double min, double max)
{
    return min + (max - min) * (rnd31(c) / (RAND_MAX + 1.0));
}

/* random_dir_no_norm, rtutility.h:189-203 */
static rt_vec3 random_dir_no_norm(ctx* c)
{
    c->cnt[RT_CNT_SHADE]++;
    double u = rnd31(c) / (RAND_MAX + 1.0);
    double v = rnd31(c) / (RAND_MAX + 1.0);
    double theta = 2 * REF_PI * u;
    rt_vec3 dir;
    if (c->portable) {
        double phi = pm_acos(2 * v - 1);
        dir.e[0] = (double)(pm_cosf((float)theta) * pm_sinf((float)phi));
        dir.e[1] = (double)(pm_sinf((float)theta) * pm_sinf((float)phi));
        dir.e[2] = (double)pm_cosf((float)phi);
    } else {
        double phi = acos(2 * v - 1);
        dir.e[0] = cosf(theta) * sinf(phi);
        dir.e[1] = sinf(theta) * sinf(phi);
        dir.e[2] = cosf(phi);
    }
    return normalize(dir);
}

/* reflected_vec, rtutility.h:205-208 */
static inline rt_vec3 reflected_vec(rt_vec3 v, rt_vec3 n) { return sub(v, mul_s(n, 2 * dot(v, n))); }

/* refracted_vec, rtutility.h:210-227 (n1, n2 squared first: reference quirk) */
static rt_vec3 refracted_vec(rt_vec3 v, rt_vec3 normal, double n1, double n2)
{
    n1 *= n1;
    n2 *= n2;
    double radical = 1 - ((n1 / n2) * (n1 / n2)) * (1 - (dot(normal, v) * dot(normal, v)));
    if (radical > 0) {
        rt_vec3 comp_tan = mul_s(sub(v, mul_s(normal, dot(v, normal))), (n1 / n2));
        rt_vec3 comp_normal = mul_s(neg(normal), sqrt(radical));
        return add(comp_tan, comp_normal);
    }
    return reflected_vec(v, normal);
}

/* rgb_to_hsl / hue_to_rgb / hsl_to_rgb, rtutility.h:81-165 */
static rt_color rgb_to_hsl(rt_color rgb)
{
    double r = rgb.e[0], g = rgb.e[1], b = rgb.e[2];
    double mx = (r > g) ? ((r > b) ? r : b) : ((g > b) ? g : b);
    double mn = (r < g) ? ((r < b) ? r : b) : ((g < b) ? g : b);
    double h = 0.0, s, l = (mx + mn) / 2.0;
    if (mx == mn) {
        h = 0.0;
        s = 0.0;
    } else {
        double d = mx - mn;
        s = (l < 0.5) ? (d / (mx + mn)) : (d / (2.0 - mx - mn));
        if (mx == r) h = (g - b) / d + ((g < b) ? 6.0 : 0.0);
        else if (mx == g) h = (b - r) / d + 2.0;
        else if (mx == b) h = (r - g) / d + 4.0;
        h /= 6.0;
    }
    return v3(h, s, l);
}

static double hue_to_rgb(double t1, double t2, double hue)
{
    if (hue < 0.0) hue += 1.0;
    if (hue > 1.0) hue -= 1.0;
    if (6.0 * hue < 1.0) return t1 + (t2 - t1) * 6.0 * hue;
    if (2.0 * hue < 1.0) return t2;
    if (3.0 * hue < 2.0) return t1 + (t2 - t1) * ((2.0 / 3.0) - hue) * 6.0;
    return t1;
}

static rt_color hsl_to_rgb(rt_color hsl)
{
    double h = hsl.e[0], s = hsl.e[1], l = hsl.e[2];
    if (s == 0.0) return v3(l, l, l);
    double t2 = (l < 0.5) ? (l * (1.0 + s)) : (l + s - l * s);
    double t1 = 2.0 * l - t2;
    return v3(hue_to_rgb(t1, t2, h + 1.0 / 3.0), hue_to_rgb(t1, t2, h), hue_to_rgb(t1, t2, h - 1.0 / 3.0));
}

/* ------------------------------------------------------------------------ */
/* geometry                                                                 */
/* ------------------------------------------------------------------------ */
/* hit_sphere, sphere.h:13-47 */
static oracle_hit hit_sphere(ctx* c, rt_point3 center, double radius, rt_ray r)
{
    oracle_hit h;
    memset(&h, 0, sizeof h);
    if (c) c->cnt[RT_CNT_SPHERE_TESTS]++;
    rt_vec3 oc = sub(r.origin, center);
    double a = dot(r.dir, r.dir);
    double b = 2.0 * dot(oc, r.dir);
    double cc = dot(oc, oc) - radius * radius;
    double disc = b * b - 4 * a * cc;
    if (disc > 0) {
        if (c) c->cnt[RT_CNT_SPHERE_DISC]++;
        double t1 = (-b - sqrt(disc)) / (2 * a);
        if (t1 >= 0.0001) {
            h.didHit = 1;
            h.dst = t1;
            h.hitPoint = ray_at(r, t1);
            h.normal = normalize(sub(ray_at(r, t1), center));
            return h;
        }
        double t2 = (-b + sqrt(disc)) / (2 * a);
        if (t2 >= 0.0001) {
            h.didHit = 1;
            h.dst = t2;
            h.hitPoint = ray_at(r, t2);
            h.normal = normalize(sub(ray_at(r, t2), center));
            return h;
        }
    }
    return h;
}

/* hit_triangle, mesh.h:70-94 (one-sided, eps 1e-6 / 1e-7); the CUDA path's
 * triangle.hu:247-270 is the same arithmetic with eps 1e-5 for dst/u/v/w */
static oracle_hit hit_triangle_eps(ctx* c, const rt_triangle* tri, rt_ray r, double eps);
static oracle_hit hit_triangle(ctx* c, const rt_triangle* tri, rt_ray r)
{
    return hit_triangle_eps(c, tri, r, 0.0000001);
}
static oracle_hit hit_triangle_eps(ctx* c, const rt_triangle* tri, rt_ray r, double eps)
{
    oracle_hit h;
    memset(&h, 0, sizeof h);
    if (c) c->cnt[RT_CNT_TRI_TESTS]++;
    rt_point3 edgeAB = sub(tri->B, tri->A);
    rt_point3 edgeAC = sub(tri->C, tri->A);
    rt_vec3 normalVect = cross(edgeAB, edgeAC);
    rt_vec3 ao = sub(r.origin, tri->A);
    rt_vec3 dao = cross(ao, r.dir);
    double det = -dot(r.dir, normalVect);
    double invDet = 1 / det;
    double dst = dot(ao, normalVect) * invDet;
    double u = dot(edgeAC, dao) * invDet;
    double v = -dot(edgeAB, dao) * invDet;
    double w = 1 - u - v;
    h.didHit = det >= 1E-6 && dst >= eps && u >= eps && v >= eps && w >= eps;
    h.dst = dst;
    if (h.didHit) {          /* read only for a hit (speed: the same values mesh.h:91-92 computes) */
        h.hitPoint = add(r.origin, mul_s(r.dir, dst));
        h.normal = normalize(normalVect);
    }
    return h;
}

/* get_barycentric_coord, texture.h:16-27 */
static rt_point3 barycentric(const rt_triangle* tri, const oracle_hit* h)
{
    double areaABC = dot(h->normal, cross(sub(tri->B, tri->A), sub(tri->C, tri->A)));
    double areaPBC = dot(h->normal, cross(sub(tri->B, h->hitPoint), sub(tri->C, h->hitPoint)));
    double areaPCA = dot(h->normal, cross(sub(tri->C, h->hitPoint), sub(tri->A, h->hitPoint)));
    rt_point3 res;
    res.e[0] = areaPBC / areaABC;
    res.e[1] = areaPCA / areaABC;
    res.e[2] = 1.0 - res.e[0] - res.e[1];
    return res;
}

/* tri_uvmapping, texture.h:44-90.  Out-of-table texel indices (reference UB)
 * are clamped into the table; DESIGN.md "Defined behaviour". */
static rt_material tri_uvmapping(const rt_triangle* tri, const oracle_hit* h, const rt_material* mat_list,
                                 int tw, int th, long long n_texels, int indice_tri, const int* quelMat)
{
    rt_point3 bary = barycentric(tri, h);
    double uu = (bary.e[0] * tri->uvA.u + bary.e[1] * tri->uvB.u + bary.e[2] * tri->uvC.u);
    double vv = (bary.e[0] * tri->uvA.v + bary.e[1] * tri->uvB.v + bary.e[2] * tri->uvC.v);
    uu = fmod(uu, 1.0);
    vv = fmod(vv, 1.0);
    if (uu < 0) uu += 1.0;
    if (vv < 0) vv += 1.0;
    int x = (int)(uu * (double)(tw));
    int y = (int)(vv * (double)(th));
    int numero_mat = quelMat[indice_tri];
    long long index = ((long long)y * tw + x) + ((long long)th * tw * numero_mat);
    if (index < 0) index = 0;
    if (index >= n_texels) index = n_texels - 1;
    rt_material res = mat_list[index];
    if (numero_mat == 1) {
        res.emissionColor = v3(1, 1, 1);
        res.emissionStrength = 1.85;
        res.alpha = 1.0;
    }
    if (numero_mat == 4) {
        res.alpha = 0.6;
        res.materialIndex = 1.33;
        res.reflectionStrength = 0.93;
    }
    if (numero_mat == 3) {
        res.alpha = 0.1;
        res.materialIndex = 1.50;
        res.reflectionStrength = 0.3;
    }
    return res;
}

/* sphere_uvmapping, texture.h:92-112 (equirect sky texel).  The texel index
 * is clamped into the table (the reference indexes unchecked). */
static rt_material sphere_uvmapping(ctx* c, const rt_sphere* s, rt_vec3 hitPoint)
{
    const rt_scene* sc = c->sc;
    const double PI = 3.1415926535897932385;               /* rtutility.h:14 */
    const double inv = 1 / s->radius;                      /* divide(), vec3.h:105-107 */
    rt_vec3 d = v3((hitPoint.e[0] - s->center.e[0]) * inv, (hitPoint.e[1] - s->center.e[1]) * inv,
                   (hitPoint.e[2] - s->center.e[2]) * inv);
    double theta = c->portable ? pm_acos(-d.e[1]) : acos(-d.e[1]);
    double phi = (c->portable ? pm_atan2(-d.e[2], d.e[0]) : atan2(-d.e[2], d.e[0])) + PI;
    double u = phi / (2 * PI), v = theta / PI;
    int x = (int)(u * (double)(sc->sky_width));
    int y = (int)(v * (double)(sc->sky_height));
    long long index = (long long)y * sc->sky_width + x;
    long long n = (long long)sc->sky_width * sc->sky_height;
    index = index < 0 ? 0 : (index >= n ? n - 1 : index);
    return sc->sky_mat_list[index];
}

/* Speed only (test infrastructure, not a reference function): a conservative
 * test whether the ray can meet the triangles' box mb_lo..mb_hi at t >= 0.
 * An accepted hit_triangle needs det >= 1e-6 and u, v, w >= 1e-7, so the exact
 * ray-plane point lies within the triangle up to the rounding of u and v
 * (first order: a few ulp of the coordinates scaled by 1/det, below 1e-8 for
 * coordinates of magnitude <= 1e3); the box is padded by 2^-16 (1 + max
 * |coordinate|), far above that, and the slab distances are widened by
 * 2^-30 relative.  Non-finite rays always scan.  oracle_set_mesh_cull(0)
 * turns it off (tests/test_oracle.py checks both give the same frames). */
static int g_mesh_cull = 1;
void oracle_set_mesh_cull(int on) { g_mesh_cull = on; }
static int meets_mesh_box(const ctx* c, rt_ray r)
{
    double t0 = 0.0, t1 = INFINITY;
    for (int k = 0; k < 3; k++) {
        const double o = r.origin.e[k], d = r.dir.e[k];
        if (!isfinite(o) || !isfinite(d)) return 1;
        const double lo = c->mb_lo.e[k], hi = c->mb_hi.e[k];
        if (d == 0.0) {
            if (o < lo || o > hi) return 0;
            continue;
        }
        double a = (lo - o) / d, b = (hi - o) / d;
        if (a > b) { const double x = a; a = b; b = x; }
        a -= fabs(a) * 0x1p-30;
        b += fabs(b) * 0x1p-30;
        if (a > t0) t0 = a;
        if (b < t1) t1 = b;
    }
    return t0 <= t1;
}

/* closest_hit, main.c:52-92 (linear scan: spheres, then triangles) */
static oracle_hit closest_hit(ctx* c, rt_ray r, int count_tex)
{
    const rt_scene* sc = c->sc;
    oracle_hit best;
    memset(&best, 0, sizeof best);
    best.didHit = 0;
    best.dst = INFINITY;
    c->cnt[RT_CNT_CASTS]++;
    for (int i = 0; i < sc->nbSpheres; i++) {
        const rt_sphere* s = &sc->sphere_list[i];
        oracle_hit h = hit_sphere(c, s->center, s->radius, r);
        if (h.didHit && h.dst < best.dst) {
            best = h;
            best.mat = s->mat;
            if (c->sky && i == sc->nbSpheres - 1) {        /* main.c:64-71 (commented out there) */
                rt_material sky_mat = sphere_uvmapping(c, s, h.hitPoint);
                best.mat.emissionColor = sky_mat.diffuseColor;
                best.mat.alpha = 1.0;
            }
        }
    }
    int tri_won = 0;
    long long n_texels = (long long)sc->nbMaterials * sc->tex_width * sc->tex_height;
    int nt = sc->nbTriangles;
    if (nt > 0 && c->mesh_cull && !meets_mesh_box(c, r)) {   /* no triangle can be hit: the scan finds none */
        c->cnt[RT_CNT_TRI_TESTS] += (unsigned long long)nt;  /* (the reference's count: it tests them all) */
        nt = 0;
    }
    for (int i = 0; i < nt; i++) {
        const rt_triangle* tri = &sc->triangle_list[i];
        oracle_hit h = hit_triangle(c, tri, r);
        if (h.didHit && h.dst < best.dst) {
            rt_material tex_mat = tri_uvmapping(tri, &h, sc->mat_list, sc->tex_width, sc->tex_height,
                                                n_texels, i, sc->quelMatPourTri);
            best = h;
            best.mat = tex_mat;
            tri_won = 1;
        }
    }
    if (count_tex && tri_won && best.didHit) c->cnt[RT_CNT_TEX_HITS]++;
    return best;
}

/* ---- CUDA path (rt.h RT_SEM_CUDA) ----------------------------------------- */
/* hit_sphere, sphere.hu:13-47: the same discriminant and roots as sphere.h,
 * accepting t1 >= 0, then t2 >= 0.001 */
static oracle_hit hit_sphere_cuda(ctx* c, rt_point3 center, double radius, rt_ray r)
{
    oracle_hit h;
    memset(&h, 0, sizeof h);
    if (c) c->cnt[RT_CNT_SPHERE_TESTS]++;
    rt_vec3 oc = sub(r.origin, center);
    double a = dot(r.dir, r.dir);
    double b = 2.0 * dot(oc, r.dir);
    double cc = dot(oc, oc) - radius * radius;
    double disc = b * b - 4 * a * cc;
    if (disc > 0) {
        if (c) c->cnt[RT_CNT_SPHERE_DISC]++;
        double t1 = (-b - sqrt(disc)) / (2 * a);
        if (t1 >= 0) {
            h.didHit = 1;
            h.dst = t1;
            h.hitPoint = ray_at(r, t1);
            h.normal = normalize(sub(ray_at(r, t1), center));
            return h;
        }
        double t2 = (-b + sqrt(disc)) / (2 * a);
        if (t2 >= 0.001) {
            h.didHit = 1;
            h.dst = t2;
            h.hitPoint = ray_at(r, t2);
            h.normal = normalize(sub(ray_at(r, t2), center));
            return h;
        }
    }
    return h;
}

/* hit_BBox, triangle.hu:42-59 (CUDA min/max on doubles are fmin/fmax) */
static int hit_bbox_cuda(const ctx* c, rt_ray r)
{
    double tmin[3], tmax[3];
    for (int k = 0; k < 3; k++) {
        double t1 = (c->bb_lo.e[k] - r.origin.e[k]) / r.dir.e[k];
        double t2 = (c->bb_hi.e[k] - r.origin.e[k]) / r.dir.e[k];
        tmin[k] = fmin(t1, t2);
        tmax[k] = fmax(t1, t2);
    }
    return fmin(fmin(tmax[0], tmax[1]), tmax[2]) - fmax(fmax(tmin[0], tmin[1]), tmin[2]) > 0;
}

/* closest_hit, main_cuda.cu:23-59: spheres, then (if the ray meets the mesh
 * box) the triangles, each with its own material (the CUDA loader's per-mesh
 * material, triangle.hu:104-105) */
static oracle_hit closest_hit_cuda(ctx* c, rt_ray r)
{
    const rt_scene* sc = c->sc;
    oracle_hit best;
    memset(&best, 0, sizeof best);
    best.dst = INFINITY;
    c->cnt[RT_CNT_CASTS]++;
    for (int i = 0; i < sc->nbSpheres; i++) {
        const rt_sphere* s = &sc->sphere_list[i];
        oracle_hit h = hit_sphere_cuda(c, s->center, s->radius, r);
        if (h.didHit && h.dst < best.dst) {
            best = h;
            best.mat = s->mat;
        }
    }
    if (sc->nbTriangles > 0 && hit_bbox_cuda(c, r)) {
        for (int i = 0; i < sc->nbTriangles; i++) {
            const rt_triangle* tri = &sc->triangle_list[i];
            oracle_hit h = hit_triangle_eps(c, tri, r, 0.00001);
            if (h.didHit && h.dst < best.dst) {
                best = h;
                best.mat = tri->mat;
            }
        }
    }
    return best;
}

/* ambient_occlusion, main.c:94-116 (nbSamples = 1); main_cuda.cu:61-84 is
 * the same with its own closest_hit */
static rt_color ambient_occlusion(ctx* c, rt_vec3 point, rt_vec3 normal, double AO_intensity)
{
    const int nbSamples = 1;
    rt_color occlusion = v3(0, 0, 0);
    for (int i = 0; i < nbSamples; ++i) {
        rt_vec3 randomDir = random_dir_no_norm(c);
        rt_vec3 hemisphereDir = add(normal, randomDir);
        rt_ray occlusionRay = {point, normalize(hemisphereDir)};
        oracle_hit oh = c->cuda ? closest_hit_cuda(c, occlusionRay) : closest_hit(c, occlusionRay, 0);
        if (oh.didHit) {
            double distance = length(sub(oh.hitPoint, point));
            double attenuation = distance / oh.dst;
            attenuation = c->portable ? pm_pow(attenuation, AO_intensity) : pow(attenuation, AO_intensity);
            occlusion = add(occlusion, v3(attenuation, attenuation, attenuation));
        }
    }
    return div_s(div_s(occlusion, nbSamples), AO_intensity);
}

/* ------------------------------------------------------------------------ */
/* IOR stack, pile.h:9-72 (array-backed; same push/pop semantics)            */
/* ------------------------------------------------------------------------ */
typedef struct { double n[2]; } ind_ref;
typedef struct { ind_ref* el; int size, cap; } pile;

static void pile_init(pile* p) { p->el = NULL; p->size = 0; p->cap = 0; }
static void pile_free(pile* p) { free(p->el); }
static void empiler(pile* p, double n1, double n2)
{
    if (p->size == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 8;
        p->el = (ind_ref*)realloc(p->el, sizeof(ind_ref) * (size_t)p->cap);
        if (!p->el) abort();
    }
    p->el[p->size].n[0] = n1;
    p->el[p->size].n[1] = n2;
    p->size++;
}
static ind_ref depiler(pile* p)
{
    ind_ref res = {{0.0, 0.0}};  /* pile.h:35-44 leaves it uninitialised; unreachable */
    if (p->size > 0) res = p->el[--p->size];
    return res;
}
static void index_suivant_pile(pile* p, double n2)   /* pile.h:61-66 */
{
    ind_ref ancien = depiler(p);
    double old_n2 = ancien.n[1];
    empiler(p, ancien.n[0], ancien.n[1]);
    empiler(p, old_n2, n2);
}
static ind_ref info_pile_actuelle(pile* p)            /* pile.h:68-72 */
{
    ind_ref res = depiler(p);
    empiler(p, res.n[0], res.n[1]);
    return res;
}

/* ------------------------------------------------------------------------ */
/* tracer, main.c:118-242                                                    */
/* ------------------------------------------------------------------------ */
static void tracer(ctx* c, rt_ray r, rt_color out[3])
{
    rt_color incomingLight = v3(0, 0, 0);
    rt_color rayColor = v3(1, 1, 1);
    rt_color albedo_color = v3(0, 0, 0);
    rt_color normal_color = v3(0, 0, 0);
    int is_alpha = 0;
    int alpha_depth = 0;
    double n1 = 0.0, n2 = 1.0;
    pile pl;
    pile_init(&pl);
    empiler(&pl, 1.0, 1.0);
    ind_ref ind;

    for (int i = 0; i < c->B; i++) {
        oracle_hit h = closest_hit(c, r, 1);
        rt_material mat = h.mat;   /* zero on a miss (reference: indeterminate) */

        if (i == 0) {
            albedo_color = mat.diffuseColor;
            normal_color = h.normal;
        }
        if (i == alpha_depth && is_alpha) {
            albedo_color = mat.diffuseColor;
            if (mat.emissionStrength > 0) albedo_color = mat.emissionColor;
            normal_color = h.normal;
            is_alpha = 0;
        }

        if (h.didHit) {
            if (i == alpha_depth && mat.emissionStrength > 0) {   /* main.c:154-160 */
                rt_color HSL = rgb_to_hsl(mat.emissionColor);
                HSL.e[2] *= 1.0;
                HSL.e[1] *= 1.0;
                rt_color newCol = hsl_to_rgb(HSL);
                out[0] = newCol;
                out[1] = newCol;
                out[2] = h.normal;
                pile_free(&pl);
                return;
            }

            r.origin = h.hitPoint;
            rt_vec3 diffuse_dir = normalize(add(h.normal, random_dir_no_norm(c)));
            rt_vec3 reflected_dir = reflected_vec(r.dir, h.normal);
            rt_vec3 diff_ref_dir = lerp(diffuse_dir, reflected_dir, mat.reflectionStrength);

            if (mat.alpha <= 0.99 && mat.alpha >= 0.0001) {        /* main.c:167-193 */
                c->cnt[RT_CNT_REFRACT]++;
                rt_vec3 normal = h.normal;
                index_suivant_pile(&pl, mat.materialIndex);
                ind = info_pile_actuelle(&pl);
                n1 = ind.n[0];
                n2 = ind.n[1];
                if (dot(r.dir, h.normal) > 0) {
                    normal = neg(h.normal);
                    ind = depiler(&pl);
                    n1 = ind.n[1];
                    n2 = ind.n[0];
                }
                rt_vec3 refracted_dir = refracted_vec(r.dir, normal, n1, n2);
                double rnd = random_double(c, 0, 1);
                if (rnd > mat.alpha) {
                    r.dir = refracted_dir;
                    continue;
                } else {
                    r.dir = diff_ref_dir;
                }
            }
            if (mat.alpha > 0.99) {
                is_alpha = 0;
                r.dir = diff_ref_dir;
            }
            if (mat.alpha < 0.0001) {                               /* main.c:200-206 */
                r.origin = h.hitPoint;
                is_alpha = 1;
                alpha_depth++;
                continue;
            }

            if (c->useAO) {                                         /* main.c:208-222 */
                rt_color emittedLight = mul_s(mat.emissionColor, mat.emissionStrength * 1.5 * c->AO);
                incomingLight = add(incomingLight, mul(emittedLight, rayColor));
                if (rayColor.e[0] > 0.5 || rayColor.e[1] > 0.5 || rayColor.e[2] > 0.5)
                    rayColor = mul(mat.diffuseColor, mul_s(rayColor, 1.3));
                rayColor = mul(mat.diffuseColor, rayColor);
                rt_color occlusion = ambient_occlusion(c, h.hitPoint, h.normal, c->AO);
                rayColor = mul(rayColor, occlusion);
            } else {                                                /* main.c:224-234 */
                rt_color emittedLight = mul_s(mat.emissionColor, mat.emissionStrength);
                incomingLight = add(incomingLight, mul(emittedLight, rayColor));
                if (rayColor.e[0] > 0.5 || rayColor.e[1] > 0.5 || rayColor.e[2] > 0.5)
                    rayColor = mul(mat.diffuseColor, mul_s(rayColor, 1.3));
                rayColor = mul(mat.diffuseColor, rayColor);
            }
        } else {
            break;
        }
    }
    (void)n2;
    pile_free(&pl);
    out[0] = incomingLight;
    out[1] = albedo_color;
    out[2] = normal_color;
}

/* tracer, main_cuda.cu:86-141.  The pre-pass cast returns emitters (HSL
 * round trip with L and S x1.20) and misses (0); the bounce loop then starts
 * from the same ray; albedo/normal are the pre-pass hit's (the function's
 * outer hitInfo, main_cuda.cu:140). */
static void tracer_cuda(ctx* c, rt_ray r, rt_color out[3])
{
    oracle_hit first = closest_hit_cuda(c, r);
    if (first.didHit) {
        if (first.mat.emissionStrength > 0) {
            rt_color HSL = rgb_to_hsl(first.mat.emissionColor);
            HSL.e[2] *= 1.20;
            HSL.e[1] *= 1.20;
            rt_color newCol = hsl_to_rgb(HSL);
            out[0] = newCol;
            out[1] = newCol;
            out[2] = first.normal;
            return;
        }
    } else {
        out[0] = out[1] = out[2] = v3(0, 0, 0);
        return;
    }
    rt_color incomingLight = v3(0, 0, 0);
    rt_color rayColor = v3(1, 1, 1);
    for (int i = 0; i < c->B; i++) {
        oracle_hit h = closest_hit_cuda(c, r);
        if (h.didHit) {
            rt_material mat = h.mat;
            r.origin = h.hitPoint;
            rt_vec3 diffuse_dir = normalize(add(h.normal, random_dir_no_norm(c)));
            rt_vec3 reflected_dir = sub(r.dir, mul_s(h.normal, 2 * dot(r.dir, h.normal)));
            r.dir = lerp(diffuse_dir, reflected_dir, mat.reflectionStrength);
            if (c->useAO) {
                rt_color emittedLight = mul_s(mat.emissionColor, mat.emissionStrength * 1.5 * c->AO);
                incomingLight = add(incomingLight, mul(emittedLight, rayColor));
                rayColor = mul(mat.diffuseColor, rayColor);
                rt_color occlusion = ambient_occlusion(c, h.hitPoint, h.normal, c->AO);
                rayColor = mul(rayColor, occlusion);
            } else {
                rt_color emittedLight = mul_s(mat.emissionColor, mat.emissionStrength);
                incomingLight = add(incomingLight, mul(emittedLight, rayColor));
                rayColor = mul(mat.diffuseColor, rayColor);
            }
        } else {
            break;
        }
    }
    out[0] = incomingLight;
    out[1] = first.mat.diffuseColor;
    out[2] = first.normal;
}

/* ------------------------------------------------------------------------ */
/* camera, camera.h:21-55; resolve, rtutility.h:56-71                        */
/* ------------------------------------------------------------------------ */
static rt_ray get_ray(double u, double v, const rt_camera* cam, double focus, double dx, double dy)
{
    rt_ray res;
    rt_vec3 direction = add(cam->coin_bas_gauche,
                            add(mul_s(cam->horizontal, u), sub(mul_s(cam->vertical, v), cam->origin)));
    rt_vec3 destination = add(cam->origin, mul_s(direction, focus));
    rt_point3 new_origin = add(cam->origin, v3(dx, dy, 0));
    res.origin = new_origin;
    res.dir = normalize(sub(destination, new_origin));
    return res;
}

static double clampd(double x, double mn, double mx)
{
    if (x < mn) return mn;
    if (x > mx) return mx;
    return x;
}

static rt_color write_color_canva(rt_color px, int spp)
{
    double r = px.e[0], g = px.e[1], b = px.e[2];
    double rapport = 1.0 / spp;
    r = sqrtf((float)(rapport * r));
    g = sqrtf((float)(rapport * g));
    b = sqrtf((float)(rapport * b));
    return v3((int)(256 * clampd(r, 0.0, 0.999)), (int)(256 * clampd(g, 0.0, 0.999)),
              (int)(256 * clampd(b, 0.0, 0.999)));
}

/* ------------------------------------------------------------------------ */
/* fill_canva, main.c:245-284, and the row-band driver main.c:404-453        */
/* ------------------------------------------------------------------------ */
typedef struct band {
    const rt_scene* sc;
    const rt_params* p;
    int start_row, end_row;
    double focus, ox, oy, AO;
    int portable;
    rt_color *canva, *albedo, *normal, *radiance;
    unsigned long long cnt[RT_NCOUNTERS];
} band;

static void init_ctx(ctx* c, const band* b)
{
    memset(c, 0, sizeof *c);
    c->sc = b->sc;
    c->B = b->p->nbRebondMax;
    c->useAO = b->p->useAO;
    c->AO = b->AO;
    c->rng = b->p->rng;
    c->portable = b->portable;
    c->sky = b->p->sky_mode == RT_SKY_LAST_SPHERE && b->sc->sky_mat_list && b->sc->nbSpheres > 0;
    c->seed = b->p->seed;
    c->cuda = b->p->semantics == RT_SEM_CUDA;
    if (!c->cuda && b->sc->nbTriangles > 0 && g_mesh_cull) {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, m = 0.0;
        int finite = 1;
        for (int i = 0; i < b->sc->nbTriangles; i++) {
            const rt_triangle* t = &b->sc->triangle_list[i];
            const rt_point3* P[3] = {&t->A, &t->B, &t->C};
            for (int q = 0; q < 3; q++)
                for (int k = 0; k < 3; k++) {
                    const double x = P[q]->e[k];
                    finite = finite && isfinite(x);
                    lo[k] = fmin(lo[k], x);
                    hi[k] = fmax(hi[k], x);
                    m = fmax(m, fabs(x));
                }
        }
        const double pad = 0x1p-16 * (1.0 + m);
        c->mesh_cull = finite;
        for (int k = 0; k < 3; k++) {
            c->mb_lo.e[k] = lo[k] - pad;
            c->mb_hi.e[k] = hi[k] + pad;
        }
    }
    if (c->cuda && b->sc->nbTriangles > 0) {           /* load_geometry_data's box, triangle.hu:142-156 */
        const rt_triangle* t0 = &b->sc->triangle_list[0];
        c->bb_lo = t0->A;
        c->bb_hi = t0->A;
        for (int i = 0; i < b->sc->nbTriangles; i++) {
            const rt_triangle* t = &b->sc->triangle_list[i];
            for (int k = 0; k < 3; k++) {
                c->bb_lo.e[k] = fmin(c->bb_lo.e[k], fmin(t->A.e[k], fmin(t->B.e[k], t->C.e[k])));
                c->bb_hi.e[k] = fmax(c->bb_hi.e[k], fmax(t->A.e[k], fmax(t->B.e[k], t->C.e[k])));
            }
        }
    }
}

static void* band_worker(void* arg)
{
    band* b = (band*)arg;
    const rt_params* p = b->p;
    const int W = p->largeur_image, H = p->hauteur_image, S = p->nbRayonParPixel;
    ctx c;
    init_ctx(&c, b);
    /* rt.h spp_chunks: P > 1 sums samples in P fixed slices, then the slice
     * sums in slice order; P = 1 is fill_canva's running sum (main.c:264-273) */
    const int P = rt_resolve_spp_chunks(p->spp_chunks, S);
    for (int j = b->start_row; j >= b->end_row; --j) {
        for (int i = 0; i < W; i++) {
            int pixel_index = j * W + i;
            rt_color tot[3] = {v3(0, 0, 0), v3(0, 0, 0), v3(0, 0, 0)};
            for (int ch = 0; ch < P; ++ch) {
                const int s0 = (int)rt_chunk_bound(ch, S, P), s1 = (int)rt_chunk_bound(ch + 1, S, P);
                rt_color part[3] = {v3(0, 0, 0), v3(0, 0, 0), v3(0, 0, 0)};
                for (int x = s0; x < s1; ++x) {
                    c.pixel = (uint32_t)pixel_index;
                    c.sample = (uint32_t)x;
                    c.n = 0;
                    c.cnt[RT_CNT_SAMPLES]++;
                    double u, v;
                    if (c.cuda) {                      /* main_cuda.cu:152-153 */
                        u = ((double)i + 0.5 + random_double(&c, -0.5, 0.5)) / (W - 1);
                        v = ((double)j + 0.5 + random_double(&c, -0.5, 0.5)) / (H - 1);
                    } else {                           /* main.c:265-266 */
                        u = ((double)i + random_double(&c, -0.5, 0.5)) / (W - 1);
                        v = ((double)j + random_double(&c, -0.5, 0.5)) / (H - 1);
                    }
                    double dx = random_double(&c, -0.5, 0.5) * b->ox;
                    double dy = random_double(&c, -0.5, 0.5) * b->oy;
                    rt_ray r = get_ray(u, v, &p->cam, b->focus, dx, dy);
                    rt_color smp[3];
                    if (c.cuda) tracer_cuda(&c, r, smp);
                    else tracer(&c, r, smp);
                    part[0] = add(part[0], smp[0]);
                    part[1] = add(part[1], smp[1]);
                    part[2] = add(part[2], smp[2]);
                }
                if (ch == 0) {
                    tot[0] = part[0];
                    tot[1] = part[1];
                    tot[2] = part[2];
                } else {
                    tot[0] = add(tot[0], part[0]);
                    tot[1] = add(tot[1], part[1]);
                    tot[2] = add(tot[2], part[2]);
                }
            }
            b->canva[pixel_index] = write_color_canva(tot[0], S);
            if (b->albedo) b->albedo[pixel_index] = div_s(tot[1], S);
            if (b->normal) b->normal[pixel_index] = div_s(tot[2], S);
            if (b->radiance) b->radiance[pixel_index] = div_s(tot[0], S);
        }
    }
    memcpy(b->cnt, c.cnt, sizeof c.cnt);
    return NULL;
}

static int validate(const rt_scene* sc, const rt_params* p)
{
    if (!sc || !p) return RT_EINVAL;
    if (p->largeur_image < 1 || p->hauteur_image < 1 || p->nbRayonParPixel < 1 || p->nbRebondMax < 0)
        return RT_EINVAL;
    if (p->rng != RT_RNG_GLIBC && p->rng != RT_RNG_PHILOX) return RT_EINVAL;
    if (p->semantics != RT_SEM_MAIN_C && p->semantics != RT_SEM_CUDA) return RT_EINVAL;
    if (p->semantics == RT_SEM_CUDA && p->sky_mode != RT_SKY_OFF) return RT_EINVAL;
    if (p->precision != RT_PREC_FP64) return RT_EINVAL;   /* the restatement is the fp64 spec only */
    if (sc->nbSpheres < 0 || sc->nbTriangles < 0) return RT_EINVAL;
    if (sc->nbSpheres > 0 && !sc->sphere_list) return RT_EINVAL;
    if (sc->nbTriangles > 0) {
        if (!sc->triangle_list || !sc->mat_list || !sc->quelMatPourTri) return RT_EINVAL;
        if (sc->tex_width < 1 || sc->tex_height < 1 || sc->nbMaterials < 1) return RT_EINVAL;
        for (int i = 0; i < sc->nbTriangles; i++)
            if (sc->quelMatPourTri[i] < 0 || sc->quelMatPourTri[i] >= sc->nbMaterials) return RT_EINVAL;
    }
    return RT_OK;
}

int oracle_render_rows(const rt_scene* scene, const rt_params* params, int row_hi, int row_lo, int nthreads,
                       int reseed, rt_color* canva, rt_color* albedo, rt_color* normal, rt_color* radiance,
                       unsigned long long* counters)
{
    int rc = validate(scene, params);
    if (rc) return rc;
    if (!canva || row_lo < 0 || row_hi >= params->hauteur_image || row_hi < row_lo) return RT_EINVAL;
    int nrows = row_hi - row_lo + 1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nrows) nthreads = nrows;

    double focus = params->focus_distance, ox = params->ouverture_x, oy = params->ouverture_y;
    double AO = params->AO_intensity;
    if (params->compat_int_truncation && params->semantics != RT_SEM_CUDA) {   /* ThreadData int fields, main.c:42-43 */
        focus = (double)(int)focus;
        ox = (double)(int)ox;
        oy = (double)(int)oy;
        AO = (double)(int)AO;
    }
    int portable = g_math_mode >= 0 ? g_math_mode : (params->rng == RT_RNG_PHILOX);
    if (params->rng == RT_RNG_GLIBC && reseed) srand(1);

    band* bands = (band*)calloc((size_t)nthreads, sizeof(band));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!bands || !th) {
        free(bands);
        free(th);
        return RT_ENOMEM;
    }
    int rows_per_thread = nrows / nthreads;   /* main.c:407-449 */
    int remaining_rows = nrows % nthreads;
    int start_row = row_hi;
    for (int t = 0; t < nthreads; t++) {
        int end_row = start_row - rows_per_thread + 1;
        if (t == nthreads - 1) end_row -= remaining_rows;
        band* b = &bands[t];
        b->sc = scene;
        b->p = params;
        b->start_row = start_row;
        b->end_row = end_row;
        b->focus = focus;
        b->ox = ox;
        b->oy = oy;
        b->AO = AO;
        b->portable = portable;
        b->canva = canva;
        b->albedo = albedo;
        b->normal = normal;
        b->radiance = radiance;
        start_row = end_row - 1;
    }
    if (nthreads == 1) {
        band_worker(&bands[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, band_worker, &bands[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    if (counters) {
        for (int t = 0; t < nthreads; t++)
            for (int k = 0; k < RT_NCOUNTERS; k++) counters[k] += bands[t].cnt[k];
    }
    free(bands);
    free(th);
    return RT_OK;
}

/* ------------------------------------------------------------------------ */
/* exported leaf functions                                                   */
/* ------------------------------------------------------------------------ */
oracle_hit oracle_hit_sphere(rt_point3 center, double radius, rt_ray r) { return hit_sphere(NULL, center, radius, r); }
oracle_hit oracle_hit_triangle(const rt_triangle* tri, rt_ray r) { return hit_triangle(NULL, tri, r); }
oracle_hit oracle_hit_sphere_cuda(rt_point3 center, double radius, rt_ray r)
{
    return hit_sphere_cuda(NULL, center, radius, r);
}
rt_material oracle_tri_uvmapping(const rt_triangle* tri, const oracle_hit* h, const rt_material* mat_list, int tw,
                                 int th, int tri_index, const int* quelMatPourTri)
{
    return tri_uvmapping(tri, h, mat_list, tw, th, (long long)1 << 62, tri_index, quelMatPourTri);
}
rt_vec3 oracle_refracted_vec(rt_vec3 v, rt_vec3 n, double n1, double n2) { return refracted_vec(v, n, n1, n2); }
rt_vec3 oracle_reflected_vec(rt_vec3 v, rt_vec3 n) { return reflected_vec(v, n); }
rt_color oracle_write_color_canva(rt_color c, int spp) { return write_color_canva(c, spp); }
rt_color oracle_rgb_to_hsl(rt_color c) { return rgb_to_hsl(c); }
rt_color oracle_hsl_to_rgb(rt_color c) { return hsl_to_rgb(c); }
rt_ray oracle_get_ray(double u, double v, const rt_camera* cam, double focus, double dx, double dy)
{
    return get_ray(u, v, cam, focus, dx, dy);
}

/* init_camera, camera.h:21-40 */
rt_camera oracle_init_camera(rt_point3 origin, rt_point3 target, rt_vec3 up, double vfov, double ratio)
{
    rt_camera cam;
    double theta = vfov * 3.1415926535897932385 / 180.0;
    double h = tan(theta / 2);
    double hauteur_viewport = 2.0 * h;
    double largeur_viewport = ratio * hauteur_viewport;
    rt_vec3 w = normalize(sub(origin, target));
    rt_vec3 u = normalize(cross(up, w));
    rt_vec3 v = cross(w, u);
    cam.origin = origin;
    cam.horizontal = mul_s(u, largeur_viewport);
    cam.vertical = mul_s(v, hauteur_viewport);
    cam.coin_bas_gauche = sub(cam.origin, add(div_s(cam.horizontal, 2), add(div_s(cam.vertical, 2), w)));
    return cam;
}

void oracle_trace_sample(const rt_scene* scene, const rt_params* params, rt_ray r, unsigned pixel, unsigned sample,
                         rt_color out[3])
{
    band b;
    memset(&b, 0, sizeof b);
    b.sc = scene;
    b.p = params;
    b.AO = params->compat_int_truncation ? (double)(int)params->AO_intensity : params->AO_intensity;
    b.portable = g_math_mode >= 0 ? g_math_mode : (params->rng == RT_RNG_PHILOX);
    ctx c;
    init_ctx(&c, &b);
    c.pixel = pixel;
    c.sample = sample;
    c.n = 0;
    tracer(&c, r, out);
}

void oracle_pile_sequence(const double* ops, const int* exit_flags, int n, double* n1_out, double* n2_out)
{
    pile pl;
    pile_init(&pl);
    empiler(&pl, 1.0, 1.0);
    for (int i = 0; i < n; i++) {
        index_suivant_pile(&pl, ops[i]);
        ind_ref ind = info_pile_actuelle(&pl);
        double n1 = ind.n[0], n2 = ind.n[1];
        if (exit_flags[i]) {
            ind = depiler(&pl);
            n1 = ind.n[1];
            n2 = ind.n[0];
        }
        n1_out[i] = n1;
        n2_out[i] = n2;
    }
    pile_free(&pl);
}

double oracle_pm_acos(double x) { return pm_acos(x); }
float oracle_pm_sinf(float x) { return pm_sinf(x); }
float oracle_pm_cosf(float x) { return pm_cosf(x); }
double oracle_pm_pow(double x, double y) { return pm_pow(x, y); }
void oracle_pm_pow_n(const double* xy, double* out, long long n)   /* pairs (x, y) */
{
    for (long long i = 0; i < n; ++i) out[i] = pm_pow(xy[2 * i], xy[2 * i + 1]);
}
double oracle_pm_atan2(double y, double x) { return pm_atan2(y, x); }

/* texel index sphere_uvmapping picks (test hook; portable: 0 libm, 1 pm_*) */
long long oracle_sky_index(rt_vec3 center, double radius, rt_vec3 hitPoint, int w, int h, int portable)
{
    rt_material* mats = (rt_material*)calloc((size_t)w * h, sizeof(rt_material));
    for (long long k = 0; k < (long long)w * h; ++k) mats[k].diffuseColor.e[0] = (double)k;
    rt_scene sc;
    memset(&sc, 0, sizeof sc);
    sc.sky_mat_list = mats;
    sc.sky_width = w;
    sc.sky_height = h;
    ctx c;
    memset(&c, 0, sizeof c);
    c.sc = &sc;
    c.portable = portable;
    rt_sphere s;
    memset(&s, 0, sizeof s);
    s.center = center;
    s.radius = radius;
    const long long k = (long long)sphere_uvmapping(&c, &s, hitPoint).diffuseColor.e[0];
    free(mats);
    return k;
}
void oracle_philox(const unsigned* ctr4, const unsigned* key2, unsigned* out4)
{
    uint32_t c[4] = {ctr4[0], ctr4[1], ctr4[2], ctr4[3]}, k[2] = {key2[0], key2[1]}, o[4];
    pm_philox4x32_10(c, k, o);
    for (int i = 0; i < 4; i++) out4[i] = o[i];
}

/* ---- exhaustive math scans (multi-threaded) ---------------------------- */
typedef struct scan_job {
    uint32_t b0, b1;           /* float bit range, inclusive-exclusive */
    long long k0, k1, step;
    unsigned long long tot, d1, d2;
} scan_job;

static void* sincos_worker(void* arg)
{
    scan_job* j = (scan_job*)arg;
    for (uint32_t b = j->b0; b < j->b1; b++) {
        float x;
        memcpy(&x, &b, 4);
        float s1 = sinf(x), s2 = pm_sinf(x), c1 = cosf(x), c2 = pm_cosf(x);
        j->tot++;
        if (memcmp(&s1, &s2, 4)) j->d1++;
        if (memcmp(&c1, &c2, 4)) j->d2++;
    }
    return NULL;
}

void oracle_scan_sincosf(float lo, float hi, int nthreads, unsigned long long* n_total,
                         unsigned long long* n_sin_diff, unsigned long long* n_cos_diff)
{
    uint32_t b0, b1;
    memcpy(&b0, &lo, 4);
    memcpy(&b1, &hi, 4);
    b1 += 1;
    if (nthreads < 1) nthreads = 1;
    scan_job* jobs = (scan_job*)calloc((size_t)nthreads, sizeof(scan_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    uint32_t span = (b1 - b0 + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        jobs[t].b0 = b0 + (uint32_t)t * span;
        jobs[t].b1 = jobs[t].b0 + span > b1 ? b1 : jobs[t].b0 + span;
        if (jobs[t].b0 > b1) jobs[t].b0 = b1;
        pthread_create(&th[t], NULL, sincos_worker, &jobs[t]);
    }
    *n_total = *n_sin_diff = *n_cos_diff = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        *n_total += jobs[t].tot;
        *n_sin_diff += jobs[t].d1;
        *n_cos_diff += jobs[t].d2;
    }
    free(jobs);
    free(th);
}

/* pm_sinf/pm_cosf against the correctly rounded float sin/cos: the x87
 * long-double sinl/cosl, rounded to float (64-bit significand; a double
 * rounding through it would need a sin value within 2^-64 relative of a
 * float midpoint). */
static void* sincos_cr_worker(void* arg)
{
    scan_job* j = (scan_job*)arg;
    for (long long b = j->k0; b < j->k1; b += j->step) {
        const uint32_t bits = (uint32_t)b;
        float x;
        memcpy(&x, &bits, 4);
        const float s1 = (float)sinl((long double)x), c1 = (float)cosl((long double)x);
        const float s2 = pm_sinf(x), c2 = pm_cosf(x);
        j->tot++;
        if (memcmp(&s1, &s2, 4)) j->d1++;
        if (memcmp(&c1, &c2, 4)) j->d2++;
    }
    return NULL;
}

void oracle_scan_sincosf_cr(float lo, float hi, long long step, int nthreads, unsigned long long* n_total,
                            unsigned long long* n_sin_diff, unsigned long long* n_cos_diff)
{
    uint32_t b0, b1;
    memcpy(&b0, &lo, 4);
    memcpy(&b1, &hi, 4);
    if (nthreads < 1) nthreads = 1;
    if (step < 1) step = 1;
    scan_job* jobs = (scan_job*)calloc((size_t)nthreads, sizeof(scan_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t].k0 = (long long)b0 + t * step;
        jobs[t].k1 = (long long)b1 + 1;
        jobs[t].step = step * nthreads;
        pthread_create(&th[t], NULL, sincos_cr_worker, &jobs[t]);
    }
    *n_total = *n_sin_diff = *n_cos_diff = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        *n_total += jobs[t].tot;
        *n_sin_diff += jobs[t].d1;
        *n_cos_diff += jobs[t].d2;
    }
    free(jobs);
    free(th);
}

static void* acos_worker(void* arg)
{
    scan_job* j = (scan_job*)arg;
    for (long long k = j->k0; k < j->k1; k += j->step) {
        double v = (double)k / (RAND_MAX + 1.0);
        double x = 2 * v - 1;
        double a1 = acos(x), a2 = pm_acos(x);
        j->tot++;
        if (memcmp(&a1, &a2, 8)) {
            j->d1++;
            float f1 = (float)a1, f2 = (float)a2;
            if (memcmp(&f1, &f2, 4)) j->d2++;
        }
    }
    return NULL;
}

void oracle_scan_acos(long long k0, long long k1, long long step, int nthreads, unsigned long long* n_total,
                      unsigned long long* n_diff, unsigned long long* n_float_diff)
{
    if (nthreads < 1) nthreads = 1;
    if (step < 1) step = 1;
    scan_job* jobs = (scan_job*)calloc((size_t)nthreads, sizeof(scan_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t].k0 = k0 + (long long)t * step;
        jobs[t].k1 = k1;
        jobs[t].step = step * nthreads;
        pthread_create(&th[t], NULL, acos_worker, &jobs[t]);
    }
    *n_total = *n_diff = *n_float_diff = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        *n_total += jobs[t].tot;
        *n_diff += jobs[t].d1;
        *n_float_diff += jobs[t].d2;
    }
    free(jobs);
    free(th);
}
