/*
 * oracle/ref_leaf_harness.c — TEST INFRASTRUCTURE (container only).
 *
 * Compiles the reference's leaf headers where they lie (-I/root/reference)
 * and exports pointer-based wrappers so tests can compare the oracle's
 * restatement with the reference's own code on identical inputs.  Nothing
 * from the reference is copied; this file only #includes it.  Output goes to
 * oracle/_ref/ (git-ignored).  main.c / denoiser.h are not included: they
 * require the absent OpenImageDenoise header.
 */
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>

#include "vec3.h"
#include "ray.h"
#include "hitinfo.h"
#include "sphere.h"
#include "rtutility.h"
#include "camera.h"
#include "mesh.h"
#include "texture.h"
#include "pile.h"

#define EXPORT __attribute__((visibility("default")))

typedef struct ref_hit {   /* mirrors oracle_hit: int didHit + HitInfo tail */
    int didHit;
    double dst;
    point3 hitPoint;
    vec3 normal;
    material mat;
} ref_hit;

static void to_ref_hit(const HitInfo* h, ref_hit* o)
{
    o->didHit = h->didHit ? 1 : 0;
    o->dst = h->dst;
    o->hitPoint = h->hitPoint;
    o->normal = h->normal;
    o->mat = h->mat;
}

EXPORT void ref_hit_sphere(const point3* center, double radius, const ray* r, ref_hit* out)
{
    HitInfo h = hit_sphere(*center, radius, *r);
    if (!h.didHit) { h.dst = 0; h.hitPoint = vec3_init(); h.normal = vec3_init(); }
    h.mat = (material){{{0, 0, 0}}, {{0, 0, 0}}, 0, 0, 0, 0};
    to_ref_hit(&h, out);
}

EXPORT void ref_hit_triangle(const triangle* tri, const ray* r, ref_hit* out)
{
    HitInfo h = hit_triangle(*tri, *r);
    h.mat = (material){{{0, 0, 0}}, {{0, 0, 0}}, 0, 0, 0, 0};
    to_ref_hit(&h, out);
}

EXPORT void ref_tri_uvmapping(const triangle* tri, const ref_hit* hin, material* mat_list, int tw, int th,
                              int tri_index, int* quelMat, material* out)
{
    HitInfo h;
    h.didHit = hin->didHit;
    h.dst = hin->dst;
    h.hitPoint = hin->hitPoint;
    h.normal = hin->normal;
    h.mat = hin->mat;
    *out = tri_uvmapping(*tri, h, mat_list, tw, th, tri_index, quelMat);
}

EXPORT void ref_sphere_uvmapping(const point3* center, double radius, const point3* hitPoint, material* mat_list,
                                 int w, int h, material* out)
{
    sphere s;
    s.center = *center;
    s.radius = radius;
    HitInfo hi;
    hi.didHit = true;
    hi.dst = 1.0;
    hi.hitPoint = *hitPoint;
    hi.normal = vec3_init();
    *out = sphere_uvmapping(s, hi, mat_list, w, h);
}

EXPORT void ref_refracted_vec(const vec3* v, const vec3* n, double n1, double n2, vec3* out)
{
    *out = refracted_vec(*v, *n, n1, n2);
}
EXPORT void ref_reflected_vec(const vec3* v, const vec3* n, vec3* out) { *out = reflected_vec(*v, *n); }
EXPORT void ref_vec3_lerp(const vec3* x, const vec3* y, double t, vec3* out) { *out = vec3_lerp(*x, *y, t); }
EXPORT void ref_write_color_canva(const color* c, int spp, color* out) { *out = write_color_canva(*c, spp); }
EXPORT void ref_rgb_to_hsl(const color* c, color* out) { *out = rgb_to_hsl(*c); }
EXPORT void ref_hsl_to_rgb(const color* c, color* out) { *out = hsl_to_rgb(*c); }
EXPORT void ref_init_camera(const point3* o, const point3* t, const vec3* up, double vfov, double ratio, camera* out)
{
    *out = init_camera(*o, *t, *up, vfov, ratio);
}
EXPORT void ref_get_ray(double u, double v, const camera* cam, double focus, double dx, double dy, ray* out)
{
    *out = get_ray(u, v, *cam, focus, dx, dy);
}
EXPORT void ref_srand(unsigned s) { srand(s); }
EXPORT int ref_rand(void) { return rand(); }
EXPORT double ref_randomDouble(double lo, double hi) { return randomDouble(lo, hi); }
EXPORT void ref_random_dir_no_norm(vec3* out) { *out = random_dir_no_norm(); }

/* Same op sequence as oracle_pile_sequence (main.c:169-181 usage). */
EXPORT void ref_pile_sequence(const double* ops, const int* exit_flags, int n, double* n1_out, double* n2_out)
{
    pile* p = init_pile();
    empiler(p, 1.0, 1.0);
    for (int i = 0; i < n; i++) {
        index_suivant_pile(p, ops[i]);
        IndRef ind = info_pile_actuelle(p);
        double n1 = ind.n[0], n2 = ind.n[1];
        if (exit_flags[i]) {
            ind = depiler(p);
            n1 = ind.n[1];
            n2 = ind.n[0];
        }
        n1_out[i] = n1;
        n2_out[i] = n2;
    }
    while (p->premier) depiler(p);
    free(p);
}

/* Loader path, mesh.h:96-234 + texture.h:175-354.  Returns the triangle
 * array (caller frees with ref_free) or NULL; *mat_list_out likewise. */
EXPORT triangle* ref_list_of_mesh(const char* obj, const char* mtl, int* nTri, int* nMat, int** quelMat)
{
    char** paths;
    int* quelSommet;
    triangle* t = list_of_mesh(obj, mtl, nTri, nMat, &paths, &quelSommet, quelMat);
    free(quelSommet);
    return t;
}

EXPORT material* ref_load_textures(const char* obj, const char* mtl, int* tw, int* th)
{
    char** paths;
    int* quelSommet;
    int* quelMat;
    int nTri, nMat;
    triangle* t = list_of_mesh(obj, mtl, &nTri, &nMat, &paths, &quelSommet, &quelMat);
    material* m = create_mat_list_mtl(paths, tw, th, nMat);
    free(t);
    free(quelSommet);
    free(quelMat);
    return m;
}

EXPORT void ref_move_mesh(double x, double y, double z, triangle* tris, int n)
{
    move_mesh(x, y, z, &tris, n);
}

EXPORT void ref_free(void* p) { free(p); }
