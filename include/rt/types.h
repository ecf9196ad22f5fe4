/*
 * rt/types.h — reference-shaped data types of the render path.
 *
 * Every struct here is byte-for-byte layout-compatible (x86-64 SysV) with the
 * type of the same role in xelema/tipe-raytracer, so a caller can hand the
 * reference's own arrays to the C-ABI with a pointer cast:
 *
 *   rt_vec3        == vec3 / point3 / color   vec3.h:7-9, 145-146    (24 B)
 *   rt_ray         == ray                     ray.h:6-9              (48 B)
 *   rt_material    == material                hitinfo.h:6-13         (80 B)
 *   rt_sphere      == sphere                  sphere.h:7-11          (112 B)
 *   rt_uv          == UV                      mesh.h:9-12            (16 B)
 *   rt_triangle    == triangle                mesh.h:14-22           (200 B)
 *   rt_camera      == camera                  camera.h:10-15         (96 B)
 *   rt_thread_data == struct ThreadData       main.c:22-46           (248 B)
 *
 * The names are prefixed so this header can be included next to the
 * reference headers (which define the unprefixed names) without clashes.
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#define RT_BOOL bool
#else
#define RT_BOOL _Bool
#endif

typedef struct rt_vec3 { double e[3]; } rt_vec3;
typedef rt_vec3 rt_point3;
typedef rt_vec3 rt_color;

typedef struct rt_ray { rt_point3 origin; rt_vec3 dir; } rt_ray;

typedef struct rt_material {
    rt_color diffuseColor;
    rt_color emissionColor;
    double emissionStrength;
    double reflectionStrength;
    double alpha;          /* <1e-4 hole, [1e-4,0.99] translucent, >0.99 opaque */
    double materialIndex;  /* index of refraction used when translucent */
} rt_material;

typedef struct rt_sphere {
    rt_point3 center;
    double radius;
    rt_material mat;
} rt_sphere;

typedef struct rt_uv { double u, v; } rt_uv;

typedef struct rt_triangle {
    rt_point3 A, B, C;
    rt_material mat;       /* unused by the render path: the texel table decides */
    rt_uv uvA, uvB, uvC;
} rt_triangle;

typedef struct rt_camera {
    rt_point3 origin;
    rt_vec3 horizontal;
    rt_vec3 vertical;
    rt_point3 coin_bas_gauche;  /* lower-left corner */
} rt_camera;

/* Layout twin of main.c:22-46 `struct ThreadData`, consumed by rt_fill_canva. */
typedef struct rt_thread_data {
    int start_row, end_row;
    rt_color* canva;
    rt_color* albedo_tab;
    rt_color* normal_tab;
    rt_color* tex_list;
    rt_material* mat_list;
    rt_material* sky_mat_list;
    rt_camera cam;
    int largeur_image, hauteur_image;
    int tex_width, tex_height;
    int sky_width, sky_height;
    int* quelMatPourTri;
    int nbRayonParPixel, nbRebondMax;
    int total_pixels;
    rt_sphere* sphere_list;
    rt_triangle* triangle_list;
    int nbSpheres, nbTriangles;
    int ouverture_x, ouverture_y, focus_distance;
    int AO_intensity;
    RT_BOOL useAO;
} rt_thread_data;

#ifdef __cplusplus
}
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

RT_STATIC_ASSERT(sizeof(rt_vec3) == 24, "vec3 layout");
RT_STATIC_ASSERT(sizeof(rt_ray) == 48, "ray layout");
RT_STATIC_ASSERT(sizeof(rt_material) == 80, "material layout");
RT_STATIC_ASSERT(offsetof(rt_material, emissionStrength) == 48, "material layout");
RT_STATIC_ASSERT(offsetof(rt_material, materialIndex) == 72, "material layout");
RT_STATIC_ASSERT(sizeof(rt_sphere) == 112, "sphere layout");
RT_STATIC_ASSERT(sizeof(rt_triangle) == 200, "triangle layout");
RT_STATIC_ASSERT(offsetof(rt_triangle, uvA) == 152, "triangle layout");
RT_STATIC_ASSERT(sizeof(rt_camera) == 96, "camera layout");
RT_STATIC_ASSERT(offsetof(rt_thread_data, cam) == 56, "ThreadData layout");
RT_STATIC_ASSERT(offsetof(rt_thread_data, quelMatPourTri) == 176, "ThreadData layout");
RT_STATIC_ASSERT(offsetof(rt_thread_data, sphere_list) == 200, "ThreadData layout");
RT_STATIC_ASSERT(offsetof(rt_thread_data, ouverture_x) == 224, "ThreadData layout");
RT_STATIC_ASSERT(offsetof(rt_thread_data, useAO) == 240, "ThreadData layout");
RT_STATIC_ASSERT(sizeof(rt_thread_data) == 248, "ThreadData layout");

#endif /* RT_TYPES_H */
