/*
 * rt/host.h — C host library (librt_host.so): the reference's host-side
 * data model around the render call.
 *
 *   rt_host_init_camera   init_camera            camera.h:21-40
 *   rt_host_load_obj      list_of_mesh           mesh.h:96-218
 *   rt_host_move_mesh     move_mesh              mesh.h:220-234
 *   rt_host_load_textures create_mat_list_mtl    texture.h:175-354
 *                         (+ Kd-only MTL materials, which the reference
 *                          loader cannot read: texture.h:182 strstr(NULL))
 *   rt_host_read_ppm      P3 reader              texture.h:145-173
 *   rt_host_write_ppm     P3 writer              main.c:457-465
 *   rt_host_cuda_materials per-mesh materials of main_cuda.cu's loader
 *                                                triangle.hu:94-105
 *
 * All functions return RT_OK or a negative RT_E* code (rt.h); nothing exits.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include "types.h"

#ifdef __cplusplus
extern "C" {
#endif

rt_camera rt_host_init_camera(rt_point3 origin, rt_point3 target, rt_vec3 up, double vfov, double ratio);

/* Loader options. */
#define RT_OBJ_COMPAT_QUADS 0   /* keep the first 3 vertices of an n-gon (mesh.h:171 sscanf) */
#define RT_OBJ_FAN_QUADS    1   /* fan-triangulate n-gons                                   */

typedef struct rt_mesh {
    rt_triangle* triangles;   int nbTriangles;
    int* quelMatPourTri;      /* per triangle, index into materials (usemtl order)    */
    int nbMaterials;
    char** material_names;    /* usemtl names, nbMaterials entries                      */
    char** texture_paths;     /* map_Kd resolved against the MTL directory, or NULL     */
    rt_vec3* kd;              /* Kd per material (0 if absent)                           */
    double* ns;               /* Ns per material (0 if absent)                           */
} rt_mesh;

int  rt_host_load_obj(const char* obj_path, const char* mtl_path, int ngon_mode, rt_mesh* out);
void rt_host_move_mesh(double x, double y, double z, rt_triangle* tris, int n);
void rt_host_free_mesh(rt_mesh* m);

/* Texel table for a loaded mesh: nbMaterials * th * tw materials, rows
 * bottom-up (texture.h:227-229).  A material with a map_Kd reads
 * <base>.ppm + <base>_alpha.ppm (base = map_Kd minus ".png"); all must share
 * one size.  With kd_fallback != 0, a material without map_Kd becomes a
 * flat texture of its Kd (alpha 1, reflectionStrength Ns/100 as
 * triangle.hu:104-105), sized like the others (1x1 if none has a map). */
int rt_host_load_textures(const rt_mesh* mesh, int kd_fallback, rt_material** mat_list, int* tw, int* th);

/* RT_SEM_CUDA materials (rt.h): each triangle's rt_triangle.mat becomes its
 * material's {Kd, black, 0, Ns/100} as main_cuda.cu's assimp loader builds
 * it per mesh (triangle.hu:94-105: float Kd and shininess, reflection =
 * (double)(shininess/100)), with alpha 1. */
void rt_host_cuda_materials(rt_mesh* mesh);

/* P3 PPM reader: returns w*h*3 values as read (rows as stored, top first). */
int rt_host_read_ppm(const char* path, int* w, int* h, int* maxval, int** values);
/* P3 writer of a canva (rows j = H-1 .. 0, "%d %d %d\n"), main.c:457-465. */
int rt_host_write_ppm(const char* path, const rt_color* canva, int W, int H);

void rt_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
