/*
 * rt_demo.c — main.c's flow (main.c:286-498) on the MI355X render path:
 * scene constants -> optional OBJ/MTL mesh + texel table -> init_camera ->
 * ONE rt_render_rows call (instead of the pthread band loop main.c:402-453)
 * -> optional denoiser hook -> P3 PPM (main.c:457-465).
 *
 *   rt_demo [-w W] [-s spp] [-b nbRebondMax] [-ao AO_intensity] [-o out.ppm]
 *           [-obj file.obj -mtl file.mtl [-move x y z]] [-devices N]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "rt/host.h"
#include "rt/rt.h"

#define C3(a, b, c) {{a, b, c}}
#define MAT(d, e, es, rs) {d, e, es, rs, 1.0, 1.0}

int main(int argc, char** argv)
{
    int W = 400, spp = 100, bounces = 5, ndev = 1, useAO = 0;
    double AO = 2.5, mx = 0, my = 0, mz = 0;
    const char *out = "render.ppm", *obj = NULL, *mtl = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-w") && i + 1 < argc) W = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s") && i + 1 < argc) spp = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-b") && i + 1 < argc) bounces = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-ao") && i + 1 < argc) { useAO = 1; AO = atof(argv[++i]); }
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!strcmp(argv[i], "-obj") && i + 1 < argc) obj = argv[++i];
        else if (!strcmp(argv[i], "-mtl") && i + 1 < argc) mtl = argv[++i];
        else if (!strcmp(argv[i], "-devices") && i + 1 < argc) ndev = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-move") && i + 3 < argc) {
            mx = atof(argv[++i]);
            my = atof(argv[++i]);
            mz = atof(argv[++i]);
        } else {
            fprintf(stderr, "usage: %s [-w W] [-s spp] [-b bounces] [-ao I] [-o out.ppm] "
                            "[-obj f.obj -mtl f.mtl [-move x y z]] [-devices N]\n", argv[0]);
            return 2;
        }
    }
    double ratio = 4.0 / 3.0;
    int H = (int)(W / ratio);
    /* README.md:46-59 sphere list, alpha = 1, materialIndex = 1 */
    rt_sphere spheres[] = {
        {C3(-501, 0, 0), 500, MAT(C3(0, 1, 0), C3(0, 0, 0), 0.0, 0.96)},
        {C3(0, -501, 0), 500, MAT(C3(1, 1, 1), C3(0, 0, 0), 0.0, 0.0)},
        {C3(501, 0, 0), 500, MAT(C3(1, 0, 0), C3(0, 0, 0), 0.0, 0.96)},
        {C3(-0.5, 1.4, -1.2), 0.5, MAT(C3(0, 0, 0), C3(1.0, 0.6, 0.2), 4.0, 0.0)},
        {C3(0.5, 1.4, -2.2), 0.5, MAT(C3(0, 0, 0), C3(0.7, 0.2, 1.0), 4.0, 0.0)},
        {C3(0.6, -1.4, -1.0), 0.5, MAT(C3(0, 0, 0), C3(0.55, 0.863, 1.0), 2.5, 0.0)},
        {C3(-0.5, -1.4, -3.1), 0.5, MAT(C3(0, 0, 0), C3(0.431, 1.0, 0.596), 2.5, 0.0)},
        {C3(0, 0, -504), 500, MAT(C3(1, 1, 1), C3(0, 0, 0), 0.0, 0.0)},
        {C3(0, 501, 0), 500, MAT(C3(1, 1, 1), C3(0, 0, 0), 0.0, 0.0)},
        {C3(0.4, -0.5, -3.3), 0.5, MAT(C3(0.784, 0.965, 1), C3(0, 0, 0), 0.0, 0.99)},
    };
    rt_scene scene;
    memset(&scene, 0, sizeof scene);
    scene.sphere_list = spheres;
    scene.nbSpheres = (int)(sizeof spheres / sizeof spheres[0]);
    rt_mesh mesh;
    memset(&mesh, 0, sizeof mesh);
    rt_material* mats = NULL;
    if (obj) {
        int rc = rt_host_load_obj(obj, mtl, RT_OBJ_COMPAT_QUADS, &mesh);
        if (rc) { fprintf(stderr, "cannot load %s (%d)\n", obj, rc); return 1; }
        rt_host_move_mesh(mx, my, mz, mesh.triangles, mesh.nbTriangles);
        int tw, th;
        rc = rt_host_load_textures(&mesh, 1, &mats, &tw, &th);
        if (rc) { fprintf(stderr, "cannot load textures (%d)\n", rc); return 1; }
        scene.triangle_list = mesh.triangles;
        scene.nbTriangles = mesh.nbTriangles;
        scene.quelMatPourTri = mesh.quelMatPourTri;
        scene.nbMaterials = mesh.nbMaterials;
        scene.mat_list = mats;
        scene.tex_width = tw;
        scene.tex_height = th;
        printf("%s : %d triangles, %d materials (%dx%d texels)\n", obj, mesh.nbTriangles, mesh.nbMaterials, tw, th);
    }
    rt_point3 origin = C3(0.34, 0.3, 0.5), target = C3(0.0, -0.5, -3);
    rt_vec3 up = C3(0, 1, 0);
    rt_params p;
    rt_params_init(&p);
    p.largeur_image = W;
    p.hauteur_image = H;
    p.nbRayonParPixel = spp;
    p.nbRebondMax = bounces;
    p.cam = rt_host_init_camera(origin, target, up, 70, ratio);
    p.focus_distance = 3;
    p.useAO = useAO;
    p.AO_intensity = AO;

    if (ndev > 1) {
        int devs[64];
        for (int i = 0; i < ndev && i < 64; i++) devs[i] = i;
        if (rt_init(ndev, devs)) { fprintf(stderr, "rt_init: %s\n", rt_last_error()); return 1; }
    }
    size_t n = (size_t)W * H;
    rt_color* canva = (rt_color*)calloc(n, sizeof(rt_color));
    rt_color* albedo = (rt_color*)calloc(n, sizeof(rt_color));
    rt_color* normal = (rt_color*)calloc(n, sizeof(rt_color));
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    int rc = rt_render_rows(&scene, &p, H - 1, 0, canva, albedo, normal);
    gettimeofday(&t1, NULL);
    if (rc) { fprintf(stderr, "rt_render_rows: %s\n", rt_last_error()); return 1; }
    double dt = (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
    fprintf(stderr, "%dx%d, %d spp, %d bounces: %.3f s, %.1f Msamples/s (end-to-end)\n", W, H, spp, bounces, dt,
            (double)n * spp / dt / 1e6);
    rc = rt_host_write_ppm(out, canva, W, H);
    free(canva);
    free(albedo);
    free(normal);
    free(mats);
    rt_host_free_mesh(&mesh);
    return rc ? 1 : 0;
}
