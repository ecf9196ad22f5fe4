/*
 * oracle/ref_tracer_harness.c — TEST INFRASTRUCTURE (container only).
 *
 * Drivers for the reference's own render composition, compiled here by
 * oracle/build_ref_tracer.sh.  That script feeds gcc ONE translation unit on
 * stdin, made of:
 *
 *   1. the system headers and leaf headers main.c:1-20 includes, in main.c's
 *      order, except main.c:9 (<OpenImageDenoise/oidn.h>) and main.c:17
 *      (denoiser.h, whose denoiser() at denoiser.h:31-91 is the only OIDN
 *      user);
 *   2. denoiser.h:11-29 verbatim (col_alb_norm, can_create,
 *      add_col_alb_norm) at denoiser.h's place in main.c's include order;
 *   3. mesh.h, texture.h, pile.h (main.c:18-20);
 *   4. main.c:22-284 verbatim (ThreadData, rendered_pixels, closest_hit,
 *      ambient_occlusion, tracer, fill_canva);
 *   5. this file.
 *
 * Each verbatim range is sha256-checked against oracle/ref_tracer.sha256
 * before it is compiled, and is read from /root/reference at build time —
 * nothing from the reference is copied into this repository, no header is
 * stubbed, and main() (main.c:286-498) / denoiser() are simply absent: the
 * render path calls neither.  Output: oracle/_ref/libref_tracer.so
 * (git-ignored, never shipped to the GPU box).
 *
 * Flags: the reference Makefile's own (gcc -O3), plus -fPIC -shared.
 *
 * This file only declares drivers; it never restates reference semantics:
 *   ref_fill_canva  — builds a struct ThreadData (main.c:22-46) and runs the
 *                     reference's fill_canva (main.c:245-284) in one pthread,
 *                     exactly as main.c:446 does for a one-thread band.
 *   ref_trace_rows  — the same loop nest (main.c:248-280, descending rows,
 *                     4 jitter draws per sample) around the reference's own
 *                     get_ray / tracer / add_col_alb_norm / write_color_canva,
 *                     but with a double AO intensity (tracer's parameter type,
 *                     main.c:118; ThreadData's int field truncates it,
 *                     main.c:43) and the pre-quantisation mean radiance
 *                     (sum/S) as a fourth plane.  Its equality with
 *                     ref_fill_canva at integer AO is itself a test.
 *
 * With -DREF_STREAM_PHILOX (oracle/_ref/libref_tracer_philox.so) the same
 * verbatim ranges are compiled with the GPU's stream spec substituted for
 * the reference's two third-party dependencies, by object-like macros
 * defined before the reference headers (build_ref_tracer.sh): glibc rand()
 * becomes draw n of sample s at pixel p of rt.h's RT_RNG_PHILOX stream, and
 * libm's acos / sinf / cosf / pow become the portable oracle/pm_math.h
 * functions the kernel implements (sqrt, sqrtf, fmod are correctly rounded
 * either way).  The reference's own tracer / closest_hit /
 * ambient_occlusion / hit tests / shading then run the kernel's exact draw
 * sequence, so the GPU's frames can be compared with the reference's code
 * directly (ref_trace_rows_philox, tests/golden/gpu_reference.json).
 */
#include <pthread.h>

#define EXPORT __attribute__((visibility("default")))

EXPORT int ref_fill_canva(const sphere* sph, int ns, const triangle* tris, int nt, const material* mats, int tw,
                          int th, const int* qm, const camera* cam, int W, int H, int spp, int bounces, int focus,
                          int ox, int oy, int useAO, int AO, int row_hi, int row_lo, color* canva, color* albedo,
                          color* normal)
{
    if (W * H < 40) return -1;   /* main.c:253 divides by total_pixels / 40 */
    struct ThreadData d;
    memset(&d, 0, sizeof d);
    d.start_row = row_hi;
    d.end_row = row_lo;
    d.canva = canva;
    d.albedo_tab = albedo;
    d.normal_tab = normal;
    d.tex_list = NULL;
    d.mat_list = (material*)mats;
    d.sky_mat_list = NULL;
    d.cam = *cam;
    d.largeur_image = W;
    d.hauteur_image = H;
    d.tex_width = tw;
    d.tex_height = th;
    d.sky_width = 0;
    d.sky_height = 0;
    d.quelMatPourTri = (int*)qm;
    d.nbRayonParPixel = spp;
    d.nbRebondMax = bounces;
    d.total_pixels = W * H;
    d.sphere_list = (sphere*)sph;
    d.triangle_list = (triangle*)tris;
    d.nbSpheres = ns;
    d.nbTriangles = nt;
    d.ouverture_x = ox;
    d.ouverture_y = oy;
    d.focus_distance = focus;
    d.AO_intensity = AO;
    d.useAO = useAO != 0;
    rendered_pixels = 0;
    pthread_t t;
    if (pthread_create(&t, NULL, fill_canva, &d) != 0) return -2;
    pthread_join(t, NULL);
    return 0;
}

EXPORT int ref_trace_rows(const sphere* sph, int ns, const triangle* tris, int nt, const material* mats, int tw,
                          int th, const int* qm, const camera* cam, int W, int H, int spp, int bounces,
                          double focus, double ox, double oy, int useAO, double AO, int row_hi, int row_lo,
                          color* canva, color* albedo, color* normal, color* radiance)
{
    if (W < 2 || H < 2 || spp < 1) return -1;
    for (int j = row_hi; j >= row_lo; --j) {
        for (int i = 0; i < W; i++) {
            const int pixel_index = j * W + i;
            col_alb_norm total = {{BLACK, BLACK, BLACK}};
            for (int x = 0; x < spp; ++x) {
                double u = ((double)i + randomDouble(-0.5, 0.5)) / (W - 1);
                double v = ((double)j + randomDouble(-0.5, 0.5)) / (H - 1);
                double dx = randomDouble(-0.5, 0.5) * ox;
                double dy = randomDouble(-0.5, 0.5) * oy;
                ray r = get_ray(u, v, *cam, focus, dx, dy);
                total = add_col_alb_norm(total, tracer(r, bounces, (sphere*)sph, ns, (triangle*)tris, nt, AO,
                                                       useAO != 0, (material*)mats, tw, th, (int*)qm, NULL, 0, 0));
            }
            canva[pixel_index] = write_color_canva(total.e[0], spp);
            if (albedo) albedo[pixel_index] = divide_scalar(total.e[1], spp);
            if (normal) normal[pixel_index] = divide_scalar(total.e[2], spp);
            if (radiance) radiance[pixel_index] = divide_scalar(total.e[0], spp);
        }
    }
    return 0;
}

EXPORT void ref_tracer_srand(unsigned s) { srand(s); }

#ifdef REF_STREAM_PHILOX
/* ref_trace_rows with the RT_RNG_PHILOX stream keyed by (seed, global pixel
 * j*W+i, sample x), summing each pixel's samples in rt.h's spp_chunks slices
 * (rt_chunk_bound: per-slice running sums, then the slice sums in slice
 * order; P = 1 is fill_canva's running sum). */
EXPORT int ref_trace_rows_philox(const sphere* sph, int ns, const triangle* tris, int nt, const material* mats,
                                 int tw, int th, const int* qm, const camera* cam, int W, int H, int spp,
                                 int bounces, double focus, double ox, double oy, int useAO, double AO,
                                 unsigned long long seed, int chunks, int row_hi, int row_lo, color* canva,
                                 color* albedo, color* normal, color* radiance)
{
    if (W < 2 || H < 2 || spp < 1) return -1;
    const int P = rt_resolve_spp_chunks(chunks, spp);
    ref_ps.seed = seed;
    for (int j = row_hi; j >= row_lo; --j) {
        for (int i = 0; i < W; i++) {
            const int pixel_index = j * W + i;
            col_alb_norm total = {{BLACK, BLACK, BLACK}};
            for (int c = 0; c < P; ++c) {
                col_alb_norm part = {{BLACK, BLACK, BLACK}};
                const int s0 = (int)rt_chunk_bound(c, spp, P), s1 = (int)rt_chunk_bound(c + 1, spp, P);
                for (int x = s0; x < s1; ++x) {
                    ref_ps.pixel = (uint32_t)pixel_index;
                    ref_ps.sample = (uint32_t)x;
                    ref_ps.n = 0;
                    double u = ((double)i + randomDouble(-0.5, 0.5)) / (W - 1);
                    double v = ((double)j + randomDouble(-0.5, 0.5)) / (H - 1);
                    double dx = randomDouble(-0.5, 0.5) * ox;
                    double dy = randomDouble(-0.5, 0.5) * oy;
                    ray r = get_ray(u, v, *cam, focus, dx, dy);
                    part = add_col_alb_norm(part, tracer(r, bounces, (sphere*)sph, ns, (triangle*)tris, nt, AO,
                                                         useAO != 0, (material*)mats, tw, th, (int*)qm, NULL, 0, 0));
                }
                total = c == 0 ? part : add_col_alb_norm(total, part);
            }
            canva[pixel_index] = write_color_canva(total.e[0], spp);
            if (albedo) albedo[pixel_index] = divide_scalar(total.e[1], spp);
            if (normal) normal[pixel_index] = divide_scalar(total.e[2], spp);
            if (radiance) radiance[pixel_index] = divide_scalar(total.e[0], spp);
        }
    }
    return 0;
}
#endif
