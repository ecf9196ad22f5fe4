/*
 * rt/rt.h — C-ABI of the MI355X path-tracing render path (librt_hip.so).
 *
 * This is the drop-in boundary for the reference's per-pixel render loop:
 *
 *   rt_fill_canva   replaces fill_canva(void*)            main.c:245-284
 *                   (same pthread start-routine signature, same ThreadData
 *                    layout; main.c:446 only swaps the function name)
 *   rt_render_rows  replaces the thread-spawn loop        main.c:402-453
 *                   and the CUDA staging + launch         main_cuda.cu:280-339
 *                   (state init :326, render_canva<<<>>> :329, D2H :332-339)
 *   rt_render_async device-resident twin of render_canva  main_cuda.cu:143-171
 *                   (caller-owned device frame, caller's HIP stream)
 *
 * Plain C types only: pointers, sizes and the reference-shaped structs of
 * rt/types.h.  All entry points return RT_OK (0) or a negative RT_E* code and
 * never exit(); the message of the last failure on the calling thread is
 * rt_last_error().
 */
#ifndef RT_RT_H
#define RT_RT_H

#include "types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rt_params gained `precision` (RT_PREC_*) and rt_params_init defaults
 *    spp_chunks to RT_SPP_CHUNKS_AUTO (a different summation grouping than
 *    the strict fill_canva order of spp_chunks = 1); build rt_params with
 *    rt_params_init so new fields read their defaults.  rt_gather_async.
 * 3: RT_CNT_BVH_STACK_OVER appended (RT_NCOUNTERS 17 -> 18): d_counters
 *    arrays of rt_count_async hold RT_NCOUNTERS entries; scenes above 65534
 *    spheres upload (exact sphere scans) instead of RT_EUNSUPPORTED.
 * 4: rt_params gained `gather` (RT_GATHER_*: rt_render_gather_async moves
 *    the slots' planes with an RCCL ncclGather by default, peer copies only
 *    on request); rt_abi_version(), rt_last_gather_transport();
 *    rt_set_fill_precision(RT_PREC_FP32) returns RT_EUNSUPPORTED.
 * A caller compares rt_abi_version() with the RT_ABI_VERSION it was built
 * against before passing rt_params or counter arrays.                   */
#define RT_ABI_VERSION 4

/* ---- status codes ------------------------------------------------------- */
#define RT_OK            0
#define RT_EINVAL       -1   /* bad argument (sizes, NULL, out-of-range index) */
#define RT_EDEVICE      -2   /* HIP runtime / device failure                   */
#define RT_ENOMEM       -3   /* host or device allocation failed                */
#define RT_EUNSUPPORTED -4   /* valid request the GPU path does not implement   */

/* ---- random-number streams ---------------------------------------------- */
/* RT_RNG_PHILOX: draw n of sample s at pixel p is word (n & 3) of
 * Philox4x32-10(key = seed, counter = {n >> 2, 0, p, s}) >> 1, i.e. the
 * hiprand/rocrand `rocrand_init(seed, (s << 32) | p, 0)` stream truncated to
 * the 31 bits glibc rand() returns (rtutility.h:229-231 semantics otherwise).
 * RT_RNG_GLIBC: one sequential glibc rand() stream (the reference's own);
 * inherently serial, so only the CPU oracle implements it.                  */
#define RT_RNG_PHILOX 0
#define RT_RNG_GLIBC  1

/* ---- scene: the reference's arrays, unchanged --------------------------- */
typedef struct rt_scene {
    const rt_sphere*   sphere_list;    int nbSpheres;      /* main.c:332-347      */
    const rt_triangle* triangle_list;  int nbTriangles;    /* mesh.h:96-218       */
    const rt_material* mat_list;       /* texel table, nbMaterials*th*tw, texture.h:175 */
    int tex_width, tex_height, nbMaterials;
    const int*         quelMatPourTri; /* per-triangle material, mesh.h:172        */
    /* Equirect sky texels (create_mat_list of the sky PPM, main.c:374), used
     * only with rt_params.sky_mode = RT_SKY_LAST_SPHERE; may be NULL. */
    const rt_material* sky_mat_list;
    int sky_width, sky_height;
} rt_scene;

/* ---- render parameters (main.c:293-347 constants, ThreadData fields) ---- */
typedef struct rt_params {
    int largeur_image, hauteur_image;  /* W, H                                   */
    int nbRayonParPixel;               /* samples per pixel S (>= 1)             */
    int nbRebondMax;                   /* bounce budget B (>= 0)                 */
    rt_camera cam;                     /* from init_camera, camera.h:21-40       */
    double focus_distance;
    double ouverture_x, ouverture_y;   /* aperture (depth of field)              */
    double AO_intensity;
    int useAO;
    int compat_int_truncation;         /* 1: truncate focus/ouverture/AO to int
                                          as ThreadData does (main.c:42-43)      */
    int rng;                           /* RT_RNG_*                               */
    int spp_chunks;                    /* 0/1: each pixel sums its samples in
                                          order s = 0..S-1 (fill_canva's order).
                                          P > 1: samples are summed in P fixed
                                          contiguous slices (rt_chunk_bound),
                                          then slice sums in slice order; a
                                          deterministic grouping (independent of
                                          GPU count) that lets one pixel's
                                          samples run on P wavefronts (the
                                          persistent task-queue kernel).
                                          RT_SPP_CHUNKS_AUTO: P = min(32, S),
                                          see rt_resolve_spp_chunks          */
    unsigned long long seed;           /* Philox key                             */
    int accel;                         /* RT_ACCEL_*: triangle traversal          */
    int sky_mode;                      /* RT_SKY_*                                */
    int semantics;                     /* RT_SEM_*: whose integrator               */
    int precision;                     /* RT_PREC_*: arithmetic of the integrator  */
    int gather;                        /* RT_GATHER_*: multi-device frame transport
                                          (rt_render_gather_async)            */
} rt_params;

/* rt_params.gather: how rt_render_gather_async brings the device slots'
 * planes to the first device.  RCCL (default): one RCCL communicator per
 * device of rt_init's list (ncclCommInitAll, made once per list) and one
 * ncclGather of each slot's planes to rank 0 over xGMI, then the assemble
 * kernel; the devices must be distinct (a list naming a device twice is
 * RT_EUNSUPPORTED -- RCCL has one rank per GPU).  PEER: hipMemcpyPeerAsync
 * per slot (also for a list that repeats a device).  Neither falls back to
 * the other; rt_last_gather_transport() names the one a call used. */
#define RT_GATHER_RCCL 0
#define RT_GATHER_PEER 1

/* rt_params.semantics.  MAIN_C (default) is main.c, the authoritative CPU
 * path.  CUDA is main_cuda.cu's integrator, the reference's
 * GPU path (§8f, an optional fidelity mode):
 *   - tracer main_cuda.cu:86-141: a pre-pass cast returns emitters as
 *     hsl_to_rgb(rgb_to_hsl(emission) with L and S x1.20) and misses as 0; the
 *     bounce loop has no alpha holes, refraction or textures, no x1.3
 *     brightening; albedo/normal are the pre-pass hit's;
 *   - hit_sphere sphere.hu:27-45 accepts t1 >= 0, then t2 >= 0.001;
 *     hit_triangle triangle.hu:247-270 uses 1e-5 for dst/u/v/w;
 *   - closest_hit main_cuda.cu:23-59 skips the triangles when the ray misses
 *     their bounding box (hit_BBox, triangle.hu:42-59; one mesh = all the
 *     triangles) and gives a triangle its own rt_triangle.mat (the CUDA
 *     loader's per-mesh material: Kd, reflection Ns/100, triangle.hu:104-105);
 *   - fill main_cuda.cu:152-156: jitter (i + 0.5 + U(-0.5, 0.5)) / (W - 1);
 *     focus, aperture and AO_intensity are doubles (compat_int_truncation is
 *     ignored), sky_mode must be OFF.
 * The draws come from the same RT_RNG_PHILOX stream and the same portable
 * sinf/cosf/acos (curand XORWOW and the __cosf/__sinf intrinsics of the CUDA
 * build are NVIDIA-specific and not reproduced), so CUDA-mode images match
 * the oracle's restatement of main_cuda.cu bit for bit, not NVIDIA output. */
#define RT_SEM_MAIN_C 0
#define RT_SEM_CUDA   1

/* rt_params.sky_mode.  OFF is main.c as shipped (the sky branch of
 * closest_hit is commented out, main.c:64-71).  LAST_SPHERE enables that
 * branch: when the last sphere is the closest hit, its emissionColor becomes
 * the sky texel sphere_uvmapping (texture.h:92-112) picks and its alpha 1. */
/* rt_params.precision.  FP64 (default and only renderable value) is the
 * reference's arithmetic in its operation order: images equal the reference's
 * own compiled composition bit for bit (tests/test_gpu_reference.py).
 * RT_PREC_FP32 (an experimental binary32 integrator, r02-r04) was removed in
 * r05: its measured 1.1-3.4e-4 per-channel RMSE against the FP64 frames was
 * above north_star's 1e-4.  It is rejected with RT_EUNSUPPORTED; the value
 * stays reserved so the struct keeps its meaning. */
#define RT_PREC_FP64 0
#define RT_PREC_FP32 1

#define RT_SKY_OFF 0
#define RT_SKY_LAST_SPHERE 1

/* rt_params.accel.  AUTO: scenes with more than 32 triangles get a BVH at
 * rt_scene_upload and closest-hit traverses it (the hit chosen is still the
 * reference's: the lexicographic minimum of (dst, triangle index) over the
 * same exact tests, DESIGN.md "BVH"); NONE: test every triangle, as
 * main.c:80-90. */
#define RT_ACCEL_AUTO 0
#define RT_ACCEL_NONE 1

/* rt_params.spp_chunks = RT_SPP_CHUNKS_AUTO selects the grouping the
 * benchmarks use: P = min(RT_SPP_CHUNKS_DEFAULT, S) slices.  It depends only
 * on S, so images are identical for any GPU count, tiling or thread count;
 * the CPU oracle resolves it with the same function.  Against the strict
 * sample order (P = 1) the grouping moves pre-gamma radiance by < 1e-12
 * RMSE (floating-point re-association of the per-pixel sum). */
#define RT_SPP_CHUNKS_AUTO    (-1)
#define RT_SPP_CHUNKS_DEFAULT 32
static inline int rt_resolve_spp_chunks(int spp_chunks, int spp)
{
    int p = spp_chunks == RT_SPP_CHUNKS_AUTO ? RT_SPP_CHUNKS_DEFAULT : spp_chunks;
    if (p <= 1 || spp <= 1) return 1;
    return p < spp ? p : spp;
}

/* Slice c (0 <= c < P) of a pixel's S samples is [rt_chunk_bound(c),
 * rt_chunk_bound(c + 1)).  Equal slices (c*S/P) when P < 5 or S < 8*P;
 * otherwise E = P - L equal slices of weight 2^L followed by L tapered ones
 * of weights 2^(L-1), ..., 2, 1, with L = 5 taper levels when P >= 8 and
 * S >= 32*P, else L = 3 (weights 8, ..., 8, 4, 2, 1).  The task-queue kernel
 * hands out slices in order, so the tasks still running when its queue
 * empties are short (the frame's tail); five levels keep that tail as fine
 * with 12 slices as three levels do with 32, i.e. with 2.7x fewer partial
 * sums per pixel.  A pure function of (c, S, P), shared by the kernels and
 * the oracle, so images stay independent of GPU count and tiling. */
static inline int rt_chunk_taper_levels(long long S, long long P)
{
    if (P >= 8 && S >= 32 * P) return 5;
    if (P >= 5 && S >= 8 * P) return 3;
    return 0;
}
static inline long long rt_chunk_bound(long long c, long long S, long long P)
{
    const int L = rt_chunk_taper_levels(S, P);
    if (!L) return c * S / P;
    const long long one = 1LL << L, E = P - L;
    const long long U = E * one + (one - 1);
    const long long w = c <= E ? one * c : one * E + one - (one >> (c - E));
    return w * S / U;
}

/* Fills defaults: RT_RNG_PHILOX, seed 1010 (main_cuda.cu's curand seed),
 * compat_int_truncation 1, spp_chunks RT_SPP_CHUNKS_AUTO, RT_ACCEL_AUTO,
 * RT_GATHER_RCCL, everything else zero. */
void rt_params_init(rt_params* p);

/* ---- lifecycle ---------------------------------------------------------- */
/* Devices used by rt_render_rows / rt_fill_canva (row tiles are dealt
 * cyclically over them).  ndev <= 0 or devices == NULL selects device 0.
 * Calling any render entry point without rt_init implies rt_init(0, NULL). */
int  rt_init(int ndev, const int* devices);
void rt_shutdown(void);
const char* rt_last_error(void);
/* RT_ABI_VERSION of the loaded library. */
int rt_abi_version(void);
/* Name of the render kernel the calling thread's last render launch used
 * ("render_kernel_q<QB=0|3|4>" = the task-queue kernel without a BVH / with
 * a deep / shallow tree; "render_kernel_q<QB=-1>" / "<QB=-2>" = its
 * sphere-only instantiations (-2: every material opaque); "<QB=3,OP>" = the
 * deep-tree one for scenes whose every material is opaque;
 * "render_kernel<BVH>" / "render_kernel" = the fixed-grid kernels,
 * "render_kernel_cuda"); "none" before the first.
 * The choice never changes a result.  Diagnostics and tests. */
const char* rt_last_render_kernel(void);
const char* rt_version(void);
int  rt_device_count(void);

/* ---- host-buffer drop-in ------------------------------------------------ */
/* Renders rows row_hi down to row_lo (inclusive; row 0 = bottom, pixel
 * index j*W+i as main.c:261) into caller-owned arrays of W*H colors.  canva
 * receives write_color_canva() values (ints 0..255 stored as double,
 * rtutility.h:56-71); albedo/normal receive the per-pixel means
 * (main.c:278-279).  albedo/normal may be NULL.  Only the named rows are
 * written.  Thread-safe for concurrent calls on disjoint rows. */
int rt_render_rows(const rt_scene* scene, const rt_params* params,
                   int row_hi, int row_lo,
                   rt_color* canva, rt_color* albedo, rt_color* normal);

/* pthread start routine with fill_canva's exact contract (main.c:245-284):
 * arg is a struct ThreadData / rt_thread_data.  Renders start_row..end_row
 * on the GPU with the Philox stream (seed 1010) and the spp_chunks grouping
 * set by rt_set_fill_spp_chunks (default RT_SPP_CHUNKS_AUTO).  Returns NULL
 * on success, (void*)1 on failure (see rt_last_error on that thread). */
void* rt_fill_canva(void* thread_data);

/* The spp_chunks rt_fill_canva renders with (ThreadData has no such field):
 * RT_SPP_CHUNKS_AUTO (default, the benchmarked task-queue kernel) or an
 * explicit P (1 = fill_canva's strict running sum, main.c:264-273).
 * Process-wide; returns the previous setting. */
int rt_set_fill_spp_chunks(int spp_chunks);

/* The rt_params.precision rt_fill_canva renders with.  Since r05 always
 * RT_PREC_FP64 (RT_PREC_FP32 was removed, see rt_params.precision):
 * RT_PREC_FP64 returns the previous setting, anything else is refused
 * (RT_PREC_FP32: RT_EUNSUPPORTED, other values: RT_EINVAL) and changes
 * nothing.  Process-wide. */
int rt_set_fill_precision(int precision);

/* rt_render_rows / rt_fill_canva keep the uploaded scene (and its BVH) of
 * the last few distinct scenes per device, keyed by the exact bytes of the
 * caller's arrays, so the NUM_THREADS calls of one frame upload it once.
 * Drops them (rt_shutdown does too); returns how many were cached. */
int rt_scene_cache_clear(void);

/* ---- device-resident interface ------------------------------------------ */
typedef struct rt_device_scene rt_device_scene;   /* opaque */

int  rt_scene_upload(int device, const rt_scene* scene, rt_device_scene** out);
void rt_scene_release(rt_device_scene* scene);

/* Which rows one launch renders.  Local tile lt in [0, n_tiles) is global
 * tile t = tile_first + lt*tile_step, covering global rows
 * row_base + t*tile_rows + y, y in [0, tile_rows); rows >= H are skipped.
 * Output row lt*tile_rows + y of the frame buffers holds that global row.
 * A contiguous band [lo, hi] is {lo, hi-lo+1, 0, 1, 1}; rank r of G with
 * cyclic k-row tiles is {0, k, r, G, ceil(ceil(H/k)/G)}. */
typedef struct rt_tiling {
    int row_base, tile_rows, tile_first, tile_step, n_tiles;
} rt_tiling;

/* Device pointers, each n_tiles*tile_rows*W colors (double3).  canva is
 * required; albedo, normal and radiance (pre-gamma mean, sum/S) optional. */
typedef struct rt_frame {
    rt_color* canva;
    rt_color* albedo;
    rt_color* normal;
    rt_color* radiance;
} rt_frame;

/* Enqueue the render on `hip_stream` (hipStream_t, NULL = null stream).
 * Asynchronous: returns after the launch. */
int rt_render_async(const rt_device_scene* scene, const rt_params* params,
                    const rt_tiling* tiling, const rt_frame* frame,
                    void* hip_stream);

/* Un-permute a rank-major gather of per-rank frames into a full W*H plane.
 * Rank r's block starts at gathered + r*rank_stride colors (rank_stride 0:
 * rows_per_rank*W, i.e. packed) and was rendered with tiling
 * {0, tile_rows, r, world, rows_per_rank/tile_rows}.  out: W*H colors. */
int rt_assemble_async(const rt_color* gathered, long long rank_stride, int world,
                      int tile_rows, int rows_per_rank, int W, int H,
                      rt_color* out, void* hip_stream);

/* ---- device-resident multi-device frame ---------------- */
/* Replaces main_cuda.cu:280-339 (one device, three D2H copies) for a device
 * destination on several devices of one node.  rt_gather_async copies slot
 * r's local plane (rows_per_rank*W colours on device src_devices[r], rendered
 * with tiling {0, tile_rows, r, world, rows_per_rank/tile_rows}) into a
 * rank-major staging block on dst_device with peer copies (xGMI), then
 * un-permutes the staging into out (W*H colours on dst_device), all on
 * hip_stream (a stream of dst_device; the caller orders the slots' renders
 * before it, e.g. with events).
 * rt_render_gather_async does the whole frame: every device of rt_init's list
 * (default: device 0) renders its cyclic tile_rows-row tiles on a pooled
 * stream of its own (after the work already enqueued on hip_stream), and the
 * requested planes of `frame` (device pointers on the list's FIRST device,
 * W*H colours each) are gathered and assembled on hip_stream.  Asynchronous;
 * images are bit-identical to one device's rt_render_async (the stream is
 * keyed by the global pixel). */
int rt_gather_async(int world, const int* src_devices, const rt_color* const* locals, int tile_rows,
                    int rows_per_rank, int W, int H, int dst_device, rt_color* out, void* hip_stream);
int rt_render_gather_async(const rt_scene* scene, const rt_params* params, int tile_rows, const rt_frame* frame,
                           void* hip_stream);
/* The transport the calling thread's last rt_render_gather_async used:
 * "rccl: ncclGather, RCCL x.y.z (library path), N ranks" or "peer:
 * hipMemcpyPeerAsync, N slots"; "none" before the first. */
const char* rt_last_gather_transport(void);
/* Peer access the gathers use from dst_device to src_device, enabled on
 * first use per pair: 1 = enabled (copy engines read over xGMI; also the
 * answer for dst == src), 0 = unavailable or refused by the runtime (e.g.
 * hipErrorPeerAccessUnsupported) or disabled with the environment variable
 * RT_PEER_ACCESS=0 -- the gathers then still work, hipMemcpyPeerAsync staging
 * each copy itself; RT_EINVAL for a device that is not visible.
 * NOTE: the distinct-device branches (peer enable, cross-device event waits,
 * xGMI copies) have only run in tests on machines with >= 2 GPUs; the
 * builder's own GPU box has one, where every slot is device 0. */
int rt_peer_access(int dst_device, int src_device);

/* ---- instrumentation (roofline accounting, tests) ----------------------- */
enum {
    RT_CNT_SAMPLES = 0,   /* camera samples traced                         */
    RT_CNT_CASTS,         /* closest-hit casts (bounce + AO)               */
    RT_CNT_SPHERE_TESTS,  /* ray-sphere tests                              */
    RT_CNT_SPHERE_DISC,   /* ... with discriminant > 0                     */
    RT_CNT_TRI_TESTS,     /* ray-triangle tests                            */
    RT_CNT_SHADE,         /* direction samples (random_dir_no_norm calls)  */
    RT_CNT_TEX_HITS,      /* closest hits on a triangle (texel fetch)      */
    RT_CNT_REFRACT,       /* refraction-branch events                      */
    RT_CNT_RNG_DRAWS,     /* 31-bit draws consumed                         */
    RT_CNT_EXACT_RESCANS, /* sphere scans redone exactly (candidate pass
                             ambiguous; GPU diagnostic, the oracle reports 0) */
    RT_CNT_BVH_NODES,     /* BVH nodes visited (GPU diagnostic)            */
    RT_CNT_BVH_TRI_TESTS, /* triangles actually tested through the BVH
                             (GPU diagnostic; RT_CNT_TRI_TESTS keeps the
                             reference's brute-force count)              */
    RT_CNT_BVH_LANE_SLOTS, /* 64 x wave-level BVH traversal steps (GPU
                             diagnostic; bvh_nodes / this = SIMD efficiency) */
    RT_CNT_LEAF_LANE_SLOTS, /* 64 x wave-level iterations of the BVH leaf
                             loop (GPU diagnostic; vs bvh_tri_tests)     */
    RT_CNT_CAST_LANE_SLOTS, /* 64 x wave-level sphere passes (GPU
                             diagnostic; vs casts)                       */
    RT_CNT_SHADE_LANE_SLOTS, /* 64 x wave-level hit resolutions (bounce
                             shading or AO tail; GPU diagnostic)         */
    RT_CNT_BVH_STACK_OVER, /* BVH stack pushes made at a depth >= the LDS
                             stack of the kernel a render of the same params
                             takes (the queue kernel's 24 / 32 / 14 entries,
                             else the fixed grid's 48; rt_kernels.hip
                             choose_render).  Must be 0: the host admits a
                             tree by its exact stack bound (rt_bvh.cpp); a
                             nonzero count means that bound is wrong (GPU
                             diagnostic, rt_count_async only).  The
                             counting walk drops pushes beyond 48 entries,
                             so when this is nonzero the BVH node and
                             triangle counts may be too low            */
    RT_NCOUNTERS
};
/* Same traversal as rt_render_async, no frame; adds event counts into the
 * device array d_counters[RT_NCOUNTERS] (unsigned long long). */
int rt_count_async(const rt_device_scene* scene, const rt_params* params,
                   const rt_tiling* tiling, unsigned long long* d_counters,
                   void* hip_stream);

/* ---- progressive rendering / checkpoint-resume ----------- */
/* Adds samples [sample_offset, sample_offset + nbRayonParPixel) of every
 * pixel of the tiling's local frame to the device accumulator d_sums (9
 * doubles per local pixel: radiance, albedo, normal sums; local_rows*W
 * entries, zero-filled by the caller before the first batch).  The stream is
 * keyed by the global sample index, so with spp_chunks = 1 the sums after any
 * sequence of batches covering samples 0..S-1 in order are bit-identical to
 * one launch of S samples (fill_canva's fold continues across batches).  With
 * spp_chunks = P > 1 a batch adds its P slice sums in slice order.  The sums
 * are plain memory: copy them out to checkpoint, back in to resume.
 * sample_offset + nbRayonParPixel must not exceed 2^32. */
int rt_accumulate_async(const rt_device_scene* scene, const rt_params* params, long long sample_offset,
                        const rt_tiling* tiling, double* d_sums, void* hip_stream);
/* Writes the frame planes of d_sums for total_spp samples per pixel
 * (write_color_canva with rapport = 1.0/total_spp, albedo/normal = sum /
 * total_spp), main.c:275-279.  params supplies W and H. */
int rt_resolve_async(const double* d_sums, const rt_params* params, int total_spp, const rt_tiling* tiling,
                     const rt_frame* frame, void* hip_stream);

/* ---- zero-throughput exit ------------------------------------------------ */
/* tracer (main.c:118-242) keeps bouncing after rayColor has become (0, 0, 0)
 * (a black-diffuse light, a green wall then a red one, an AO miss); those
 * bounces add exactly 0.  Render launches end such paths early when that is
 * provably exact for the scene and parameters (bounded materials, and with
 * AO 0 < AO_intensity <= 1000 and coordinates within 2^20), so frames are
 * bit-identical either way; only the work done, and so rt_count_async's
 * cast/shade/draw counts, differ.  Process-wide, default on; 0 reproduces
 * the reference's counts (tests).  Returns the previous setting. */
int rt_set_zero_throughput_exit(int enable);

/* ---- denoiser hook (denoiser.h:31-91, called at main.c:455) -------------- */
/* denoiser()'s signature.  main.c runs it once on the finished frame when
 * useDenoiser is set; the OIDN library itself is not part of this one. */
typedef void (*rt_denoise_fn)(int largeur_image, int hauteur_image, rt_color* canva, rt_camera cam,
                              rt_color* albedo, rt_color* normal);
/* Installs (NULL clears; default NULL) the hook rt_render_rows calls after it
 * has written a whole frame (row_hi = H-1, row_lo = 0) including the albedo
 * and normal planes, on the calling thread, with params->cam. */
void rt_set_denoise_hook(rt_denoise_fn fn);
rt_denoise_fn rt_get_denoise_hook(void);

/* The OIDN "RT" filter's buffer formats (denoiser.h:44-60, 80-84): float3
 * planes color = (float)canva / 255.0f, albedo/normal = (float)value, and
 * back canva = (int)(color * 255.0f).  Host versions, and a device pack of a
 * device frame for a GPU denoiser (caller's stream; albedo/normal planes are
 * skipped when their pointers are NULL). */
int rt_denoise_pack(int W, int H, const rt_color* canva, const rt_color* albedo, const rt_color* normal,
                    float* color3, float* albedo3, float* normal3);
int rt_denoise_unpack(int W, int H, const float* color3, rt_color* canva);
int rt_denoise_pack_async(int W, int H, const rt_frame* frame, float* color3, float* albedo3, float* normal3,
                          void* hip_stream);

/* Device-math self test: evaluates one device primitive on n host inputs
 * (synchronous, device 0).  op: 0 acos, 1 sinf, 2 cosf, 3 pow(x, y),
 * 4 sqrt, 5 x/y, 6 sqrtf, 7 philox word (in[0..3] = ctr, in[4..5] = key as
 * integers in doubles; returns 4 words per input), 8 normalize (3 doubles in,
 * 3 out, vec3.h:137-139), 9 atan2(y, x).  Inputs are read as pairs (x, y)
 * for binary ops. */
int rt_selftest_math(int op, const double* in, double* out, int n);

/* Exhaustive check of the sampler's fast phi path (random_dir_no_norm,
 * rtutility.h:196-200): for every rand() value r in [r0, r0 + n) (r < 2^31),
 * sinf/cosf of (float)acos(2 r/2^31 - 1) from the fast path against the full
 * portable path.  counts[0] = inputs that take the fallback, counts[1] =
 * inputs whose fast result differs (0 is the correctness bar).  Synchronous,
 * device 0. */
int rt_verify_sampler_phi(unsigned long long r0, unsigned long long n, unsigned long long counts[2]);

/* Stress check of the sphere candidate pass (closest_hit's sphere half,
 * main.c:59-78): for n rays (origin xyz, direction xyz: 6 doubles each) the
 * candidate pass with its exact fallback against the plain exact scan of
 * hit_sphere.  counts[0] = rays sent to the exact fallback, counts[1] = rays
 * whose winner or distance differs (0 is the correctness bar).  Synchronous,
 * device 0. */
int rt_verify_sphere_pass(const rt_scene* scene, const double* rays, long long n, unsigned long long counts[2]);

/* Stress check of the kernel's normalize (vec3.h:137-139, a / sqrt(a.a)):
 * n pseudo-random vectors (Philox keyed by seed; unit-scale, n + dir sums,
 * common and per-component binary scales 2^-450..2^450) through the fast
 * exact path against the IEEE sqrt and divisions.  counts[0] = vectors on the
 * fast path, counts[1] = results that differ in any bit (0 is the
 * correctness bar).  Synchronous, device 0. */
int rt_verify_normalize(unsigned long long seed, unsigned long long n, unsigned long long counts[2]);

/* Stress check of the texel lookup's affine fast path (tri_uvmapping +
 * get_barycentric_coord, texture.h:16-27,44-90): point i (3 doubles in pts)
 * taken as a hit on triangle tri[i] of the scene (at most 32 triangles, so in
 * the caller's order; the hit normal is the triangle's unit normal) through the
 * affine uv map when its rounding bound makes the texel certain, against the
 * reference's barycentric operations.  counts[0] = points the fast path
 * decides, counts[1] = points where it picks another texel (0 is the
 * correctness bar).  A scene whose triangles all have uv 0 has no map
 * (RT_EUNSUPPORTED).  Synchronous, device 0. */
int rt_verify_texel_map(const rt_scene* scene, const double* pts, const int* tri, long long n,
                        unsigned long long counts[2]);

#ifdef __cplusplus
}
#endif
#endif /* RT_RT_H */
