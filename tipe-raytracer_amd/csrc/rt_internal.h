// rt_internal.h — device-side scene layout and launch descriptors shared by
// the C-ABI (rt_api.cpp) and the kernels (rt_kernels.hip).
//
// HBM layout of one uploaded scene (DESIGN.md "Data layout"):
//   SphCand [ns_pad] 32 B  center, |C|^2 - radius^2 — the candidate pass,
//                          scanned wave-uniformly through the scalar unit,
//                          two records per s_load_dwordx16; padded to an even
//                          count with never-hit records (k = +inf)
//   SphGeo  [ns_pad] 32 B  center, radius^2 — the exact reference test
//                          (winner, fallback scan; r2 = -inf padding)
//   DevMat  [ns]     80 B  sphere material — gathered for the winner only
//   TriGeo  [nt]     96 B  A, B-A, C-A, N  — scanned wave-uniformly
//   TriTex  [nt]    136 B  B, C, uvA/B/C, material, unit normal, area terms — winner only
//   BvhNode4[nodes] 128 B  four child boxes (rt_bvh.h) when nt > 32; the
//   int     [nt]           triangle arrays are then in leaf order and
//                          tri_orig maps back to the caller's order
//   DevMat  [nm*th*tw]     texel table (reference `material` records)
//   DevMat  [nt]           rt_triangle.mat per triangle (RT_SEM_CUDA materials)
//   double  [ns][3]        the colour an emitting sphere shows when seen
//                          directly: hsl_to_rgb(rgb_to_hsl(emission))
// Per launch: a 18-double uniform block (camera, focus, aperture, AO, W-1,
// H-1) read through the scalar unit where used, and, when the samples of a
// pixel are split over P chunks, a [P][pixels][9] partial-sum scratch.
#pragma once
#include <cstdint>

namespace rt {

struct BvhNode4;                                      // rt_bvh.h
struct BvhNodeH;                                      // rt_bvh.h (64-byte form)

struct SphGeo { double cx, cy, cz, r2; };            // r2 = radius*radius (sphere.h:22)
// Candidate-pass record (rt_kernels.hip spheres_closest): center and
// k = |C|^2 - r2 (host, long double), so c*a = a*|o|^2 - 2a*o.C + a*k is an
// FMA chain; padding records have k = +inf (never hit).
struct SphCand { double cx, cy, cz, k; };
struct DevMat {                                       // == material, hitinfo.h:6-13
    double dr, dg, db;       // diffuseColor
    double er, eg, eb;       // emissionColor
    double es, rs, alpha, ior;
};
struct TriGeo {                                       // mesh.h:72-74 precomputed
    double ax, ay, az;
    double abx, aby, abz;
    double acx, acy, acz;
    double nx, ny, nz;       // cross(B-A, C-A), unnormalised
};
struct TriTex {                                       // what tri_uvmapping reads
    double bx, by, bz, cx, cy, cz;
    double uau, uav, ubu, ubv, ucu, ucv;
    int mat;                 // quelMatPourTri[i]
    int tex0;                // the texel index when every uv is 0 (it is then (0, 0) of
                             // material mat for any finite hit), else -1
    double unx, uny, unz;    // vec3_normalize(N) (mesh.h:91), host-computed: the hit normal
    double area;             // get_barycentric_coord's areaABC = dot(un, N) (texture.h:18)
};
static_assert(sizeof(SphGeo) == 32, "SphGeo");
static_assert(sizeof(SphCand) == 32, "SphCand");
static_assert(sizeof(DevMat) == 80, "DevMat");
static_assert(sizeof(TriGeo) == 96, "TriGeo");
static_assert(sizeof(TriTex) == 136, "TriTex");
// tri_uvmapping's u, v as affine functions of the hit point (rt_api.cpp
// tri_uv_affine): u(P) = u0 + gu.(P - A), v(P) = v0 + gv.(P - A), with
// tw*|u_ref - u| <= eu (th*|v_ref - v| <= ev) for every P within diam
// (max-norm) of A, u_ref being the reference's rounded u; diam < 0: no fast
// path for this triangle
struct TriUV {
    double gux, guy, guz, u0;
    double gvx, gvy, gvz, v0;
    double eu, ev, diam;
};
static_assert(sizeof(TriUV) == 88, "TriUV");

// uniform block (doubles)
enum : int {
    U_CAM_O = 0, U_CAM_H = 3, U_CAM_V = 6, U_CAM_C = 9,
    U_FOCUS = 12, U_OX, U_OY, U_AO, U_WM1, U_HM1,
    U_RC_WM1, U_RC_HM1,      // rcp_refined(W-1), rcp_refined(H-1) (device-computed), or 0: plain division
    U_COUNT
};

// Everything one render launch needs, passed by value as the kernel argument.
struct KParams {
    // scene
    const SphGeo* sph;
    const SphCand* sph_cand; // candidate-pass records [ns_pad]
    double cand_lmax;        // >= max_k |C_k| + R_k (+inf: candidate pass off, exact scans)
    const DevMat* sph_mat;
    const TriGeo* tri;
    const TriTex* tri_tex;
    const TriUV* tri_uv;     // (textured scenes) the affine texel map, null: every hit takes the exact path
    const DevMat* texels;
    const double* uni;       // U_COUNT doubles
    const BvhNode4* bvh;     // 4-wide triangle BVH (rt_bvh.h), or null: brute-force scan
    const BvhNodeH* bvhh;    // the same tree in 64-byte nodes (the queue kernel's), or null
    const int* tri_orig;     // triangle k's index in the caller's list (null: k)
    const DevMat* sky;       // sky texels when sky mode is on, else null
    const DevMat* tri_mat;   // rt_triangle.mat per triangle (leaf order with a BVH): RT_SEM_CUDA
    int cuda;                // rt.h RT_SEM_CUDA (render_kernel_cuda)
    int f32;                 // always 0: RT_PREC_FP32 was removed in r05 (field kept: kernarg layout)
    double cbb[6];           // RT_SEM_CUDA: the triangles' box (lo xyz, hi xyz), hit_BBox
    const double* sph_rinv;  // 1/radius per sphere (sphere_uvmapping's divide)
    const double* sph_disp;  // per sphere: hsl round trip of its emission (main.c:155-158), 3 doubles
    int sky_w, sky_h;
    double bvh_srel, bvh_sabs;   // distance-cull slack (rt_bvh.cpp)
    float bvh_rbox;              // >= |every bound| of the tree's boxes (single-precision slab margin)
    int bvh_stack;               // traversal stack entries the tree can need (rt_bvh.h BvhBuild::stack4)
    int bvh_steps;               // queue kernel: node visits per lane and round (host: by tree depth)
    int bvh_nodes;               // 4-wide nodes (breadth-first order: the top levels first)
    int ns, ns_pad, nt;
    int tw, th;
    long long n_texels;
    // image / integrator
    int W, H, S, B;
    int useAO;
    int zero_exit;           // paths end once rayColor == 0 (host: only where exact, LanePath::zero_rc)
    int tex_const;           // TriTex::tex0 stands for tri_texel (host: every triangle has one,
                             // and every coordinate and ray origin is within 2^100, so the
                             // barycentrics of a hit are finite)
    int cam_pin;             // aperture 0 and no -0 camera coordinate: co + (jx*0, jy*0, 0) == co exactly
    uint32_t key0, key1;
    int chunks;              // samples of a pixel split into this many chunks
    int chunk_taper;         // rt_chunk_bound's taper levels L (0: equal slices)
    unsigned chunk_den;      // rt_chunk_bound's divisor: chunks, or (chunks - L) 2^L + 2^L - 1 tapered
    // tiling
    int row_base, tile_rows, tile_first, tile_step, n_tiles, row_end;
    int local_rows;          // n_tiles * tile_rows
    int band_y0, band_rows;  // local rows [band_y0, band_y0 + band_rows) of this launch (partials are per band)
    // outputs (device, local frame of local_rows x W colors)
    double* canva;
    double* albedo;
    double* normal;
    double* radiance;
    double* partial;         // chunks > 1: [chunks][band_rows*W][9]
    double* sums;            // accumulate mode (rt_accumulate_async): [local_rows*W][9] running sums, or null
    long long s_base;        // global index of this launch's first sample (Philox counter word 3)
    unsigned* task_ctr;      // render_kernel_q's task counter (zeroed per band launch), or null
    unsigned npx_here;       // render_kernel_q: pixels of this band that exist (tasks = npx_here * chunks)
    unsigned qm_npx, qm_w, qm_tile, qm_chunks;   // floor((2^32-1)/d) for d = npx_here, W, tile_rows,
                                                 // chunks (udiv_q); qm_chunks 0: 64-bit chunk starts
    unsigned long long* trace;   // render_kernel_q diagnostics (RT_QUEUE_TRACE), normally null
    unsigned long long* counters;
    int opaque;              // every sphere material opaque: !(alpha < 0.0001) && !(alpha <= 0.99) (no hole,
                             // no refraction; the queue kernel's QB = -2 instantiation).  Last, so the
                             // other fields keep their kernarg offsets (and the kernels their SMEM loads)
    int opaque_all;          // ... and so is every triangle material: every texel, no material index 3 or 4
                             // (tri_material's alpha overrides); the deep-tree OPQ instantiation
    int ns_cand;             // spheres the candidate pass scans: ns_pad, or 0 when cand_lmax is +inf (every
                             // ray then takes the exact scan: non-finite spheres, or more than 65534
                             // spheres, whose slots do not fit RT_CAND_TAG's 16 bits)
    int stack_cap;           // BVH stack entries of the kernel launch_render picks for this launch
                             // (choose_render; host-set): what COUNT runs check pushes against
    double bvh_rb;           // the origin bound R_b the tree's padding assumed (rt_bvh.h r_scene)
    double bvh_kdelta;       // padding growth per unit of origin beyond it (rt_bvh.h k_delta)
    float bvh_rb_f;          // a float with rb_f (1 + 2^-23) <= R_b (the walk's cheap "inside" test)
    int bvh_far;             // some ray origin may lie beyond R_b: a sphere or the camera does
};

// The render kernel launch_render takes and its BVH walk's LDS stack entries
// (rt_kernels.hip choose_render).
struct RenderChoice {
    bool queue;              // render_kernel_q (else the fixed-grid render_kernel / render_kernel_cuda)
    int qb;                  // render_kernel_q's QB
    bool opq;                // ... its OPQ instantiation
    int stack_cap;           // stack entries of the chosen kernel's BVH walk (0 without a BVH)
};
RenderChoice choose_render(const KParams& kp, bool task_ok);

struct UniBlock { double v[U_COUNT]; };

// launchers (rt_kernels.hip)
int launch_set_uniforms(const UniBlock& u, double* d_uni, void* stream);
int launch_render(const KParams& kp, void* stream);
// Name of the render kernel the calling thread's last launch_render chose.
const char* last_render_kernel();
int launch_count(const KParams& kp, void* stream);
int launch_assemble(const double* gathered, long long rank_stride, int world, int tile_rows,
                    int rows_per_rank, int W, int H, double* out, void* stream);
int launch_selftest(int op, const double* d_in, double* d_out, int n, void* stream);
int launch_verify_phi(unsigned long long r0, unsigned long long n, unsigned long long* d_counts);
int launch_verify_normalize(unsigned long long seed, unsigned long long n, unsigned long long* d_counts);
int launch_verify_spheres(const KParams& kp, const double* d_rays, long long n, unsigned long long* d_counts);
int launch_verify_texel(const KParams& kp, const double* d_pts, const int* d_tri, long long n,
                        unsigned long long* d_counts);
int launch_resolve(const KParams& kp, void* stream);
int launch_denoise_pack(long long npx, const double* canva, const double* albedo, const double* normal,
                        float* color3, float* albedo3, float* normal3, void* stream);

}  // namespace rt
