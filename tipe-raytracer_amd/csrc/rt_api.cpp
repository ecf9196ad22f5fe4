// rt_api.cpp — C-ABI of librt_hip.so (include/rt/rt.h): validation, scene
// upload into the HBM layout of rt_internal.h, launch descriptors, the
// host-buffer drop-ins (rt_render_rows / rt_fill_canva) and diagnostics.
// Every HIP call is checked; failures return RT_E* and set rt_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt/rt.h"
#include "rt_internal.h"
#include "rt_bvh.h"
#include "rt_rccl.h"

using namespace rt;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(RT_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                                \
    } while (0)

std::mutex g_mu;
std::vector<int> g_devices;
bool g_inited = false;

// Restores the caller's current device on scope exit (torch owns it in bench).
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess) ok = true;
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int validate_scene(const rt_scene* sc)
{
    if (!sc) return fail(RT_EINVAL, "scene is NULL");
    if (sc->nbSpheres < 0 || sc->nbTriangles < 0) return fail(RT_EINVAL, "negative primitive count");
    if (sc->nbSpheres > 0 && !sc->sphere_list) return fail(RT_EINVAL, "sphere_list is NULL");
    if (sc->nbTriangles > 0) {
        if (!sc->triangle_list || !sc->mat_list || !sc->quelMatPourTri)
            return fail(RT_EINVAL, "triangles need triangle_list, mat_list and quelMatPourTri");
        if (sc->tex_width < 1 || sc->tex_height < 1 || sc->nbMaterials < 1)
            return fail(RT_EINVAL, "texture table %dx%d x %d materials", sc->tex_width, sc->tex_height,
                        sc->nbMaterials);
        for (int i = 0; i < sc->nbTriangles; ++i)
            if (sc->quelMatPourTri[i] < 0 || sc->quelMatPourTri[i] >= sc->nbMaterials)
                return fail(RT_EINVAL, "quelMatPourTri[%d] = %d outside [0, %d)", i, sc->quelMatPourTri[i],
                            sc->nbMaterials);
    }
    if (sc->sky_mat_list && (sc->sky_width < 1 || sc->sky_height < 1))
        return fail(RT_EINVAL, "sky table %dx%d", sc->sky_width, sc->sky_height);
    return RT_OK;
}

int validate_params(const rt_params* p)
{
    if (!p) return fail(RT_EINVAL, "params is NULL");
    if (p->largeur_image < 1 || p->hauteur_image < 1)
        return fail(RT_EINVAL, "image %dx%d", p->largeur_image, p->hauteur_image);
    if (p->nbRayonParPixel < 1) return fail(RT_EINVAL, "nbRayonParPixel %d < 1", p->nbRayonParPixel);
    if (p->nbRebondMax < 0) return fail(RT_EINVAL, "nbRebondMax %d < 0", p->nbRebondMax);
    if (p->rng == RT_RNG_GLIBC)
        return fail(RT_EUNSUPPORTED,
                    "RT_RNG_GLIBC is one sequential rand() stream with data-dependent draw counts; "
                    "only the CPU oracle replays it");
    if (p->rng != RT_RNG_PHILOX) return fail(RT_EINVAL, "unknown rng %d", p->rng);
    if (p->accel != RT_ACCEL_AUTO && p->accel != RT_ACCEL_NONE) return fail(RT_EINVAL, "unknown accel %d", p->accel);
    if (p->sky_mode != RT_SKY_OFF && p->sky_mode != RT_SKY_LAST_SPHERE)
        return fail(RT_EINVAL, "unknown sky_mode %d", p->sky_mode);
    if (p->semantics != RT_SEM_MAIN_C && p->semantics != RT_SEM_CUDA)
        return fail(RT_EINVAL, "unknown semantics %d", p->semantics);
    if (p->semantics == RT_SEM_CUDA && p->sky_mode != RT_SKY_OFF)
        return fail(RT_EINVAL, "sky_mode needs RT_SEM_MAIN_C (main_cuda.cu has no sky)");
    if (p->precision == RT_PREC_FP32)
        return fail(RT_EUNSUPPORTED, "RT_PREC_FP32 was removed (r05): its 1.1-3.4e-4 per-channel RMSE against the "
                                     "reference exceeded north_star's 1e-4; only the bit-exact FP64 path renders");
    if (p->precision != RT_PREC_FP64) return fail(RT_EINVAL, "unknown precision %d", p->precision);
    if (p->gather != RT_GATHER_RCCL && p->gather != RT_GATHER_PEER)
        return fail(RT_EINVAL, "unknown gather transport %d", p->gather);
    if ((unsigned long long)p->largeur_image * (unsigned long long)p->hauteur_image > 0xffffffffull)
        return fail(RT_EUNSUPPORTED, "pixel index exceeds the 32-bit Philox counter word");
    return RT_OK;
}

int validate_tiling(const rt_tiling* t)
{
    if (!t) return fail(RT_EINVAL, "tiling is NULL");
    if (t->tile_rows < 1 || t->tile_step < 1 || t->tile_first < 0 || t->n_tiles < 0 || t->row_base < 0)
        return fail(RT_EINVAL, "bad tiling {%d,%d,%d,%d,%d}", t->row_base, t->tile_rows, t->tile_first,
                    t->tile_step, t->n_tiles);
    if ((long long)t->n_tiles * t->tile_rows > (1ll << 30)) return fail(RT_EINVAL, "tiling too large");
    return RT_OK;
}

}  // namespace

namespace {
std::atomic<rt_denoise_fn> g_denoise{nullptr};
}

struct rt_device_scene {
    int device = 0;
    int ns = 0, ns_pad = 0, nt = 0, tw = 1, th = 1;
    long long n_texels = 0;
    SphGeo* sph = nullptr;
    SphCand* sph_cand = nullptr;
    double cand_lmax = HUGE_VAL;
    DevMat* sph_mat = nullptr;
    TriGeo* tri = nullptr;
    TriTex* tri_tex = nullptr;
    TriUV* tri_uv = nullptr;         // affine texel map per triangle (scenes that are not all uv-less)
    DevMat* texels = nullptr;
    BvhNode4* bvh = nullptr;         // 4-wide BVH; null: no BVH (few triangles)
    BvhNodeH* bvhh = nullptr;        // the same tree in 64-byte nodes, or null (does not fit binary16)
    DevMat* sky = nullptr;           // sky texels (scene->sky_mat_list), or null
    DevMat* tri_mat = nullptr;       // rt_triangle.mat per triangle (RT_SEM_CUDA)
    double cbb[6] = {0, 0, 0, 0, 0, 0};   // triangles' box (RT_SEM_CUDA hit_BBox)
    double* sph_rinv = nullptr;      // 1/radius per sphere
    double* sph_disp = nullptr;      // hsl round trip of each sphere's emission
    int sky_w = 0, sky_h = 0;
    int* tri_orig = nullptr;         // leaf order -> caller's triangle index
    int bvh_nodes = 0, bvh_depth = 0, bvh_stack4 = 0;
    double s_rel = 0.0, s_abs = 0.0, r_scene = 0.0, k_delta = 0.0;
    double sph_bound = 0.0;          // max over spheres of max_a |c_a| + r (+inf for a non-finite one)
    float bvh_rbox = 0.0f;           // >= every |bound| of the BVH's boxes
    bool mats_bounded = false;       // every diffuse/emission/strength finite, |x| <= 2^100
    bool sph_opaque = false;         // every sphere material takes main.c's opaque branch (no hole, no refraction)
    bool tri_opaque = false;         // ... every texel too, and no triangle uses material index 3 or 4
    double coord_max = HUGE_VAL;     // max |coordinate| of the spheres (|C_a| + R) and triangle vertices
    bool all_tex0 = false;           // every triangle's uv are 0: its texel is TriTex::tex0
};

namespace {

std::atomic<int> g_zero_exit{1};

// The shading fields a zero rayColor multiplies (LanePath::zero_rc).
bool shading_bounded(const DevMat& m, double lim = 0x1p100)
{
    const double v[7] = {m.dr, m.dg, m.db, m.er, m.eg, m.eb, m.es};
    for (double x : v)
        if (!(std::fabs(x) <= lim)) return false;
    return true;
}

// rgb_to_hsl then hsl_to_rgb (rtutility.h:81-165, main.c:155-158): the colour
// tracer adds when a primary ray sees an emitter.  It depends on the
// emission alone, so each sphere's is computed here once, with the same IEEE
// operations in the same order as the kernel's hsl_roundtrip (which still
// serves triangles and the sky sphere, whose material depends on the hit).
double hue_to_rgb_host(double t1, double t2, double hue)
{
    if (hue < 0.0) hue += 1.0;
    if (hue > 1.0) hue -= 1.0;
    if (6.0 * hue < 1.0) return t1 + (t2 - t1) * 6.0 * hue;
    if (2.0 * hue < 1.0) return t2;
    if (3.0 * hue < 2.0) return t1 + (t2 - t1) * (2.0 / 3.0 - hue) * 6.0;
    return t1;
}
void hsl_roundtrip_host(const rt_vec3& rgb, double out[3])
{
    const double r = rgb.e[0], g = rgb.e[1], b = rgb.e[2];
    const double mx = (r > g) ? ((r > b) ? r : b) : ((g > b) ? g : b);
    const double mn = (r < g) ? ((r < b) ? r : b) : ((g < b) ? g : b);
    double h = 0.0, sat, l = (mx + mn) / 2.0;
    if (mx == mn) {
        h = 0.0;
        sat = 0.0;
    } else {
        const double d = mx - mn;
        sat = (l < 0.5) ? (d / (mx + mn)) : (d / (2.0 - mx - mn));
        if (mx == r) h = (g - b) / d + ((g < b) ? 6.0 : 0.0);
        else if (mx == g) h = (b - r) / d + 2.0;
        else if (mx == b) h = (r - g) / d + 4.0;
        h /= 6.0;
    }
    if (sat == 0.0) {
        out[0] = out[1] = out[2] = l;
        return;
    }
    const double t2 = (l < 0.5) ? (l * (1.0 + sat)) : (l + sat - l * sat);
    const double t1 = 2.0 * l - t2;
    const double third = 1.0 / 3.0;
    out[0] = hue_to_rgb_host(t1, t2, h + third);
    out[1] = hue_to_rgb_host(t1, t2, h);
    out[2] = hue_to_rgb_host(t1, t2, h - third);
}

// tri_uvmapping's texture coordinates (texture.h:16-27, 44-90) as affine
// functions of the hit point.  The reference forms b0 = n.((B-P)x(C-P)) / areaABC
// and b1 = n.((C-P)x(A-P)) / areaABC with n the hit normal (the triangle's unit
// normal un) and areaABC = TriTex::area; in exact arithmetic b0 = (n.N +
// ((B-C)x n).(P-A)) / area and b1 = ((C-A)x n).(P-A) / area for EVERY P (the
// component of P along n cancels in n.((B-P)x(C-P))), so u = uC + b0 (uA-uC) +
// b1 (uB-uC) = u0 + gu.(P-A).  Rounding bound of the reference's u against that,
// for P with |P - A|_max <= diam (so every |P - V|_max <= R = 2 diam), Q =
// |n|_1 R^2 / area, |b_i| <= 2Q: the cross products' components are within 8u R^2,
// each area within 14u |n|_1 R^2, each b within u (38Q + 3), and u_ref within
// sum|uv| u (54Q + 7) (u = 2^-53); the kernel's evaluation (three subtractions,
// three fma, the rounded gradient and u0, the multiplication by tw) adds at most
// 10u (|u0| + |gu|_1 diam) tw.  Stored: eu = tw (4 x the first + the second)
// + 4u tw (the reference's own frac * tw rounding) -- in tw units.
void tri_uv_affine(const TriGeo& g, const TriTex& x, int tw, int th, TriUV& o)
{
    typedef long double L;
    const L u = 0x1p-53L;
    const L Ax = g.ax, Ay = g.ay, Az = g.az, Bx = x.bx, By = x.by, Bz = x.bz, Cx = x.cx, Cy = x.cy, Cz = x.cz;
    const L nx = x.unx, ny = x.uny, nz = x.unz, area = x.area;
    const L nN = nx * (L)g.nx + ny * (L)g.ny + nz * (L)g.nz;
    const L dmax = std::max({std::fabs(Bx - Ax), std::fabs(By - Ay), std::fabs(Bz - Az), std::fabs(Cx - Ax),
                             std::fabs(Cy - Ay), std::fabs(Cz - Az), std::fabs(Cx - Bx), std::fabs(Cy - By),
                             std::fabs(Cz - Bz)});
    o = TriUV{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -1.0};
    if (!(area > 0) || !std::isfinite((double)area) || !(dmax > 0) || !std::isfinite((double)dmax)) return;
    // grad b0 = (B - C) x n / area, grad b1 = (C - A) x n / area
    const L p0x = (By - Cy) * nz - (Bz - Cz) * ny, p0y = (Bz - Cz) * nx - (Bx - Cx) * nz, p0z = (Bx - Cx) * ny - (By - Cy) * nx;
    const L p1x = (Cy - Ay) * nz - (Cz - Az) * ny, p1y = (Cz - Az) * nx - (Cx - Ax) * nz, p1z = (Cx - Ax) * ny - (Cy - Ay) * nx;
    const L b0A = nN / area;                 // b0 at A (1 up to areaABC's rounding), b1 at A = 0
    const L uA = x.uau, uB = x.ubu, uC = x.ucu, vA = x.uav, vB = x.ubv, vC = x.ucv;
    const L gux = (p0x * (uA - uC) + p1x * (uB - uC)) / area, guy = (p0y * (uA - uC) + p1y * (uB - uC)) / area,
            guz = (p0z * (uA - uC) + p1z * (uB - uC)) / area;
    const L gvx = (p0x * (vA - vC) + p1x * (vB - vC)) / area, gvy = (p0y * (vA - vC) + p1y * (vB - vC)) / area,
            gvz = (p0z * (vA - vC) + p1z * (vB - vC)) / area;
    const L u0 = uC + b0A * (uA - uC), v0 = vC + b0A * (vA - vC);
    const L R = 2 * dmax;
    const L n1 = std::fabs(nx) + std::fabs(ny) + std::fabs(nz);
    const L Q = n1 * R * R / area;
    const L su = std::fabs(uA) + std::fabs(uB) + std::fabs(uC), sv = std::fabs(vA) + std::fabs(vB) + std::fabs(vC);
    const L gu1 = std::fabs(gux) + std::fabs(guy) + std::fabs(guz), gv1 = std::fabs(gvx) + std::fabs(gvy) + std::fabs(gvz);
    const L mu = std::fabs(u0) + gu1 * dmax, mv = std::fabs(v0) + gv1 * dmax;   // |u(P)|, |v(P)| bounds
    const L eu = tw * (4 * su * u * (54 * Q + 7) + 10 * u * mu + 4 * u);
    const L ev = th * (4 * sv * u * (54 * Q + 7) + 10 * u * mv + 4 * u);
    // the kernel converts floor(tw u) to int: keep |tw u| well inside 2^31
    if (!std::isfinite((double)eu) || !std::isfinite((double)ev) || tw * mu > 0x1p29L || th * mv > 0x1p29L ||
        eu > 0.25L || ev > 0.25L)
        return;
    o = TriUV{(double)gux, (double)guy, (double)guz, (double)u0, (double)gvx, (double)gvy, (double)gvz, (double)v0,
              (double)(eu * (1 + 0x1p-20L)), (double)(ev * (1 + 0x1p-20L)), (double)dmax};
}

DevMat to_dev(const rt_material& m)
{
    return DevMat{m.diffuseColor.e[0],  m.diffuseColor.e[1],  m.diffuseColor.e[2], m.emissionColor.e[0],
                  m.emissionColor.e[1], m.emissionColor.e[2], m.emissionStrength,  m.reflectionStrength,
                  m.alpha,              m.materialIndex};
}

void free_scene(rt_device_scene* s)
{
    if (!s) return;
    DeviceGuard g(s->device);
    (void)hipFree(s->sph);
    (void)hipFree(s->sph_cand);
    (void)hipFree(s->sph_mat);
    (void)hipFree(s->tri);
    (void)hipFree(s->tri_tex);
    (void)hipFree(s->tri_uv);
    (void)hipFree(s->texels);
    (void)hipFree(s->bvh);
    (void)hipFree(s->bvhh);
    (void)hipFree(s->sky);
    (void)hipFree(s->tri_mat);
    (void)hipFree(s->sph_rinv);
    (void)hipFree(s->sph_disp);
    (void)hipFree(s->tri_orig);
    delete s;
}

template <class T>
int upload(T** dst, const std::vector<T>& src)
{
    if (src.empty()) return RT_OK;
    HIP_TRY(hipMalloc((void**)dst, src.size() * sizeof(T)));
    HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return RT_OK;
}

int ensure_init_locked()
{
    if (g_inited) return RT_OK;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (n < 1) return fail(RT_EDEVICE, "no HIP device");
    g_devices.assign(1, 0);
    g_inited = true;
    return RT_OK;
}

int make_kparams(const rt_device_scene* sc, const rt_params* p, const rt_tiling* t, KParams& kp, double* uni)
{
    std::memset(&kp, 0, sizeof kp);
    kp.sph = sc->sph;
    kp.sph_cand = sc->sph_cand;
    kp.cand_lmax = sc->cand_lmax;
    kp.sph_mat = sc->sph_mat;
    kp.tri = sc->tri;
    kp.tri_tex = sc->tri_tex;
    kp.tri_uv = sc->tri_uv;
    kp.texels = sc->texels;
    kp.tri_orig = sc->tri_orig;
    kp.sph_rinv = sc->sph_rinv;
    kp.sph_disp = sc->sph_disp;
    kp.tri_mat = sc->tri_mat;
    kp.cuda = p->semantics == RT_SEM_CUDA ? 1 : 0;
    kp.f32 = 0;                      // (RT_PREC_FP32 removed in r05; the field keeps the kernarg layout)
    for (int i = 0; i < 6; ++i) kp.cbb[i] = sc->cbb[i];
    if (p->sky_mode == RT_SKY_LAST_SPHERE && sc->sky && sc->ns > 0) {
        kp.sky = sc->sky;
        kp.sky_w = sc->sky_w;
        kp.sky_h = sc->sky_h;
    }
    kp.ns = sc->ns;
    kp.ns_pad = sc->ns_pad;
    kp.ns_cand = std::isfinite(sc->cand_lmax) ? sc->ns_pad : 0;
    kp.nt = sc->nt;
    kp.tw = sc->tw;
    kp.th = sc->th;
    kp.n_texels = sc->n_texels;
    kp.W = p->largeur_image;
    kp.H = p->hauteur_image;
    kp.S = p->nbRayonParPixel;
    kp.B = p->nbRebondMax;
    for (int i = 0; i < 3; ++i) {
        uni[U_CAM_O + i] = p->cam.origin.e[i];
        uni[U_CAM_H + i] = p->cam.horizontal.e[i];
        uni[U_CAM_V + i] = p->cam.vertical.e[i];
        uni[U_CAM_C + i] = p->cam.coin_bas_gauche.e[i];
    }
    double focus = p->focus_distance, ox = p->ouverture_x, oy = p->ouverture_y, AO = p->AO_intensity;
    if (p->compat_int_truncation && p->semantics != RT_SEM_CUDA) {   // ThreadData int fields, main.c:42-43
        focus = (double)(int)focus;
        ox = (double)(int)ox;
        oy = (double)(int)oy;
        AO = (double)(int)AO;
    }
    uni[U_FOCUS] = focus;
    uni[U_OX] = ox;
    uni[U_OY] = oy;
    // camera.h:49-54: the ray starts at origin + (jx*ox, jy*oy, 0); with ox = oy = 0
    // the offsets are +-0 and the sum is the origin itself unless a coordinate is -0
    kp.cam_pin = ox == 0.0 && oy == 0.0 && !(p->cam.origin.e[0] == 0.0 && std::signbit(p->cam.origin.e[0])) &&
                 !(p->cam.origin.e[1] == 0.0 && std::signbit(p->cam.origin.e[1])) &&
                 !(p->cam.origin.e[2] == 0.0 && std::signbit(p->cam.origin.e[2]));
    kp.opaque = sc->sph_opaque ? 1 : 0;
    kp.opaque_all = sc->sph_opaque && (sc->nt == 0 || sc->tri_opaque) ? 1 : 0;
    uni[U_AO] = AO;
    uni[U_WM1] = (double)(p->largeur_image - 1);    // main.c:265 (largeur_image-1)
    uni[U_HM1] = (double)(p->hauteur_image - 1);
    uni[U_RC_WM1] = uni[U_RC_HM1] = 0.0;            // refined on the device (set_uniforms_kernel)
    kp.useAO = p->useAO ? 1 : 0;
    kp.key0 = (uint32_t)p->seed;
    kp.key1 = (uint32_t)(p->seed >> 32);
    kp.chunks = rt_resolve_spp_chunks(p->spp_chunks, p->nbRayonParPixel);
    kp.chunk_taper = rt_chunk_taper_levels(kp.S, kp.chunks);      // rt.h rt_chunk_bound
    kp.chunk_den = kp.chunk_taper ? (unsigned)(kp.chunks - kp.chunk_taper) * (1u << kp.chunk_taper) +
                                        ((1u << kp.chunk_taper) - 1u)
                                  : (unsigned)kp.chunks;
    kp.row_base = t->row_base;
    kp.tile_rows = t->tile_rows;
    kp.tile_first = t->tile_first;
    kp.tile_step = t->tile_step;
    kp.n_tiles = t->n_tiles;
    kp.row_end = p->hauteur_image;
    kp.local_rows = t->n_tiles * t->tile_rows;
    // The BVH padding assumed every ray origin within r_scene (rt_bvh.cpp);
    // primary rays start at the camera origin + (dx, dy, 0), |dx| <= |ox|/2.
    double cam = 0.0;
    for (int i = 0; i < 3; ++i) cam = std::max(cam, std::fabs(p->cam.origin.e[i]));
    cam += 0.5 * (std::fabs(ox) + std::fabs(oy));
    if (!std::isfinite(cam) || !std::isfinite(p->cam.origin.e[0]) || !std::isfinite(p->cam.origin.e[1]) ||
        !std::isfinite(p->cam.origin.e[2]))
        cam = HUGE_VAL;                  // std::max drops NaN: no gate below may pass on a NaN camera
    // Zero-throughput exit (rt_kernels.hip LanePath::zero_rc): exact when the
    // shading values are bounded and, with AO, the AO factor stays finite.
    kp.zero_exit = g_zero_exit.load() && p->semantics != RT_SEM_CUDA && sc->mats_bounded &&
                   (!kp.useAO || (AO > 0.0 && AO <= 1000.0 && std::fmax(sc->coord_max, cam) <= 0x1p20));
    // TriTex::tex0 (constant texels of uv-less triangles): a hit point P is then
    // within ~2^101 of the origin, the signed areas of get_barycentric_coord stay
    // below 2^205 and areaABC >= |N| (1 - 2^-50) with |N| >= 1e-6 / |d| for any
    // hit (det >= 1e-6), so the barycentrics are finite and u = v = +-0
    kp.tex_const = sc->all_tex0 && std::fmax(sc->coord_max, cam) <= 0x1p100;
    // (origins beyond r_scene -- the camera, hit points on far spheres -- widen
    // the walk's margins per ray, rt_kernels.hip ray32; a non-finite camera
    // takes the every-triangle scan)
    if (sc->bvh && p->accel == RT_ACCEL_AUTO && std::isfinite(cam)) {
        kp.bvh = sc->bvh;
        kp.bvhh = sc->bvhh;
        kp.bvh_srel = sc->s_rel;
        kp.bvh_sabs = sc->s_abs;
        kp.bvh_rb = sc->r_scene;
        kp.bvh_kdelta = sc->k_delta;
        {
            float rf = (float)sc->r_scene;            // rb_f (1 + 2^-23) <= R_b
            while (rf > 0.0f && (double)rf * (1.0 + 0x1p-23) > sc->r_scene) rf = std::nextafter(rf, 0.0f);
            kp.bvh_rb_f = rf;
            // origins: the camera (+ aperture), hit points on the spheres and on
            // the triangles (inside R_b by construction)
            kp.bvh_far = !(cam <= sc->r_scene && sc->sph_bound <= sc->r_scene);
        }
        kp.bvh_rbox = sc->bvh_rbox;
        // the traversal stack's uint16 entries (node indices): entries the tree can
        // need (rt_bvh.cpp's exact bound), or more than any stack when an index
        // would not fit
        kp.bvh_stack = (sc->bvh_nodes < 0x8000 && sc->nt <= 0x8000) ? sc->bvh_stack4 : 1 << 30;
        // shallow trees finish most walks in one round with 4 visits; deeper ones
        // do best with 3 (measured: sweep depth4 3: 3395 -> 3542 at 4; C4 depth4 7:
        // 1134 at 3, 1122 at 4)
        kp.bvh_steps = sc->bvh_depth <= 4 ? 4 : 3;
        kp.bvh_nodes = sc->bvh_nodes;
    }
    return RT_OK;
}

// Stream-ordered scratch (uniform block, chunk partials) around one launch.
// The device's default memory pool keeps freed blocks (release threshold
// raised once), so repeated launches do not re-map memory.
// Bytes of chunk partials per launch (RT_PARTIAL_BUDGET overrides; tests use
// a small budget to exercise the banding).
size_t partial_budget()
{
    const char* e = std::getenv("RT_PARTIAL_BUDGET");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (size_t)v : ((size_t)4 << 30);
}

int launch_on_stream(KParams& kp, const double* uni, hipStream_t st, bool count)
{
    static std::once_flag pool_once[64];
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev >= 0 && dev < 64) {
        std::call_once(pool_once[dev], [dev]() {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
                uint64_t thr = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
            }
        });
    }
    double* d_uni = nullptr;
    double* d_part = nullptr;
    // uniform block + render_kernel_q's task counter (on its own 64-byte line)
    HIP_TRY(hipMallocAsync((void**)&d_uni, (U_COUNT + 16) * sizeof(double), st));
    UniBlock ub;
    for (int i = 0; i < U_COUNT; ++i) ub.v[i] = uni[i];
    hipError_t e = (hipError_t)launch_set_uniforms(ub, d_uni, st);
    // With spp_chunks > 1 the per-chunk partial sums ([chunks][rows*W][9]
    // doubles) are bounded by kPartialBudget: taller frames are rendered in
    // row bands that reuse one partial buffer (pixels are independent, so
    // banding does not change any result).  See partial_budget().
    int band = kp.local_rows;
    if (kp.chunks > 1 && !count) {
        const size_t per_row = (size_t)kp.chunks * kp.W * 9 * sizeof(double);
        const size_t rows = std::max<size_t>(16, partial_budget() / per_row / 16 * 16);
        band = (int)std::min<size_t>(rows, (size_t)kp.local_rows);
        if (e == hipSuccess) e = hipMallocAsync((void**)&d_part, per_row * band, st);
    }
    kp.uni = d_uni;
    kp.partial = d_part;
    // the queue kernel numbers tasks (chunk, pixel of the band) in 32 bits
    kp.task_ctr = (d_part && (unsigned long long)band * kp.W * kp.chunks < (1ull << 31))
                      ? (unsigned*)(d_uni + ((U_COUNT + 7) / 8 + 1) * 8) : nullptr;
    // the stack of the kernel a render of these params takes (a count run emulates
    // the render's banding to find out whether that render has the task counter)
    {
        int band_r = kp.local_rows;
        if (kp.chunks > 1) {
            const size_t per_row = (size_t)kp.chunks * kp.W * 9 * sizeof(double);
            band_r = (int)std::min<size_t>(std::max<size_t>(16, partial_budget() / per_row / 16 * 16),
                                           (size_t)kp.local_rows);
        }
        const bool task_ok = kp.chunks > 1 && (unsigned long long)band_r * kp.W * kp.chunks < (1ull << 31);
        kp.stack_cap = choose_render(kp, count ? task_ok : kp.task_ctr != nullptr).stack_cap;
    }
    for (int y0 = 0; e == hipSuccess && y0 < kp.local_rows; y0 += band) {
        kp.band_y0 = y0;
        kp.band_rows = band;
        e = (hipError_t)(count ? launch_count(kp, st) : launch_render(kp, st));
    }
    if (d_part) (void)hipFreeAsync(d_part, st);
    (void)hipFreeAsync(d_uni, st);
    if (e != hipSuccess) return fail(RT_EDEVICE, "render launch: %s", hipGetErrorString(e));
    return RT_OK;
}

// ---- host-buffer drop-in plumbing (rt_render_rows / rt_fill_canva) --------
// main.c runs fill_canva on NUM_THREADS pthreads (main.c:404-453); each of
// them becomes one rt_render_rows call.  So that those calls neither re-upload
// the scene (and rebuild its BVH) nor serialise on hipFree/hipStreamDestroy:
//  * uploaded scenes are cached per device, keyed by the exact bytes of the
//    caller's arrays (a changed array is a different scene, never stale);
//  * streams come from a per-device pool, each with a pinned staging buffer
//    for its D2H copy, reused across calls;
//  * frame planes are stream-ordered allocations (hipMallocAsync) from the
//    device pool whose release threshold launch_on_stream raises.
std::atomic<int> g_fill_chunks{RT_SPP_CHUNKS_AUTO};
std::atomic<int> g_fill_prec{RT_PREC_FP64};

struct PooledStream {
    int device = 0;
    hipStream_t st = nullptr;
    void* host = nullptr;            // pinned staging for the D2H copy
    size_t host_bytes = 0;
    hipEvent_t plane_done[3] = {nullptr, nullptr, nullptr};   // D2H of each output plane
    hipError_t reserve_host(size_t n)
    {
        if (n <= host_bytes) return hipSuccess;
        if (host) (void)hipHostFree(host);
        host = nullptr;
        host_bytes = 0;
        const hipError_t e = hipHostMalloc(&host, n, hipHostMallocDefault);
        if (e == hipSuccess) host_bytes = n;
        return e;
    }
};

std::mutex g_pool_mu;
std::vector<PooledStream*> g_pool_free;    // idle streams (any device); destroyed by rt_shutdown

int stream_pool_get(int device, PooledStream** out)
{
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool_free.size(); ++i)
            if (g_pool_free[i]->device == device) {
                *out = g_pool_free[i];
                g_pool_free.erase(g_pool_free.begin() + (long)i);
                return RT_OK;
            }
    }
    DeviceGuard g(device);
    PooledStream* ps = new PooledStream();
    ps->device = device;
    hipError_t e = hipStreamCreateWithFlags(&ps->st, hipStreamNonBlocking);
    for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ps->plane_done[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (hipEvent_t ev : ps->plane_done)
            if (ev) (void)hipEventDestroy(ev);
        if (ps->st) (void)hipStreamDestroy(ps->st);
        delete ps;
        return fail(RT_EDEVICE, "device %d stream: %s", device, hipGetErrorString(e));
    }
    *out = ps;
    return RT_OK;
}

void stream_pool_put(PooledStream* ps)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool_free.push_back(ps);
}

// Idle pooled streams and their pinned staging buffers (streams a call still
// holds go back to the pool when it returns and are released by the next
// rt_shutdown).
void stream_pool_clear()
{
    std::vector<PooledStream*> idle;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        idle.swap(g_pool_free);
    }
    for (PooledStream* ps : idle) {
        DeviceGuard g(ps->device);
        (void)hipStreamSynchronize(ps->st);
        (void)hipStreamDestroy(ps->st);
        for (hipEvent_t ev : ps->plane_done)
            if (ev) (void)hipEventDestroy(ev);
        if (ps->host) (void)hipHostFree(ps->host);
        delete ps;
    }
}

// fn(i0, i1) over [0, n) split into nthr contiguous ranges, the first on
// the calling thread (host-side scatter of a frame's rows)
std::atomic<int> g_calls_in_flight{0};    // rt_render_rows calls running (rt_fill_canva's threads)

template <class F>
void par_ranges(int n, int nthr, const F& fn)
{
    nthr = std::max(1, std::min(nthr, n));
    if (nthr == 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nthr - 1);
    for (int t = 1; t < nthr; ++t) th.emplace_back(fn, (int)((long long)n * t / nthr), (int)((long long)n * (t + 1) / nthr));
    fn(0, (int)((long long)n / nthr));
    for (auto& x : th) x.join();
}

// Exact bytes of everything rt_scene_upload reads.
std::vector<unsigned char> scene_key(const rt_scene* sc)
{
    std::vector<unsigned char> k;
    auto put = [&k](const void* p, size_t n) {
        const unsigned char* b = (const unsigned char*)p;
        k.insert(k.end(), b, b + n);
    };
    const int hdr[7] = {sc->nbSpheres, sc->nbTriangles, sc->tex_width, sc->tex_height, sc->nbMaterials,
                        sc->sky_mat_list ? sc->sky_width : -1, sc->sky_mat_list ? sc->sky_height : -1};
    put(hdr, sizeof hdr);
    if (sc->nbSpheres > 0) put(sc->sphere_list, sizeof(rt_sphere) * (size_t)sc->nbSpheres);
    if (sc->nbTriangles > 0) {
        put(sc->triangle_list, sizeof(rt_triangle) * (size_t)sc->nbTriangles);
        put(sc->quelMatPourTri, sizeof(int) * (size_t)sc->nbTriangles);
        put(sc->mat_list, sizeof(rt_material) * (size_t)sc->nbMaterials * sc->tex_width * sc->tex_height);
    }
    if (sc->sky_mat_list) put(sc->sky_mat_list, sizeof(rt_material) * (size_t)sc->sky_width * sc->sky_height);
    return k;
}

struct CachedScene {
    int device;
    std::vector<unsigned char> key;
    std::shared_ptr<rt_device_scene> ds;
    unsigned long long used;
};
// The cache is a heap object that is never destroyed: a process that exits
// without rt_shutdown (main.c's drop-in flow never calls it) must not run
// free_scene -> hipFree from a static destructor after the HIP runtime may
// already be torn down; the driver reclaims the device memory at exit.
std::mutex g_cache_mu;
std::vector<CachedScene>& g_cache = *new std::vector<CachedScene>();   // at most kCacheEntries, LRU evicted
unsigned long long g_cache_clock = 0;
constexpr size_t kCacheEntries = 4;

// The device copy of *sc on `device`, uploaded on first use.  Held under the
// cache lock: concurrent callers of one new scene wait for its single upload.
int scene_cache_get(int device, const rt_scene* sc, std::shared_ptr<rt_device_scene>& out)
{
    std::vector<unsigned char> key = scene_key(sc);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (CachedScene& c : g_cache)
        if (c.device == device && c.key == key) {
            c.used = ++g_cache_clock;
            out = c.ds;
            return RT_OK;
        }
    rt_device_scene* ds = nullptr;
    const int rc = rt_scene_upload(device, sc, &ds);
    if (rc) return rc;
    if (g_cache.size() >= kCacheEntries) {
        size_t lru = 0;
        for (size_t i = 1; i < g_cache.size(); ++i)
            if (g_cache[i].used < g_cache[lru].used) lru = i;
        g_cache.erase(g_cache.begin() + (long)lru);    // in-flight users keep their reference
    }
    g_cache.push_back(CachedScene{device, std::move(key), std::shared_ptr<rt_device_scene>(ds, free_scene),
                                  ++g_cache_clock});
    out = g_cache.back().ds;
    return RT_OK;
}

int scene_cache_clear()
{
    std::lock_guard<std::mutex> lk(g_cache_mu);
    const int n = (int)g_cache.size();
    g_cache.clear();
    return n;
}

}  // namespace

extern "C" {

void rt_params_init(rt_params* p)
{
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->rng = RT_RNG_PHILOX;
    p->seed = 1010ull;
    p->compat_int_truncation = 1;
    p->spp_chunks = RT_SPP_CHUNKS_AUTO;
}

int rt_init(int ndev, const int* devices)
{
    std::lock_guard<std::mutex> lk(g_mu);
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (n < 1) return fail(RT_EDEVICE, "no HIP device");
    std::vector<int> devs;             // committed only when every id is visible
    if (ndev <= 0 || !devices) {
        devs.push_back(0);
    } else {
        for (int i = 0; i < ndev; ++i) {
            if (devices[i] < 0 || devices[i] >= n)
                return fail(RT_EINVAL, "device %d is not visible (%d device%s)", devices[i], n, n == 1 ? "" : "s");
            devs.push_back(devices[i]);
        }
    }
    g_devices.swap(devs);
    g_inited = true;
    return RT_OK;
}

void rt_shutdown(void)
{
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_devices.clear();
        g_inited = false;
    }
    scene_cache_clear();
    stream_pool_clear();
    rccl_release();
}

const char* rt_last_error(void) { return g_err.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_render_kernel(void) { return last_render_kernel(); }

const char* rt_version(void)
{
#define RT_STR2(x) #x
#define RT_STR(x) RT_STR2(x)
    return "tipe-raytracer-mi355x 0.6 (abi " RT_STR(RT_ABI_VERSION) ", gfx950; precision FP64, bit-exact against "
           "the reference's own composition; RT_PREC_FP32 removed (RT_EUNSUPPORTED); rt_params_init defaults "
           "spp_chunks to RT_SPP_CHUNKS_AUTO, a fixed per-pixel slice grouping; multi-device gathers over RCCL "
           "(RT_GATHER_RCCL) or peer copies (RT_GATHER_PEER))";
#undef RT_STR
#undef RT_STR2
}

int rt_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_scene_upload(int device, const rt_scene* scene, rt_device_scene** out)
{
    if (!out) return fail(RT_EINVAL, "out is NULL");
    *out = nullptr;
    int rc = validate_scene(scene);
    if (rc) return rc;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(RT_EINVAL, "device %d of %d", device, n);
    DeviceGuard guard(device);
    if (!guard.ok) return fail(RT_EDEVICE, "hipSetDevice(%d) failed", device);

    // Spheres padded to an even count with never-hit records (r2 = -inf makes
    // the discriminant -inf): the kernel reads them two per s_load_dwordx16.
    // The candidate pass keeps the winner's slot in 16 mantissa bits (RT_CAND_TAG):
    // above 65534 spheres it is switched off (cand_lmax = +inf, KParams::ns_cand = 0)
    // and every ray takes the exact reference scan -- correct for any count, slower.
    const int ns_pad = (scene->nbSpheres + 1) & ~1;
    std::vector<SphGeo> sph((size_t)ns_pad, SphGeo{0.0, 0.0, 0.0, -HUGE_VAL});
    std::vector<SphCand> cand((size_t)ns_pad, SphCand{0.0, 0.0, 0.0, HUGE_VAL});
    std::vector<DevMat> sph_mat((size_t)scene->nbSpheres);
    std::vector<double> sph_rinv((size_t)scene->nbSpheres);
    std::vector<double> sph_disp((size_t)scene->nbSpheres * 3);
    // Candidate-pass bound L >= |C_k| + R_k for every sphere (rounded up, at
    // least 2^-20); a non-finite sphere makes it +inf, which turns the
    // candidate pass into the exact scan (rt_kernels.hip spheres_closest).
    long double lmax = 0x1p-20L;
    for (int i = 0; i < scene->nbSpheres; ++i) {
        const rt_sphere& s = scene->sphere_list[i];
        const double r2 = s.radius * s.radius;
        sph[i] = SphGeo{s.center.e[0], s.center.e[1], s.center.e[2], r2};
        const long double cx = s.center.e[0], cy = s.center.e[1], cz = s.center.e[2];
        const long double c2 = cx * cx + cy * cy + cz * cz;
        cand[i] = SphCand{s.center.e[0], s.center.e[1], s.center.e[2], (double)(c2 - (long double)r2)};
        const long double L = (std::sqrt(c2) + std::fabs((long double)s.radius)) * (1.0L + 0x1p-40L);
        lmax = std::isfinite((double)L) && !std::isnan((double)cand[i].k) ? std::max(lmax, L) : (long double)HUGE_VAL;
        sph_mat[i] = to_dev(s.mat);
        sph_rinv[i] = 1 / s.radius;                    // divide(v, t) = v * (1/t), vec3.h:105-107
        hsl_roundtrip_host(s.mat.emissionColor, &sph_disp[3 * (size_t)i]);
    }
    const double cand_lmax = std::isfinite((double)lmax) && scene->nbSpheres <= 65534
                                 ? std::nextafter((double)lmax, HUGE_VAL) : HUGE_VAL;
    std::vector<DevMat> sky;
    if (scene->sky_mat_list)
        for (long long i = 0; i < (long long)scene->sky_width * scene->sky_height; ++i)
            sky.push_back(to_dev(scene->sky_mat_list[i]));
    std::vector<TriGeo> tri((size_t)scene->nbTriangles);
    std::vector<TriTex> tex((size_t)scene->nbTriangles);
    std::vector<DevMat> tri_mat((size_t)scene->nbTriangles);
    double cbb[6] = {0, 0, 0, 0, 0, 0};
    if (scene->nbTriangles > 0) {                    // load_geometry_data's box, triangle.hu:142-156
        for (int a = 0; a < 3; ++a) cbb[a] = cbb[3 + a] = scene->triangle_list[0].A.e[a];
        for (int i = 0; i < scene->nbTriangles; ++i) {
            const rt_triangle& t = scene->triangle_list[i];
            for (int a = 0; a < 3; ++a) {
                cbb[a] = std::fmin(cbb[a], std::fmin(t.A.e[a], std::fmin(t.B.e[a], t.C.e[a])));
                cbb[3 + a] = std::fmax(cbb[3 + a], std::fmax(t.A.e[a], std::fmax(t.B.e[a], t.C.e[a])));
            }
        }
    }
    for (int i = 0; i < scene->nbTriangles; ++i) {
        const rt_triangle& t = scene->triangle_list[i];
        const double abx = t.B.e[0] - t.A.e[0], aby = t.B.e[1] - t.A.e[1], abz = t.B.e[2] - t.A.e[2];
        const double acx = t.C.e[0] - t.A.e[0], acy = t.C.e[1] - t.A.e[1], acz = t.C.e[2] - t.A.e[2];
        TriGeo& g = tri[i];
        g.ax = t.A.e[0];
        g.ay = t.A.e[1];
        g.az = t.A.e[2];
        g.abx = abx;
        g.aby = aby;
        g.abz = abz;
        g.acx = acx;
        g.acy = acy;
        g.acz = acz;
        g.nx = aby * acz - abz * acy;          // vec3_cross, vec3.h:121-127
        g.ny = abz * acx - abx * acz;
        g.nz = abx * acy - aby * acx;
        TriTex& x = tex[i];
        x.bx = t.B.e[0];
        x.by = t.B.e[1];
        x.bz = t.B.e[2];
        x.cx = t.C.e[0];
        x.cy = t.C.e[1];
        x.cz = t.C.e[2];
        x.uau = t.uvA.u;
        x.uav = t.uvA.v;
        x.ubu = t.uvB.u;
        x.ubv = t.uvB.v;
        x.ucu = t.uvC.u;
        x.ucv = t.uvC.v;
        x.mat = scene->quelMatPourTri[i];
        x.tex0 = -1;
        if (t.uvA.u == 0.0 && t.uvA.v == 0.0 && t.uvB.u == 0.0 && t.uvB.v == 0.0 && t.uvC.u == 0.0 &&
            t.uvC.v == 0.0) {
            // tri_uvmapping (texture.h:44-90) with every uv 0: u = v = +-0 for
            // finite barycentrics, so x = y = 0 and the index is tw*th*mat (clamped
            // into the table as the kernel clamps it)
            const long long nt = (long long)scene->nbMaterials * scene->tex_width * scene->tex_height;
            long long idx = (long long)scene->tex_height * scene->tex_width * x.mat;
            idx = idx < 0 ? 0 : idx;
            idx = idx >= nt ? nt - 1 : idx;
            if (nt > 0 && nt < (1LL << 31)) x.tex0 = (int)idx;
        }
        // hit_triangle's normal, vec3_normalize(normalVect) (mesh.h:91, vec3.h:137-139):
        // a pure function of the triangle, computed once here with the reference's
        // operations (IEEE sqrt and divisions, no contraction) instead of per hit
        const double nl = std::sqrt((g.nx * g.nx + g.ny * g.ny) + g.nz * g.nz);
        x.unx = g.nx / nl;
        x.uny = g.ny / nl;
        x.unz = g.nz / nl;
        // get_barycentric_coord's areaABC (texture.h:18) with the hit normal n = un:
        // dot(n, cross(B - A, C - A)) = dot(un, N), constant per triangle
        x.area = (x.unx * g.nx + x.uny * g.ny) + x.unz * g.nz;
        tri_mat[i] = to_dev(t.mat);
    }
    // Triangle BVH (rt_bvh.cpp) over scenes with more than 32 triangles; the
    // triangle arrays are then stored in leaf order.  r_scene bounds the
    // triangles' coordinates (so every hit point on them) and the spheres
    // whose hit points cost the padding little (bvh_origin_radius); the padding
    // assumes origins within it, and rays from farther out (the camera, hit
    // points on large spheres such as main.c:346's radius-1e5 sky) widen the
    // walk's margins by the rest (rt_kernels.hip ray32).  Against r_scene over
    // every sphere: RTX_MAP/nature under the sky 700 -> 808 Msamples/s at 64 spp
    // (r06, tools/probes/nature_radius.py)
    BvhBuild bvh;
    if (scene->nbTriangles > 32) {           // (a BVH over C3's 5 triangles: 5118 -> 4482 Msamples/s)
        double r = 1.0;
        for (int i = 0; i < scene->nbTriangles; ++i) {
            const rt_triangle& t = scene->triangle_list[i];
            for (int a = 0; a < 3; ++a)
                r = std::max({r, std::fabs(t.A.e[a]), std::fabs(t.B.e[a]), std::fabs(t.C.e[a])});
        }
        std::vector<double> sb((size_t)scene->nbSpheres);
        for (int i = 0; i < scene->nbSpheres; ++i) {
            const rt_sphere& q = scene->sphere_list[i];
            double b = 0.0;
            for (int a = 0; a < 3; ++a) b = std::max(b, std::fabs(q.center.e[a]) + std::fabs(q.radius));
            sb[(size_t)i] = std::isfinite(b) ? b : HUGE_VAL;
        }
        if (std::isfinite(r)) r = bvh_origin_radius(tri.data(), scene->nbTriangles, r, sb.data(), scene->nbSpheres);
        if (std::isfinite(r) && build_bvh(tri.data(), scene->nbTriangles, r, bvh)) {
            std::vector<TriGeo> tri2(tri.size());
            std::vector<TriTex> tex2(tex.size());
            std::vector<DevMat> mat2(tri_mat.size());
            for (size_t k = 0; k < tri.size(); ++k) {
                tri2[k] = tri[(size_t)bvh.order[k]];
                tex2[k] = tex[(size_t)bvh.order[k]];
                mat2[k] = tri_mat[(size_t)bvh.order[k]];
            }
            tri.swap(tri2);
            tex.swap(tex2);
            tri_mat.swap(mat2);
        }
    }
    std::vector<DevMat> texels;
    long long n_texels = 0;
    if (scene->nbTriangles > 0) {
        n_texels = (long long)scene->nbMaterials * scene->tex_width * scene->tex_height;
        if (n_texels >= (1LL << 31))     // the kernels index texels in 32 bits (160 GiB of texels)
            return fail(RT_EUNSUPPORTED, "%lld texels >= 2^31", n_texels);
        texels.resize((size_t)n_texels);
        for (long long i = 0; i < n_texels; ++i) texels[(size_t)i] = to_dev(scene->mat_list[i]);
    }

    bool mats_bounded = true;
    double coord_max = 0.0;
    for (const std::vector<DevMat>* v : {&sph_mat, &texels, &sky})
        for (const DevMat& m : *v) {
            mats_bounded = mats_bounded && shading_bounded(m);
        }
    for (int i = 0; i < scene->nbSpheres; ++i) {
        const rt_sphere& q = scene->sphere_list[i];
        for (int a = 0; a < 3; ++a) coord_max = std::fmax(coord_max, std::fabs(q.center.e[a]) + std::fabs(q.radius));
        if (!std::isfinite(q.radius)) coord_max = HUGE_VAL;
    }
    for (int i = 0; i < scene->nbTriangles; ++i) {
        const rt_triangle& t = scene->triangle_list[i];
        for (int a = 0; a < 3; ++a)
            coord_max = std::fmax(coord_max, std::fmax(std::fabs(t.A.e[a]), std::fmax(std::fabs(t.B.e[a]), std::fabs(t.C.e[a]))));
    }
    // fmax drops NaN operands: a non-finite coordinate anywhere makes the bound
    // infinite, so the gates that read it (zero_exit, tex_const) hold by construction
    for (int i = 0; i < scene->nbSpheres; ++i)
        for (int a = 0; a < 3; ++a)
            if (!std::isfinite(scene->sphere_list[i].center.e[a])) coord_max = HUGE_VAL;
    for (int i = 0; i < scene->nbTriangles; ++i) {
        const rt_triangle& t = scene->triangle_list[i];
        for (int a = 0; a < 3; ++a)
            if (!std::isfinite(t.A.e[a]) || !std::isfinite(t.B.e[a]) || !std::isfinite(t.C.e[a])) coord_max = HUGE_VAL;
    }

    rt_device_scene* ds = new rt_device_scene();
    ds->device = device;
    ds->mats_bounded = mats_bounded;
    const auto opaque_mat = [](const DevMat& m) { return !(m.alpha < 0.0001) && !(m.alpha <= 0.99); };
    ds->sph_opaque = std::all_of(sph_mat.begin(), sph_mat.end(), opaque_mat);
    // tri_material (rt_kernels.hip): the texel's alpha, overridden for
    // material indices 1 (1.0), 3 (0.1) and 4 (0.6); the texel index is
    // clamped into the whole table, so every texel counts
    ds->tri_opaque = std::all_of(texels.begin(), texels.end(), opaque_mat);
    for (int i = 0; i < scene->nbTriangles && ds->tri_opaque; ++i)
        if (scene->quelMatPourTri[i] == 3 || scene->quelMatPourTri[i] == 4) ds->tri_opaque = false;
    ds->coord_max = coord_max;
    ds->all_tex0 = scene->nbTriangles > 0 &&
                   std::all_of(tex.begin(), tex.end(), [](const TriTex& x) { return x.tex0 >= 0; });
    // the affine texel map (rt_kernels.hip tri_texel's fast path), in leaf order
    std::vector<TriUV> tri_uv;
    if (scene->nbTriangles > 0 && !ds->all_tex0) {
        tri_uv.resize(tex.size());
        for (size_t i = 0; i < tex.size(); ++i)
            tri_uv_affine(tri[i], tex[i], scene->tex_width, scene->tex_height, tri_uv[i]);
    }
    ds->ns = scene->nbSpheres;
    ds->ns_pad = ns_pad;
    ds->cand_lmax = cand_lmax;
    for (int i = 0; i < 6; ++i) ds->cbb[i] = cbb[i];
    ds->nt = scene->nbTriangles;
    ds->tw = scene->nbTriangles > 0 ? scene->tex_width : 1;
    ds->th = scene->nbTriangles > 0 ? scene->tex_height : 1;
    ds->n_texels = n_texels;
    ds->sky_w = scene->sky_mat_list ? scene->sky_width : 0;
    ds->sky_h = scene->sky_mat_list ? scene->sky_height : 0;
    ds->bvh_nodes = (int)bvh.nodes4.size();
    ds->bvh_depth = bvh.depth4;
    ds->bvh_stack4 = bvh.stack4;
    ds->s_rel = bvh.s_rel;
    ds->s_abs = bvh.s_abs;
    ds->r_scene = bvh.r_scene;
    for (int i = 0; i < scene->nbSpheres; ++i) {
        const rt_sphere& q = scene->sphere_list[i];
        double b = 0.0;
        for (int a = 0; a < 3; ++a) b = std::max(b, std::fabs(q.center.e[a]) + std::fabs(q.radius));
        ds->sph_bound = std::isfinite(b) ? std::max(ds->sph_bound, b) : HUGE_VAL;   // (max keeps +inf)
    }
    ds->k_delta = bvh.k_delta;
    {
        float rb = 0.0f;             // the single-precision slab margin's coordinate bound
        for (const BvhNode4& nd : bvh.nodes4)
            for (int c = 0; c < 4; ++c)
                if (nd.count[c] >= 0)
                    for (int a = 0; a < 3; ++a) rb = std::max({rb, std::fabs(nd.lo[a][c]), std::fabs(nd.hi[a][c])});
        ds->bvh_rbox = std::isfinite(rb) ? rb * (1.0f + 0x1p-20f) : HUGE_VALF;
    }
    std::vector<BvhNodeH> nodesh;
    {
        float rbh = 0.0f;
        if (!bvh.nodes4.empty() && pack_bvh_h(bvh.nodes4, nodesh, rbh))
            ds->bvh_rbox = std::max(ds->bvh_rbox, rbh * (1.0f + 0x1p-20f));   // one bound serves both forms
        else
            nodesh.clear();
    }
    if ((rc = upload(&ds->sph, sph)) || (rc = upload(&ds->sph_cand, cand)) || (rc = upload(&ds->sph_mat, sph_mat)) || (rc = upload(&ds->tri, tri)) ||
        (rc = upload(&ds->tri_tex, tex)) || (rc = upload(&ds->tri_uv, tri_uv)) || (rc = upload(&ds->texels, texels)) ||
        (rc = upload(&ds->bvh, bvh.nodes4)) || (rc = upload(&ds->bvhh, nodesh)) || (rc = upload(&ds->tri_orig, bvh.order)) ||
        (rc = upload(&ds->sky, sky)) || (rc = upload(&ds->sph_rinv, sph_rinv)) || (rc = upload(&ds->sph_disp, sph_disp)) ||
        (rc = upload(&ds->tri_mat, tri_mat))) {
        free_scene(ds);
        return rc;
    }
    *out = ds;
    return RT_OK;
}

void rt_scene_release(rt_device_scene* scene) { free_scene(scene); }

int rt_render_async(const rt_device_scene* scene, const rt_params* params, const rt_tiling* tiling,
                    const rt_frame* frame, void* hip_stream)
{
    if (!scene) return fail(RT_EINVAL, "scene is NULL");
    int rc;
    if ((rc = validate_params(params)) || (rc = validate_tiling(tiling))) return rc;
    if (!frame || !frame->canva) return fail(RT_EINVAL, "frame.canva is NULL");
    KParams kp;
    double uni[U_COUNT];
    make_kparams(scene, params, tiling, kp, uni);
    kp.canva = (double*)frame->canva;
    kp.albedo = (double*)frame->albedo;
    kp.normal = (double*)frame->normal;
    kp.radiance = (double*)frame->radiance;
    if (kp.local_rows == 0 || kp.W == 0) return RT_OK;
    DeviceGuard guard(scene->device);
    return launch_on_stream(kp, uni, (hipStream_t)hip_stream, false);
}

int rt_accumulate_async(const rt_device_scene* scene, const rt_params* params, long long sample_offset,
                        const rt_tiling* tiling, double* d_sums, void* hip_stream)
{
    if (!scene) return fail(RT_EINVAL, "scene is NULL");
    int rc;
    if ((rc = validate_params(params)) || (rc = validate_tiling(tiling))) return rc;
    if (!d_sums) return fail(RT_EINVAL, "d_sums is NULL");
    if (sample_offset < 0 || sample_offset + params->nbRayonParPixel > (1ll << 32))
        return fail(RT_EINVAL, "samples [%lld, %lld) exceed the 32-bit Philox sample word", sample_offset,
                    sample_offset + params->nbRayonParPixel);
    KParams kp;
    double uni[U_COUNT];
    make_kparams(scene, params, tiling, kp, uni);
    kp.sums = d_sums;
    kp.s_base = sample_offset;
    if (kp.local_rows == 0 || kp.W == 0) return RT_OK;
    DeviceGuard guard(scene->device);
    return launch_on_stream(kp, uni, (hipStream_t)hip_stream, false);
}

int rt_resolve_async(const double* d_sums, const rt_params* params, int total_spp, const rt_tiling* tiling,
                     const rt_frame* frame, void* hip_stream)
{
    int rc;
    if ((rc = validate_tiling(tiling))) return rc;
    if (!params || params->largeur_image < 1 || params->hauteur_image < 1) return fail(RT_EINVAL, "bad params");
    if (!d_sums || !frame || !frame->canva) return fail(RT_EINVAL, "NULL buffer");
    if (total_spp < 1) return fail(RT_EINVAL, "total_spp %d < 1", total_spp);
    KParams kp;
    std::memset(&kp, 0, sizeof kp);
    kp.W = params->largeur_image;
    kp.H = params->hauteur_image;
    kp.S = total_spp;
    kp.row_base = tiling->row_base;
    kp.tile_rows = tiling->tile_rows;
    kp.tile_first = tiling->tile_first;
    kp.tile_step = tiling->tile_step;
    kp.n_tiles = tiling->n_tiles;
    kp.row_end = params->hauteur_image;
    kp.local_rows = tiling->n_tiles * tiling->tile_rows;
    kp.sums = (double*)d_sums;
    kp.canva = (double*)frame->canva;
    kp.albedo = (double*)frame->albedo;
    kp.normal = (double*)frame->normal;
    kp.radiance = (double*)frame->radiance;
    if (kp.local_rows == 0) return RT_OK;
    const int e = launch_resolve(kp, hip_stream);
    if (e) return fail(RT_EDEVICE, "resolve launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int rt_count_async(const rt_device_scene* scene, const rt_params* params, const rt_tiling* tiling,
                   unsigned long long* d_counters, void* hip_stream)
{
    if (!scene) return fail(RT_EINVAL, "scene is NULL");
    int rc;
    if ((rc = validate_params(params)) || (rc = validate_tiling(tiling))) return rc;
    if (!d_counters) return fail(RT_EINVAL, "d_counters is NULL");
    KParams kp;
    double uni[U_COUNT];
    make_kparams(scene, params, tiling, kp, uni);
    kp.counters = d_counters;
    if (kp.local_rows == 0) return RT_OK;
    DeviceGuard guard(scene->device);
    return launch_on_stream(kp, uni, (hipStream_t)hip_stream, true);
}

int rt_assemble_async(const rt_color* gathered, long long rank_stride, int world, int tile_rows, int rows_per_rank,
                      int W, int H, rt_color* out, void* hip_stream)
{
    if (!gathered || !out) return fail(RT_EINVAL, "NULL buffer");
    if (world < 1 || tile_rows < 1 || rows_per_rank < 0 || W < 1 || H < 1 || rows_per_rank % tile_rows ||
        rank_stride < 0)
        return fail(RT_EINVAL, "bad assemble geometry");
    if (rank_stride == 0) rank_stride = (long long)rows_per_rank * W;
    if (rank_stride < (long long)rows_per_rank * W) return fail(RT_EINVAL, "rank_stride overlaps rank blocks");
    const long long tiles = (H + tile_rows - 1) / tile_rows;
    if ((long long)world * (rows_per_rank / tile_rows) < tiles)
        return fail(RT_EINVAL, "gather holds %d tiles/rank x %d ranks < %lld tiles", rows_per_rank / tile_rows,
                    world, tiles);
    const int e = launch_assemble((const double*)gathered, rank_stride, world, tile_rows, rows_per_rank, W, H,
                                  (double*)out, hip_stream);
    if (e) return fail(RT_EDEVICE, "assemble launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

// ---- device-resident multi-device frame ----------------------
// main_cuda.cu:280-339 renders on one device and copies the three planes to
// the host.  Several devices of one node: each renders its cyclic row tiles,
// and the tiles travel device to device over xGMI (peer copies on the
// destination's copy engines: a gather into one device is G-1 point-to-point
// transfers, which is all ncclGather, rccl.h:745, would issue for it inside one
// process), then the assemble kernel un-permutes them into row order.
namespace {

// Peer access of dst to src, enabled once per pair.  Status: 1 = enabled
// (the copy engines read src over xGMI), 0 = not available, refused
// (e.g. hipErrorPeerAccessUnsupported) or switched off with the environment
// variable RT_PEER_ACCESS=0; hipMemcpyPeerAsync then stages the copy through
// the host itself, so the gather still works, only slower.
std::mutex g_peer_mu;
std::vector<std::array<int, 3>> g_peer;      // (dst, src, status)

int enable_peer(int dst, int src)
{
    if (dst == src) return 1;
    std::lock_guard<std::mutex> lk(g_peer_mu);
    for (auto& d : g_peer)
        if (d[0] == dst && d[1] == src) return d[2];
    int status = 0;
    const char* env = std::getenv("RT_PEER_ACCESS");
    int can = 0;
    if (!(env && env[0] == '0') && hipDeviceCanAccessPeer(&can, dst, src) == hipSuccess && can) {
        DeviceGuard g(dst);
        const hipError_t e = hipDeviceEnablePeerAccess(src, 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) status = 1;
        (void)hipGetLastError();     // a refusal must not poison the next call's error check
    }
    g_peer.push_back({dst, src, status});
    return status;
}

// One plane: slot r's rows_per_rank*W colours (device src_dev[r]) into the
// rank-major staging block r on dst_dev, then assemble into out (W*H).
int gather_plane(int world, const int* src_dev, const rt_color* const* locals, int tile_rows, int rows_per_rank,
                 int W, int H, int dst_dev, rt_color* staging, rt_color* out, hipStream_t st)
{
    const size_t n = (size_t)rows_per_rank * W;
    for (int r = 0; r < world; ++r) {
        if (!locals[r]) return fail(RT_EINVAL, "locals[%d] is NULL", r);
        enable_peer(dst_dev, src_dev[r]);
        const hipError_t e = hipMemcpyPeerAsync(staging + (size_t)r * n, dst_dev, locals[r], src_dev[r],
                                                n * sizeof(rt_color), st);
        if (e != hipSuccess) return fail(RT_EDEVICE, "peer copy %d -> %d: %s", src_dev[r], dst_dev, hipGetErrorString(e));
    }
    const int e = launch_assemble((const double*)staging, (long long)n, world, tile_rows, rows_per_rank, W, H,
                                  (double*)out, st);
    if (e) return fail(RT_EDEVICE, "assemble launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int check_gather_geometry(int world, int tile_rows, int rows_per_rank, int W, int H)
{
    if (world < 1 || tile_rows < 1 || rows_per_rank < 0 || W < 1 || H < 1 || rows_per_rank % tile_rows)
        return fail(RT_EINVAL, "bad gather geometry");
    const long long tiles = (H + tile_rows - 1) / tile_rows;
    if ((long long)world * (rows_per_rank / tile_rows) < tiles)
        return fail(RT_EINVAL, "%d ranks x %d tiles < %lld tiles", world, rows_per_rank / tile_rows, tiles);
    return RT_OK;
}

}  // namespace

int rt_peer_access(int dst_device, int src_device)
{
    const int n = rt_device_count();
    if (dst_device < 0 || dst_device >= n || src_device < 0 || src_device >= n)
        return fail(RT_EINVAL, "peer pair %d <- %d: %d visible device%s", dst_device, src_device, n, n == 1 ? "" : "s");
    return enable_peer(dst_device, src_device);
}

int rt_gather_async(int world, const int* src_devices, const rt_color* const* locals, int tile_rows,
                    int rows_per_rank, int W, int H, int dst_device, rt_color* out, void* hip_stream)
{
    int rc;
    if (!src_devices || !locals || !out) return fail(RT_EINVAL, "NULL argument");
    if ((rc = check_gather_geometry(world, tile_rows, rows_per_rank, W, H))) return rc;
    DeviceGuard g(dst_device);
    hipStream_t st = (hipStream_t)hip_stream;
    rt_color* staging = nullptr;
    HIP_TRY(hipMallocAsync((void**)&staging, (size_t)world * rows_per_rank * W * sizeof(rt_color), st));
    rc = gather_plane(world, src_devices, locals, tile_rows, rows_per_rank, W, H, dst_device, staging, out, st);
    (void)hipFreeAsync(staging, st);
    return rc;
}

namespace {
thread_local std::string g_gather_transport = "none";
}

const char* rt_last_gather_transport(void) { return g_gather_transport.c_str(); }

int rt_render_gather_async(const rt_scene* scene, const rt_params* params, int tile_rows, const rt_frame* frame,
                           void* hip_stream)
{
    int rc;
    if ((rc = validate_scene(scene)) || (rc = validate_params(params))) return rc;
    if (!frame || !frame->canva) return fail(RT_EINVAL, "frame.canva is NULL");
    if (tile_rows < 1) return fail(RT_EINVAL, "tile_rows %d < 1", tile_rows);
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if ((rc = ensure_init_locked())) return rc;
        devs = g_devices;
    }
    const int G = (int)devs.size(), W = params->largeur_image, H = params->hauteur_image;
    // RT_GATHER_RCCL: one rank per device, so the list must not repeat one; the
    // communicators are made (once per list) before anything is enqueued
    const bool rccl = params->gather == RT_GATHER_RCCL;
    if (rccl) {
        for (int a = 0; a < G; ++a)
            for (int b = a + 1; b < G; ++b)
                if (devs[(size_t)a] == devs[(size_t)b])
                    return fail(RT_EUNSUPPORTED, "RT_GATHER_RCCL needs distinct devices (rt_init's list names device %d "
                                                 "twice; RCCL has one rank per GPU): use RT_GATHER_PEER", devs[(size_t)a]);
        std::string err;
        if (rccl_comms(devs, err)) return fail(RT_EDEVICE, "RCCL: %s", err.c_str());
    }
    const int dst = devs[0];
    const int n_tiles = (((H + tile_rows - 1) / tile_rows) + G - 1) / G;      // per slot (rows >= H skipped)
    const int rows_pr = n_tiles * tile_rows;
    rt_color* outs[4] = {frame->canva, frame->albedo, frame->normal, frame->radiance};
    int nplanes = 0;
    for (rt_color* o : outs) nplanes += o ? 1 : 0;
    const size_t plane = (size_t)rows_pr * W;                            // colours per plane and slot
    hipStream_t dst_st = (hipStream_t)hip_stream;

    struct Slot {
        std::shared_ptr<rt_device_scene> sc;
        PooledStream* ps = nullptr;
        rt_color* buf = nullptr;
        hipEvent_t ev = nullptr;
    };
    std::vector<Slot> slots((size_t)G);
    auto release = [&]() {           // stream-ordered: nothing here waits for the GPU
        for (auto& s : slots) {
            if (!s.ps) continue;
            DeviceGuard g(s.ps->device);
            if (s.buf) (void)hipFreeAsync(s.buf, s.ps->st);
            if (s.ev) (void)hipEventDestroy(s.ev);
            stream_pool_put(s.ps);
            s.ps = nullptr;
        }
    };
    // 1. every slot renders its tiles on its own device and pooled stream,
    //    after whatever the caller enqueued on hip_stream before this call
    hipEvent_t go = nullptr;
    {
        DeviceGuard g(dst);
        HIP_TRY(hipEventCreateWithFlags(&go, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(go, dst_st));
    }
    for (int q = 0; q < G && rc == RT_OK; ++q) {
        Slot& s = slots[(size_t)q];
        if ((rc = scene_cache_get(devs[(size_t)q], scene, s.sc)) || (rc = stream_pool_get(devs[(size_t)q], &s.ps))) break;
        DeviceGuard g(devs[(size_t)q]);
        hipError_t e = hipStreamWaitEvent(s.ps->st, go, 0);
        if (e == hipSuccess) e = hipMallocAsync((void**)&s.buf, plane * nplanes * sizeof(rt_color), s.ps->st);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            rc = fail(RT_EDEVICE, "device %d frame: %s", devs[(size_t)q], hipGetErrorString(e));
            break;
        }
        rt_tiling t{0, tile_rows, q, G, n_tiles};
        KParams kp;
        double uni[U_COUNT];
        make_kparams(s.sc.get(), params, &t, kp, uni);
        rt_color* nxt = s.buf;
        double** dstp[4] = {&kp.canva, &kp.albedo, &kp.normal, &kp.radiance};
        for (int pl = 0; pl < 4; ++pl) {
            *dstp[pl] = outs[pl] ? (double*)nxt : nullptr;
            if (outs[pl]) nxt += plane;
        }
        if ((rc = launch_on_stream(kp, uni, s.ps->st, false))) break;
        if ((e = hipEventRecord(s.ev, s.ps->st)) != hipSuccess)
            rc = fail(RT_EDEVICE, "device %d event: %s", devs[(size_t)q], hipGetErrorString(e));
    }
    // 2. the destination's stream waits for every slot, gathers each plane over
    //    xGMI and un-permutes it; 3. each slot frees its planes after the copies
    if (rc == RT_OK) {
        DeviceGuard g(dst);
        for (int q = 0; q < G && rc == RT_OK; ++q) {
            const hipError_t e = hipStreamWaitEvent(dst_st, slots[(size_t)q].ev, 0);
            if (e != hipSuccess) rc = fail(RT_EDEVICE, "wait: %s", hipGetErrorString(e));
        }
        rt_color* staging = nullptr;
        const size_t per_slot = rccl ? plane * nplanes : plane;             // colours staged per slot
        if (rc == RT_OK) {
            const hipError_t e = hipMallocAsync((void**)&staging, (size_t)G * per_slot * sizeof(rt_color), dst_st);
            if (e != hipSuccess) rc = fail(RT_ENOMEM, "gather staging: %s", hipGetErrorString(e));
        }
        if (rccl && rc == RT_OK) {
            // every slot's planes (contiguous in its buffer) in one ncclGather to
            // rank 0, rank 0's part on hip_stream (which waited for its render),
            // the others' on their own streams after their renders; then one
            // assemble per plane from the rank-major staging
            std::vector<const void*> send((size_t)G);
            std::vector<hipStream_t> sst((size_t)G);
            for (int q = 0; q < G; ++q) {
                send[(size_t)q] = slots[(size_t)q].buf;
                sst[(size_t)q] = q == 0 ? dst_st : slots[(size_t)q].ps->st;
            }
            std::string err;
            if (rccl_gather(devs, send, staging, per_slot * 3, sst, err)) rc = fail(RT_EDEVICE, "RCCL: %s", err.c_str());
            for (int k = 0; k < nplanes && rc == RT_OK; ++k) {
                int pl = -1;
                for (int j = 0, m = 0; j < 4; ++j)
                    if (outs[j] && m++ == k) pl = j;
                const int e = launch_assemble((const double*)(staging + (size_t)k * plane), (long long)per_slot, G,
                                              tile_rows, rows_pr, W, H, (double*)outs[pl], dst_st);
                if (e) rc = fail(RT_EDEVICE, "assemble launch: %s", hipGetErrorString((hipError_t)e));
            }
            if (rc == RT_OK)
                g_gather_transport = "rccl: ncclGather, " + rccl_describe() + ", " + std::to_string(G) + " ranks";
        } else {
            int k = 0;
            for (int pl = 0; pl < 4 && rc == RT_OK; ++pl) {
                if (!outs[pl]) continue;
                std::vector<const rt_color*> loc((size_t)G);
                for (int q = 0; q < G; ++q) loc[(size_t)q] = slots[(size_t)q].buf + (size_t)k * plane;
                rc = gather_plane(G, devs.data(), loc.data(), tile_rows, rows_pr, W, H, dst, staging, outs[pl], dst_st);
                ++k;
            }
            if (rc == RT_OK) g_gather_transport = "peer: hipMemcpyPeerAsync, " + std::to_string(G) + " slots";
        }
        if (staging) (void)hipFreeAsync(staging, dst_st);
        if (rc == RT_OK) {
            // the slots free their planes only after the copies that read them
            hipError_t e = hipEventRecord(go, dst_st);            // reused: "the copies are done"
            if (e != hipSuccess) rc = fail(RT_EDEVICE, "gather event: %s", hipGetErrorString(e));
            for (int q = 0; q < G && rc == RT_OK; ++q) {
                DeviceGuard gq(devs[(size_t)q]);
                if ((e = hipStreamWaitEvent(slots[(size_t)q].ps->st, go, 0)) != hipSuccess)
                    rc = fail(RT_EDEVICE, "device %d wait: %s", devs[(size_t)q], hipGetErrorString(e));
            }
        }
    }
    if (rc != RT_OK) {
        // Keep the error message.  Copies already queued on the destination's
        // stream may still read slot planes, and the slots may still render
        // into them: drain both before release() hands the memory back.
        {
            DeviceGuard g(dst);
            (void)hipStreamSynchronize(dst_st);
        }
        for (auto& s : slots)
            if (s.ps) {
                DeviceGuard gq(s.ps->device);
                (void)hipStreamSynchronize(s.ps->st);
            }
    }
    release();
    {
        DeviceGuard g(dst);
        (void)hipEventDestroy(go);
    }
    return rc;
}

int rt_render_rows(const rt_scene* scene, const rt_params* params, int row_hi, int row_lo, rt_color* canva,
                   rt_color* albedo, rt_color* normal)
{
    int rc;
    if ((rc = validate_scene(scene)) || (rc = validate_params(params))) return rc;
    if (!canva) return fail(RT_EINVAL, "canva is NULL");
    if (row_lo < 0 || row_hi >= params->hauteur_image || row_hi < row_lo)
        return fail(RT_EINVAL, "rows %d..%d outside [0, %d)", row_hi, row_lo, params->hauteur_image);
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if ((rc = ensure_init_locked())) return rc;
        devs = g_devices;
    }
    const int W = params->largeur_image;
    const int nrows = row_hi - row_lo + 1;
    const int ndev = (int)devs.size();
    struct InFlight {
        InFlight() { ++g_calls_in_flight; }
        ~InFlight() { --g_calls_in_flight; }
    } in_flight;
    // One device: one band.  Several: cyclic 1-row tiles (load balance: the
    // busiest device renders at most one row more than the average).
    const int k = ndev == 1 ? nrows : 1;
    const int ntiles = (nrows + k - 1) / k;
    rt_color* outs[3] = {canva, albedo, normal};
    const int nplanes = 3;

    struct Slot {
        std::shared_ptr<rt_device_scene> sc;
        PooledStream* ps = nullptr;
        double* buf = nullptr;      // device planes canva | albedo | normal (only the requested ones)
        int n_tiles = 0;
        size_t plane = 0;           // doubles per plane
    };
    std::vector<Slot> slots((size_t)ndev);
    auto cleanup = [&]() {
        for (auto& s : slots) {
            if (!s.ps) continue;
            DeviceGuard g(s.ps->device);
            if (s.buf) (void)hipFreeAsync(s.buf, s.ps->st);
            (void)hipStreamSynchronize(s.ps->st);
            stream_pool_put(s.ps);
            s.ps = nullptr;
        }
    };
    // 1. every device: cached scene, pooled stream, stream-ordered planes, launch
    for (int q = 0; q < ndev; ++q) {
        Slot& s = slots[(size_t)q];
        s.n_tiles = ntiles > q ? (ntiles - q + ndev - 1) / ndev : 0;
        if (s.n_tiles == 0) continue;
        if ((rc = scene_cache_get(devs[(size_t)q], scene, s.sc))) {
            cleanup();
            return rc;
        }
        if ((rc = stream_pool_get(devs[(size_t)q], &s.ps))) {
            cleanup();
            return rc;
        }
        DeviceGuard g(devs[(size_t)q]);
        s.plane = (size_t)s.n_tiles * k * W * 3;
        size_t nbuf = 0;
        for (int pl = 0; pl < nplanes; ++pl) nbuf += outs[pl] ? s.plane : 0;
        hipError_t e = hipMallocAsync((void**)&s.buf, nbuf * sizeof(double), s.ps->st);
        if (e != hipSuccess) {
            cleanup();
            return fail(RT_EDEVICE, "device %d frame: %s", devs[(size_t)q], hipGetErrorString(e));
        }
        rt_tiling t{row_lo, k, q, ndev, s.n_tiles};
        KParams kp;
        double uni[U_COUNT];
        make_kparams(s.sc.get(), params, &t, kp, uni);
        kp.row_end = row_hi + 1;
        double* nxt = s.buf;
        double** dst[3] = {&kp.canva, &kp.albedo, &kp.normal};
        for (int pl = 0; pl < nplanes; ++pl) {
            *dst[pl] = outs[pl] ? nxt : nullptr;
            if (outs[pl]) nxt += s.plane;
        }
        if ((rc = launch_on_stream(kp, uni, s.ps->st, false))) {
            cleanup();
            return rc;
        }
    }
    // 2. every device: D2H of the requested planes into its stream's pinned
    //    staging buffer, one copy and event per plane, all enqueued before
    //    any wait (the devices' copies overlap)
    for (int q = 0; q < ndev; ++q) {
        Slot& s = slots[(size_t)q];
        if (s.n_tiles == 0) continue;
        DeviceGuard g(devs[(size_t)q]);
        size_t nbuf = 0;
        for (int pl = 0; pl < nplanes; ++pl) nbuf += outs[pl] ? s.plane : 0;
        hipError_t e = s.ps->reserve_host(nbuf * sizeof(double));
        size_t off = 0;
        for (int pl = 0; pl < nplanes && e == hipSuccess; ++pl) {
            if (!outs[pl]) continue;
            e = hipMemcpyAsync((double*)s.ps->host + off, s.buf + off, s.plane * sizeof(double), hipMemcpyDeviceToHost,
                               s.ps->st);
            if (e == hipSuccess) e = hipEventRecord(s.ps->plane_done[pl], s.ps->st);
            off += s.plane;
        }
        if (e != hipSuccess) {
            cleanup();
            return fail(RT_EDEVICE, "device %d copy: %s", devs[(size_t)q], hipGetErrorString(e));
        }
    }
    // 3. each device and plane as its copy lands: scatter its rows into the
    //    caller's array on several host threads (the next plane is still in
    //    flight meanwhile)
    // (concurrent calls, e.g. rt_fill_canva's pthreads, share the threads)
    const int nthr = std::max(1, std::min(8, (int)std::thread::hardware_concurrency() / 2) / g_calls_in_flight.load());
    for (int q = 0; q < ndev; ++q) {
        Slot& s = slots[(size_t)q];
        if (s.n_tiles == 0) continue;
        DeviceGuard g(devs[(size_t)q]);
        const double* src0 = (const double*)s.ps->host;
        for (int pl = 0; pl < nplanes; ++pl) {
            if (!outs[pl]) continue;
            const hipError_t e = hipEventSynchronize(s.ps->plane_done[pl]);
            if (e != hipSuccess) {
                cleanup();
                return fail(RT_EDEVICE, "device %d render/copy: %s", devs[(size_t)q], hipGetErrorString(e));
            }
            // tile lt of this device = caller rows row_lo + (q + lt * ndev) * k + [0, k)
            auto scatter = [&, src0, pl](int lt0, int lt1) {
                for (int lt = lt0; lt < lt1; ++lt) {
                    const int gr0 = row_lo + (q + lt * ndev) * k;
                    const int nr = std::min(k, row_hi + 1 - gr0);
                    if (nr > 0)
                        std::memcpy(outs[pl] + (size_t)gr0 * W, src0 + (size_t)lt * k * W * 3,
                                    sizeof(double) * 3 * (size_t)W * nr);
                }
            };
            if (ndev == 1) {       // one band: split its rows instead of its single tile
                const double* src = src0;
                auto rows = [&, src, pl](int r0, int r1) {
                    if (r1 > r0)
                        std::memcpy(outs[pl] + (size_t)(row_lo + r0) * W, src + (size_t)r0 * W * 3,
                                    sizeof(double) * 3 * (size_t)W * (r1 - r0));
                };
                par_ranges(nrows, nrows * (size_t)W * 24 >= (4u << 20) ? nthr : 1, rows);
            } else {
                par_ranges(s.n_tiles, (size_t)s.n_tiles * k * W * 24 >= (4u << 20) ? nthr : 1, scatter);
            }
            src0 += s.plane;
        }
    }
    cleanup();
    // main.c:455: denoiser() on the finished frame
    const rt_denoise_fn hook = g_denoise.load();
    if (hook && row_hi == params->hauteur_image - 1 && row_lo == 0 && albedo && normal)
        hook(W, params->hauteur_image, canva, params->cam, albedo, normal);
    return RT_OK;
}

void rt_set_denoise_hook(rt_denoise_fn fn) { g_denoise.store(fn); }
int rt_set_zero_throughput_exit(int enable) { return g_zero_exit.exchange(enable ? 1 : 0); }
int rt_set_fill_spp_chunks(int spp_chunks)
{
    if (spp_chunks < RT_SPP_CHUNKS_AUTO) spp_chunks = 1;
    return g_fill_chunks.exchange(spp_chunks);
}
int rt_set_fill_precision(int precision)
{
    // RT_PREC_FP32 was removed (r05): rt_fill_canva renders FP64 only
    if (precision == RT_PREC_FP32)
        return fail(RT_EUNSUPPORTED, "RT_PREC_FP32 was removed (r05); rt_fill_canva renders FP64");
    if (precision != RT_PREC_FP64) return fail(RT_EINVAL, "unknown precision %d", precision);
    return g_fill_prec.exchange(RT_PREC_FP64);
}
int rt_scene_cache_clear(void) { return scene_cache_clear(); }
rt_denoise_fn rt_get_denoise_hook(void) { return g_denoise.load(); }

int rt_denoise_pack(int W, int H, const rt_color* canva, const rt_color* albedo, const rt_color* normal,
                    float* color3, float* albedo3, float* normal3)
{
    if (W < 1 || H < 1 || !canva || !color3) return fail(RT_EINVAL, "bad denoise_pack arguments");
    const size_t n = (size_t)W * H;
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) {
            color3[3 * i + c] = (float)canva[i].e[c] / 255.0f;          // denoiser.h:44-48
            if (albedo && albedo3) albedo3[3 * i + c] = (float)albedo[i].e[c];
            if (normal && normal3) normal3[3 * i + c] = (float)normal[i].e[c];
        }
    return RT_OK;
}

int rt_denoise_unpack(int W, int H, const float* color3, rt_color* canva)
{
    if (W < 1 || H < 1 || !canva || !color3) return fail(RT_EINVAL, "bad denoise_unpack arguments");
    const size_t n = (size_t)W * H;
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) canva[i].e[c] = (int)(color3[3 * i + c] * 255.0f);   // denoiser.h:80-84
    return RT_OK;
}

int rt_denoise_pack_async(int W, int H, const rt_frame* frame, float* color3, float* albedo3, float* normal3,
                          void* hip_stream)
{
    if (W < 1 || H < 1 || !frame || !frame->canva || !color3)
        return fail(RT_EINVAL, "bad denoise_pack_async arguments");
    const int e = launch_denoise_pack((long long)W * H, (const double*)frame->canva,
                                      albedo3 ? (const double*)frame->albedo : nullptr,
                                      normal3 ? (const double*)frame->normal : nullptr, color3, albedo3, normal3,
                                      hip_stream);
    if (e) return fail(RT_EDEVICE, "denoise pack launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

void* rt_fill_canva(void* arg)
{
    const rt_thread_data* d = (const rt_thread_data*)arg;
    if (!d) {
        fail(RT_EINVAL, "thread data is NULL");
        return (void*)1;
    }
    int nmat = 0;
    for (int i = 0; i < d->nbTriangles; ++i)
        if (d->quelMatPourTri && d->quelMatPourTri[i] + 1 > nmat) nmat = d->quelMatPourTri[i] + 1;
    rt_scene sc;
    std::memset(&sc, 0, sizeof sc);
    sc.sphere_list = d->sphere_list;
    sc.nbSpheres = d->nbSpheres;
    sc.triangle_list = d->triangle_list;
    sc.nbTriangles = d->nbTriangles;
    sc.mat_list = d->mat_list;
    sc.tex_width = d->tex_width;
    sc.tex_height = d->tex_height;
    sc.nbMaterials = nmat;
    sc.quelMatPourTri = d->quelMatPourTri;
    sc.sky_mat_list = d->sky_mat_list;        // carried like ThreadData does; sky_mode stays OFF (main.c)
    sc.sky_width = d->sky_width;
    sc.sky_height = d->sky_height;
    rt_params p;
    rt_params_init(&p);
    p.largeur_image = d->largeur_image;
    p.hauteur_image = d->hauteur_image;
    p.nbRayonParPixel = d->nbRayonParPixel;
    p.nbRebondMax = d->nbRebondMax;
    p.cam = d->cam;
    p.focus_distance = d->focus_distance;     // already int in ThreadData
    p.ouverture_x = d->ouverture_x;
    p.ouverture_y = d->ouverture_y;
    p.AO_intensity = d->AO_intensity;
    p.useAO = d->useAO ? 1 : 0;
    p.compat_int_truncation = 0;
    p.spp_chunks = g_fill_chunks.load();
    p.precision = g_fill_prec.load();
    const int rc = rt_render_rows(&sc, &p, d->start_row, d->end_row, d->canva, d->albedo_tab, d->normal_tab);
    return rc == RT_OK ? nullptr : (void*)1;
}

int rt_selftest_math(int op, const double* in, double* out, int n)
{
    if (!in || !out || n < 0 || op < 0 || op > 9) return fail(RT_EINVAL, "bad selftest arguments");
    if (n == 0) return RT_OK;
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = ensure_init_locked();
        if (rc) return rc;
        dev = g_devices[0];
    }
    DeviceGuard guard(dev);
    const size_t nin = (size_t)n * (op == 7 ? 6 : op == 8 ? 3 : (op == 3 || op == 5 || op == 9) ? 2 : 1);
    const size_t nout = (size_t)n * (op == 7 ? 4 : op == 8 ? 3 : 1);
    double *d_in = nullptr, *d_out = nullptr;
    HIP_TRY(hipMalloc((void**)&d_in, nin * sizeof(double)));
    hipError_t e = hipMalloc((void**)&d_out, nout * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(d_in, in, nin * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = (hipError_t)launch_selftest(op, d_in, d_out, n, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d_out, nout * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(RT_EDEVICE, "selftest: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_verify_sphere_pass(const rt_scene* scene, const double* rays, long long n, unsigned long long counts[2])
{
    if (!counts || !rays || n < 0) return fail(RT_EINVAL, "bad verify arguments");
    counts[0] = counts[1] = 0;
    if (n == 0) return RT_OK;
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = ensure_init_locked();
        if (rc) return rc;
        dev = g_devices[0];
    }
    rt_device_scene* ds = nullptr;
    int rc = rt_scene_upload(dev, scene, &ds);
    if (rc) return rc;
    DeviceGuard guard(dev);
    KParams kp;
    std::memset(&kp, 0, sizeof kp);
    kp.sph = ds->sph;
    kp.sph_cand = ds->sph_cand;
    kp.cand_lmax = ds->cand_lmax;
    kp.ns = ds->ns;
    kp.ns_pad = ds->ns_pad;
    kp.ns_cand = std::isfinite(ds->cand_lmax) ? ds->ns_pad : 0;
    double* d_rays = nullptr;
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc((void**)&d_rays, (size_t)n * 6 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&d, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, (size_t)n * 6 * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = (hipError_t)launch_verify_spheres(kp, d_rays, n, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(counts, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    (void)hipFree(d);
    rt_scene_release(ds);
    if (e != hipSuccess) return fail(RT_EDEVICE, "verify_sphere_pass: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_verify_texel_map(const rt_scene* scene, const double* pts, const int* tri, long long n,
                        unsigned long long counts[2])
{
    if (!counts || !pts || !tri || n < 0 || !scene) return fail(RT_EINVAL, "bad verify arguments");
    counts[0] = counts[1] = 0;
    if (scene->nbTriangles < 1 || scene->nbTriangles > 32)
        return fail(RT_EUNSUPPORTED, "verify_texel_map: 1-32 triangles (caller order), got %d", scene->nbTriangles);
    for (long long i = 0; i < n; ++i)
        if (tri[i] < 0 || tri[i] >= scene->nbTriangles) return fail(RT_EINVAL, "tri[%lld] = %d", i, tri[i]);
    if (n == 0) return RT_OK;
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = ensure_init_locked();
        if (rc) return rc;
        dev = g_devices[0];
    }
    rt_device_scene* ds = nullptr;
    int rc = rt_scene_upload(dev, scene, &ds);
    if (rc) return rc;
    if (!ds->tri_uv) {
        rt_scene_release(ds);
        return fail(RT_EUNSUPPORTED, "verify_texel_map: the scene has no affine texel map (every uv 0)");
    }
    DeviceGuard guard(dev);
    KParams kp;
    std::memset(&kp, 0, sizeof kp);
    kp.tri = ds->tri;
    kp.tri_tex = ds->tri_tex;
    kp.tri_uv = ds->tri_uv;
    kp.tw = ds->tw;
    kp.th = ds->th;
    kp.n_texels = ds->n_texels;
    double* d_pts = nullptr;
    int* d_tri = nullptr;
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc((void**)&d_pts, (size_t)n * 3 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&d_tri, (size_t)n * sizeof(int));
    if (e == hipSuccess) e = hipMalloc((void**)&d, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemcpy(d_pts, pts, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_tri, tri, (size_t)n * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = (hipError_t)launch_verify_texel(kp, d_pts, d_tri, n, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(counts, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d_pts);
    (void)hipFree(d_tri);
    (void)hipFree(d);
    rt_scene_release(ds);
    if (e != hipSuccess) return fail(RT_EDEVICE, "verify_texel_map: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_verify_sampler_phi(unsigned long long r0, unsigned long long n, unsigned long long counts[2])
{
    if (!counts || r0 > (1ull << 31) || n > (1ull << 31) - r0) return fail(RT_EINVAL, "bad verify range");
    counts[0] = counts[1] = 0;
    if (n == 0) return RT_OK;
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = ensure_init_locked();
        if (rc) return rc;
        dev = g_devices[0];
    }
    DeviceGuard guard(dev);
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 2 * sizeof(unsigned long long)));
    hipError_t e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = (hipError_t)launch_verify_phi(r0, n, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(counts, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_EDEVICE, "verify_sampler_phi: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_verify_normalize(unsigned long long seed, unsigned long long n, unsigned long long counts[2])
{
    if (!counts) return fail(RT_EINVAL, "verify_normalize: counts is NULL");
    counts[0] = counts[1] = 0;
    if (n == 0) return RT_OK;
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = ensure_init_locked();
        if (rc) return rc;
        dev = g_devices[0];
    }
    DeviceGuard guard(dev);
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 2 * sizeof(unsigned long long)));
    hipError_t e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = (hipError_t)launch_verify_normalize(seed, n, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(counts, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_EDEVICE, "verify_normalize: %s", hipGetErrorString(e));
    return RT_OK;
}

}  // extern "C"
