// rt_kernels.hip — the per-pixel path-tracing kernel for gfx950 (CDNA4).
//
// One thread renders one pixel: the nbRayonParPixel sample loop, the
// nbRebondMax bounce loop, closest-hit scans, shading and AO all run in
// registers; the only HBM traffic is the final 3-4 colors per pixel.
//
// Semantics follow main.c (the authoritative CPU path), not main_cuda.cu:
//   fill_canva        main.c:245-284      -> render_kernel
//   tracer            main.c:118-242      -> trace()
//   closest_hit       main.c:52-92        -> closest_hit()
//   ambient_occlusion main.c:94-116       -> ao_factor()
//   hit_sphere        sphere.h:13-47, hit_triangle mesh.h:70-94,
//   tri_uvmapping     texture.h:44-90, get_ray camera.h:42-55,
//   random_dir_no_norm / refracted_vec / hsl  rtutility.h:81-231,
//   write_color_canva rtutility.h:56-71
// Every floating-point operation is the reference's, in its association
// order, one IEEE rounding each (built with -ffp-contract=off): results are
// bit-identical to the CPU restatement in RT_RNG_PHILOX mode.
//
// MI355X mapping (DESIGN.md "Kernel"):
//  * geometry is scanned in the same order by every lane of a wave, so the
//    sphere/triangle records are read through constant-address-space
//    pointers -> scalar (SMEM) loads into SGPRs, broadcast to 64 lanes for
//    free; nothing is staged per lane;
//  * per-lane divergent data (the winner's material, texels) is fetched once
//    per bounce from L1/L2;
//  * the IOR stack of pile.h reduces to one register (top n2), see trace();
//  * 256-thread blocks = four 8x8-pixel waves (ray coherence), 16x16 tiles.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "rt/rt.h"
#include "rt_internal.h"
#include "rt_device_math.h"

namespace rt {

#define RT_CONST __attribute__((address_space(4)))

struct V3 {
    double x, y, z;
};
__device__ __forceinline__ V3 v3(double a, double b, double c) { return V3{a, b, c}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 muls(V3 a, double t) { return v3(a.x * t, a.y * t, a.z * t); }
__device__ __forceinline__ V3 divs(V3 a, double t) { return v3(a.x / t, a.y / t, a.z / t); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 u, V3 v)
{
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
__device__ __forceinline__ V3 normalize(V3 a) { return divs(a, sqrt(dot(a, a))); }   // vec3.h:137-139

struct Mat {
    V3 diff, emis;
    double es, rs, alpha, ior;
};
__device__ __forceinline__ Mat load_mat(const DevMat* m)
{
    const DevMat r = *m;
    return Mat{v3(r.dr, r.dg, r.db), v3(r.er, r.eg, r.eb), r.es, r.rs, r.alpha, r.ior};
}

// Per-thread event counters (COUNT instantiation only).
struct Cnt {
    unsigned long long c[RT_NCOUNTERS];
};

enum : int { HIT_NONE = 0, HIT_SPHERE = 1, HIT_TRI = 2 };

// closest_hit, main.c:52-92: linear scan, spheres then triangles; a strictly
// closer hit replaces the record.  Returns the winner (kind, index, t).
template <bool COUNT>
__device__ __forceinline__ int closest_hit(const KParams& kp, const V3 o, const V3 d, double& t_best, int& idx,
                                           Cnt& cnt)
{
    const SphGeo* __restrict__ sph = kp.sph;
    const TriGeo* __restrict__ tri = kp.tri;
    const double a = dot(d, d);          // sphere.h:20 (same for every sphere)
    const double two_a = 2 * a;          // sphere.h:27,36
    const double four_a = 4 * a;         // sphere.h:24 `4*a*c` == (4*a)*c
    double best = __longlong_as_double(0x7ff0000000000000ll);   // INFINITY, main.c:56
    int kind = HIT_NONE, win = -1;
    if (COUNT) {
        cnt.c[RT_CNT_CASTS] += 1;
        cnt.c[RT_CNT_SPHERE_TESTS] += (unsigned long long)kp.ns;
        cnt.c[RT_CNT_TRI_TESTS] += (unsigned long long)kp.nt;
    }
    for (int k = 0; k < kp.ns; ++k) {                     // hit_sphere, sphere.h:13-47
        const SphGeo s = sph[k];
        const double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
        const double b = 2.0 * (ocx * d.x + ocy * d.y + ocz * d.z);
        const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - s.r2;
        const double disc = b * b - four_a * c;
        if (disc > 0) {
            if (COUNT) cnt.c[RT_CNT_SPHERE_DISC] += 1;
            const double sq = sqrt(disc);
            // t1 = (-b - sq)/(2a) is taken iff t1 >= 1e-4; a negative
            // numerator decides that without the division (2a > 0).
            const double n1 = -b - sq;
            double t = 0.0;
            bool hit = false;
            if (!(n1 < 0.0)) {
                t = n1 / two_a;
                hit = t >= 0.0001;
            }
            if (!hit) {
                const double n2 = -b + sq;
                if (!(n2 < 0.0)) {
                    t = n2 / two_a;
                    hit = t >= 0.0001;
                }
            }
            if (hit && t < best) {
                best = t;
                kind = HIT_SPHERE;
                win = k;
            }
        }
    }
    for (int k = 0; k < kp.nt; ++k) {                     // hit_triangle, mesh.h:70-94
        const TriGeo g = tri[k];
        const double det = -(d.x * g.nx + d.y * g.ny + d.z * g.nz);
        if (det >= 1E-6) {
            const V3 ao = v3(o.x - g.ax, o.y - g.ay, o.z - g.az);
            const V3 dao = cross(ao, d);
            const double invDet = 1 / det;
            const double dst = (ao.x * g.nx + ao.y * g.ny + ao.z * g.nz) * invDet;
            if (dst >= 0.0000001 && dst < best) {
                const double u = (g.acx * dao.x + g.acy * dao.y + g.acz * dao.z) * invDet;
                const double v = -(g.abx * dao.x + g.aby * dao.y + g.abz * dao.z) * invDet;
                const double w = 1 - u - v;
                if (u >= 0.0000001 && v >= 0.0000001 && w >= 0.0000001) {
                    best = dst;
                    kind = HIT_TRI;
                    win = k;
                }
            }
        }
    }
    t_best = best;
    idx = win;
    return kind;
}

// tri_uvmapping + get_barycentric_coord, texture.h:16-27,44-90.
__device__ __forceinline__ Mat tri_material(const KParams& kp, int k, const V3 P, const V3 n)
{
    const TriGeo g = kp.tri[k];
    const TriTex tx = kp.tri_tex[k];
    const V3 A = v3(g.ax, g.ay, g.az), B = v3(tx.bx, tx.by, tx.bz), C = v3(tx.cx, tx.cy, tx.cz);
    const double areaABC = dot(n, v3(g.nx, g.ny, g.nz));      // cross(B-A, C-A) == N
    const double areaPBC = dot(n, cross(B - P, C - P));
    const double areaPCA = dot(n, cross(C - P, A - P));
    const double b0 = areaPBC / areaABC;
    const double b1 = areaPCA / areaABC;
    const double b2 = 1.0 - b0 - b1;
    double u = (b0 * tx.uau + b1 * tx.ubu + b2 * tx.ucu);
    double v = (b0 * tx.uav + b1 * tx.ubv + b2 * tx.ucv);
    u = u - trunc(u);                 // fmod(u, 1.0): exact
    v = v - trunc(v);
    if (u < 0) u += 1.0;
    if (v < 0) v += 1.0;
    const int x = (int)(u * (double)(kp.tw));
    const int y = (int)(v * (double)(kp.th));
    const int m = tx.mat;
    long long index = ((long long)y * kp.tw + x) + ((long long)kp.th * kp.tw * m);
    index = index < 0 ? 0 : index;                       // reference UB -> clamp
    index = index >= kp.n_texels ? kp.n_texels - 1 : index;
    Mat res = load_mat(kp.texels + index);
    if (m == 1) {
        res.emis = v3(1, 1, 1);
        res.es = 1.85;
        res.alpha = 1.0;
    }
    if (m == 4) {
        res.alpha = 0.6;
        res.ior = 1.33;
        res.rs = 0.93;
    }
    if (m == 3) {
        res.alpha = 0.1;
        res.ior = 1.50;
        res.rs = 0.3;
    }
    return res;
}

// random_dir_no_norm, rtutility.h:189-203 (float sinf/cosf of double args)
template <bool COUNT>
__device__ __forceinline__ V3 random_dir(Stream& st, Cnt& cnt)
{
    if (COUNT) cnt.c[RT_CNT_SHADE] += 1;
    const double u = unit31(st.next31());
    const double v = unit31(st.next31());
    const double theta = 0x1.921fb54442d18p+2 * u;        // 2*PI*u
    const double phi = pm_acos(2 * v - 1);
    float st_, ct_, sp_, cp_;
    pm_sincosf((float)theta, st_, ct_);
    pm_sincosf((float)phi, sp_, cp_);
    const V3 dir = v3((double)(ct_ * sp_), (double)(st_ * sp_), (double)cp_);
    return normalize(dir);
}

// refracted_vec, rtutility.h:210-227 (indices squared: reference quirk)
__device__ __forceinline__ V3 refracted(V3 v, V3 nrm, double n1, double n2)
{
    n1 *= n1;
    n2 *= n2;
    const double cn = dot(nrm, v);
    const double radical = 1 - ((n1 / n2) * (n1 / n2)) * (1 - (cn * cn));
    if (radical > 0) {
        const V3 comp_tan = muls(v - muls(nrm, dot(v, nrm)), (n1 / n2));
        const V3 comp_normal = muls(v3(-nrm.x, -nrm.y, -nrm.z), sqrt(radical));
        return comp_tan + comp_normal;
    }
    return v - muls(nrm, 2 * dot(v, nrm));
}

// rgb_to_hsl / hsl_to_rgb round trip, rtutility.h:81-165 (main.c:155-158)
__device__ __forceinline__ double hue_to_rgb(double t1, double t2, double hue)
{
    if (hue < 0.0) hue += 1.0;
    if (hue > 1.0) hue -= 1.0;
    if (6.0 * hue < 1.0) return t1 + (t2 - t1) * 6.0 * hue;
    if (2.0 * hue < 1.0) return t2;
    if (3.0 * hue < 2.0) return t1 + (t2 - t1) * ((2.0 / 3.0) - hue) * 6.0;
    return t1;
}
__device__ __forceinline__ V3 hsl_roundtrip(V3 rgb)
{
    const double r = rgb.x, g = rgb.y, b = rgb.z;
    const double mx = (r > g) ? ((r > b) ? r : b) : ((g > b) ? g : b);
    const double mn = (r < g) ? ((r < b) ? r : b) : ((g < b) ? g : b);
    double h = 0.0, s, l = (mx + mn) / 2.0;
    if (mx == mn) {
        h = 0.0;
        s = 0.0;
    } else {
        const double d = mx - mn;
        s = (l < 0.5) ? (d / (mx + mn)) : (d / (2.0 - mx - mn));
        if (mx == r) h = (g - b) / d + ((g < b) ? 6.0 : 0.0);
        else if (mx == g) h = (b - r) / d + 2.0;
        else if (mx == b) h = (r - g) / d + 4.0;
        h /= 6.0;
    }
    l *= 1.0;
    s *= 1.0;
    if (s == 0.0) return v3(l, l, l);
    const double t2 = (l < 0.5) ? (l * (1.0 + s)) : (l + s - l * s);
    const double t1 = 2.0 * l - t2;
    return v3(hue_to_rgb(t1, t2, h + 1.0 / 3.0), hue_to_rgb(t1, t2, h), hue_to_rgb(t1, t2, h - 1.0 / 3.0));
}

// ambient_occlusion, main.c:94-116: one cast, only distance/dst matters.
template <bool COUNT>
__device__ __forceinline__ double ao_factor(const KParams& kp, const V3 p, const V3 n, Stream& st, Cnt& cnt)
{
    const V3 rd = random_dir<COUNT>(st, cnt);
    const V3 dir = normalize(n + rd);
    double t;
    int idx;
    const int kind = closest_hit<COUNT>(kp, p, dir, t, idx, cnt);
    double occ = 0.0;
    if (kind != HIT_NONE) {
        const V3 hp = p + muls(dir, t);
        const V3 df = hp - p;
        const double distance = sqrt(dot(df, df));
        double att = distance / t;
        att = pm_pow(att, kp.AO);
        occ = occ + att;
    }
    return (occ / 1.0) / kp.AO;
}

// tracer, main.c:118-242.  The IOR stack (pile.h) is reduced to `top_n2`:
// every translucent hit pushes (top.n2, m) (index_suivant_pile) and, when
// exiting, pops that same pair again, so the stack only ever changes on
// entry and only its top n2 is ever read (DESIGN.md "IOR stack").
template <bool COUNT>
__device__ __forceinline__ void trace(const KParams& kp, V3 o, V3 d, Stream& st, V3& out_rad, V3& out_alb,
                                      V3& out_nrm, Cnt& cnt)
{
    V3 inc = v3(0, 0, 0), rc = v3(1, 1, 1), alb = v3(0, 0, 0), nrm = v3(0, 0, 0);
    bool is_alpha = false;
    int alpha_depth = 0;
    double top_n2 = 1.0;
    for (int i = 0; i < kp.B; i++) {
        double t;
        int idx;
        const int kind = closest_hit<COUNT>(kp, o, d, t, idx, cnt);
        V3 hp = v3(0, 0, 0), hn = v3(0, 0, 0);
        Mat mat = Mat{v3(0, 0, 0), v3(0, 0, 0), 0.0, 0.0, 0.0, 0.0};
        if (kind == HIT_SPHERE) {
            const SphGeo s = kp.sph[idx];
            hp = o + muls(d, t);                         // ray_at
            hn = normalize(hp - v3(s.cx, s.cy, s.cz));
            mat = load_mat(kp.sph_mat + idx);
        } else if (kind == HIT_TRI) {
            if (COUNT) cnt.c[RT_CNT_TEX_HITS] += 1;
            const TriGeo g = kp.tri[idx];
            hp = o + muls(d, t);
            hn = normalize(v3(g.nx, g.ny, g.nz));
            mat = tri_material(kp, idx, hp, hn);
        }
        if (i == 0) {
            alb = mat.diff;
            nrm = hn;
        }
        if (i == alpha_depth && is_alpha) {
            alb = mat.es > 0 ? mat.emis : mat.diff;
            nrm = hn;
            is_alpha = false;
        }
        if (kind == HIT_NONE) break;
        if (i == alpha_depth && mat.es > 0) {            // direct view of a light
            const V3 col = hsl_roundtrip(mat.emis);
            out_rad = col;
            out_alb = col;
            out_nrm = hn;
            return;
        }
        o = hp;
        const V3 diffuse_dir = normalize(hn + random_dir<COUNT>(st, cnt));
        const V3 reflected_dir = d - muls(hn, 2 * dot(d, hn));
        const V3 dr = diffuse_dir + muls(reflected_dir - diffuse_dir, mat.rs);
        if (mat.alpha <= 0.99 && mat.alpha >= 0.0001) {  // refraction, main.c:167-193
            if (COUNT) cnt.c[RT_CNT_REFRACT] += 1;
            V3 nn = hn;
            double n1, n2;
            if (dot(d, hn) > 0) {                        // leaving: pop restores the stack
                nn = v3(-hn.x, -hn.y, -hn.z);
                n1 = mat.ior;
                n2 = top_n2;
            } else {                                     // entering: push (top.n2, ior)
                n1 = top_n2;
                n2 = mat.ior;
                top_n2 = mat.ior;
            }
            const V3 refr = refracted(d, nn, n1, n2);
            const double rnd = 0.0 + 1.0 * unit31(st.next31());
            if (rnd > mat.alpha) {
                d = refr;
                continue;
            }
            d = dr;
        }
        if (mat.alpha > 0.99) {
            is_alpha = false;
            d = dr;
        }
        if (mat.alpha < 0.0001) {                        // alpha hole: pass through
            is_alpha = true;
            alpha_depth++;
            continue;
        }
        if (kp.useAO) {
            const V3 em = muls(mat.emis, mat.es * 1.5 * kp.AO);
            inc = inc + mulv(em, rc);
            if (rc.x > 0.5 || rc.y > 0.5 || rc.z > 0.5) rc = mulv(mat.diff, muls(rc, 1.3));
            rc = mulv(mat.diff, rc);
            const double occ = ao_factor<COUNT>(kp, hp, hn, st, cnt);
            rc = mulv(rc, v3(occ, occ, occ));
        } else {
            const V3 em = muls(mat.emis, mat.es);
            inc = inc + mulv(em, rc);
            if (rc.x > 0.5 || rc.y > 0.5 || rc.z > 0.5) rc = mulv(mat.diff, muls(rc, 1.3));
            rc = mulv(mat.diff, rc);
        }
    }
    out_rad = inc;
    out_alb = alb;
    out_nrm = nrm;
}

// write_color_canva, rtutility.h:56-71 (sqrtf of the float-rounded product)
__device__ __forceinline__ double resolve(double sum, double rapport)
{
    double r = (double)sqrtf((float)(rapport * sum));
    r = r < 0.0 ? 0.0 : (r > 0.999 ? 0.999 : r);
    return (double)(int)(256 * r);
}

__device__ __forceinline__ void store3(double* base, long long i, V3 v)
{
    base[3 * i + 0] = v.x;
    base[3 * i + 1] = v.y;
    base[3 * i + 2] = v.z;
}

// fill_canva, main.c:245-284: one thread = one pixel, all S samples.
template <bool COUNT>
__global__ __launch_bounds__(256) void render_kernel(const KParams kp)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    Cnt cnt;
    if (COUNT)
        for (int k = 0; k < RT_NCOUNTERS; ++k) cnt.c[k] = 0;
    bool valid = x < kp.W && ly < kp.local_rows;
    int g = 0;
    if (valid) {
        const int lt = ly / kp.tile_rows, yy = ly - lt * kp.tile_rows;
        g = kp.row_base + (kp.tile_first + lt * kp.tile_step) * kp.tile_rows + yy;
        valid = g < kp.row_end;
    }
    if (valid) {
        const V3 co = v3(kp.cam_o[0], kp.cam_o[1], kp.cam_o[2]);
        const V3 ch = v3(kp.cam_h[0], kp.cam_h[1], kp.cam_h[2]);
        const V3 cv = v3(kp.cam_v[0], kp.cam_v[1], kp.cam_v[2]);
        const V3 cc = v3(kp.cam_c[0], kp.cam_c[1], kp.cam_c[2]);
        const double wm1 = (double)(kp.W - 1), hm1 = (double)(kp.H - 1);
        const uint32_t pixel = (uint32_t)g * (uint32_t)kp.W + (uint32_t)x;
        V3 srad = v3(0, 0, 0), salb = v3(0, 0, 0), snrm = v3(0, 0, 0);
        for (int s = 0; s < kp.S; ++s) {
            Stream st;
            st.start(pixel, (uint32_t)s, kp.key0, kp.key1);
            const double ju = -0.5 + 1.0 * unit31(st.next31());     // randomDouble(-0.5, 0.5)
            const double jv = -0.5 + 1.0 * unit31(st.next31());
            const double jx = -0.5 + 1.0 * unit31(st.next31());
            const double jy = -0.5 + 1.0 * unit31(st.next31());
            const double u = ((double)x + ju) / wm1;
            const double v = ((double)g + jv) / hm1;
            const double dx = jx * kp.ox, dy = jy * kp.oy;
            // get_ray, camera.h:42-55
            const V3 dir = cc + (muls(ch, u) + (muls(cv, v) - co));
            const V3 dest = co + muls(dir, kp.focus);
            const V3 no = co + v3(dx, dy, 0);
            const V3 rd = normalize(dest - no);
            V3 rad, alb, nrm;
            trace<COUNT>(kp, no, rd, st, rad, alb, nrm, cnt);
            srad = srad + rad;
            salb = salb + alb;
            snrm = snrm + nrm;
            if (COUNT) {
                cnt.c[RT_CNT_SAMPLES] += 1;
                cnt.c[RT_CNT_RNG_DRAWS] += st.n;
            }
        }
        if (!COUNT) {
            const long long li = (long long)ly * kp.W + x;
            const double rapport = 1.0 / kp.S;
            store3(kp.canva, li, v3(resolve(srad.x, rapport), resolve(srad.y, rapport), resolve(srad.z, rapport)));
            const double S = (double)kp.S;
            if (kp.albedo) store3(kp.albedo, li, divs(salb, S));
            if (kp.normal) store3(kp.normal, li, divs(snrm, S));
            if (kp.radiance) store3(kp.radiance, li, divs(srad, S));
        }
    }
    if (COUNT) {
        for (int k = 0; k < RT_NCOUNTERS; ++k) {
            unsigned long long v = cnt.c[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (lane == 0 && v) atomicAdd(kp.counters + k, v);
        }
    }
}

// Un-permute a rank-major gather of cyclic row tiles into the full frame.
__global__ __launch_bounds__(256) void assemble_kernel(const double* __restrict__ gathered, long long rank_stride,
                                                       int world, int tile_rows, int rows_per_rank, int W, int H,
                                                       double* __restrict__ out)
{
    const long long n = (long long)W * H * 3;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const long long px = e / 3;
        const int c = (int)(e - px * 3);
        const int g = (int)(px / W), i = (int)(px - (long long)g * W);
        const int t = g / tile_rows, y = g - t * tile_rows;
        const int r = t % world, lt = t / world;
        const long long src = (long long)r * rank_stride + ((long long)lt * tile_rows + y) * W + i;
        out[e] = gathered[src * 3 + c];
    }
}

// Device-math self test (rt_selftest_math).
__global__ void selftest_kernel(int op, const double* __restrict__ in, double* __restrict__ out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (op) {
    case 0: out[i] = pm_acos(in[i]); break;
    case 1: {
        float s, c;
        pm_sincosf((float)in[i], s, c);
        out[i] = (double)s;
        break;
    }
    case 2: {
        float s, c;
        pm_sincosf((float)in[i], s, c);
        out[i] = (double)c;
        break;
    }
    case 3: out[i] = pm_pow(in[2 * i], in[2 * i + 1]); break;
    case 4: out[i] = sqrt(in[i]); break;
    case 5: out[i] = in[2 * i] / in[2 * i + 1]; break;
    case 6: out[i] = (double)sqrtf((float)in[i]); break;
    case 7: {
        const double* q = in + 6 * i;
        const Philox p = philox4x32_10((uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3],
                                       (uint32_t)q[4], (uint32_t)q[5]);
        out[4 * i + 0] = p.w0;
        out[4 * i + 1] = p.w1;
        out[4 * i + 2] = p.w2;
        out[4 * i + 3] = p.w3;
        break;
    }
    default: out[i] = 0.0;
    }
}

static int grid_for(const KParams& kp, dim3& grid)
{
    grid = dim3((unsigned)((kp.W + 15) / 16), (unsigned)((kp.local_rows + 15) / 16), 1);
    return 0;
}

int launch_render(const KParams& kp, void* stream)
{
    dim3 grid;
    grid_for(kp, grid);
    hipLaunchKernelGGL(render_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, kp);
    return (int)hipGetLastError();
}

int launch_count(const KParams& kp, void* stream)
{
    dim3 grid;
    grid_for(kp, grid);
    hipLaunchKernelGGL(render_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, kp);
    return (int)hipGetLastError();
}

int launch_assemble(const double* gathered, long long rank_stride, int world, int tile_rows, int rows_per_rank, int W,
                    int H, double* out, void* stream)
{
    const long long n = (long long)W * H * 3;
    long long blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, gathered,
                       rank_stride, world, tile_rows, rows_per_rank, W, H, out);
    return (int)hipGetLastError();
}

int launch_selftest(int op, const double* d_in, double* d_out, int n, void* stream)
{
    hipLaunchKernelGGL(selftest_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, op,
                       d_in, d_out, n);
    return (int)hipGetLastError();
}

}  // namespace rt
