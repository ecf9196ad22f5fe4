// rt_bvh.cpp — host build of the triangle BVH used by the render kernel
// (the reference scans every triangle, main.c:80-90, and
// its CUDA path only has a per-mesh slab box, triangle.hu:42-59).
//
// Binary BVH, full-sweep SAH over the three axes, one triangle per leaf
// (kLeaf; more only at the depth cap).  Each node stores the boxes
// of BOTH children (float, rounded outward), so one 64-byte node fetch
// decides both descents.  Node 0
// is the root split; triangles are reordered into leaf order and the kernel
// keeps each one's original index for the reference's tie-break.
//
// Exactness: the BVH only decides which triangles are *tested*; every test
// is the reference arithmetic and the winner is the lexicographic minimum of
// (dst, original index) -- what the reference's in-order strict-< scan
// returns.  So culling must never drop a triangle that could win or tie.
// The boxes are padded, and the kernel's distance cull carries a slack, by
// rigorous bounds on the rounding error of the reference test (DESIGN.md
// "BVH"): with det >= 1e-6 (mesh.h:79) the computed barycentrics of an
// accepted hit are within eps_k of exact ones, so the ray meets triangle k's
// plane inside k's box grown by
//     delta_k = (e1+e2) * (2^-44 * 1e6 * ((e1+e2)*4R + 6*e1*e2) + 2^-48)
// (e1, e2 = |B-A|, |C-A|; R bounds every coordinate and ray origin), and the
// computed dst is within  2^-44 * 1e6 * maxN * (t + R)  of that plane hit
// (maxN = max |N|).  The constants carry a factor >= 8 over the
// first-order bounds (3-term dot/cross products, one division).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_bvh.h"

namespace rt {
namespace {

struct Box {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
    double hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    void grow(const Box& b)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    void grow(const double* p)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
        }
    }
    double area() const
    {
        if (lo[0] > hi[0]) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

struct Prim {
    Box box;
    double c[3];
    int idx;
};

struct Ref {
    bool leaf;
    int index;   // node index, or first prim of the leaf
    int count;
    Box box;
};

int kLeaf = 1;                // leaf size target (RT_BVH_LEAF overrides, for tuning; 1 measured best with the queue kernel)

// Outward rounding of a double bound to float.
float down(double x)
{
    float f = (float)x;
    return (double)f > x ? std::nextafter(f, -HUGE_VALF) : f;
}
float up(double x)
{
    float f = (float)x;
    return (double)f < x ? std::nextafter(f, HUGE_VALF) : f;
}

struct Builder {
    std::vector<Prim>& P;
    std::vector<BvhNode>& nodes;
    int max_depth = 0;

    Ref leaf(int b, int e, const Box& box) { return Ref{true, b, e - b, box}; }

    // Full-sweep SAH: every axis, every split between centroid-sorted
    // primitives (ties by index, so the build is deterministic), or -1 at the
    // depth cap.  Against r01-r04's 16 bins on the widest centroid axis: C4
    // +1.1 %, sweep scene -0.6 % (profiles/r04_bvh/ab.txt).
    int split(int b, int e, int depth)
    {
        const int n = e - b;
        if (n <= kLeaf || depth >= kMaxDepth) return -1;
        std::vector<double> rarea((size_t)n);
        double best = HUGE_VAL;
        int best_axis = -1, best_i = -1;
        for (int a = 0; a < 3; ++a) {
            std::sort(P.begin() + b, P.begin() + e, [a](const Prim& x, const Prim& y) {
                return x.c[a] < y.c[a] || (x.c[a] == y.c[a] && x.idx < y.idx);
            });
            Box r;
            for (int i = n - 1; i >= 1; --i) {
                r.grow(P[(size_t)(b + i)].box);
                rarea[(size_t)i] = r.area();
            }
            Box l;
            for (int i = 1; i < n; ++i) {              // left = [b, b + i)
                l.grow(P[(size_t)(b + i - 1)].box);
                const double cost = l.area() * i + rarea[(size_t)i] * (n - i);
                if (cost < best) {
                    best = cost;
                    best_axis = a;
                    best_i = i;
                }
            }
        }
        if (best_axis < 0) return -1;
        if (best_axis != 2)
            std::sort(P.begin() + b, P.begin() + e, [a = best_axis](const Prim& x, const Prim& y) {
                return x.c[a] < y.c[a] || (x.c[a] == y.c[a] && x.idx < y.idx);
            });
        return b + best_i;
    }

    Ref build(int b, int e, int depth)
    {
        Box box;
        for (int i = b; i < e; ++i) {
            box.grow(P[(size_t)i].box);
        }
        max_depth = std::max(max_depth, depth);
        if (e - b <= kLeaf || depth >= kMaxDepth) return leaf(b, e, box);
        const int mid = split(b, e, depth);
        if (mid < 0) return leaf(b, e, box);
        const int idx = (int)nodes.size();
        nodes.emplace_back();
        const Ref L = build(b, mid, depth + 1);
        const Ref R = build(mid, e, depth + 1);
        BvhNode& nd = nodes[(size_t)idx];
        const Ref* ch[2] = {&L, &R};
        for (int c = 0; c < 2; ++c) {
            for (int a = 0; a < 3; ++a) {
                nd.lo[c][a] = down(ch[c]->box.lo[a]);
                nd.hi[c][a] = up(ch[c]->box.hi[a]);
            }
            nd.child[c] = ch[c]->index;
            nd.count[c] = ch[c]->leaf ? ch[c]->count : 0;
        }
        return Ref{false, idx, 0, box};
    }
};

double norm3(double x, double y, double z) { return std::sqrt(x * x + y * y + z * z); }

// Collapse of the binary tree into 4-wide nodes: a node's children are its
// binary children, with the internal child of largest box area replaced by
// its own two children while fewer than four.  Boxes are copied (already
// rounded outward).
struct Elem {
    float lo[3], hi[3];
    int ref, count;          // count 0: binary node index
};

float area(const Elem& e)
{
    const float x = e.hi[0] - e.lo[0], y = e.hi[1] - e.lo[1], z = e.hi[2] - e.lo[2];
    return x * y + y * z + z * x;
}

Elem elem_of(const BvhNode& n, int c)
{
    Elem e;
    for (int a = 0; a < 3; ++a) {
        e.lo[a] = n.lo[c][a];
        e.hi[a] = n.hi[c][a];
    }
    e.ref = n.child[c];
    e.count = n.count[c];
    return e;
}

int collapse(const std::vector<BvhNode>& bin, int b, std::vector<BvhNode4>& out, int depth, int& max_depth)
{
    max_depth = std::max(max_depth, depth);
    std::vector<Elem> ch = {elem_of(bin[(size_t)b], 0), elem_of(bin[(size_t)b], 1)};
    while (ch.size() < 4) {
        int best = -1;
        for (int i = 0; i < (int)ch.size(); ++i)
            if (ch[(size_t)i].count == 0 && (best < 0 || area(ch[(size_t)i]) > area(ch[(size_t)best]))) best = i;
        if (best < 0) break;
        const BvhNode& n = bin[(size_t)ch[(size_t)best].ref];
        ch[(size_t)best] = elem_of(n, 0);
        ch.push_back(elem_of(n, 1));
    }
    const int idx = (int)out.size();
    out.emplace_back();
    int child[4] = {0, 0, 0, 0}, count[4] = {-1, -1, -1, -1};
    for (int i = 0; i < (int)ch.size(); ++i) {
        child[i] = ch[(size_t)i].count > 0 ? ch[(size_t)i].ref
                                           : collapse(bin, ch[(size_t)i].ref, out, depth + 1, max_depth);
        count[i] = ch[(size_t)i].count;
    }
    BvhNode4& nd = out[(size_t)idx];
    for (int i = 0; i < 4; ++i) {
        for (int a = 0; a < 3; ++a) {
            nd.lo[a][i] = i < (int)ch.size() ? ch[(size_t)i].lo[a] : 0.0f;
            nd.hi[a][i] = i < (int)ch.size() ? ch[(size_t)i].hi[a] : 0.0f;
        }
        nd.child[i] = child[i];
        nd.count[i] = count[i];
    }
    return idx;
}

}  // namespace

double bvh_pad_slope(const TriGeo* tri, int nt, double* median_e)
{
    double maxE = 0.0;
    std::vector<double> es((size_t)std::max(nt, 0));
    for (int i = 0; i < nt; ++i) {
        const TriGeo& g = tri[i];
        es[(size_t)i] = norm3(g.abx, g.aby, g.abz) + norm3(g.acx, g.acy, g.acz);
        maxE = std::max(maxE, es[(size_t)i]);
    }
    if (median_e) {
        *median_e = 0.0;
        if (nt > 0) {
            std::nth_element(es.begin(), es.begin() + nt / 2, es.end());
            *median_e = es[(size_t)(nt / 2)];
        }
    }
    return (maxE * maxE * 4.0 * std::ldexp(1e6, -44) + std::ldexp(1.0, -48)) * (1.0 + std::ldexp(1.0, -40));
}

double bvh_origin_radius(const TriGeo* tri, int nt, double tri_bound, const double* sphere_bounds, int ns)
{
    double med = 0.0;
    const double k = bvh_pad_slope(tri, nt, &med);
    // the largest origin radius whose padding stays within 2^-12 of the median
    // triangle's size: spheres inside it (e.g. the README box's radius-500 walls
    // around the C4 tree) cost the tree nothing and their hit points no per-ray
    // margin; larger ones (main.c:346's radius-1e5 sky) stay outside
    const double cap = std::max(tri_bound, std::ldexp(med, -12) / k);
    double r = tri_bound;
    for (int i = 0; i < ns; ++i)
        if (sphere_bounds[i] <= cap) r = std::max(r, sphere_bounds[i]);
    return r;
}

bool build_bvh(const TriGeo* tri, int nt, double r_scene, BvhBuild& out)
{
    out = BvhBuild();
    if (const char* e = std::getenv("RT_BVH_LEAF")) kLeaf = std::max(1, std::min(16, std::atoi(e)));
    if (nt <= kLeaf) return false;
    // The SAH build makes leaves of kLeaf triangles except where the depth cap
    // binds, so a mesh of more than 65535 * kLeaf triangles gets >= 65535
    // internal nodes, which the uint16 traversal stack entries refuse (checked
    // again below): refuse before paying for the sweep build.
    if ((nt + kLeaf - 1) / kLeaf - 1 >= 65535) return false;
    double maxN = 0.0;
    std::vector<Prim> P((size_t)nt);
    for (int i = 0; i < nt; ++i) {
        const TriGeo& g = tri[i];
        const double e1 = norm3(g.abx, g.aby, g.abz), e2 = norm3(g.acx, g.acy, g.acz);
        maxN = std::max(maxN, norm3(g.nx, g.ny, g.nz));
        const double delta = (e1 + e2) * (std::ldexp(1e6, -44) * ((e1 + e2) * 4.0 * r_scene + 6.0 * e1 * e2) +
                                          std::ldexp(1.0, -48)) +
                             std::ldexp(r_scene, -48);
        const double A[3] = {g.ax, g.ay, g.az};
        const double B[3] = {g.ax + g.abx, g.ay + g.aby, g.az + g.abz};
        const double C[3] = {g.ax + g.acx, g.ay + g.acy, g.az + g.acz};
        Prim& p = P[(size_t)i];
        p.box.grow(A);
        p.box.grow(B);
        p.box.grow(C);
        for (int a = 0; a < 3; ++a) {
            p.box.lo[a] -= delta + std::fabs(p.box.lo[a]) * std::ldexp(1.0, -50);
            p.box.hi[a] += delta + std::fabs(p.box.hi[a]) * std::ldexp(1.0, -50);
            p.c[a] = 0.5 * (p.box.lo[a] + p.box.hi[a]);
        }
        p.idx = i;
    }
    Builder bld{P, out.nodes};
    const Ref root = bld.build(0, nt, 0);
    if (root.leaf || out.nodes.size() >= 65535) {        // uint16 traversal stack entries
        out = BvhBuild();
        return false;
    }
    out.order.resize((size_t)nt);
    for (int i = 0; i < nt; ++i) out.order[(size_t)i] = P[(size_t)i].idx;
    out.depth = bld.max_depth;
    collapse(out.nodes, 0, out.nodes4, 0, out.depth4);
    // Breadth-first node order: the top levels are the first nodes (the queue
    // kernel keeps the first ones in LDS).  Child indices are renumbered.
    {
        const size_t n4 = out.nodes4.size();
        std::vector<int> order;                  // new position -> old index
        order.reserve(n4);
        order.push_back(0);
        for (size_t h = 0; h < order.size(); ++h) {
            const BvhNode4& nd = out.nodes4[(size_t)order[h]];
            for (int c = 0; c < 4; ++c)
                if (nd.count[c] == 0) order.push_back(nd.child[c]);
        }
        std::vector<int> pos(n4, -1);
        for (size_t i = 0; i < order.size(); ++i) pos[(size_t)order[i]] = (int)i;
        std::vector<BvhNode4> bfs(order.size());
        for (size_t i = 0; i < order.size(); ++i) {
            bfs[i] = out.nodes4[(size_t)order[i]];
            for (int c = 0; c < 4; ++c)
                if (bfs[i].count[c] == 0) bfs[i].child[c] = pos[(size_t)bfs[i].child[c]];
        }
        out.nodes4.swap(bfs);
    }
    // Traversal stack bound: bvh_step (rt_kernels.hip) pushes every hit
    // internal child but the one it enters, and every entry on the stack was
    // pushed at an ancestor of the current node, so the stack never holds more
    // than the maximum over root-to-node paths of sum(internal children - 1).
    // (Breadth-first order: children after parents.)
    {
        std::vector<int> need(out.nodes4.size(), 0);
        for (size_t i = out.nodes4.size(); i-- > 0;) {
            int k = 0, m = 0;
            for (int c = 0; c < 4; ++c)
                if (out.nodes4[i].count[c] == 0) {
                    ++k;
                    m = std::max(m, need[(size_t)out.nodes4[i].child[c]]);
                }
            need[i] = std::max(0, k - 1) + m;
        }
        out.stack4 = need.empty() ? 0 : need[0];
    }
    if (out.stack4 > kStack4 || out.nodes4.size() >= 65535) {
        out = BvhBuild();
        return false;
    }
    const double k = std::ldexp(1e6, -44) * maxN;
    out.s_rel = k + std::ldexp(1.0, -48);
    out.s_abs = k * r_scene + std::ldexp(r_scene, -48);
    out.r_scene = r_scene;
    // delta(R) above is affine in R with slope (e1+e2)^2 4 2^-44 1e6 + 2^-48, the
    // distance slack S_abs = s_rel R: a ray from |o|_inf = R' > r_scene needs the
    // boxes wider by at most k_delta (R' - r_scene) and S_abs = s_rel R' (the walk
    // adds both per ray, rt_kernels.hip ray32); rounded up
    out.k_delta = bvh_pad_slope(tri, nt, nullptr);
    return std::isfinite(out.k_delta);
}

// ---- 64-byte nodes (BvhNodeH) ------------------------------------------------
namespace {

// binary16 <-> double by bits (normal, subnormal, zero; no inf/NaN here)
double h2d(unsigned short h)
{
    const int e = (h >> 10) & 0x1f, m = h & 0x3ff;
    const double v = e == 0 ? std::ldexp((double)m, -24) : std::ldexp((double)(m | 0x400), e - 25);
    return (h & 0x8000) ? -v : v;
}
// the binary16 bit pattern next above / below h (finite h; false at overflow)
bool h_up(unsigned short& h)
{
    if (h == 0x8000) h = 0x0001;                       // -0 -> smallest positive
    else if (h & 0x8000) h = (unsigned short)(h - 1);  // negative: toward zero
    else {
        if (h >= 0x7bff) return false;                 // 65504 has no finite successor
        h = (unsigned short)(h + 1);
    }
    return true;
}
bool h_down(unsigned short& h)
{
    if (h == 0x0000) h = 0x8001;
    else if (h & 0x8000) {
        if (h >= 0xfbff) return false;
        h = (unsigned short)(h + 1);
    } else h = (unsigned short)(h - 1);
    return true;
}
// the largest binary16 <= x, or the smallest >= x (x finite); false beyond 65504
bool h_round(double x, bool up, unsigned short& h)
{
    if (!(std::fabs(x) <= 65504.0)) return false;
    // nearest by search from a coarse start: frexp/ldexp give the bits directly
    const double ax = std::fabs(x);
    unsigned short b;
    if (ax < std::ldexp(1.0, -14)) {
        b = (unsigned short)std::nearbyint(ax * std::ldexp(1.0, 24));
    } else {
        int e;
        const double f = std::frexp(ax, &e);           // ax = f 2^e, f in [0.5, 1)
        long m = std::lrint(std::ldexp(f, 11));        // 11 significant bits
        if (m == 2048) { m = 1024; ++e; }
        b = (unsigned short)(((e - 1 + 15) << 10) | (m & 0x3ff));
        if (((b >> 10) & 0x1f) >= 31) return false;
    }
    h = (unsigned short)(x < 0.0 ? (b | 0x8000) : b);
    if (x == 0.0) h = 0;
    while (up ? h2d(h) < x : h2d(h) > x)
        if (!(up ? h_up(h) : h_down(h))) return false;
    return true;
}

}  // namespace

bool pack_bvh_h(const std::vector<BvhNode4>& nodes4, std::vector<BvhNodeH>& out, float& rbox)
{
    out.assign(nodes4.size(), BvhNodeH{});
    double rb = 0.0;
    for (size_t i = 0; i < nodes4.size(); ++i) {
        const BvhNode4& n = nodes4[i];
        BvhNodeH& h = out[i];
        double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
        for (int c = 0; c < 4; ++c)
            if (n.count[c] >= 0)
                for (int a = 0; a < 3; ++a) lo[a] = std::fmin(lo[a], (double)n.lo[a][c]);
        double org[3];
        for (int a = 0; a < 3; ++a) {
            if (!std::isfinite(lo[a])) lo[a] = 0.0;
            if (!h_round(lo[a], false, h.org[a])) return false;
            org[a] = h2d(h.org[a]);
            rb = std::fmax(rb, std::fabs(org[a]));
        }
        h.cnt = 0;
        for (int c = 0; c < 4; ++c) {
            int nib;
            if (n.count[c] < 0) nib = 15;
            else if (n.count[c] > 14) return false;
            else nib = n.count[c];
            if (n.count[c] >= 0 && (n.child[c] < 0 || n.child[c] > 0xffff)) return false;
            h.cnt = (unsigned short)(h.cnt | (nib << (4 * c)));
            h.child[c] = (unsigned short)(n.count[c] >= 0 ? n.child[c] : 0);
            for (int a = 0; a < 3; ++a) {
                if (n.count[c] < 0) {
                    h.plo[a][c] = h.phi[a][c] = 0;
                    continue;
                }
                // org + rel in double is exact (two binary16 values), so the
                // comparisons below are exact; step outward until they hold
                unsigned short ql, qh;
                if (!h_round((double)n.lo[a][c] - org[a], false, ql) || !h_round((double)n.hi[a][c] - org[a], true, qh))
                    return false;
                while (org[a] + h2d(ql) > (double)n.lo[a][c])
                    if (!h_down(ql)) return false;
                while (org[a] + h2d(qh) < (double)n.hi[a][c])
                    if (!h_up(qh)) return false;
                h.plo[a][c] = ql;
                h.phi[a][c] = qh;
                rb = std::fmax(rb, std::fmax(std::fabs(org[a] + h2d(ql)), std::fabs(org[a] + h2d(qh))));
                rb = std::fmax(rb, std::fabs(org[a]) + std::fmax(std::fabs(h2d(ql)), std::fabs(h2d(qh))));
            }
        }
    }
    rbox = (float)rb;
    if ((double)rbox < rb) rbox = std::nextafter(rbox, HUGE_VALF);
    return std::isfinite(rbox);
}

}  // namespace rt
