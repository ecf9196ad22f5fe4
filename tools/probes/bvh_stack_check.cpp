// Host check of BvhBuild::stack4 (rt_bvh.cpp), the traversal-stack bound the
// launcher admits trees to the queue kernel's 24-entry LDS stack by.  It runs
// bvh_step's push rule (rt_kernels.hip: every hit internal child but the one
// entered is pushed) as a depth-first walk in which every child box is hit,
// entering the first or the last internal child, and for random rays against
// the float boxes; the largest stack size of every walk must stay <= stack4.  Input: triangles as 9 doubles per line on
// stdin, then the ray count as argv[1].  Used by tests/test_bvh_stack.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "rt_bvh.h"
using namespace rt;

static bool slab(const BvhNode4& n, int c, const double* o, const double* inv)
{
    double t0 = -HUGE_VAL, t1 = HUGE_VAL;
    const float* lo[3] = {n.lo[0], n.lo[1], n.lo[2]};
    const float* hi[3] = {n.hi[0], n.hi[1], n.hi[2]};
    for (int a = 0; a < 3; ++a) {
        double p = (lo[a][c] - o[a]) * inv[a], q = (hi[a][c] - o[a]) * inv[a];
        if (p > q) std::swap(p, q);
        t0 = std::fmax(t0, p);
        t1 = std::fmin(t1, q);
    }
    return t0 <= t1 && t1 >= 0.0;
}

// max stack size of the walk; hit(node, child) decides the child boxes
template <class HIT>
static int walk(const std::vector<BvhNode4>& N, HIT hit, bool last = false)
{
    std::vector<int> stk;
    int node = 0, peak = 0;
    for (;;) {
        int next = -1;
        for (int c = 0; c < 4; ++c) {
            if (N[(size_t)node].count[c] != 0 || !hit(node, c)) continue;
            if (next < 0) next = N[(size_t)node].child[c];
            else if (last) {
                stk.push_back(next);
                next = N[(size_t)node].child[c];
            } else stk.push_back(N[(size_t)node].child[c]);
        }
        peak = std::max(peak, (int)stk.size());
        if (next >= 0) {
            node = next;
            continue;
        }
        if (stk.empty()) break;
        node = stk.back();
        stk.pop_back();
    }
    return peak;
}

int main(int argc, char** argv)
{
    const int nrays = argc > 1 ? std::atoi(argv[1]) : 0;
    std::vector<TriGeo> tri;
    double v[9], r = 0.0;
    while (std::scanf("%lf %lf %lf %lf %lf %lf %lf %lf %lf", v, v + 1, v + 2, v + 3, v + 4, v + 5, v + 6, v + 7, v + 8) == 9) {
        TriGeo g;
        g.ax = v[0]; g.ay = v[1]; g.az = v[2];
        g.abx = v[3] - v[0]; g.aby = v[4] - v[1]; g.abz = v[5] - v[2];
        g.acx = v[6] - v[0]; g.acy = v[7] - v[1]; g.acz = v[8] - v[2];
        g.nx = g.aby * g.acz - g.abz * g.acy; g.ny = g.abz * g.acx - g.abx * g.acz; g.nz = g.abx * g.acy - g.aby * g.acx;
        tri.push_back(g);
        for (double x : v) r = std::fmax(r, std::fabs(x));
    }
    BvhBuild b;
    if (!build_bvh(tri.data(), (int)tri.size(), r, b)) {
        std::printf("{\"bvh\": false}\n");
        return 0;
    }
    const int all = std::max(walk(b.nodes4, [](int, int) { return true; }),
                             walk(b.nodes4, [](int, int) { return true; }, true));
    int rays = 0;
    std::srand(12345);
    const auto u = [] { return std::rand() / (double)RAND_MAX * 2.0 - 1.0; };
    for (int k = 0; k < nrays; ++k) {
        double o[3] = {u() * r, u() * r, u() * r}, d[3] = {u(), u(), u()}, inv[3];
        for (int a = 0; a < 3; ++a) inv[a] = 1.0 / d[a];
        rays = std::max(rays, walk(b.nodes4, [&](int n, int c) { return slab(b.nodes4[(size_t)n], c, o, inv); }));
    }
    std::printf("{\"bvh\": true, \"nodes\": %zu, \"depth4\": %d, \"stack4\": %d, \"all_hit_peak\": %d, \"ray_peak\": %d}\n",
                b.nodes4.size(), b.depth4, b.stack4, all, rays);
    return 0;
}
