// Host SAH cost of the 4-wide tree build_bvh makes (rt_bvh.cpp): expected
// node visits and triangle tests per random ray through the root box
// (surface-area ratios), the proxy used to compare tree builders before a
// GPU A/B.  Input: triangles as 9 doubles per line on stdin (bvh_cost.sh).
#include <cmath>
#include <cstdio>
#include <vector>
#include "rt_bvh.h"
using namespace rt;
static double area(const double* lo, const double* hi)
{
    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return 2.0 * (x * y + y * z + z * x);
}
int main()
{
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
    if (!build_bvh(tri.data(), (int)tri.size(), r, b)) { std::printf("no bvh\n"); return 1; }
    // a node's own box = union of its children's; visits = sum A(node)/A(root)
    const size_t n = b.nodes4.size();
    std::vector<double> nlo(3 * n, HUGE_VAL), nhi(3 * n, -HUGE_VAL);
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 4; ++c)
            if (b.nodes4[i].count[c] >= 0)
                for (int a = 0; a < 3; ++a) {
                    nlo[3 * i + a] = std::fmin(nlo[3 * i + a], b.nodes4[i].lo[a][c]);
                    nhi[3 * i + a] = std::fmax(nhi[3 * i + a], b.nodes4[i].hi[a][c]);
                }
    const double a0 = area(&nlo[0], &nhi[0]);
    double visits = 0.0, tests = 0.0;
    for (size_t i = 0; i < n; ++i) {
        visits += area(&nlo[3 * i], &nhi[3 * i]) / a0;
        for (int c = 0; c < 4; ++c)
            if (b.nodes4[i].count[c] > 0) {
                double lo[3], hi[3];
                for (int a = 0; a < 3; ++a) { lo[a] = b.nodes4[i].lo[a][c]; hi[a] = b.nodes4[i].hi[a][c]; }
                tests += area(lo, hi) / a0 * b.nodes4[i].count[c];
            }
    }
    std::printf("{\"nodes\": %zu, \"depth4\": %d, \"stack4\": %d, \"sah_node_visits\": %.3f, \"sah_tri_tests\": %.3f}\n",
                n, b.depth4, b.stack4, visits, tests);
    return 0;
}
