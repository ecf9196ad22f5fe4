// Host check of pack_bvh_h (rt_bvh.cpp): every 64-byte node's binary16
// planes contain the 128-byte node's float boxes exactly, and the decoded
// counts / children equal the 4-wide tree's.  Input: triangles as 9 doubles
// per line (A, B, C) on stdin.  Build: tools/probes/bvh_h_check.sh
#include <cmath>
#include <cstdio>
#include <vector>
#include "rt_bvh.h"
using namespace rt;
static double h2d(unsigned short h)
{
    const int e = (h >> 10) & 0x1f, m = h & 0x3ff;
    const double v = e == 0 ? std::ldexp((double)m, -24) : std::ldexp((double)(m | 0x400), e - 25);
    return (h & 0x8000) ? -v : v;
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
    std::vector<BvhNodeH> h;
    float rbox = 0;
    if (!pack_bvh_h(b.nodes4, h, rbox)) {      // does not fit binary16: the kernel keeps 128-byte nodes
        std::printf("{\"nodes\": %zu, \"packed\": false, \"depth4\": %d}\n", b.nodes4.size(), b.depth4);
        return 0;
    }
    long bad = 0;
    double grow = 0.0, vol = 0.0;
    for (size_t i = 0; i < h.size(); ++i)
        for (int c = 0; c < 4; ++c) {
            const int nib = (h[i].cnt >> (4 * c)) & 15, cnt = nib == 15 ? -1 : nib;
            if (cnt != b.nodes4[i].count[c]) ++bad;
            if (cnt < 0) continue;
            if (h[i].child[c] != b.nodes4[i].child[c]) ++bad;
            double g = 1.0, e = 1.0;
            for (int a = 0; a < 3; ++a) {
                const double lo = h2d(h[i].org[a]) + h2d(h[i].plo[a][c]), hi = h2d(h[i].org[a]) + h2d(h[i].phi[a][c]);
                if (!(lo <= b.nodes4[i].lo[a][c]) || !(hi >= b.nodes4[i].hi[a][c])) ++bad;
                if (!(std::fabs(lo) <= rbox && std::fabs(hi) <= rbox)) ++bad;
                g *= hi - lo;
                e *= (double)b.nodes4[i].hi[a][c] - b.nodes4[i].lo[a][c];
            }
            grow += g; vol += e;
        }
    std::printf("{\"nodes\": %zu, \"packed\": true, \"depth4\": %d, \"violations\": %ld, \"volume_growth\": %.6f, \"rbox\": %.6g}\n",
                h.size(), b.depth4, bad, grow / vol, rbox);
    return bad != 0;
}
