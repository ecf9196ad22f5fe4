// rt_bvh.h — triangle BVH layout shared by the host builder (rt_bvh.cpp), the
// C-ABI (rt_api.cpp) and the kernel (rt_kernels.hip).
#pragma once
#include <vector>

#include "rt_internal.h"

namespace rt {

constexpr int kMaxDepth = 30;       // the kernel's LDS stack holds kMaxDepth + 1 entries

// One internal node: the padded boxes of both children (one 64-byte fetch
// per visit).  Bounds are the padded double boxes rounded OUTWARD to float
// (storage only: the slab test runs in double), so every float box contains
// its double box.  count[c] > 0: child c is a leaf of count[c] triangles
// starting at child[c] (leaf order); count[c] == 0: child[c] is a node index.
struct BvhNode {
    float lo[2][3];
    float hi[2][3];
    int child[2];
    int count[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode");

// 4-wide node collapsed from the binary tree (what the kernel traverses):
// float boxes of up to four children, SoA by axis.  count[c] > 0: leaf of
// count[c] triangles from child[c]; 0: child[c] is a node index; -1: empty.
struct BvhNode4 {
    float lo[3][4];
    float hi[3][4];
    int child[4];
    int count[4];
};
static_assert(sizeof(BvhNode4) == 128, "BvhNode4");

constexpr int kStack4 = 48;         // kernel LDS stack entries (3 pushes per 4-wide level)

struct BvhBuild {
    std::vector<BvhNode> nodes;     // binary tree, node 0 = root split
    std::vector<BvhNode4> nodes4;   // collapsed 4-wide tree, node 0 = root
    std::vector<int> order;         // leaf order -> original triangle index
    int depth = 0;                  // binary depth
    int depth4 = 0;                 // 4-wide depth (stack bound: 3 * depth4 + 1 <= kStack4)
    double s_rel = 0.0, s_abs = 0.0;   // distance-cull slack (rt_bvh.cpp header)
    double r_scene = 0.0;              // coordinate bound the padding assumed
};

// Builds over nt precomputed triangles whose coordinates (and every ray
// origin) are bounded by r_scene in magnitude.  false: no BVH (too few
// triangles or too many nodes) -> brute-force scan.
bool build_bvh(const TriGeo* tri, int nt, double r_scene, BvhBuild& out);

}  // namespace rt
