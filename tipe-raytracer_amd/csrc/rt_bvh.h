// rt_bvh.h — triangle BVH layout shared by the host builder (rt_bvh.cpp), the
// C-ABI (rt_api.cpp) and the kernel (rt_kernels.hip).
#pragma once
#include <vector>

#include "rt_internal.h"

namespace rt {

constexpr int kMaxDepth = 30;       // binary build depth cap (leaves below it hold several triangles); the
                                    // kernels admit a tree by its exact stack bound (BvhBuild::stack4 vs
                                    // kStack4 / kStackQ / kStackQ4), not by its depth

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

// The same 4-wide node in 64 bytes for the queue kernel (r03): binary16
// planes relative to a binary16 node origin, rounded outward, so that
//   org + plo <= the float lo bound and org + phi >= the float hi bound
// hold exactly (the box only grows: every culling decision stays
// conservative).  Rows as BvhNode4's: plo[a] (a = x, y, z), then phi[a], 8
// bytes each (four children); the 16-byte tail holds the origin, the four
// 4-bit counts (0 internal, 1-14 leaf of that many triangles, 15 empty) and
// the 16-bit child indices (node, or first triangle in leaf order).  The
// kernel's slab test reads the halves straight into v_fma_mix_f32.
struct BvhNodeH {
    unsigned short plo[3][4];
    unsigned short phi[3][4];
    unsigned short org[3];
    unsigned short cnt;             // count of child c in bits 4c..4c+3
    unsigned short child[4];
};
static_assert(sizeof(BvhNodeH) == 64, "BvhNodeH");

// Packs nodes4 into BvhNodeH; false when a value does not fit (|coordinate|
// beyond binary16's range, a leaf of more than 14 triangles, a child index
// above 65535).  rbox: >= |org| + |plane| over every node (the slab
// margin's coordinate bound for the packed planes).
bool pack_bvh_h(const std::vector<BvhNode4>& nodes4, std::vector<BvhNodeH>& out, float& rbox);

struct BvhBuild {
    std::vector<BvhNode> nodes;     // binary tree, node 0 = root split
    std::vector<BvhNode4> nodes4;   // collapsed 4-wide tree, node 0 = root
    std::vector<int> order;         // leaf order -> original triangle index
    int depth = 0;                  // binary depth
    int depth4 = 0;                 // 4-wide depth
    int stack4 = 0;                 // traversal stack entries the tree can need (<= 3 * depth4; <= kStack4)
    double s_rel = 0.0, s_abs = 0.0;   // distance-cull slack (rt_bvh.cpp header)
    double r_scene = 0.0;              // coordinate bound the padding assumed
    double k_delta = 0.0;              // >= d(padding)/dR of every triangle: a ray whose origin
                                       // lies at R' > r_scene widens the boxes by k_delta (R' - r_scene)
};

// Builds over nt precomputed triangles whose coordinates are bounded by
// r_scene in magnitude; the padding assumes ray origins within r_scene too,
// and the walk widens it per ray for origins beyond (k_delta, rt_kernels.hip
// ray32).  false: no BVH (too few triangles or too many nodes) -> brute-force
// scan.
bool build_bvh(const TriGeo* tri, int nt, double r_scene, BvhBuild& out);
// >= d(padding)/dR of every triangle (BvhBuild::k_delta); median_e: the
// median e1 + e2 (may be null).
double bvh_pad_slope(const TriGeo* tri, int nt, double* median_e);
// The origin radius to build with: the triangles' coordinate bound, raised to
// cover every sphere (sphere_bounds[i] = max_a |c_a| + r) whose hit points the
// padding can include at a cost below 2^-12 of the median triangle's size.
double bvh_origin_radius(const TriGeo* tri, int nt, double tri_bound, const double* sphere_bounds, int ns);

}  // namespace rt
