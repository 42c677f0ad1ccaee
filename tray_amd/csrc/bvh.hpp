// Exact-culling BVH shared by the host builder (tray_bvh.cpp) and the kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/tray.h"

namespace tray {

constexpr int kBvhLeafMax = 4;
// Below this many spheres the linear scan is used (no BVH is built).
constexpr int kBvhMinSpheres = 16;

// 32 B, depth-first order. An inner node's first child is the next node; `skip`
// is the node after this subtree (nodes.size() = end of traversal).
// leaf = -1 for inner nodes, else (first slot << 3) | count.
struct BvhNode {
    float lo[3];
    float hi[3];
    int32_t skip;
    int32_t leaf;
};
static_assert(sizeof(BvhNode) == 32, "BvhNode layout");

struct Bvh {
    std::vector<BvhNode> nodes;
    std::vector<double4> geo;   // {cx, cy, cz, R*R} in leaf-slot order
    std::vector<int32_t> idx;   // original list index of each slot
    double bound = 0;           // M: every box coordinate lies in [-M, M]
};

// Returns false on non-finite input (the caller then uses the linear scan).
bool build_bvh(const tray_sphere* spheres, int32_t n, Bvh* out, int leaf_max = kBvhLeafMax);

}  // namespace tray
