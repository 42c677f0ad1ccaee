// Exact-culling 4-wide BVH shared by the host builder (tray_bvh.cpp) and the kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/tray.h"

namespace tray {

constexpr int kBvhWidth = 4;
// Spheres per leaf: 1 by default (every sphere gets its own padded box, which
// is then the FP32 pre-test of its FP64 intersection); up to 4 when the node
// count must shrink.
constexpr int kBvhLeafMax = 4;
// Below this many spheres the linear scan is used (no BVH is built).
constexpr int kBvhMinSpheres = 16;
// child[] value of an unused child slot.
constexpr int32_t kBvhEmpty = 0x7fffffff;
// Traversal stack entries are 16-bit node indices.
constexpr int32_t kBvhMaxNodes = 65535;

// 128 B: the boxes of up to four children, SoA by axis so one node is seven
// 16-byte LDS reads; box[a][0] / box[a][1] are the low / high planes on axis a
// (16 B apart, so a lane picks its near and far planes by address).
// child[k] >= 0: inner node index; child[k] < 0: leaf ~((first slot << 3) |
// count); kBvhEmpty: unused (its box is empty: lo = +inf, hi = -inf).
struct Bvh4Node {
    float box[3][2][kBvhWidth];  // [axis][lo, hi][child]
    int32_t child[kBvhWidth];
    int32_t pad[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node layout");

struct Bvh {
    std::vector<Bvh4Node> nodes;  // nodes[0] is the root (always an inner node)
    std::vector<double4> geo;     // {cx, cy, cz, R*R} in leaf-slot order
    std::vector<int32_t> idx;     // original list index of each slot
    double bound = 0;             // M: every box coordinate lies in [-M, M]
    int32_t stack_max = 0;        // deepest stack the near-first traversal can build
    int leaf_max = 1;
};

// Returns false on non-finite input or a tree the kernel cannot index (the
// caller then uses the linear scan).
bool build_bvh(const tray_sphere* spheres, int32_t n, Bvh* out, int leaf_max = 1);

}  // namespace tray
