// Exact-culling 4-wide BVH shared by the host builder (tray_bvh.cpp) and the kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/tray.h"

namespace tray {

#ifndef TRAY_BVH_WIDTH
#define TRAY_BVH_WIDTH 4
#endif
constexpr int kBvhWidth = TRAY_BVH_WIDTH;  // children per node: 4 or 8
static_assert(kBvhWidth == 4 || kBvhWidth == 8, "BVH width");
// Spheres per leaf: 1 by default (every sphere gets its own padded box, which
// is then the FP32 pre-test of its FP64 intersection); up to 4 when the node
// count must shrink.
constexpr int kBvhLeafMax = 4;
// Below this many spheres the linear scan is used (no BVH is built).
constexpr int kBvhMinSpheres = 16;
// Child references are 16 bits: an inner node index (< 0x8000), 0x8000 | leaf
// index, or kBvhNone for an unused child slot (whose box is empty).
constexpr uint32_t kBvhLeafBit = 0x8000u;
constexpr uint32_t kBvhNone = 0xFFFFu;
constexpr int32_t kBvhMaxNodes = 0x8000;
constexpr int32_t kBvhMaxLeaves = 0x7FFF;
// A sphere whose box dwarfs the rest of the scene (a ground sphere) is not put
// in the tree: every traversal tests it first (nearly every ray would visit
// it anyway), which also seeds the culling distance. At most kBvhGlobals, each
// with a box surface kBvhGlobalRatio times that of all the other spheres.
constexpr int kBvhGlobals = 2;
constexpr double kBvhGlobalRatio = 16.0;

// 128 B: the boxes of up to four children, SoA by axis so one node is seven
// 16-byte LDS reads; box[a][0] / box[a][1] are the low / high planes on axis a
// (16 B apart, so a lane picks its near and far planes by address). An unused
// child's box is empty (lo = +inf, hi = -inf) and its ref is kBvhNone.
struct Bvh4Node {
    float box[3][2][kBvhWidth];  // [axis][lo, hi][child]
    uint32_t ref[kBvhWidth];     // 16-bit child references (above)
    uint32_t pad[kBvhWidth == 4 ? 4 : 0];
};
static_assert(sizeof(Bvh4Node) % 32 == 0, "Bvh4Node layout");

struct Bvh {
    std::vector<Bvh4Node> nodes;  // nodes[0] is the root (always an inner node)
    std::vector<int32_t> leaves;  // per leaf: (first slot << 3) | sphere count (leaf_max 1: slot == leaf index)
    std::vector<double4> geo;     // {cx, cy, cz, R*R} in leaf-slot order
    std::vector<int32_t> idx;     // original list index of each slot
    double bound = 0;             // M: every box coordinate lies in [-M, M]
    int32_t stack_max = 0;        // deepest stack the ordered traversal can build
    int leaf_max = 1;
    int32_t n_global = 0;         // spheres tested before the tree: the last n_global slots
};

// Returns false on non-finite input or a tree the kernel cannot index (the
// caller then uses the linear scan).
bool build_bvh(const tray_sphere* spheres, int32_t n, Bvh* out, int leaf_max = 1);
// Build variants for offline comparison (tools/bvh_sim.cpp); the defaults are build_bvh's.
struct BvhOptions {
    bool sweep = false;  // full-sweep SAH instead of 32 bins
    int collapse = 0;    // 0: open the largest-area child; 1: the largest area x primitive count
};
bool build_bvh_opts(const tray_sphere* spheres, int32_t n, Bvh* out, int leaf_max, const BvhOptions& opt);

}  // namespace tray
