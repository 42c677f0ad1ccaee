// Internal launch interface between the C-ABI glue (tray_abi.hip) and the
// megakernel (tray_kernel.hip). Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "bvh.hpp"

namespace tray {

enum : int32_t { kLambertian = 1, kMetal = 2, kDielectric = 3 };
enum : int32_t { kOutRGBF64 = 0, kOutRGBF32 = 1, kOutRGBA8 = 2 };

// Sphere geometry is staged into LDS as double4 {cx, cy, cz, R*R} (32 B).
// Up to 160 KiB of LDS per workgroup on gfx950 -> 5120 spheres; larger scenes
// read the same array from global memory (L2/L1-resident).
// BVH workgroups: TRAY_BVH_BLOCK lanes each, TRAY_BVH_WAVES_PER_SIMD waves per
// SIMD, so (4 SIMDs x waves x 64) / block workgroups share a CU and its LDS.
#ifndef TRAY_BVH_WAVES_PER_SIMD
#define TRAY_BVH_WAVES_PER_SIMD 4
#endif
#ifndef TRAY_BVH_BLOCK
#define TRAY_BVH_BLOCK (256 * TRAY_BVH_WAVES_PER_SIMD)
#endif
constexpr int kBvhBlocksPerCU = 256 * TRAY_BVH_WAVES_PER_SIMD / TRAY_BVH_BLOCK;
// KernelParams::coop_lanes unless the "coop_lanes" debug knob says otherwise.
#ifndef TRAY_COOP_LANES
#define TRAY_COOP_LANES 2
#endif
#ifdef TRAY_PROFILE
constexpr size_t kMaxLDSBytes = (160 * 1024) / kBvhBlocksPerCU - 2048;  // diagnostic builds: 2 KB of counters
#else
constexpr size_t kMaxLDSBytes = (160 * 1024) / kBvhBlocksPerCU;
#endif

// Per-sphere shading record, read only for the closest hit (64 B).
struct MatRec {
    double albedo[3];  // Dielectric (attenuation 1): albedo[0], [1] hold Schlick's r0 for the
                       // front (ratio 1/RefIdx) and back (ratio RefIdx) faces, ray/materials.go:67-68
    double param;   // Metal.Fuzz / Dielectric.RefIdx
    double radius;  // Sphere.Radius (normal = (P - C) / R, ray/objects.go:100)
    double rinv;    // RN(1 / Radius): exact quotients via div_rcp (tray_kernel.hip)
    double pinv;    // RN(1 / RefIdx) = Go's 1.0/d.RefIdx (ray/materials.go:48)
    int32_t type;
    int32_t pad;
};

struct CamRec {
    double position[3];
    double pixel00[3];
    double pixel_x[3];
    double pixel_y[3];
    double defocus_u[3];
    double defocus_v[3];
    double aperture;
};

struct V3 {
    double x, y, z;
};

// Traversal stack slots per lane beyond the depth bound (Bvh::stack_max): slot
// 0, the scratch slot of a push, and the two slots above the top that the
// branch-free three-entry push writes unconditionally (tray_kernel.hip trav_node).
constexpr int32_t kStackSlack = 3;

// Unsigned 32-bit division by a launch-invariant divisor d >= 1 (Granlund and
// Montgomery 1994, the round-up method): with l = ceil(log2 d) and
// m = floor(2^32 (2^l - d) / d) + 1, t = mulhi(n, m) gives
// n / d = (t + ((n - t) >> min(l, 1))) >> max(l - 1, 0) for every n < 2^32.
// Five integer instructions on the device, no FP64 conversion.
struct FastDiv {
    uint32_t d, m, s1, s2;
};
inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    FastDiv f;
    f.d = d;
    f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    f.s1 = l < 1 ? l : 1;
    f.s2 = l > 1 ? l - 1 : 0;
    return f;
}

struct KernelParams {
    const double4* geo;  // n_pad entries: n spheres, then NaN padding (never hit)
    const MatRec* mat;
    uint32_t* queue;     // work-item counter: zero at launch (allocation, then each resolve pass)
    int32_t n;
    int32_t n_pad;       // round_up(n, 4) + 4
    int32_t tiles_x;     // 8x8 pixel tiles per compact row band
    uint32_t nchunks;    // 64-item chunks of the band's work items (one item = one sample)
    uint32_t pool_chunks;  // chunks a workgroup takes from the queue per atomic (set by launch_render)
    uint32_t items;      // band work items: passes x frame_items
    uint32_t frame_items;  // one pass's items of the band: 8x8-tile-padded pixels x spp
    uint32_t passes, pass0;  // progressive passes pass0 .. pass0 + passes - 1 in this launch
    FastDiv div_passes;       // (pixel x passes + pass) -> (pixel, pass): a pixel's passes are consecutive items
    uint32_t wave_chunks;     // chunks a wave reserves per pool take (take_chunk)
    uint32_t late_at;         // from this chunk on, single-chunk takes
    size_t out_frame_bytes;  // output stride between passes
    int32_t j0, band_rows;  // the band: compact rows [j0, j0 + band_rows)
    FastDiv div_spp, div_tiles_x, div_tile_rows;  // item decoding; compact row -> image row
    double* samples;     // per-item path colours (3 doubles), summed by the resolve kernel; with
                         // on-chip accumulation (acc_slots > 0) the same buffer holds AccPartial records
    // Fixed-point accumulation (acc_shift > 0, rays_per_pixel a multiple of 64 or 16 / 32):
    // the background is pre-scaled by 2^acc_shift, each sample's scaled colour is rounded to
    // an integer and the integers are summed exactly (order-free); 0: FP64 sum in sample order.
    int32_t acc_shift;
    int32_t acc_slots;   // >0: per-wave LDS accumulators (slots per wave), partial per 64-item chunk
    uint32_t acc_off;    // byte offset of the accumulator region in the kernel's dynamic LDS
    uint32_t acc_rshift;  // items per chunk record = 2^acc_rshift: 6 (64 | r) or log2 r (r = 16, 32)
    const Bvh4Node* nodes;  // exact-culling 4-wide BVH (tray_bvh.cpp), root first
    const int32_t* leaves;  // per leaf: (first slot << 3) | count
    int32_t leaf_single;    // 1: every leaf holds one sphere and its index is its slot
    const double4* bgeo;    // spheres in leaf-slot order
    const int32_t* bidx;    // original index per slot
    const MatRec* bmat;     // shading record per slot
    int32_t n_nodes, n_slots, n_leaves;
    int32_t n_global;       // spheres tested before the tree: slots [n_slots - n_global, n_slots)
    int32_t stack_cap;      // traversal stack slots per lane (Bvh::stack_max + kStackSlack)
    int32_t stack_lds;      // slots kept in LDS (set by launch_render)
    uint32_t* stack_ovf;    // slots beyond the LDS ones, stride = grid lanes
    unsigned long long* stats;  // nullable: [segments, sphere tests, box tests]
    int32_t width, height, spp, max_depth;
    int32_t y_start, rows, tile_rows, tile_count, tile_index;
    int32_t out_format;
    double ray_radius;
    double focus_time;  // FocusDistance / FocalLength (ray/camera.go:134)
    uint32_t key[4];  // the draw key of the seed (rng.hpp draw_key, include/tray.h)
    CamRec cam;
    V3 bg_a, bg_b;
    void* out;
    uint32_t* segments;
    const double* srgb;  // TRAY_OUT_RGBA8: the 256-entry encoder table (tray::srgb_thresholds)
    unsigned long long* progress;  // nullable, HOST-mapped: samples finished per 8-row tile row of the compact rows
    const uint4* cand;   // nullable (BVH only): primary-ray candidate record per compact pixel (launch_cand_build)
    // Expensive-first work order ("Work order"; on-chip sums only), per band:
    // tile_order (nullable: band order) lists the band's 8x8 tiles in the order their
    // work items are handed out; tile_cost (nullable: no counting) receives each tile's
    // Scene.Hit calls (the chunk records carry their counts, the resolve adds them), from
    // which launch_render's tile_order_kernel builds the next launch's order.
    const uint32_t* tile_order;
    uint32_t* tile_cost;
    FastDiv div_chunks_per_tile;  // 64-item chunks per tile: rays_per_pixel x passes
    // The drain's wave-wide Scene.Hit ("The drain"): once a wave's queue has
    // run dry and it holds at most this many paths, each of their segments is one scan of
    // every sphere by the whole wave instead of a one-lane traversal. 0: off.
    uint32_t coop_lanes;
};

struct LaunchPlan;
// Enqueues the render of `plan` (plan_launch of the same p and use_bvh): the
// megakernel and resolve pass of every band. `samples_bytes` is the capacity
// of p.samples, sized from plan.buffer_bytes by the caller (an internal
// invariant, checked: hipErrorInvalidValue before anything is enqueued).
// With p.tile_cost set (a counting launch; on-chip sums only), `order_out` (one
// word per tile of p's rows) receives the next launch's work order; p.tile_order
// may be the same buffer (each band's order is rewritten after its megakernel).
hipError_t launch_render(KernelParams p, bool use_bvh, const LaunchPlan& plan, hipStream_t stream,
                         size_t samples_bytes, uint32_t* order_out = nullptr);

// Fixed-point accumulation. A sample's colour c (already scaled by 2^k through
// the background) is rounded to the integer v = rint(c), |v| <= 2^kAccBits; any
// sum of at most 64 such integers is itself an integer of magnitude <= 2^53, so
// FP64 adds it exactly: a chunk's sum (64 samples of one pixel) does not depend
// on the order in which its samples finish, and the resolve pass adds a pixel's
// chunk sums as 64-bit integers. A NaN sample makes its channel's sum NaN.
constexpr int32_t kAccBits = 47;
// A frame whose colour bound leaves the scale 2^k below 2^kAccMinShift (the
// absolute resolution of a sample, 2^-k) keeps the FP64 sum in sample order.
constexpr int32_t kAccMinShift = 44;
// One chunk's sums in global memory (exact integers held as doubles): 32 B.
struct AccPartial {
    double sum[3];
    double pad;
};
static_assert(sizeof(AccPartial) == 32, "AccPartial layout");
// In LDS each open chunk has TRAY_ACC_COPIES sets of three sums; lane l adds to
// set l % copies, so fewer lanes of a wave hit one address in one instruction.
#ifndef TRAY_ACC_COPIES
#define TRAY_ACC_COPIES 2
#endif
constexpr int32_t kAccCopies = TRAY_ACC_COPIES;
constexpr size_t kAccSlotBytes = (size_t)kAccCopies * 3 * sizeof(double);
// Per slot also one 32-bit count of the chunk's Scene.Hit calls (the work order's cost).
constexpr size_t kAccCountBytes = sizeof(uint32_t);
constexpr int32_t kAccSlotsMax = 64;  // per wave (the free-slot mask is 64 bits)
constexpr int32_t kAccSlotsMin = 8;

// Where a launch keeps things (launch_render; render_async_impl sizes its
// buffers from it): the scene layout, stack slots in LDS, LDS bytes, and
// whether the chunk accumulators fit next to them.
struct LaunchLayout {
    int lds_mode;
    int32_t stack_lds;
    size_t lds;
    int32_t acc_slots;  // 0: accumulate through the per-sample buffer
    uint32_t acc_off;
    uint32_t acc_rshift;  // KernelParams::acc_rshift (6 when acc_slots is 0)
};
// Rays per pixel whose samples can be summed in fixed point, on chip: 64 | r (a
// 64-item chunk is one pixel-pass's samples, or part of them) or r = 16 / 32 (a
// chunk is 64 / r whole pixel-passes). Smaller r would leave too few slots.
constexpr bool acc_groupable(int32_t spp) { return spp > 0 && (spp % 64 == 0 || spp == 16 || spp == 32); }
// log2 of the items per chunk record for rays per pixel `spp`.
constexpr uint32_t acc_record_shift(int32_t spp) { return spp % 64 == 0 ? 6u : spp == 32 ? 5u : 4u; }
LaunchLayout launch_layout(const KernelParams& p, bool use_bvh);
// Device bytes of the per-sample buffer or (acc_slots > 0) the chunk partials
// (one per 2^rshift samples).
size_t accum_buffer_bytes(int32_t width, int32_t rows, uint64_t spp, bool partials, uint32_t rshift = 6);
// Everything a launch decides from p and the debug knobs, decided ONCE
// (plan_launch) and handed to launch_render, so the buffer the caller sizes
// from it and the bands the launch runs cannot disagree.
struct LaunchPlan {
    LaunchLayout layout;
    int32_t band_tiles;   // 8-row tile rows per launch band
    size_t buffer_bytes;  // per-sample buffer or chunk records of one band
};
LaunchPlan plan_launch(const KernelParams& p, bool use_bvh);

// Primary-ray candidates: for every compact pixel of p's rows, the
// tree spheres (leaf slots) that any camera ray of the pixel can reach, by a
// conservative bound on the beam from the lens disc through the pixel's
// anti-aliasing disc; a record holds up to kCandSlots slots, or
// kCandOverflow (that pixel's camera rays traverse the BVH). Needs p's camera,
// image, row, BVH geometry and shading record fields.
// The build runs in two passes: 8x8 tiles of pixels first (up to
// kCandTileSlots spheres per tile), then each pixel over its tile's list;
// `out` must hold cand_workspace_bytes(width, rows) (the records, then the
// tile lists).
constexpr uint32_t kCandSlots = 7;
constexpr uint32_t kCandTileSlots = 64;
constexpr uint32_t kCandOverflow = 0xFFFFu;
size_t cand_workspace_bytes(int32_t width, int32_t rows);
hipError_t launch_cand_build(const KernelParams& p, uint4* out, hipStream_t stream);

// ColorF.ToSRGBA over n device pixels (3 doubles each) into RGBA8 words, with the
// threshold table `srgb` (device, 256 doubles) that makes it bit-identical to the
// host encoder.
hipError_t launch_to_srgba(const double* rgb, size_t n_pixels, uint32_t* rgba, const double* srgb,
                           hipStream_t stream);

// Samples per launch band (the sample buffer holds one band: 24 B per sample);
// the band_samples debug knob (include/tray_debug.h) lowers it (tests exercise bands).
#ifndef TRAY_BAND_LOG2
#define TRAY_BAND_LOG2 30
#endif
constexpr uint64_t kMaxBandSamples = 1ull << TRAY_BAND_LOG2;  // 2^30: 25.8 GB of sample buffer (of 288 GB of HBM)
// With on-chip chunk sums the buffer holds one 32-B record per 64 samples, so a band
// is bounded by the 32-bit item indices instead: 2^31 samples (1 GB of records).
#ifndef TRAY_BAND_LOG2_ACC
#define TRAY_BAND_LOG2_ACC 31
#endif
constexpr uint64_t kMaxBandSamplesAcc = 1ull << TRAY_BAND_LOG2_ACC;
static_assert(TRAY_BAND_LOG2_ACC <= 31, "item indices are 32-bit: a band holds at most 2^31 samples");
// The band limit of a launch with (partials) or without on-chip chunk sums.
uint64_t max_band_samples(bool partials = false);
// Bytes of sample buffer launch_render needs for `rows` compact rows.
size_t sample_buffer_bytes(int32_t width, int32_t rows, uint64_t spp);
// False when one 8-row band has more than 2^31 samples (item indices are 32-bit).
bool band_fits(int32_t width, uint64_t spp);

// LDS the BVH kernel needs to hold the whole BVH scene (plus its traversal
// stacks) on chip; above kMaxLDSBytes it reads the scene from global memory.
size_t bvh_scene_lds_bytes(int32_t n_nodes, int32_t n_slots, int32_t n_leaves, int32_t stack_cap);
// Where the BVH kernel keeps a scene: mode 1 nodes, geometry and leaf table in
// LDS; 2 nodes and leaf table in LDS, geometry in global memory; 0 all in global
// memory. `rank` orders plans by speed (higher is faster; tray_kernel.hip).
struct LdsPlan {
    int mode, rank;
};
LdsPlan bvh_lds_plan(int32_t n_nodes, int32_t n_slots, int32_t n_leaves, int32_t stack_cap);
// Bytes of global stack-overflow area a render of a scene with this stack bound
// needs on `device` (0 when the whole stack fits in LDS).
size_t bvh_stack_overflow_bytes(int32_t stack_cap, int device);

// Padded geometry length for n spheres (see KernelParams::geo).
inline int32_t padded_spheres(int32_t n) { return ((n + 3) / 4) * 4 + 4; }

}  // namespace tray
