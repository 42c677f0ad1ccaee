// tray_abi.hip — the C-ABI (include/tray.h) around the megakernel.
//
// Replaces the hot half of (*Tracer).Render / RenderLines (ray/tracer.go:48-155):
// scene flattening + upload, one kernel launch per row set, copy-out. The Go
// host's defaulting (ray/tracer.go:50-84) happens BEFORE these calls, in the
// caller (tray_amd/ray.py or a cgo shim), exactly as Render does it.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tray.h"
#include "../../include/tray_debug.h"
#include "tray_internal.hpp"
#include "bvh.hpp"
#include "rng.hpp"
#include "tray_kernel.hpp"

namespace tray {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// tray_debug.h knobs: a value and a set bit per knob, read at each render.
static std::atomic<long long> g_knob_value[kKnobCount];
static std::atomic<bool> g_knob_set[kKnobCount];
static const char* const kKnobNames[kKnobCount] = {
    "acc_slots", "band_samples", "bvh_leaf", "bvh_lds_mode", "stack_lds_slots", "node_deep", "primary_candidates",
    "resolve_staged", "wave_chunks", "scene_contexts", "grid_reserve", "work_order", "coop_lanes"};

bool debug_knob(DebugKnob k, long long* v) {
    if (!g_knob_set[k].load(std::memory_order_acquire)) return false;
    *v = g_knob_value[k].load(std::memory_order_relaxed);
    return true;
}

static int knob_index(const char* name) {
    for (int i = 0; i < kKnobCount; ++i)
        if (name && strcmp(name, kKnobNames[i]) == 0) return i;
    return -1;
}

static int hip_fail(hipError_t e, const char* what) {
    return fail(TRAY_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define TRAY_HIP(call)                                  \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

// One render slot of a device for the synchronous entry points: a stream, the
// output workspaces, and the last scene the slot uploaded (reused while the
// caller passes the same scene again, as main.go does on every resize).
// tray_render uses slot 0; tray_render_devices uses slot j for the j-th time a
// device appears in its list (each slot's renders are ordered on its stream).
struct Slot {
    hipStream_t stream = nullptr;
    void* out_ws = nullptr;
    size_t out_ws_bytes = 0;
    uint32_t* seg_ws = nullptr;
    size_t seg_ws_bytes = 0;
    tray_scene_s* cached = nullptr;
    std::vector<tray_sphere> cached_spheres;
    tray_background cached_bg;
    // Live progress: samples finished per 8-row tile row of the slot's compact
    // rows, in host-mapped coherent memory the kernel adds to (system-scope
    // atomics) and the calling thread polls.
    unsigned long long* prog_host = nullptr;
    unsigned long long* prog_dev = nullptr;  // its device address
    size_t prog_bytes = 0;
};

// Per-device state: render slots and the sRGB encoder table of
// tray_linear_to_srgba_async.
struct DeviceState {
    std::mutex mu;
    bool checked = false;
    bool usable = false;
    std::deque<Slot> slots;  // a deque: growing it keeps references to existing slots valid
    double* srgb = nullptr;  // tray::srgb_thresholds on the device
    Slot& slot(size_t j) {
        if (slots.size() <= j) slots.resize(j + 1);
        return slots[j];
    }
};

static std::mutex g_devices_mu;
static std::vector<DeviceState*> g_devices;

// Set while a progress callback runs on this thread: the entry points that
// take a device's lock refuse to run from inside one (the render that called
// back still holds that lock), instead of deadlocking.
thread_local bool g_in_progress_callback = false;

static int refuse_reentry(const char* fn) {
    return fail(TRAY_ERR_INVALID_ARGUMENT,
                std::string(fn) + " called from a tray_progress_fn: the library is not re-entrant from its callbacks");
}

static int visible_devices(int* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        *count = 0;
        return TRAY_OK;
    }
    *count = n;
    return TRAY_OK;
}

static int device_state(int32_t device, DeviceState** out) {
    int n = 0;
    visible_devices(&n);
    if (n <= 0) return fail(TRAY_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(TRAY_ERR_INVALID_ARGUMENT, "device ordinal out of range");
    std::lock_guard<std::mutex> lk(g_devices_mu);
    if ((int)g_devices.size() < n) g_devices.resize(n, nullptr);
    if (!g_devices[device]) g_devices[device] = new DeviceState();
    DeviceState* st = g_devices[device];
    if (!st->checked) {
        hipDeviceProp_t prop;
        TRAY_HIP(hipGetDeviceProperties(&prop, device));
        st->usable = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
        st->checked = true;
        if (!st->usable)
            return fail(TRAY_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
        // The runtime sets up its path for pageable copies of >= 64 KB on their
        // first use (7-13 ms, tools/hip_h2d_costs.hip); a small first render
        // never triggers it, so without this the first render of a larger scene
        // would pay it. Paid here, with the device's other one-time costs.
        int prev = 0;
        (void)hipGetDevice(&prev);
        if (hipSetDevice(device) == hipSuccess) {
            constexpr size_t kWarmBytes = 256 << 10;
            std::vector<char> h(kWarmBytes, 0);
            void* d = nullptr;
            if (hipMalloc(&d, kWarmBytes) == hipSuccess) {
                (void)hipMemcpy(d, h.data(), kWarmBytes, hipMemcpyHostToDevice);
                (void)hipMemcpy(h.data(), d, kWarmBytes, hipMemcpyDeviceToHost);
                (void)hipFree(d);
            }
        }
        (void)hipSetDevice(prev);
    }
    if (!st->usable) return fail(TRAY_ERR_NO_DEVICE, "device is not gfx950");
    *out = st;
    return TRAY_OK;
}

int device_usable(int32_t device) {
    DeviceState* st = nullptr;
    return device_state(device, &st);
}

}  // namespace tray

// What a primary-ray candidate list depends on (compared byte for byte).
struct CandKey {
    tray_camera cam;
    double ray_radius;
    int32_t width, height, y_start, rows, tile_rows, tile_count, tile_index, multi_sample;
};

// The mutable device state ONE render uses while it runs: the work-queue word
// (zero between launches: zeroed at allocation, then by each band's resolve
// pass), the per-sample buffer or chunk records of a launch band, the primary-ray
// candidate records of the last camera and row set it rendered, and the
// traversal-stack overflow area (deep BVHs). `done` is recorded on the render's
// stream after each launch that used it. A scene holds a few of these, so that
// renders of one scene on different streams (or threads) run concurrently
// without sharing any of it, as several goroutines may Render one read-only
// *Scene at once (ray/tracer.go:48, ray/objects.go:37-46).
struct LaunchCtx {
    uint32_t* queue = nullptr;
    double* samples = nullptr;
    size_t samples_bytes = 0;
    uint4* cand = nullptr;
    size_t cand_bytes = 0;
    bool cand_valid = false;
    CandKey cand_key;
    uint32_t* stack_ovf = nullptr;
    size_t ovf_bytes = 0;
    // Work order (launch_render): per 8x8 tile of the rows, the Scene.Hit calls a
    // counting launch measured and the order the next launches hand tiles out in,
    // valid for `order_key` (camera, rows, tiling, rays per pixel, depth).
    uint32_t* tile_cost = nullptr;
    size_t tile_cost_bytes = 0;
    uint32_t* tile_order = nullptr;
    size_t tile_order_bytes = 0;
    bool order_valid = false;
    CandKey order_key;
    int32_t order_spp = 0, order_depth = 0;
    hipEvent_t done = nullptr;
    bool launched = false;          // `done` has been recorded
    hipStream_t last_stream = nullptr;
    uint64_t last_use = 0;          // the scene's launch count at its last launch
};

// Launch contexts per scene: renders beyond this many in flight at once wait
// (on the device, hipStreamWaitEvent) for the least recently used one.
constexpr int kSceneContexts = 4;

// A scene resident on one device. Its arrays are read-only after the upload;
// everything a render writes lives in a launch context (above), taken under the
// scene's mutex for the time it takes to enqueue the render.
struct tray_scene_s {
    int32_t device;
    int32_t n;
    int32_t n_pad;
    double4* geo;  // n_pad entries, NaN-padded (see tray::KernelParams::geo)
    tray::MatRec* mat;
    tray::V3 bg_a, bg_b;
    double max_att;  // max(1, |albedo| of every Lambertian/Metal sphere): bounds a path's throughput
    // exact-culling BVH (absent for tiny or non-finite scenes)
    bool has_bvh;
    double bvh_bound;
    int32_t n_nodes, n_slots, n_leaves, stack_cap, leaf_max, n_global;
    tray::Bvh4Node* nodes;
    int32_t* leaves;
    size_t ovf_bytes;  // traversal-stack overflow area a render needs (deep BVHs only; per context)
    double4* bgeo;
    int32_t* bidx;
    tray::MatRec* bmat;
    // One device allocation holds geo, mat, srgb and the BVH arrays (the pointers
    // above point into it).
    void* arena;
    double* srgb;  // the RGBA8 encoder table (tray::srgb_thresholds), 256 doubles
    std::mutex mu;  // guards ctx and launches
    std::vector<LaunchCtx*> ctx;
    uint64_t launches;
};

using namespace tray;

static int validate_spheres(const tray_sphere* s, int32_t n) {
    if (n < 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "negative sphere count");
    if (n > 0 && !s) return fail(TRAY_ERR_INVALID_ARGUMENT, "null sphere array");
    for (int32_t i = 0; i < n; ++i) {
        if (s[i].material < TRAY_LAMBERTIAN || s[i].material > TRAY_DIELECTRIC)
            return fail(TRAY_ERR_UNSUPPORTED, "sphere " + std::to_string(i) + ": unsupported material kind " +
                                                  std::to_string(s[i].material));
        if (s[i].reserved != 0)
            return fail(TRAY_ERR_INVALID_ARGUMENT, "sphere " + std::to_string(i) + ": reserved field must be 0");
    }
    return TRAY_OK;
}

static int validate_params(const tray_params* p) {
    if (!p) return fail(TRAY_ERR_INVALID_ARGUMENT, "null params");
    if (p->width <= 0 || p->height <= 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "width/height must be > 0");
    if ((uint64_t)p->width * (uint64_t)p->height > 0xFFFFFFFFull)
        return fail(TRAY_ERR_TOO_LARGE, "image has more than 2^32 pixels (RNG pixel counter is 32-bit)");
    if (p->max_depth <= 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "max_depth must be > 0 (Render defaults it to 10)");
    if (p->rays_per_pixel <= 0)
        return fail(TRAY_ERR_INVALID_ARGUMENT, "rays_per_pixel must be > 0 (Render defaults it to 1)");
    if (!std::isfinite(p->ray_radius)) return fail(TRAY_ERR_INVALID_ARGUMENT, "ray_radius must be finite");
    if (p->y_start < 0 || p->y_end > p->height || p->y_start > p->y_end)
        return fail(TRAY_ERR_INVALID_ARGUMENT, "row range outside the image");
    if (p->tile_rows < 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "tile_rows must be >= 0");
    if (p->tile_rows > 0 && (p->tile_count < 1 || p->tile_index < 0 || p->tile_index >= p->tile_count))
        return fail(TRAY_ERR_INVALID_ARGUMENT, "tile_index must be in [0, tile_count)");
    if (p->output < TRAY_OUT_RGB_F64 || p->output > TRAY_OUT_RGBA8)
        return fail(TRAY_ERR_INVALID_ARGUMENT, "unknown output format");
    if (p->flags & ~(TRAY_FLAG_LINEAR_SCAN | TRAY_FLAG_ORDERED_SUM))
        return fail(TRAY_ERR_INVALID_ARGUMENT, "unknown flags");
    if (p->pass < 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "pass must be >= 0");
    if (((uint64_t)p->pass + 1u) * (uint64_t)p->rays_per_pixel > 0x100000000ull)
        return fail(TRAY_ERR_TOO_LARGE, "pass x rays_per_pixel exceeds the 32-bit RNG sample word");
    return TRAY_OK;
}

static size_t bytes_per_pixel(int32_t fmt) {
    return fmt == TRAY_OUT_RGB_F64 ? 24 : fmt == TRAY_OUT_RGB_F32 ? 12 : 4;
}

extern "C" {
#pragma GCC visibility push(default)

int32_t tray_abi_version(void) { return TRAY_ABI_VERSION; }

int tray_debug_set(const char* name, int64_t value) {
    const int i = knob_index(name);
    if (i < 0) return fail(TRAY_ERR_INVALID_ARGUMENT, std::string("unknown debug knob: ") + (name ? name : "(null)"));
    g_knob_value[i].store((long long)value, std::memory_order_relaxed);
    g_knob_set[i].store(true, std::memory_order_release);
    return TRAY_OK;
}

int tray_debug_clear(const char* name) {
    if (!name) {
        for (int i = 0; i < kKnobCount; ++i) g_knob_set[i].store(false, std::memory_order_release);
        return TRAY_OK;
    }
    const int i = knob_index(name);
    if (i < 0) return fail(TRAY_ERR_INVALID_ARGUMENT, std::string("unknown debug knob: ") + name);
    g_knob_set[i].store(false, std::memory_order_release);
    return TRAY_OK;
}

const char* tray_last_error(void) { return g_last_error.c_str(); }

int tray_device_count(int32_t* count) {
    if (!count) return fail(TRAY_ERR_INVALID_ARGUMENT, "null count");
    int n = 0;
    visible_devices(&n);
    int usable = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++usable;
    }
    *count = usable;
    return TRAY_OK;
}

int32_t tray_params_rows(const tray_params* p) {
    if (!p || p->y_end <= p->y_start) return 0;
    const int32_t total = p->y_end - p->y_start;
    if (p->tile_rows <= 0) return total;
    if (p->tile_count < 1 || p->tile_index < 0 || p->tile_index >= p->tile_count) return 0;
    const int32_t ntiles = (total + p->tile_rows - 1) / p->tile_rows;
    int32_t rows = 0;
    for (int32_t t = p->tile_index; t < ntiles; t += p->tile_count) {
        const int32_t left = total - t * p->tile_rows;
        rows += left < p->tile_rows ? left : p->tile_rows;
    }
    return rows;
}

int tray_scene_upload(const tray_sphere* spheres, int32_t n, const tray_background* bg, int32_t device,
                      tray_scene_t* out) {
    if (!out || !bg) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    int rc = validate_spheres(spheres, n);
    if (rc) return rc;
    DeviceState* st = nullptr;
    rc = device_state(device, &st);
    if (rc) return rc;
    TRAY_HIP(hipSetDevice(device));
    const int32_t n_pad = padded_spheres(n);
    const double qnan = std::nan("");
    std::vector<double4> geo((size_t)n_pad, make_double4(qnan, qnan, qnan, qnan));
    std::vector<MatRec> mat((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        const tray_sphere& s = spheres[i];
        // R*R precomputed: identical bits to Sphere.Hit's s.Radius*s.Radius (ray/objects.go:85).
        geo[i] = make_double4(s.center[0], s.center[1], s.center[2], s.radius * s.radius);
        MatRec& m = mat[i];
        m.albedo[0] = s.albedo[0];
        m.albedo[1] = s.albedo[1];
        m.albedo[2] = s.albedo[2];
        m.param = s.param;
        m.radius = s.radius;
        m.rinv = 1.0 / s.radius;  // correctly rounded on the host
        m.pinv = 1.0 / s.param;
        if (s.material == TRAY_DIELECTRIC) {  // Reflectance's r0 for both faces (same ops as the kernel)
            for (int f = 0; f < 2; ++f) {
                const double ref_idx = f == 0 ? m.pinv : s.param;
                double r0 = (1 - ref_idx) / (1 + ref_idx);
                r0 *= r0;
                m.albedo[f] = r0;
            }
        }
        m.type = s.material;
        m.pad = 0;
    }
    // The leaf size whose LDS plan ranks best (tray_kernel.hip bvh_lds_plan),
    // the smallest on ties: one sphere per leaf while the scene and its stack
    // fit the CU's LDS, else a few spheres per leaf (fewer nodes).
    Bvh bvh;
    bool has_bvh = false;
    if (n >= kBvhMinSpheres) {
        int rank = -1, leaf_lo = 1, leaf_hi = kBvhLeafMax;
        long long leaf = 0;
        if (debug_knob(kKnobBvhLeaf, &leaf))  // A/B: one leaf size only
            leaf_lo = leaf_hi = (int)std::max(1LL, std::min((long long)kBvhLeafMax, leaf));
        for (int leaf_max = leaf_lo; leaf_max <= leaf_hi; leaf_max *= 2) {
            Bvh b;
            if (!build_bvh(spheres, n, &b, leaf_max)) continue;
            const int32_t cap = b.stack_max + kStackSlack;  // + scratch slots (tray_kernel.hpp)
            if (bvh_scene_lds_bytes(0, 0, 0, cap) > kMaxLDSBytes) continue;  // stack alone too deep
            const int r = bvh_lds_plan((int32_t)b.nodes.size(), (int32_t)b.geo.size(), (int32_t)b.leaves.size(), cap).rank;
            if (r > rank) {
                bvh = std::move(b);
                has_bvh = true;
                rank = r;
            }
            if (rank == 4) break;
        }
    }
    tray_scene_s* sc = new tray_scene_s();
    sc->device = device;
    sc->has_bvh = has_bvh;
    sc->bvh_bound = bvh.bound;
    sc->n_nodes = (int32_t)bvh.nodes.size();
    sc->n_slots = (int32_t)bvh.geo.size();
    sc->n_leaves = (int32_t)bvh.leaves.size();
    sc->leaves = nullptr;
    sc->ovf_bytes = 0;
    sc->launches = 0;
    sc->stack_cap = bvh.stack_max + kStackSlack;
    sc->leaf_max = has_bvh ? bvh.leaf_max : 0;
    sc->n_global = has_bvh ? bvh.n_global : 0;
    sc->nodes = nullptr;
    sc->bgeo = nullptr;
    sc->bidx = nullptr;
    sc->bmat = nullptr;
    sc->srgb = nullptr;
    std::vector<MatRec> bmat(bvh.idx.size());
    for (size_t i = 0; i < bvh.idx.size(); ++i) {
        const int32_t k = bvh.idx[i];
        if (k >= 0 && k < n) bmat[i] = mat[(size_t)k];
        else memset(&bmat[i], 0, sizeof(MatRec));
    }
    sc->n = n;
    sc->n_pad = n_pad;
    sc->geo = nullptr;
    sc->mat = nullptr;
    sc->max_att = 1.0;
    for (int32_t i = 0; i < n; ++i)
        if (spheres[i].material != TRAY_DIELECTRIC)  // Dielectric attenuates by exactly 1
            for (int c = 0; c < 3; ++c) {
                const double a = std::fabs(spheres[i].albedo[c]);
                sc->max_att = a > sc->max_att || a != a ? (a != a ? HUGE_VAL : a) : sc->max_att;
            }
    sc->bg_a = V3{bg->color_a[0], bg->color_a[1], bg->color_a[2]};
    sc->bg_b = V3{bg->color_b[0], bg->color_b[1], bg->color_b[2]};
    // One arena, filled from one host image with one copy: eleven allocations
    // and seven synchronous copies took the C2 upload from 0.31 to 0.44 ms
    // (tools/e2e_breakdown.py, profiles/r2g_e2e_breakdown.jsonl).
    struct Part {
        void** dst;
        const void* src;  // nullptr: zeros
        size_t bytes;
    };
    const Part parts[] = {
        {(void**)&sc->geo, geo.data(), sizeof(double4) * (size_t)n_pad},
        {(void**)&sc->srgb, srgb_thresholds(), 256 * sizeof(double)},
        {(void**)&sc->mat, mat.data(), sizeof(MatRec) * (size_t)n},
        {(void**)&sc->nodes, bvh.nodes.data(), has_bvh ? sizeof(Bvh4Node) * bvh.nodes.size() : 0},
        {(void**)&sc->leaves, bvh.leaves.data(), has_bvh ? sizeof(int32_t) * bvh.leaves.size() : 0},
        {(void**)&sc->bgeo, bvh.geo.data(), has_bvh ? sizeof(double4) * bvh.geo.size() : 0},
        {(void**)&sc->bidx, bvh.idx.data(), has_bvh ? sizeof(int32_t) * bvh.idx.size() : 0},
        {(void**)&sc->bmat, bmat.data(), has_bvh ? sizeof(MatRec) * bmat.size() : 0},
    };
    constexpr size_t kAlign = 256;
    size_t total = 0;
    for (const Part& q : parts) total += (q.bytes + kAlign - 1) / kAlign * kAlign;
    std::vector<uint8_t> image(total, 0);
    size_t at = 0;
    std::vector<size_t> offsets;
    for (const Part& q : parts) {
        offsets.push_back(at);
        if (q.src && q.bytes) memcpy(image.data() + at, q.src, q.bytes);
        at += (q.bytes + kAlign - 1) / kAlign * kAlign;
    }
    sc->arena = nullptr;
    hipError_t e = hipMalloc(&sc->arena, total);
    if (e == hipSuccess) e = hipMemcpy(sc->arena, image.data(), total, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        for (size_t i = 0; i < sizeof(parts) / sizeof(parts[0]); ++i)  // empty arrays stay null
            *parts[i].dst = parts[i].bytes ? static_cast<uint8_t*>(sc->arena) + offsets[i] : nullptr;
    }
    if (has_bvh) sc->ovf_bytes = bvh_stack_overflow_bytes(bvh.stack_max + kStackSlack, device);
    if (e != hipSuccess) {
        (void)hipFree(sc->arena);
        delete sc;
        return hip_fail(e, "scene upload");
    }
    *out = sc;
    return TRAY_OK;
}

int tray_scene_get_info(tray_scene_t sc, tray_scene_info* out) {
    if (!sc || !out) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof(*out));
    out->n_spheres = sc->n;
    out->has_bvh = sc->has_bvh ? 1 : 0;
    out->leaf_max = sc->leaf_max;
    out->n_nodes = sc->n_nodes;
    out->n_leaves = sc->n_leaves;
    out->stack_depth = sc->has_bvh ? sc->stack_cap - kStackSlack : 0;
    out->lds_resident = sc->has_bvh ? bvh_lds_plan(sc->n_nodes, sc->n_slots, sc->n_leaves, sc->stack_cap).mode : 0;
    out->n_global = sc->n_global;
    out->bound = sc->bvh_bound;
    return TRAY_OK;
}

static void free_ctx(LaunchCtx* c) {
    if (c->launched) (void)hipEventSynchronize(c->done);  // its last render, on whatever stream
    if (c->queue) (void)hipFree(c->queue);
    // Pool allocations (grow_ctx_buffer), idle now: released on the null stream.
    for (void* b : {(void*)c->samples, (void*)c->cand, (void*)c->stack_ovf, (void*)c->tile_cost, (void*)c->tile_order})
        if (b) (void)hipFreeAsync(b, nullptr);
    if (c->done) (void)hipEventDestroy(c->done);
    delete c;
}

int tray_scene_release(tray_scene_t sc) {
    if (!sc) return TRAY_OK;
    (void)hipSetDevice(sc->device);
    {
        std::lock_guard<std::mutex> lk(sc->mu);
        for (LaunchCtx* c : sc->ctx) free_ctx(c);  // waits for the renders still enqueued
        sc->ctx.clear();
    }
    if (sc->arena) (void)hipFree(sc->arena);
    delete sc;
    return TRAY_OK;
}

// Primary-ray candidate lists (on unless the "primary_candidates" knob is 0, an
// A/B and test switch), for scenes whose tree has at most kCandMaxSpheres
// spheres (the build tests every tree sphere against every 8x8 tile's beam).
constexpr int32_t kCandMaxSpheres = 16384;
static bool cand_enabled() {
    long long v = 1;
    return !debug_knob(kKnobPrimaryCandidates, &v) || v != 0;
}
// Expensive-first work order (on unless the "work_order" knob is 0, an A/B and test switch).
static bool work_order_enabled() {
    long long v = 1;
    return !debug_knob(kKnobWorkOrder, &v) || v != 0;
}

// The fixed-point scale 2^k of a render (tray_kernel.hpp), or 0 for the FP64
// sum in sample order. Fixed point needs 64 | rays_per_pixel or rays_per_pixel
// 16 / 32 (acc_groupable: a 64-item chunk is then part of one pixel-pass or
// whole pixel-passes) and a colour bound that leaves k >= kAccMinShift:
// a sample's colour is its throughput (a product of <= max_depth attenuations,
// each <= max_att) times a convex combination of the two background colours,
// so |c| <= C = max|bg| * max_att^max_depth (x 1.001 for rounding). k is the
// largest shift with C * 2^k <= 2^kAccBits (tray_kernel.hpp).
// TRAY_FLAG_ORDERED_SUM selects the FP64 sum in sample order (include/tray.h).
static int32_t fixed_point_shift(const tray_scene_s* sc, const tray_params* p) {
    if (!acc_groupable(p->rays_per_pixel)) return 0;
    if (p->flags & TRAY_FLAG_ORDERED_SUM) return 0;
    double bg = 0.0;
    const double comps[6] = {sc->bg_a.x, sc->bg_a.y, sc->bg_a.z, sc->bg_b.x, sc->bg_b.y, sc->bg_b.z};
    for (double c : comps) {
        if (!std::isfinite(c)) return 0;
        bg = std::max(bg, std::fabs(c));
    }
    if (!std::isfinite(sc->max_att)) return 0;
    const double bound = bg * std::pow(sc->max_att, (double)p->max_depth) * 1.001;
    if (!(bound < 0x1p20)) return 0;
    int e = 0;
    std::frexp(std::max(bound, 0x1p-300), &e);  // bound < 2^e
    if (p->rays_per_pixel > (1 << 15)) return 0;  // the pixel's total r x 2^47 must stay below 2^63
    const int32_t k = kAccBits - e;
    return k >= kAccMinShift ? std::min(k, 600) : 0;
}

// The kernel parameters of a render of `p` on `sc` (everything but the output,
// instrumentation and workspace pointers) and whether it runs the BVH kernel.
static int prepare_render(tray_scene_t sc, const tray_camera* cam, const tray_params* p, int32_t n_passes,
                          KernelParams& k, bool& use_bvh) {
    if (!sc || !cam) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    int rc = validate_params(p);
    if (rc) return rc;
    if (n_passes < 1) return fail(TRAY_ERR_INVALID_ARGUMENT, "n_passes must be >= 1");
    if (((uint64_t)p->pass + (uint64_t)n_passes) * (uint64_t)p->rays_per_pixel > 0x100000000ull)
        return fail(TRAY_ERR_TOO_LARGE, "(pass + n_passes) x rays_per_pixel exceeds the 32-bit RNG sample word");
    const uint64_t spp_launch = (uint64_t)p->rays_per_pixel * (uint64_t)n_passes;
    if (!band_fits(p->width, spp_launch))
        return fail(TRAY_ERR_TOO_LARGE, "width x rays_per_pixel x passes too large (8 rows of samples exceed 2^31)");
    memset(&k, 0, sizeof(k));
    k.geo = sc->geo;
    k.mat = sc->mat;
    k.n = sc->n;
    k.n_pad = sc->n_pad;
    k.width = p->width;
    k.height = p->height;
    k.spp = p->rays_per_pixel;
    k.max_depth = p->max_depth;
    k.y_start = p->y_start;
    k.rows = tray_params_rows(p);
    k.tile_rows = p->tile_rows;
    k.tile_count = p->tile_rows > 0 ? p->tile_count : 1;
    k.tile_index = p->tile_rows > 0 ? p->tile_index : 0;
    k.out_format = p->output;
    k.ray_radius = p->ray_radius;
    k.focus_time = cam->focus_distance / cam->focal_length;  // ray/camera.go:134
    {
        const DrawKey dk = draw_key(p->seed);  // include/tray.h, ABI 6
        k.key[0] = dk.k0, k.key[1] = dk.k1, k.key[2] = dk.k2, k.key[3] = dk.k3;
    }
    memcpy(k.cam.position, cam->position, sizeof(k.cam.position));
    memcpy(k.cam.pixel00, cam->pixel00, sizeof(k.cam.pixel00));
    memcpy(k.cam.pixel_x, cam->pixel_x, sizeof(k.cam.pixel_x));
    memcpy(k.cam.pixel_y, cam->pixel_y, sizeof(k.cam.pixel_y));
    memcpy(k.cam.defocus_u, cam->defocus_u, sizeof(k.cam.defocus_u));
    memcpy(k.cam.defocus_v, cam->defocus_v, sizeof(k.cam.defocus_v));
    k.cam.aperture = cam->aperture;
    k.bg_a = sc->bg_a;
    k.bg_b = sc->bg_b;
    k.acc_shift = fixed_point_shift(sc, p);
    if (k.acc_shift > 0) {  // the scale rides on the background: every colour is then scaled (exactly)
        for (V3* v : {&k.bg_a, &k.bg_b}) {
            v->x = std::ldexp(v->x, k.acc_shift);
            v->y = std::ldexp(v->y, k.acc_shift);
            v->z = std::ldexp(v->z, k.acc_shift);
        }
    }
    k.passes = (uint32_t)n_passes;
    k.pass0 = (uint32_t)p->pass;
    k.out_frame_bytes = (size_t)k.rows * (size_t)p->width * bytes_per_pixel(p->output);
    k.srgb = sc->srgb;
    k.nodes = sc->nodes;
    k.bgeo = sc->bgeo;
    k.bidx = sc->bidx;
    k.bmat = sc->bmat;
    k.n_nodes = sc->n_nodes;
    k.n_slots = sc->n_slots;
    k.n_leaves = sc->n_leaves;
    k.n_global = sc->n_global;
    k.leaves = sc->leaves;
    k.leaf_single = sc->leaf_max == 1 ? 1 : 0;
    k.stack_cap = sc->stack_cap;
    {
        long long coop = TRAY_COOP_LANES;
        (void)debug_knob(kKnobCoopLanes, &coop);  // A/B and tests: the drain's wave-wide Scene.Hit
        k.coop_lanes = (uint32_t)std::max(0LL, std::min(coop, 64LL));
    }
    // The BVH's conservative FP32 box test assumes every ray origin lies within
    // [-M, M]^3 (tray_bvh.cpp): hit points do; check the camera and lens disc.
    double cam_extent = 0;
    for (int i = 0; i < 3; ++i) cam_extent = std::max(cam_extent, std::fabs(cam->position[i]));
    cam_extent += std::fabs(cam->defocus_u[0]) + std::fabs(cam->defocus_u[1]) + std::fabs(cam->defocus_u[2]) +
                  std::fabs(cam->defocus_v[0]) + std::fabs(cam->defocus_v[1]) + std::fabs(cam->defocus_v[2]);
    use_bvh = sc->has_bvh && !(p->flags & TRAY_FLAG_LINEAR_SCAN) && cam_extent <= sc->bvh_bound;
    return TRAY_OK;
}

// The scene's launch context for a render on `stream` (called with sc->mu held):
// the one last used on this stream (stream order already serialises it), else
// an idle one (never launched, or its last render has finished), else a new one
// while the scene has fewer than kSceneContexts, else the least recently used,
// which the stream then waits for on the device. Either way the stream is made
// to wait for the context's last render, so nothing it enqueues can overlap it.
static int take_ctx(tray_scene_t sc, hipStream_t stream, LaunchCtx** out) {
    long long cap = kSceneContexts;
    if (debug_knob(kKnobSceneContexts, &cap)) cap = std::max(1LL, std::min(cap, 64LL));
    LaunchCtx* pick = nullptr;
    for (LaunchCtx* c : sc->ctx)
        if (c->launched && c->last_stream == stream && (!pick || c->last_use > pick->last_use)) pick = c;
    if (!pick)
        for (LaunchCtx* c : sc->ctx)
            if ((!c->launched || hipEventQuery(c->done) == hipSuccess) && (!pick || c->last_use > pick->last_use))
                pick = c;
    if (!pick && (long long)sc->ctx.size() < cap) {
        LaunchCtx* c = new LaunchCtx();
        hipError_t e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->queue), 256);
        // Zeroed in the render's stream order: a hipMemset on the null stream is not
        // ordered before a launch on a non-blocking stream.
        if (e == hipSuccess) e = hipMemsetAsync(c->queue, 0, sizeof(uint32_t), stream);
        if (e == hipSuccess) e = hipEventRecord(c->done, stream);  // a later user waits for the zeroing
        if (e == hipSuccess) {
            c->launched = true;
            c->last_stream = stream;
        }
        if (e != hipSuccess) {
            free_ctx(c);
            return hip_fail(e, "launch context");
        }
        sc->ctx.push_back(c);
        pick = c;
    }
    if (!pick)
        for (LaunchCtx* c : sc->ctx)
            if (!pick || c->last_use < pick->last_use) pick = c;
    if (pick->launched && hipEventQuery(pick->done) != hipSuccess)
        TRAY_HIP(hipStreamWaitEvent(stream, pick->done, 0));
    *out = pick;
    return TRAY_OK;
}

// Grows a context buffer to `bytes` (contents not kept) in the order of the
// render's `stream`, without blocking the host: the old buffer goes back with
// hipFreeAsync on `stream`, which take_ctx has already ordered after the
// context's last render (hipStreamWaitEvent on its event, or stream order when
// that render ran on `stream`), and the new one comes from the device's
// stream-ordered pool (hipMallocAsync). A plain hipFree synchronises the whole
// device on ROCm: under the scene's mutex it held this thread, and every other
// thread enqueueing on the scene, until the longest render in flight ended
// (include/tray.h presents the async calls as enqueue-only). Every context
// buffer is a pool allocation, so free_ctx releases them the same way.
static hipError_t grow_ctx_buffer(void** buf, size_t* have, size_t bytes, hipStream_t stream) {
    if (*have >= bytes) return hipSuccess;
    if (*buf) {
        const hipError_t e = hipFreeAsync(*buf, stream);
        if (e != hipSuccess) return e;
        *buf = nullptr;
        *have = 0;
    }
    const hipError_t e = hipMallocAsync(buf, bytes, stream);
    if (e == hipSuccess) *have = bytes;
    else *buf = nullptr;
    return e;
}

static int render_async_impl(tray_scene_t sc, const tray_camera* cam, const tray_params* p, void* out_device,
                             uint32_t* segments_device, unsigned long long* stats_device, void* stream_arg,
                             int32_t n_passes = 1, unsigned long long* progress_device = nullptr) {
    if (!out_device) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    KernelParams k;
    bool use_bvh = false;
    int rc = prepare_render(sc, cam, p, n_passes, k, use_bvh);
    if (rc) return rc;
    k.out = out_device;
    k.segments = segments_device;
    k.stats = stats_device;
    k.progress = progress_device;
    const hipStream_t stream = static_cast<hipStream_t>(stream_arg);
    TRAY_HIP(hipSetDevice(sc->device));
    const LaunchPlan plan = plan_launch(k, use_bvh);  // decided once: the buffer and the bands agree
    std::lock_guard<std::mutex> lk(sc->mu);
    LaunchCtx* c = nullptr;
    rc = take_ctx(sc, stream, &c);
    if (rc) return rc;
    // From here on something may be enqueued on `stream` that uses the context
    // (its queue zeroing, a candidate build, a band): every exit records the
    // context's event after it, so the next user waits for it.
    auto finish = [&](hipError_t e, const char* what) -> int {
        const hipError_t r = hipEventRecord(c->done, stream);
        c->launched = c->launched || r == hipSuccess;
        c->last_stream = stream;
        c->last_use = ++sc->launches;
        if (e == hipSuccess && r != hipSuccess) {  // nothing marks the render's end: wait for it here
            (void)hipStreamSynchronize(stream);
            e = r;
            what = "hipEventRecord";
        }
        if (e != hipSuccess) {
            if (r != hipSuccess) (void)hipStreamSynchronize(stream);
            return hip_fail(e, what);
        }
        return TRAY_OK;
    };
    hipError_t e = grow_ctx_buffer(reinterpret_cast<void**>(&c->samples), &c->samples_bytes, plan.buffer_bytes, stream);
    if (e == hipSuccess && use_bvh && k.stack_cap > plan.layout.stack_lds)
        e = grow_ctx_buffer(reinterpret_cast<void**>(&c->stack_ovf), &c->ovf_bytes, sc->ovf_bytes, stream);
    if (e != hipSuccess) return finish(e, "launch context buffers");
    k.queue = c->queue;
    k.samples = c->samples;
    k.stack_ovf = c->stack_ovf;
    CandKey key;  // what the candidate records (and, with r and depth, the work order) depend on
    memset(&key, 0, sizeof(key));
    key.cam = *cam;
    key.ray_radius = p->ray_radius;
    key.width = p->width, key.height = p->height, key.y_start = p->y_start, key.rows = k.rows;
    key.tile_rows = k.tile_rows, key.tile_count = k.tile_count, key.tile_index = k.tile_index;
    key.multi_sample = p->rays_per_pixel > 1;
    // Work order: the order a counting launch of this key measured, else (with on-chip
    // sums) count now; the frame's bits do not depend on the order.
    uint32_t* order_out = nullptr;
    bool counting = false;
    // One launch band only: an order lists the band's tiles, so it holds for any launch of
    // the key with the same (single) band; multi-band launches (C3-C5 at 16 frames) keep
    // band order and neither use nor count one.
    // Live progress (tray_render_progress) keeps band order too: rows then finish from the
    // top as in Go's RenderLines (ray/tracer.go:126-128), where cost order would finish every
    // row near the end.
    const bool one_band = (int64_t)plan.band_tiles * 8 >= (int64_t)k.rows;
    if (work_order_enabled() && one_band && !progress_device) {
        const size_t tile_bytes = (size_t)((p->width + 7) / 8) * (size_t)((k.rows + 7) / 8) * sizeof(uint32_t);
        const bool same = c->order_valid && c->order_spp == p->rays_per_pixel && c->order_depth == p->max_depth &&
                          memcmp(&key, &c->order_key, sizeof(key)) == 0 && c->tile_order_bytes >= tile_bytes;
        if (same) {
            k.tile_order = c->tile_order;
        } else if (plan.layout.acc_slots > 0) {
            c->order_valid = false;
            e = grow_ctx_buffer(reinterpret_cast<void**>(&c->tile_cost), &c->tile_cost_bytes, tile_bytes, stream);
            if (e == hipSuccess)
                e = grow_ctx_buffer(reinterpret_cast<void**>(&c->tile_order), &c->tile_order_bytes, tile_bytes, stream);
            if (e == hipSuccess) e = hipMemsetAsync(c->tile_cost, 0, tile_bytes, stream);
            if (e != hipSuccess) return finish(e, "work order buffers");
            k.tile_cost = c->tile_cost;
            order_out = c->tile_order;
            counting = true;
        }
    }
    if (use_bvh && cand_enabled() && sc->n_slots - sc->n_global <= kCandMaxSpheres) {
        if (!c->cand_valid || memcmp(&key, &c->cand_key, sizeof(key)) != 0) {
            c->cand_valid = false;
            e = grow_ctx_buffer(reinterpret_cast<void**>(&c->cand), &c->cand_bytes,
                                cand_workspace_bytes(p->width, k.rows), stream);
            if (e == hipSuccess) e = launch_cand_build(k, c->cand, stream);
            if (e != hipSuccess) return finish(e, "candidate lists");
            c->cand_key = key;
            c->cand_valid = true;
        }
        k.cand = c->cand;
    }
    e = launch_render(k, use_bvh, plan, stream, c->samples_bytes, order_out);
    if (e == hipSuccess && counting) {  // the next launch of this key hands its tiles out by cost
        c->order_valid = true;
        c->order_key = key;
        c->order_spp = p->rays_per_pixel;
        c->order_depth = p->max_depth;
    }
    return finish(e, "launch_render");
}

int tray_render_plan_get(tray_scene_t sc, const tray_camera* cam, const tray_params* p, int32_t n_passes,
                         tray_render_plan* out) {
    if (!out) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof(*out));
    KernelParams k;
    bool use_bvh = false;
    int rc = prepare_render(sc, cam, p, n_passes, k, use_bvh);
    if (rc) return rc;
    const LaunchPlan plan = plan_launch(k, use_bvh);
    const LaunchLayout& L = plan.layout;
    out->fixed_point_shift = k.acc_shift;
    out->acc_slots = L.acc_slots;
    out->bvh = use_bvh ? 1 : 0;
    out->lds_layout = L.lds_mode;
    out->stack_lds = use_bvh ? L.stack_lds : 0;
    out->lds_bytes = (int64_t)L.lds;
    out->buffer_bytes = (int64_t)plan.buffer_bytes;
    return TRAY_OK;
}

int tray_render_async(tray_scene_t sc, const tray_camera* cam, const tray_params* p, void* out_device,
                      uint32_t* segments_device, void* stream) {
    return render_async_impl(sc, cam, p, out_device, segments_device, nullptr, stream);
}

int tray_render_passes_async(tray_scene_t sc, const tray_camera* cam, const tray_params* p, int32_t n_passes,
                             void* out_device, void* stream) {
    return render_async_impl(sc, cam, p, out_device, nullptr, nullptr, stream, n_passes);
}

int tray_render_stats_async(tray_scene_t sc, const tray_camera* cam, const tray_params* p, float* out_device,
                            uint64_t* stats_device, void* stream) {
    if (!stats_device) return fail(TRAY_ERR_INVALID_ARGUMENT, "null stats");
    if (!p) return fail(TRAY_ERR_INVALID_ARGUMENT, "null params");
    tray_params q = *p;
    q.output = TRAY_OUT_RGB_F32;
    return render_async_impl(sc, cam, &q, out_device, nullptr, reinterpret_cast<unsigned long long*>(stats_device),
                             stream);
}

// Grows a device workspace to `bytes` (contents not kept).
static hipError_t grow(void** buf, size_t* have, size_t bytes) {
    if (*have >= bytes) return hipSuccess;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    const hipError_t e = hipMalloc(buf, bytes);
    if (e == hipSuccess) *have = bytes;
    return e;
}

// The scene of a slot: its cached upload when the caller passes the same
// spheres and background as last time (compared byte for byte; the caller's
// arrays are copied, never retained), else a fresh upload that replaces it.
// Called with the device's mutex held.
static int cached_scene(Slot& sl, const tray_sphere* spheres, int32_t n, const tray_background* bg, int32_t device,
                        tray_scene_t* out) {
    const bool same = sl.cached && (int32_t)sl.cached_spheres.size() == n &&
                      (n == 0 || memcmp(sl.cached_spheres.data(), spheres, sizeof(tray_sphere) * (size_t)n) == 0) &&
                      memcmp(&sl.cached_bg, bg, sizeof(*bg)) == 0;
    if (!same) {
        tray_scene_t old = sl.cached;
        sl.cached = nullptr;
        sl.cached_spheres.clear();
        tray_scene_t sc = nullptr;
        const int rc = tray_scene_upload(spheres, n, bg, device, &sc);
        if (rc) {
            if (old) tray_scene_release(old);
            return rc;
        }
        if (old) {
            // The slot's renders are synchronous, so the old scene's launch
            // contexts are idle: the new scene takes them over (their sample and
            // candidate buffers) instead of allocating its own (a C2 frame's 1.4-GB
            // sample buffer: 0.28 ms of hipFree + hipMalloc per new scene,
            // profiles/r2g_e2e_breakdown.jsonl). Their candidate lists and work
            // orders were the old scene's.
            {
                std::lock_guard<std::mutex> la(old->mu);
                std::lock_guard<std::mutex> lb(sc->mu);
                std::swap(sc->ctx, old->ctx);
                std::swap(sc->launches, old->launches);
                for (LaunchCtx* c : sc->ctx) c->cand_valid = c->order_valid = false;
            }
            tray_scene_release(old);
        }
        sl.cached = sc;
        if (n > 0) sl.cached_spheres.assign(spheres, spheres + n);
        sl.cached_bg = *bg;
    }
    *out = sl.cached;
    return TRAY_OK;
}

// Stream and output workspaces of a slot for `npix` pixels.
static hipError_t prepare_slot(Slot& sl, size_t out_bytes, size_t seg_bytes) {
    hipError_t e = hipSuccess;
    if (!sl.stream) e = hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = grow(&sl.out_ws, &sl.out_ws_bytes, out_bytes);
    if (e == hipSuccess && seg_bytes) e = grow(reinterpret_cast<void**>(&sl.seg_ws), &sl.seg_ws_bytes, seg_bytes);
    return e;
}

// The slot's progress counters for `rows` compact rows (one per 8-row tile row),
// zeroed. The slot's stream is idle here (synchronous entry points only).
static hipError_t prepare_progress(Slot& sl, int32_t rows) {
    const size_t bytes = (size_t)((rows + 7) / 8) * sizeof(unsigned long long);
    if (sl.prog_bytes < bytes) {
        if (sl.prog_host) (void)hipHostFree(sl.prog_host);
        sl.prog_host = nullptr;
        sl.prog_dev = nullptr;
        sl.prog_bytes = 0;
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&sl.prog_host), bytes,
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&sl.prog_dev), sl.prog_host, 0);
        if (e != hipSuccess) return e;
        sl.prog_bytes = bytes;
    }
    memset(sl.prog_host, 0, bytes);
    return hipSuccess;
}

// One rendering shard whose progress counters the calling thread polls.
struct ProgressWatch {
    int device;
    Slot* slot;
    int32_t rows;        // compact rows of the shard
    uint64_t per_row;    // samples of one row: width x rays_per_pixel
    std::vector<uint8_t> done;  // per tile row: reported
};

// Poll every watched shard's counters until all their streams are idle, and
// report the rows of each tile row whose samples have all finished
// (ProgressFunc, ray/tracer.go:126-128: per row, while rendering). A
// device-to-host copy could not be used: it would queue behind the persistent
// grid that holds every CU. Returns the rows reported; `e` gets a stream error.
static int32_t poll_progress(std::vector<ProgressWatch>& ws, tray_progress_fn progress, void* user, hipError_t& e) {
    int32_t reported = 0;
    for (ProgressWatch& w : ws) w.done.assign((size_t)((w.rows + 7) / 8), 0);
    while (true) {
        bool busy = false;
        for (ProgressWatch& w : ws) {
            (void)hipSetDevice(w.device);
            const hipError_t q = hipStreamQuery(w.slot->stream);
            if (q == hipErrorNotReady) busy = true;
            else if (q != hipSuccess && e == hipSuccess) e = q;
        }
        if (!busy || e != hipSuccess) break;
        std::this_thread::sleep_for(std::chrono::microseconds(500));
        int32_t fresh = 0;
        for (ProgressWatch& w : ws) {
            const volatile unsigned long long* counts = w.slot->prog_host;
            for (size_t t = 0; t < w.done.size(); ++t) {
                const int32_t r = std::min(8, w.rows - 8 * (int32_t)t);
                if (!w.done[t] && (uint64_t)counts[t] >= (uint64_t)r * w.per_row) {
                    w.done[t] = 1;
                    fresh += r;
                }
            }
        }
        if (fresh) {
            g_in_progress_callback = true;
            progress(fresh, user);
            g_in_progress_callback = false;
            reported += fresh;
        }
    }
    return reported;
}

static void report_rest(tray_progress_fn progress, void* user, int32_t rows, int32_t reported) {
    if (!progress || reported >= rows) return;
    g_in_progress_callback = true;
    progress(rows - reported, user);
    g_in_progress_callback = false;
}

int tray_render(const tray_sphere* spheres, int32_t n, const tray_background* bg, const tray_camera* cam,
                const tray_params* p, int32_t device, void* out, uint32_t* segments_out) {
    return tray_render_progress(spheres, n, bg, cam, p, device, out, segments_out, nullptr, nullptr);
}

int tray_render_progress(const tray_sphere* spheres, int32_t n, const tray_background* bg, const tray_camera* cam,
                         const tray_params* p, int32_t device, void* out, uint32_t* segments_out,
                         tray_progress_fn progress, void* user) {
    if (g_in_progress_callback) return refuse_reentry("tray_render");
    if (!bg || !cam || !out) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    int rc = validate_params(p);
    if (rc) return rc;
    rc = validate_spheres(spheres, n);
    if (rc) return rc;
    DeviceState* st = nullptr;
    rc = device_state(device, &st);
    if (rc) return rc;
    const int32_t rows = tray_params_rows(p);
    const size_t npix = (size_t)rows * (size_t)p->width;
    if (npix == 0) return TRAY_OK;
    std::lock_guard<std::mutex> lk(st->mu);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    tray_scene_t sc = nullptr;
    Slot& sl = st->slot(0);
    rc = cached_scene(sl, spheres, n, bg, device, &sc);
    if (rc) return rc;
    const size_t out_bytes = npix * bytes_per_pixel(p->output);
    const size_t seg_bytes = npix * sizeof(uint32_t);
    e = prepare_slot(sl, out_bytes, segments_out ? seg_bytes : 0);
    if (e == hipSuccess && progress) e = prepare_progress(sl, rows);
    if (e != hipSuccess) return hip_fail(e, "workspace");
    rc = render_async_impl(sc, cam, p, sl.out_ws, segments_out ? sl.seg_ws : nullptr, nullptr, sl.stream, 1,
                           progress ? sl.prog_dev : nullptr);
    if (rc) {  // a band may already be enqueued: let it finish before the slot can be reused
        (void)hipStreamSynchronize(sl.stream);
        return rc;
    }
    // Before the copies: a copy into pageable caller memory returns only once done.
    int32_t reported = 0;
    if (progress) {
        std::vector<ProgressWatch> ws{ProgressWatch{device, &sl, rows, (uint64_t)p->width * (uint64_t)p->rays_per_pixel, {}}};
        reported = poll_progress(ws, progress, user, e);
        if (e != hipSuccess) {  // the launch may still write the slot's workspaces and counters
            (void)hipStreamSynchronize(sl.stream);
            return hip_fail(e, "render");
        }
    }
    e = hipMemcpyAsync(out, sl.out_ws, out_bytes, hipMemcpyDeviceToHost, sl.stream);
    if (e == hipSuccess && segments_out)
        e = hipMemcpyAsync(segments_out, sl.seg_ws, seg_bytes, hipMemcpyDeviceToHost, sl.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(sl.stream);
    if (e != hipSuccess) return hip_fail(e, "render");
    report_rest(progress, user, rows, reported);
    return TRAY_OK;
}

int tray_render_devices(const tray_sphere* spheres, int32_t n, const tray_background* bg, const tray_camera* cam,
                        const tray_params* p, const int32_t* devices, int32_t n_devices, void* out,
                        uint32_t* segments_out) {
    return tray_render_devices_progress(spheres, n, bg, cam, p, devices, n_devices, out, segments_out, nullptr,
                                        nullptr);
}

int tray_render_devices_progress(const tray_sphere* spheres, int32_t n, const tray_background* bg,
                                 const tray_camera* cam, const tray_params* p, const int32_t* devices,
                                 int32_t n_devices, void* out, uint32_t* segments_out, tray_progress_fn progress,
                                 void* user) {
    if (g_in_progress_callback) return refuse_reentry("tray_render_devices");
    if (!bg || !cam || !out || !devices) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    if (n_devices < 1 || n_devices > 1024) return fail(TRAY_ERR_INVALID_ARGUMENT, "n_devices must be in [1, 1024]");
    int rc = validate_params(p);
    if (rc) return rc;
    if (p->tile_rows != 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "tray_render_devices tiles the rows itself: tile_rows must be 0");
    rc = validate_spheres(spheres, n);
    if (rc) return rc;
    // Every distinct device, locked in ascending order (no lock-order inversion between callers).
    std::vector<int32_t> uniq(devices, devices + n_devices);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    std::vector<DeviceState*> states(uniq.size());
    for (size_t i = 0; i < uniq.size(); ++i) {
        rc = device_state(uniq[i], &states[i]);
        if (rc) return rc;
    }
    std::vector<std::unique_lock<std::mutex>> locks;
    for (DeviceState* st : states) locks.emplace_back(st->mu);
    const int32_t rows = tray_params_rows(p);
    if (rows == 0) return TRAY_OK;
    const size_t row_bytes = (size_t)p->width * bytes_per_pixel(p->output);
    const size_t seg_row_bytes = (size_t)p->width * sizeof(uint32_t);
    struct Shard {
        int32_t device;
        Slot* slot;
        tray_params params;
        int32_t rows;
    };
    std::vector<Shard> shards((size_t)n_devices);
    std::vector<int32_t> used(uniq.size(), 0);
    hipError_t e = hipSuccess;
    // Shard k renders the interleaved 1-row tiles k, k + n, ... of the row set
    // (tile k -> shard k mod n), each on its own slot and stream.
    auto drain = [&](int32_t upto) {  // let what is enqueued finish before the slots can be reused
        for (int32_t j = 0; j < upto; ++j)
            if (shards[(size_t)j].rows > 0 && shards[(size_t)j].slot->stream) {
                (void)hipSetDevice(shards[(size_t)j].device);
                (void)hipStreamSynchronize(shards[(size_t)j].slot->stream);
            }
    };
    for (int32_t k = 0; k < n_devices; ++k) {
        const size_t u = (size_t)(std::lower_bound(uniq.begin(), uniq.end(), devices[k]) - uniq.begin());
        Shard& sh = shards[(size_t)k];
        sh.device = devices[k];
        sh.slot = &states[u]->slot((size_t)used[u]++);
        sh.params = *p;
        sh.params.tile_rows = 1;
        sh.params.tile_count = n_devices;
        sh.params.tile_index = k;
        sh.rows = tray_params_rows(&sh.params);
        if (sh.rows == 0) continue;
        e = hipSetDevice(sh.device);
        if (e != hipSuccess) {
            drain(k);
            return hip_fail(e, "hipSetDevice");
        }
        tray_scene_t sc = nullptr;
        rc = cached_scene(*sh.slot, spheres, n, bg, sh.device, &sc);
        if (rc) {
            drain(k);
            return rc;
        }
        e = prepare_slot(*sh.slot, (size_t)sh.rows * row_bytes, segments_out ? (size_t)sh.rows * seg_row_bytes : 0);
        if (e == hipSuccess && progress) e = prepare_progress(*sh.slot, sh.rows);
        if (e != hipSuccess) {
            drain(k);
            return hip_fail(e, "workspace");
        }
        rc = render_async_impl(sc, cam, &sh.params, sh.slot->out_ws, segments_out ? sh.slot->seg_ws : nullptr, nullptr,
                               sh.slot->stream, 1, progress ? sh.slot->prog_dev : nullptr);
        if (rc) {
            drain(k + 1);
            return rc;
        }
    }
    // With progress, every shard's counters are polled until all the renders
    // are done, before the copies (a copy into pageable memory blocks).
    int32_t reported = 0;
    if (progress) {
        std::vector<ProgressWatch> ws;
        for (const Shard& sh : shards)
            if (sh.rows > 0)
                ws.push_back(ProgressWatch{sh.device, sh.slot, sh.rows,
                                           (uint64_t)p->width * (uint64_t)p->rays_per_pixel, {}});
        reported = poll_progress(ws, progress, user, e);
    }
    // Scatter each shard's compact rows into image order (shard k's i-th row is
    // row k + i * n of the row set) with one strided copy each.
    for (int32_t k = 0; k < n_devices && e == hipSuccess; ++k) {
        const Shard& sh = shards[(size_t)k];
        if (sh.rows == 0) continue;
        e = hipSetDevice(sh.device);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(static_cast<char*>(out) + (size_t)k * row_bytes, (size_t)n_devices * row_bytes,
                                 sh.slot->out_ws, row_bytes, row_bytes, (size_t)sh.rows, hipMemcpyDeviceToHost,
                                 sh.slot->stream);
        if (e == hipSuccess && segments_out)
            e = hipMemcpy2DAsync(segments_out + (size_t)k * p->width, (size_t)n_devices * seg_row_bytes,
                                 sh.slot->seg_ws, seg_row_bytes, seg_row_bytes, (size_t)sh.rows,
                                 hipMemcpyDeviceToHost, sh.slot->stream);
    }
    for (int32_t k = 0; k < n_devices; ++k) {  // drain every stream even after an error
        const Shard& sh = shards[(size_t)k];
        if (sh.rows == 0 || !sh.slot->stream) continue;
        (void)hipSetDevice(sh.device);
        const hipError_t s2 = hipStreamSynchronize(sh.slot->stream);
        if (e == hipSuccess) e = s2;
    }
    if (e != hipSuccess) return hip_fail(e, "render");
    report_rest(progress, user, rows, reported);
    return TRAY_OK;
}

int tray_linear_to_srgba_async(const double* rgb_device, size_t n_pixels, uint8_t* rgba_device, int32_t device,
                               void* stream) {
    if (g_in_progress_callback) return refuse_reentry("tray_linear_to_srgba_async");
    if ((!rgb_device || !rgba_device) && n_pixels) return fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    DeviceState* st = nullptr;
    int rc = device_state(device, &st);
    if (rc) return rc;
    TRAY_HIP(hipSetDevice(device));
    {
        std::lock_guard<std::mutex> lk(st->mu);
        if (!st->srgb) {
            double* t = nullptr;
            TRAY_HIP(hipMalloc(&t, 256 * sizeof(double)));
            const hipError_t e = hipMemcpy(t, srgb_thresholds(), 256 * sizeof(double), hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                (void)hipFree(t);
                return hip_fail(e, "sRGB table");
            }
            st->srgb = t;
        }
    }
    TRAY_HIP(launch_to_srgba(rgb_device, n_pixels, reinterpret_cast<uint32_t*>(rgba_device), st->srgb,
                             static_cast<hipStream_t>(stream)));
    return TRAY_OK;
}

// Frees what the synchronous entry points keep on device d (slots: cached
// scene with its sample and candidate buffers, workspaces, streams, progress
// counters; the sRGB table). Lock order: a render takes st->mu and then, inside
// (tray_scene_upload -> device_state), g_devices_mu; so this is called WITHOUT
// g_devices_mu, on a DeviceState looked up under it (they are never deleted).
static void release_device(DeviceState* st, int d) {
    if (!st) return;
    std::lock_guard<std::mutex> lk2(st->mu);
    (void)hipSetDevice(d);
    for (Slot& sl : st->slots) {
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
        if (sl.cached) tray_scene_release(sl.cached);
        if (sl.out_ws) (void)hipFree(sl.out_ws);
        if (sl.seg_ws) (void)hipFree(sl.seg_ws);
        if (sl.prog_host) (void)hipHostFree(sl.prog_host);
        if (sl.stream) (void)hipStreamDestroy(sl.stream);
    }
    st->slots.clear();
    if (st->srgb) (void)hipFree(st->srgb);
    st->srgb = nullptr;
}

// The device states to release (all when device < 0), copied under g_devices_mu
// and released after dropping it (see release_device).
static std::vector<std::pair<DeviceState*, int>> devices_to_release(int32_t device) {
    std::vector<std::pair<DeviceState*, int>> v;
    std::lock_guard<std::mutex> lk(g_devices_mu);
    for (size_t d = 0; d < g_devices.size(); ++d)
        if (g_devices[d] && (device < 0 || (size_t)device == d)) v.emplace_back(g_devices[d], (int)d);
    return v;
}

int tray_release_cache(int32_t device) {
    if (g_in_progress_callback) return refuse_reentry("tray_release_cache");
    for (auto& [st, d] : devices_to_release(device)) release_device(st, d);
    return TRAY_OK;
}

int tray_shutdown(void) {
    if (g_in_progress_callback) return refuse_reentry("tray_shutdown");
    for (auto& [st, d] : devices_to_release(-1)) release_device(st, d);
    scale_release_staging();
    return TRAY_OK;
}

#pragma GCC visibility pop
}  // extern "C"
