// tray_scale.hip — the terminal view's downscale on the device (SURVEY.md §8(f)
// row 4): main.go:119-128 scales the rendered image.RGBA to the terminal's
// size with golang.org/x/image/draw (v0.35.0, go.mod:11; not vendored) —
// BiLinear.Scale when supersampling (> 1), NearestNeighbor.Scale when the
// image is smaller than the terminal (< 1), op Over onto a fresh image.
//
// The published algorithm of that package, in its op order (FP64, no FMA):
//   * BiLinear is Kernel{Support 1, At(t) = 1 - t}. newDistrib gives every
//     destination column (row) its source taps: centre (x + 0.5) s - 0.5 with
//     s = src / dst, support widened to s when shrinking (argument scaled by
//     1 / s), taps with t >= 1 or weight 0 dropped, and 1 / total weight.
//   * scaleX: tmp[y][x] = (sum over taps, in order, of (byte * 0x101) * w) *
//     ((1 / total) / 0xffff), per channel of the premultiplied RGBA source.
//   * scaleY: sum over the vertical taps of tmp * w, colour clamped to alpha,
//     ftou(v * (1 / total)) = int32(0xffff v + 0.5) clamped to [0, 0xffff],
//     then Over: dst = (dst * (0xffff - a) * 0x101 / 0xffff + src) >> 8.
//   * NearestNeighbor: source pixel ((2 x + 1) sw / 2 dw, (2 y + 1) sh / 2 dh)
//     in integers, then the same Over.
// The taps (a few KB) are built on the host; one thread per pixel of each pass
// accumulates in tap order, so the device bytes equal the oracle's restatement
// (oracle/tray_oracle.c oracle_scale_*). Parity with the Go library itself is
// unpinned: neither the module nor a fixture is in the reference tree.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <list>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tray.h"
#include "tray_internal.hpp"

namespace tray {

struct ScaleSource {
    int32_t i, j;           // taps [i, j)
    double inv_total;       // 1 / total weight
    double inv_total_ffff;  // (1 / total weight) / 0xffff
};
struct ScaleTap {
    int32_t coord;
    int32_t pad;
    double weight;
};

// newDistrib(BiLinear, dw, sw) of x/image/draw.
static void bilinear_taps(int32_t dw, int32_t sw, std::vector<ScaleSource>& src, std::vector<ScaleTap>& taps) {
    const double support = 1.0;
    const double scale = (double)sw / (double)dw;
    double half = support, arg_scale = 1.0;
    if (scale > 1) {
        half *= scale;
        arg_scale = 1 / scale;
    }
    src.resize((size_t)dw);
    for (int32_t x = 0; x < dw; ++x) {
        const double center = ((double)x + 0.5) * scale - 0.5;
        int32_t i = (int32_t)floor(center - half);
        if (i < 0) i = 0;
        int32_t j = (int32_t)ceil(center + half);
        if (j > sw) {
            j = sw;
            if (j < i) j = i;
        }
        double total = 0.0;
        const int32_t first = (int32_t)taps.size();
        for (int32_t c = i; c < j; ++c) {
            const double t = fabs((center - (double)c) * arg_scale);
            if (t >= support) continue;
            const double w = 1 - t;
            if (w == 0) continue;
            total += w;
            taps.push_back(ScaleTap{c, 0, w});
        }
        total = 1 / total;
        src[(size_t)x] = ScaleSource{first, (int32_t)taps.size(), total, total / 0xffff};
    }
}

__device__ __forceinline__ uint32_t ftou(double f) {
    const double v = 0xffff * f + 0.5;
    const int32_t i = !(v < 2147483648.0) ? INT32_MAX : !(v > -2147483649.0) ? INT32_MIN : (int32_t)v;
    return i > 0xffff ? 0xffffu : i > 0 ? (uint32_t)i : 0u;
}

// dst pixel (4 bytes) Over a premultiplied 16-bit source colour.
__device__ __forceinline__ uint32_t over(uint32_t d, uint32_t r, uint32_t g, uint32_t b, uint32_t a) {
    const uint32_t a1 = (0xffffu - a) * 0x101u;
    const uint32_t o0 = ((d & 0xFFu) * a1 / 0xffffu + r) >> 8;
    const uint32_t o1 = (((d >> 8) & 0xFFu) * a1 / 0xffffu + g) >> 8;
    const uint32_t o2 = (((d >> 16) & 0xFFu) * a1 / 0xffffu + b) >> 8;
    const uint32_t o3 = ((d >> 24) * a1 / 0xffffu + a) >> 8;
    return (o0 & 0xFFu) | ((o1 & 0xFFu) << 8) | ((o2 & 0xFFu) << 16) | ((o3 & 0xFFu) << 24);
}

__global__ __launch_bounds__(256) void scale_x_kernel(const uint32_t* src, int32_t sw, int32_t sh, int32_t dw,
                                                     const ScaleSource* hs, const ScaleTap* ht, double4* tmp) {
    const size_t k = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= (size_t)dw * (size_t)sh) return;
    const int32_t y = (int32_t)(k / (size_t)dw), x = (int32_t)(k % (size_t)dw);
    const ScaleSource s = hs[x];
    double pr = 0, pg = 0, pb = 0, pa = 0;
    for (int32_t t = s.i; t < s.j; ++t) {
        const uint32_t p = src[(size_t)y * (size_t)sw + (size_t)ht[t].coord];
        const double w = ht[t].weight;
        pr += (double)((p & 0xFFu) * 0x101u) * w;
        pg += (double)(((p >> 8) & 0xFFu) * 0x101u) * w;
        pb += (double)(((p >> 16) & 0xFFu) * 0x101u) * w;
        pa += (double)((p >> 24) * 0x101u) * w;
    }
    tmp[k] = make_double4(pr * s.inv_total_ffff, pg * s.inv_total_ffff, pb * s.inv_total_ffff, pa * s.inv_total_ffff);
}

__global__ __launch_bounds__(256) void scale_y_over_kernel(const double4* tmp, int32_t dw, int32_t dh,
                                                          const ScaleSource* vs, const ScaleTap* vt, uint32_t* dst) {
    const size_t k = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= (size_t)dw * (size_t)dh) return;
    const int32_t y = (int32_t)(k / (size_t)dw), x = (int32_t)(k % (size_t)dw);
    const ScaleSource s = vs[y];
    double pr = 0, pg = 0, pb = 0, pa = 0;
    for (int32_t t = s.i; t < s.j; ++t) {
        const double4 p = tmp[(size_t)vt[t].coord * (size_t)dw + (size_t)x];
        const double w = vt[t].weight;
        pr += p.x * w;
        pg += p.y * w;
        pb += p.z * w;
        pa += p.w * w;
    }
    if (pr > pa) pr = pa;
    if (pg > pa) pg = pa;
    if (pb > pa) pb = pa;
    dst[k] = over(dst[k], ftou(pr * s.inv_total), ftou(pg * s.inv_total), ftou(pb * s.inv_total),
                  ftou(pa * s.inv_total));
}

__global__ __launch_bounds__(256) void scale_nearest_kernel(const uint32_t* src, int32_t sw, int32_t sh,
                                                           int32_t dw, int32_t dh, uint32_t* dst) {
    const size_t k = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= (size_t)dw * (size_t)dh) return;
    const uint64_t dy = k / (size_t)dw, dx = k % (size_t)dw;
    const uint64_t sy = (2 * dy + 1) * (uint64_t)sh / (2 * (uint64_t)dh);
    const uint64_t sx = (2 * dx + 1) * (uint64_t)sw / (2 * (uint64_t)dw);
    const uint32_t p = src[sy * (uint64_t)sw + sx];
    dst[k] = over(dst[k], (p & 0xFFu) * 0x101u, ((p >> 8) & 0xFFu) * 0x101u, ((p >> 16) & 0xFFu) * 0x101u,
                  (p >> 24) * 0x101u);
}

static int hip_err(hipError_t e, const char* what) {
    return fail(TRAY_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// Pinned host buffers for the tap tables, each reusable once the event recorded
// after its last copy has fired. A handful per process (one per scale in flight).
struct Staging {
    void* host = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    int device = -1;
    bool busy = false;
};
static std::mutex g_staging_mu;
// A list: entries keep their addresses while others are added or erased
// (scale_release_staging may erase idle entries while another thread holds a
// taken one outside the lock).
static std::list<Staging> g_staging;

// A buffer of >= bytes on the current device whose last copy has completed.
static hipError_t staging_take(size_t bytes, Staging** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_staging_mu);
    Staging* pick = nullptr;
    for (Staging& s : g_staging) {
        if (s.busy || s.device != dev || hipEventQuery(s.done) != hipSuccess) continue;
        if (s.bytes >= bytes) {
            pick = &s;
            break;
        }
        if (!pick) pick = &s;  // idle but too small: grow it
    }
    if (!pick) {
        hipEvent_t done = nullptr;
        e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
        if (e != hipSuccess) return e;  // nothing added: no entry without an event
        g_staging.emplace_back();
        pick = &g_staging.back();
        pick->device = dev;
        pick->done = done;
    }
    if (pick->bytes < bytes) {
        if (pick->host) (void)hipHostFree(pick->host);
        pick->host = nullptr;
        pick->bytes = 0;
        const size_t want = std::max<size_t>(bytes, 64 << 10);
        e = hipHostMalloc(&pick->host, want, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        pick->bytes = want;
    }
    pick->busy = true;
    *out = pick;
    return hipSuccess;
}

static void staging_give(Staging* s) {
    std::lock_guard<std::mutex> lk(g_staging_mu);
    s->busy = false;
}

void scale_release_staging() {
    std::lock_guard<std::mutex> lk(g_staging_mu);
    for (auto it = g_staging.begin(); it != g_staging.end();) {
        if (it->busy || (it->done && hipEventSynchronize(it->done) != hipSuccess)) {
            ++it;  // in use by a concurrent call, or its device failed: left as is
            continue;
        }
        if (it->host) (void)hipHostFree(it->host);
        if (it->done) (void)hipEventDestroy(it->done);
        it = g_staging.erase(it);
    }
}

// Enqueues the scale on `stream` (device buffers); workspace is stream-ordered.
static int scale_enqueue(const uint8_t* src, int32_t sw, int32_t sh, uint8_t* dst, int32_t dw, int32_t dh,
                         int32_t filter, hipStream_t stream) {
    const size_t n = (size_t)dw * (size_t)dh;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
    if (filter == TRAY_SCALE_NEAREST) {
        hipLaunchKernelGGL(scale_nearest_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, s32, sw, sh,
                           dw, dh, d32);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? TRAY_OK : hip_err(e, "scale");
    }
    std::vector<ScaleSource> hs, vs;
    std::vector<ScaleTap> ht, vt;
    bilinear_taps(dw, sw, hs, ht);
    bilinear_taps(dh, sh, vs, vt);
    // one workspace: [hs][vs][ht][vt][tmp], 16-B aligned parts
    auto al = [](size_t b) { return (b + 15) / 16 * 16; };
    const size_t b_hs = al(hs.size() * sizeof(ScaleSource)), b_vs = al(vs.size() * sizeof(ScaleSource));
    const size_t b_ht = al(ht.size() * sizeof(ScaleTap)), b_vt = al(vt.size() * sizeof(ScaleTap));
    const size_t b_tmp = (size_t)dw * (size_t)sh * sizeof(double4);
    std::vector<uint8_t> head(b_hs + b_vs + b_ht + b_vt, 0);
    memcpy(head.data(), hs.data(), hs.size() * sizeof(ScaleSource));
    memcpy(head.data() + b_hs, vs.data(), vs.size() * sizeof(ScaleSource));
    memcpy(head.data() + b_hs + b_vs, ht.data(), ht.size() * sizeof(ScaleTap));
    memcpy(head.data() + b_hs + b_vs + b_ht, vt.data(), vt.size() * sizeof(ScaleTap));
    uint8_t* ws = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&ws), head.size() + b_tmp, stream);
    if (e != hipSuccess) return hip_err(e, "scale workspace");
    // The tap tables (a few KB) go through a pinned staging buffer that stays
    // untouched until the copy, enqueued on `stream`, has run (its event): the
    // call neither blocks nor leaves the caller's stream order.
    Staging* stg = nullptr;
    e = staging_take(head.size(), &stg);
    if (e == hipSuccess) {
        memcpy(stg->host, head.data(), head.size());
        e = hipMemcpyAsync(ws, stg->host, head.size(), hipMemcpyHostToDevice, stream);
        if (e == hipSuccess) {
            e = hipEventRecord(stg->done, stream);
            // No event covers the copy: let it finish before the buffer can be taken again.
            if (e != hipSuccess) (void)hipStreamSynchronize(stream);
        }
        staging_give(stg);
    }
    const ScaleSource* d_hs = reinterpret_cast<const ScaleSource*>(ws);
    const ScaleSource* d_vs = reinterpret_cast<const ScaleSource*>(ws + b_hs);
    const ScaleTap* d_ht = reinterpret_cast<const ScaleTap*>(ws + b_hs + b_vs);
    const ScaleTap* d_vt = reinterpret_cast<const ScaleTap*>(ws + b_hs + b_vs + b_ht);
    double4* tmp = reinterpret_cast<double4*>(ws + head.size());
    if (e == hipSuccess) {
        const size_t nx = (size_t)dw * (size_t)sh;
        hipLaunchKernelGGL(scale_x_kernel, dim3((uint32_t)((nx + 255) / 256)), dim3(256), 0, stream, s32, sw, sh, dw,
                           d_hs, d_ht, tmp);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(scale_y_over_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, tmp, dw, dh,
                           d_vs, d_vt, d32);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(ws, stream);
    if (e == hipSuccess) e = f;
    return e == hipSuccess ? TRAY_OK : hip_err(e, "scale");
}

static int scale_check(const void* src, int32_t sw, int32_t sh, const void* dst, int32_t dw, int32_t dh,
                       int32_t filter) {
    if (!src || !dst) return fail(TRAY_ERR_INVALID_ARGUMENT, "null image");
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return fail(TRAY_ERR_INVALID_ARGUMENT, "image sizes must be > 0");
    if ((uint64_t)sw * (uint64_t)sh > (1ull << 31) || (uint64_t)dw * (uint64_t)dh > (1ull << 31))
        return fail(TRAY_ERR_TOO_LARGE, "image larger than 2^31 pixels");
    if (filter != TRAY_SCALE_NEAREST && filter != TRAY_SCALE_BILINEAR)
        return fail(TRAY_ERR_INVALID_ARGUMENT, "unknown scale filter");
    return TRAY_OK;
}

}  // namespace tray

using namespace tray;

extern "C" {
#pragma GCC visibility push(default)

int tray_scale_rgba_async(const uint8_t* src_device, int32_t src_width, int32_t src_height, uint8_t* dst_device,
                          int32_t dst_width, int32_t dst_height, int32_t filter, int32_t device, void* stream) {
    int rc = scale_check(src_device, src_width, src_height, dst_device, dst_width, dst_height, filter);
    if (rc) return rc;
    rc = device_usable(device);
    if (rc) return rc;
    const hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_err(e, "hipSetDevice");
    return scale_enqueue(src_device, src_width, src_height, dst_device, dst_width, dst_height, filter,
                         static_cast<hipStream_t>(stream));
}

int tray_scale_rgba(const uint8_t* src, int32_t src_width, int32_t src_height, uint8_t* dst, int32_t dst_width,
                    int32_t dst_height, int32_t filter, int32_t device) {
    int rc = scale_check(src, src_width, src_height, dst, dst_width, dst_height, filter);
    if (rc) return rc;
    rc = device_usable(device);
    if (rc) return rc;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_err(e, "hipSetDevice");
    const size_t sb = (size_t)src_width * (size_t)src_height * 4, db = (size_t)dst_width * (size_t)dst_height * 4;
    uint8_t *ds = nullptr, *dd = nullptr;
    hipStream_t st = nullptr;
    e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ds), sb);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&dd), db);
    if (e == hipSuccess) e = hipMemcpyAsync(ds, src, sb, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dd, dst, db, hipMemcpyHostToDevice, st);  // Over blends onto dst
    rc = e == hipSuccess ? scale_enqueue(ds, src_width, src_height, dd, dst_width, dst_height, filter, st)
                         : hip_err(e, "scale upload");
    if (rc == TRAY_OK) {
        e = hipMemcpyAsync(dst, dd, db, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = hip_err(e, "scale");
    }
    if (st) (void)hipStreamSynchronize(st);
    (void)hipFree(ds);
    (void)hipFree(dd);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}

#pragma GCC visibility pop
}  // extern "C"
