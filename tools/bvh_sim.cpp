// bvh_sim — offline cost of a BVH build for the kernel's traversal (host only).
//
// Traces C2-like paths on the CPU with the oracle (camera rays, Scene.Hit,
// Scatter: oracle/libtray_oracle.so), collects every secondary segment (the
// camera rays take the candidate lists on the device, not the tree), and
// replays the megakernel's traversal of a tree built by tray_bvh.cpp for each:
// the ground (out-of-tree spheres) first, then FP32 slab tests of the four
// child boxes culled by the current hit, the nearest hit child next and the
// others pushed, one cull per pop (trav_node / trav_leaf / stack_pop in
// tray_kernel.hip). Counts node visits, box tests and sphere tests per
// segment, and checks every closest hit against the oracle's linear scan.
//
//   make -C tools bvh_sim && tools/bvh_sim [pixels] [spp] [leaf_max]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../tray_amd/csrc/bvh.hpp"

extern "C" {
void oracle_camera_initialize(double* setup13, int w, int h, double* cam21);
int oracle_rich_scene(uint64_t seed, int half, tray_sphere* out, int cap);
void oracle_get_ray(const double* cam, uint64_t seed, uint32_t pixel, uint32_t sample, double px, double py, double ox,
                    double oy, double origin[3], double dir[3]);
int oracle_scene_hit(const tray_sphere* s, int n, const double o[3], const double d[3], double t0, double t1,
                     double rec[8]);
int oracle_scatter(const tray_sphere* s, const double io[3], const double id[3], const double p[3], const double nrm[3],
                   int front, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce, double att[3],
                   double so[3], double sd[3]);
}

using namespace tray;

struct Seg {
    double o[3], d[3];
};

struct Count {
    double nodes = 0, boxes = 0, spheres = 0, segs = 0, mismatches = 0, pushes = 0;
};

static float up(double v) {
    float f = (float)v;
    if ((double)f < v) f = nextafterf(f, INFINITY);
    return f;
}

// Sphere.Hit root under the kernel's rule (test_geo): t = r1 > 1e-6 ? r1 : r2.
static bool sphere_t(const double4& g, const Seg& s, double& t) {
    const double a = s.d[0] * s.d[0] + s.d[1] * s.d[1] + s.d[2] * s.d[2];
    const double ox = g.x - s.o[0], oy = g.y - s.o[1], oz = g.z - s.o[2];
    const double h = s.d[0] * ox + s.d[1] * oy + s.d[2] * oz;
    const double c = (ox * ox + oy * oy + oz * oz) - g.w;
    const double disc = h * h - a * c;
    if (disc < 0) return false;
    const double sq = sqrt(disc);
    double r = (h - sq) / a;
    if (!(r > 1e-6)) r = (h + sq) / a;
    t = r;
    return r > 1e-6;
}

static void trace(const Bvh& b, const Seg& s, Count& c, int* hit_index) {
    double closest = INFINITY;
    int slot = -1;
    const int ns = (int)b.geo.size();
    auto test = [&](int k) {
        double t;
        c.spheres += 1;
        if (sphere_t(b.geo[k], s, t) && (t < closest || (t == closest && slot >= 0 && b.idx[k] < b.idx[slot]))) {
            closest = t;
            slot = k;
        }
    };
    for (int g = ns - b.n_global; g < ns; ++g) test(g);
    float ix = 1.0f / (float)s.d[0], iy = 1.0f / (float)s.d[1], iz = 1.0f / (float)s.d[2];
    if (!std::isfinite(ix)) ix = 1e30f;
    if (!std::isfinite(iy)) iy = 1e30f;
    if (!std::isfinite(iz)) iz = 1e30f;
    const float oix = (float)s.o[0] * ix, oiy = (float)s.o[1] * iy, oiz = (float)s.o[2] * iz;
    float tlim = up(closest);
    std::vector<uint32_t> stack;  // sort keys
    uint32_t cur = 0;
    auto key_tn = [](uint32_t k) {
        const uint32_t u = k & 0xFFFF0000u;
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    const int culls = getenv("BVH_SIM_CULLS") ? atoi(getenv("BVH_SIM_CULLS")) : 1;
    auto pop = [&]() -> uint32_t {  // stack_pop: at most `culls` entries beyond tlim skipped (the kernel: 1)
        for (int k = 0; !stack.empty(); ++k) {
            const uint32_t key = stack.back();
            stack.pop_back();
            if (!(key_tn(key) > tlim) || k + 1 >= culls) {
                if (key_tn(key) > tlim && stack.empty()) return kBvhNone;  // the empty-stack sentinel culls too
                return key & 0xFFFFu;
            }
        }
        return kBvhNone;
    };
    while (cur != kBvhNone) {
        if (cur < kBvhLeafBit) {
            const Bvh4Node& nd = b.nodes[cur];
            c.nodes += 1;
            uint32_t key[4];
            for (int k = 0; k < 4; ++k) {
                if (nd.ref[k] != kBvhNone) c.boxes += 1;
                const float lx = ix < 0 ? nd.box[0][1][k] : nd.box[0][0][k], hx = ix < 0 ? nd.box[0][0][k] : nd.box[0][1][k];
                const float ly = iy < 0 ? nd.box[1][1][k] : nd.box[1][0][k], hy = iy < 0 ? nd.box[1][0][k] : nd.box[1][1][k];
                const float lz = iz < 0 ? nd.box[2][1][k] : nd.box[2][0][k], hz = iz < 0 ? nd.box[2][0][k] : nd.box[2][1][k];
                const float tn = fmaxf(fmaxf(fmaxf(fmaf(lx, ix, -oix), fmaf(ly, iy, -oiy)), fmaf(lz, iz, -oiz)), 0.0f);
                const float tf = fminf(fminf(fminf(fmaf(hx, ix, -oix), fmaf(hy, iy, -oiy)), fmaf(hz, iz, -oiz)), tlim);
                uint32_t u;
                memcpy(&u, &tn, 4);
                key[k] = tn <= tf ? ((u & 0xFFFF0000u) | nd.ref[k]) : ~0u;
            }
            static const int order_mode = getenv("BVH_SIM_ORDER") ? atoi(getenv("BVH_SIM_ORDER")) : 0;
            if (order_mode == 0) {
                std::sort(key, key + 4);  // the kernel: full sort, nearest visited, the rest pushed far-to-near
            } else {  // 1: nearest first, the rest in child order (hit keys before misses)
                int m = 0;
                for (int k = 1; k < 4; ++k)
                    if (key[k] < key[m]) m = k;
                std::swap(key[0], key[m]);
                std::stable_partition(key + 1, key + 4, [](uint32_t x) { return x != ~0u; });
                if (order_mode == 2) std::reverse(key + 1, key + 1 + (int)std::count_if(key + 1, key + 4, [](uint32_t x) { return x != ~0u; }));
            }
            if (key[0] != ~0u) {
                for (int k = 3; k >= 1; --k)
                    if (key[k] != ~0u) {
                        stack.push_back(key[k]);
                        c.pushes += 1;
                    }
                cur = key[0] & 0xFFFFu;
            } else {
                cur = pop();
            }
        } else {
            const int32_t info = b.leaves[cur & (kBvhLeafBit - 1u)];
            for (int k = 0; k < (info & 7); ++k) test((info >> 3) + k);
            tlim = up(closest);
            cur = pop();
        }
    }
    *hit_index = slot >= 0 ? b.idx[slot] : -1;
}

int main(int argc, char** argv) {
    const int pixels = argc > 1 ? atoi(argv[1]) : 4000;
    const int spp = argc > 2 ? atoi(argv[2]) : 8;
    const int leaf_max = argc > 3 ? atoi(argv[3]) : 1;
    BvhOptions opt;
    opt.sweep = argc > 4 && atoi(argv[4]) != 0;
    opt.collapse = argc > 5 ? atoi(argv[5]) : 0;
    const int half = argc > 6 ? atoi(argv[6]) : 11;
    const uint64_t scene_seed = argc > 7 ? strtoull(argv[7], nullptr, 10) : 2;
    const int W = 1280, H = 720, depth = 50;
    const uint64_t seed = scene_seed;
    std::vector<tray_sphere> sc(4 * (2 * half) * (2 * half) + 8);
    const int n = oracle_rich_scene(seed, half, sc.data(), (int)sc.size());
    sc.resize(n);
    double setup[13] = {13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0, 10.0, 10.0, 0.1}, cam[21];
    oracle_camera_initialize(setup, W, H, cam);
    // Secondary segments of C2-like paths (a fixed pseudo-random pixel sample).
    std::vector<Seg> segs;
    uint64_t st = 12345;
    auto rnd = [&]() {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(st >> 11) * 0x1p-53;
    };
    for (int q = 0; q < pixels; ++q) {
        const int x = (int)(rnd() * W), y = (int)(rnd() * H);
        for (int s = 0; s < spp; ++s) {
            Seg r;
            const double ang = 2 * M_PI * rnd(), rad = 0.5 * sqrt(rnd());
            oracle_get_ray(cam, seed, (uint32_t)(y * W + x), (uint32_t)s, x, y, rad * cos(ang), rad * sin(ang), r.o, r.d);
            for (int bounce = 0; bounce < depth; ++bounce) {
                if (bounce > 0) segs.push_back(r);
                double rec[8];
                const int m = oracle_scene_hit(sc.data(), n, r.o, r.d, 1e-6, INFINITY, rec);
                if (m < 0) break;
                double att[3], so[3], sd[3];
                if (bounce + 1 >= depth) break;
                if (oracle_scatter(&sc[m], r.o, r.d, rec, rec + 3, (int)rec[7], seed, (uint32_t)(y * W + x),
                                   (uint32_t)s, (uint32_t)bounce, att, so, sd) != 1)
                    break;
                memcpy(r.o, so, sizeof so);
                memcpy(r.d, sd, sizeof sd);
            }
        }
    }
    Bvh b;
    if (!build_bvh_opts(sc.data(), n, &b, leaf_max, opt)) {
        fprintf(stderr, "build failed\n");
        return 1;
    }
    Count c;
    for (const Seg& s : segs) {
        int got = -1;
        trace(b, s, c, &got);
        double rec[8];
        const int want = oracle_scene_hit(sc.data(), n, s.o, s.d, 1e-6, INFINITY, rec);
        c.mismatches += got != want;
        c.segs += 1;
    }
    printf("{\"sweep\": %d, \"collapse\": %d, \"spheres\": %d, \"leaf_max\": %d, \"nodes_in_tree\": %zu, \"stack_max\": %d, \"segments\": %.0f, "
           "\"node_visits_per_seg\": %.4f, \"box_tests_per_seg\": %.4f, \"sphere_tests_per_seg\": %.4f, "
           "\"pushes_per_seg\": %.4f, \"mismatches\": %.0f}\n",
           (int)opt.sweep, opt.collapse, n, leaf_max, b.nodes.size(), b.stack_max, c.segs, c.nodes / c.segs, c.boxes / c.segs, c.spheres / c.segs,
           c.pushes / c.segs, c.mismatches);
    return c.mismatches == 0 ? 0 : 2;
}
