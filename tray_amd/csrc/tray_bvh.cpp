// tray_bvh.cpp — host-side BVH build for exact-culling traversal.
//
// The reference scans every object per ray (Scene.Hit, ray/objects.go:37-46).
// Each sphere's candidate root depends only on (ray, sphere), so the scan's
// result is the lexicographic minimum of (t_i, i) over all spheres. Visiting
// spheres in ANY order with the rule "accept t < closest, or t == closest with a
// lower index" yields the same hit, PROVIDED no sphere that could win is
// skipped. The BVH below only skips a subtree when a conservative FP32 slab
// test proves its (padded) box is missed or lies beyond the current closest hit.
//
// Padding bound: with ray origin o rounded to float, 1/d in float and the slab
// arithmetic in float (unit roundoff u = 2^-24), the computed slab parameter is
// off by at most u*|o| + 4u*|lo - o| (+ second order) in position units, i.e.
// <= 9u*M for coordinates bounded by M. Boxes are padded by 4e-6*M (> 60u*M)
// and rounded outward to float, so the float interval always contains the
// exact interval of the unpadded sphere box. The kernel requires every ray
// origin to satisfy |o| <= M (hit points lie inside the boxes; the camera is
// checked at launch, else the linear scan is used).

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "bvh.hpp"

namespace tray {

namespace {

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    double area() const {
        if (!(hi[0] >= lo[0])) return 0.0;
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct Prim {
    Box box;
    double c[3];
    int32_t index;
};

struct Builder {
    std::vector<Prim> prims;
    std::vector<BvhNode> nodes;
    std::vector<double4> geo;
    std::vector<int32_t> idx;
    double pad = 0;
    int leaf_max = kBvhLeafMax;

    static float down(double v) {
        float f = (float)v;
        if ((double)f > v) f = nextafterf(f, -INFINITY);
        return f;
    }
    static float up(double v) {
        float f = (float)v;
        if ((double)f < v) f = nextafterf(f, INFINITY);
        return f;
    }

    // Emit the subtree over prims[b, e) in depth-first order; returns node index.
    int build(int b, int e, const tray_sphere* s) {
        Box box;
        for (int i = b; i < e; ++i) box.grow(prims[i].box);
        const int me = (int)nodes.size();
        nodes.push_back(BvhNode{});
        for (int k = 0; k < 3; ++k) {
            nodes[me].lo[k] = down(box.lo[k] - pad);
            nodes[me].hi[k] = up(box.hi[k] + pad);
        }
        const int count = e - b;
        if (count <= leaf_max) {
            const int slot = (int)geo.size();
            for (int i = b; i < e; ++i) {
                const tray_sphere& sp = s[prims[i].index];
                geo.push_back(make_double4(sp.center[0], sp.center[1], sp.center[2], sp.radius * sp.radius));
                idx.push_back(prims[i].index);
            }
            nodes[me].leaf = (slot << 3) | count;
            nodes[me].skip = me + 1;
            return me;
        }
        const int mid = split(b, e, box);
        build(b, mid, s);
        build(mid, e, s);
        nodes[me].leaf = -1;
        nodes[me].skip = (int)nodes.size();
        return me;
    }

    // Binned SAH over centroids; falls back to a median split on degenerate input.
    int split(int b, int e, const Box& box) {
        constexpr int kBins = 32;
        double cmin[3], cmax[3];
        for (int k = 0; k < 3; ++k) {
            cmin[k] = INFINITY;
            cmax[k] = -INFINITY;
        }
        for (int i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                cmin[k] = std::min(cmin[k], prims[i].c[k]);
                cmax[k] = std::max(cmax[k], prims[i].c[k]);
            }
        double best_cost = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int k = 0; k < 3; ++k) {
            const double ext = cmax[k] - cmin[k];
            if (!(ext > 0)) continue;
            Box bins[kBins];
            int cnt[kBins] = {};
            for (int i = b; i < e; ++i) {
                int bi = (int)((prims[i].c[k] - cmin[k]) / ext * kBins);
                bi = std::min(std::max(bi, 0), kBins - 1);
                bins[bi].grow(prims[i].box);
                cnt[bi]++;
            }
            double right_area[kBins];
            int right_cnt[kBins];
            Box acc;
            int c = 0;
            for (int i = kBins - 1; i > 0; --i) {
                acc.grow(bins[i]);
                c += cnt[i];
                right_area[i] = acc.area();
                right_cnt[i] = c;
            }
            Box left;
            int lc = 0;
            for (int i = 0; i < kBins - 1; ++i) {
                left.grow(bins[i]);
                lc += cnt[i];
                if (lc == 0 || right_cnt[i + 1] == 0) continue;
                const double cost = left.area() * lc + right_area[i + 1] * right_cnt[i + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = k;
                    best_bin = i;
                }
            }
        }
        int mid;
        if (best_axis >= 0) {
            const int k = best_axis;
            const double ext = cmax[k] - cmin[k];
            Prim* m = std::partition(prims.data() + b, prims.data() + e, [&](const Prim& p) {
                int bi = (int)((p.c[k] - cmin[k]) / ext * kBins);
                bi = std::min(std::max(bi, 0), kBins - 1);
                return bi <= best_bin;
            });
            mid = (int)(m - prims.data());
        } else {
            mid = b;
        }
        if (mid <= b || mid >= e) {  // all centroids equal: split by list position
            mid = b + (e - b) / 2;
        }
        // Keep each side's primitives in list order (deterministic, index-ordered leaves).
        std::sort(prims.begin() + b, prims.begin() + mid, [](const Prim& x, const Prim& y) { return x.index < y.index; });
        std::sort(prims.begin() + mid, prims.begin() + e, [](const Prim& x, const Prim& y) { return x.index < y.index; });
        return mid;
    }
};

}  // namespace

bool build_bvh(const tray_sphere* s, int32_t n, Bvh* out, int leaf_max) {
    out->nodes.clear();
    out->geo.clear();
    out->idx.clear();
    out->bound = 0;
    if (n <= 0) return true;
    Builder B;
    B.prims.resize((size_t)n);
    double m = 0;
    for (int32_t i = 0; i < n; ++i) {
        Prim& p = B.prims[(size_t)i];
        const double r = fabs(s[i].radius);
        for (int k = 0; k < 3; ++k) {
            p.box.lo[k] = s[i].center[k] - r;
            p.box.hi[k] = s[i].center[k] + r;
            p.c[k] = s[i].center[k];
            m = std::max(m, std::max(fabs(p.box.lo[k]), fabs(p.box.hi[k])));
        }
        p.index = i;
        if (!std::isfinite(m)) return false;
    }
    m = std::max(m, 1.0);
    B.pad = 4e-6 * m;
    B.leaf_max = std::min(std::max(leaf_max, 1), kBvhLeafMax);
    out->bound = m;
    B.build(0, n, s);
    out->nodes.swap(B.nodes);
    out->geo.swap(B.geo);
    out->idx.swap(B.idx);
    return true;
}

}  // namespace tray
