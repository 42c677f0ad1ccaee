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
//
// Build: binned SAH over sphere centroids into a binary tree (object-median
// splits once a branch gets deep, so depth stays bounded), then collapsed into
// 4-wide nodes by repeatedly opening the largest-area inner child. Spheres
// whose boxes dwarf the rest (kBvhGlobals) stay out of the tree and are tested
// at the start of every traversal: visiting them first is one more any-order
// visit, so the result is unchanged.

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

// Binary node: leaf when count > 0 (prims [first, first + count)).
struct Node2 {
    Box box;
    int32_t left = -1, right = -1;
    int32_t first = 0, count = 0;
};

// Past this depth splits are object medians: depth <= kSahDepth + log2(n).
constexpr int kSahDepth = 32;

struct Builder {
    std::vector<Prim> prims;
    std::vector<Prim> scratch;  // split(): the right side while the left is compacted
    std::vector<Node2> bin;
    std::vector<Bvh4Node> nodes;
    std::vector<int32_t> leaves;
    std::vector<double4> geo;
    std::vector<int32_t> idx;
    double pad = 0;
    int leaf_max = 1;
    int32_t stack_max = 0;
    BvhOptions opt;

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

    int build2(int b, int e, int depth) {
        const int me = (int)bin.size();
        bin.push_back(Node2{});
        Box box;
        for (int i = b; i < e; ++i) box.grow(prims[i].box);
        bin[me].box = box;
        if (e - b <= leaf_max) {
            bin[me].first = b;
            bin[me].count = e - b;
            return me;
        }
        const int mid = split(b, e, depth);
        const int l = build2(b, mid, depth + 1);
        const int r = build2(mid, e, depth + 1);
        bin[me].left = l;
        bin[me].right = r;
        return me;
    }

    // Binned SAH over centroids; object median when deep or degenerate.
    int split(int b, int e, int depth) {
        if (opt.sweep) return split_sweep(b, e, depth);
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
        for (int k = 0; k < 3 && depth < kSahDepth; ++k) {
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
            // Only the occupied bins matter: an empty bin's box grows nothing
            // (min/max with +-inf are exact) and a split after it has the same
            // two sides, hence the same cost, as the split after the last
            // occupied bin before it, which comes first and wins the tie.
            int occ[kBins], m = 0;
            for (int i = 0; i < kBins; ++i)
                if (cnt[i]) occ[m++] = i;
            double right_area[kBins];
            int right_cnt[kBins];
            Box acc;
            int c = 0;
            for (int j = m - 1; j > 0; --j) {  // right side of the split before occupied bin j
                acc.grow(bins[occ[j]]);
                c += cnt[occ[j]];
                right_area[j] = acc.area();
                right_cnt[j] = c;
            }
            Box left;
            int lc = 0;
            for (int j = 0; j + 1 < m; ++j) {
                left.grow(bins[occ[j]]);
                lc += cnt[occ[j]];
                const double cost = left.area() * lc + right_area[j + 1] * right_cnt[j + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = k;
                    best_bin = occ[j];
                }
            }
        }
        int mid = b;
        if (best_axis >= 0) {
            // Stable: [b, e) is in list order (see below), so both sides stay in it.
            const int k = best_axis;
            const double ext = cmax[k] - cmin[k];
            scratch.clear();
            int w = b;
            for (int i = b; i < e; ++i) {
                int bi = (int)((prims[i].c[k] - cmin[k]) / ext * kBins);
                bi = std::min(std::max(bi, 0), kBins - 1);
                if (bi <= best_bin) prims[w++] = prims[i];  // w <= i: forward compaction keeps the order
                else scratch.push_back(prims[i]);
            }
            std::copy(scratch.begin(), scratch.end(), prims.begin() + w);
            mid = w;
        }
        if (mid <= b || mid >= e) {  // median along the widest centroid extent (ties: list order)
            int k = 0;
            for (int a = 1; a < 3; ++a)
                if (cmax[a] - cmin[a] > cmax[k] - cmin[k]) k = a;
            mid = b + (e - b) / 2;
            std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e, [k](const Prim& x, const Prim& y) {
                return x.c[k] < y.c[k] || (x.c[k] == y.c[k] && x.index < y.index);
            });
            // Keep each side's primitives in list order (deterministic, index-ordered leaves).
            const auto by_index = [](const Prim& x, const Prim& y) { return x.index < y.index; };
            std::sort(prims.begin() + b, prims.begin() + mid, by_index);
            std::sort(prims.begin() + mid, prims.begin() + e, by_index);
        }
        return mid;
    }

    // Full-sweep SAH (tools/bvh_sim): every split between consecutive centroids
    // along each axis (ties in list order), cost A_L N_L + A_R N_R.
    int split_sweep(int b, int e, int depth) {
        const int n = e - b;
        double best = INFINITY;
        int best_axis = -1, best_at = -1;
        std::vector<Prim> tmp(prims.begin() + b, prims.begin() + e);
        std::vector<double> right(n + 1);
        for (int k = 0; k < 3 && depth < kSahDepth; ++k) {
            std::stable_sort(tmp.begin(), tmp.end(), [k](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
            Box acc;
            for (int i = n - 1; i >= 1; --i) {
                acc.grow(tmp[i].box);
                right[i] = acc.area() * (n - i);
            }
            Box left;
            for (int i = 1; i < n; ++i) {
                left.grow(tmp[i - 1].box);
                if (tmp[i].c[k] == tmp[i - 1].c[k]) continue;  // no plane between equal centroids
                const double cost = left.area() * i + right[i];
                if (cost < best) {
                    best = cost;
                    best_axis = k;
                    best_at = i;
                }
            }
        }
        if (best_axis < 0) {
            const int mid = b + n / 2;
            int k = 0;
            double ext[3];
            for (int a = 0; a < 3; ++a) {
                double lo = INFINITY, hi = -INFINITY;
                for (int i = b; i < e; ++i) lo = std::min(lo, prims[i].c[a]), hi = std::max(hi, prims[i].c[a]);
                ext[a] = hi - lo;
            }
            for (int a = 1; a < 3; ++a)
                if (ext[a] > ext[k]) k = a;
            std::stable_sort(prims.begin() + b, prims.begin() + e, [k](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
            const auto by_index = [](const Prim& x, const Prim& y) { return x.index < y.index; };
            std::sort(prims.begin() + b, prims.begin() + mid, by_index);
            std::sort(prims.begin() + mid, prims.begin() + e, by_index);
            return mid;
        }
        const int k = best_axis;
        std::stable_sort(tmp.begin(), tmp.end(), [k](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
        const auto by_index = [](const Prim& x, const Prim& y) { return x.index < y.index; };
        std::sort(tmp.begin(), tmp.begin() + best_at, by_index);
        std::sort(tmp.begin() + best_at, tmp.end(), by_index);
        std::copy(tmp.begin(), tmp.end(), prims.begin() + b);
        return b + best_at;
    }

    // Which inner child the collapse opens next (opt.collapse): 0 the largest
    // area, 1 the largest area x primitive count.
    double open_score(int c) const {
        const double a = bin[c].box.area();
        if (opt.collapse == 1) return a * (double)count_of(c);
        return a;
    }
    int count_of(int c) const {
        if (bin[c].count > 0) return bin[c].count;
        return count_of(bin[c].left) + count_of(bin[c].right);
    }

    // Emit the 4-wide node for binary inner node `n` (pre-order); `depth_stack`
    // = stack entries its ancestors may have left. Returns the node index.
    int collapse(int n, int32_t depth_stack, const tray_sphere* s) {
        int ch[kBvhWidth] = {bin[n].left, bin[n].right, -1, -1};
        int cnt = 2;
        while (cnt < kBvhWidth) {  // open the largest-area inner child
            int pick = -1;
            double pick_area = -1;
            for (int k = 0; k < cnt; ++k)
                if (bin[ch[k]].count == 0 && open_score(ch[k]) > pick_area) {
                    pick = k;
                    pick_area = open_score(ch[k]);
                }
            if (pick < 0) break;
            const int c = ch[pick];
            ch[pick] = bin[c].left;
            ch[cnt++] = bin[c].right;
        }
        const int me = (int)nodes.size();
        nodes.push_back(Bvh4Node{});
        // The traversal visits the nearest hit child and pushes the others.
        const int32_t here = depth_stack + (cnt - 1);
        stack_max = std::max(stack_max, here);
        for (int k = 0; k < kBvhWidth; ++k) {
            if (k >= cnt) {
                for (int a = 0; a < 3; ++a) {
                    nodes[me].box[a][0][k] = INFINITY;
                    nodes[me].box[a][1][k] = -INFINITY;
                }
                nodes[me].ref[k] = kBvhNone;
                continue;
            }
            const Node2& c = bin[ch[k]];
            for (int a = 0; a < 3; ++a) {
                nodes[me].box[a][0][k] = down(c.box.lo[a] - pad);
                nodes[me].box[a][1][k] = up(c.box.hi[a] + pad);
            }
            if (c.count > 0) {
                const int slot = (int)geo.size();
                for (int i = c.first; i < c.first + c.count; ++i) {
                    const tray_sphere& sp = s[prims[i].index];
                    geo.push_back(make_double4(sp.center[0], sp.center[1], sp.center[2], sp.radius * sp.radius));
                    idx.push_back(prims[i].index);
                }
                nodes[me].ref[k] = kBvhLeafBit | (uint32_t)leaves.size();
                leaves.push_back((slot << 3) | c.count);
            } else {
                const int sub = collapse(ch[k], here, s);
                nodes[me].ref[k] = (uint32_t)sub;
            }
        }
        return me;
    }
};

}  // namespace

bool build_bvh(const tray_sphere* s, int32_t n, Bvh* out, int leaf_max) {
    return build_bvh_opts(s, n, out, leaf_max, BvhOptions{});
}

bool build_bvh_opts(const tray_sphere* s, int32_t n, Bvh* out, int leaf_max, const BvhOptions& opt) {
    out->nodes.clear();
    out->leaves.clear();
    out->geo.clear();
    out->idx.clear();
    out->bound = 0;
    out->stack_max = 0;
    out->n_global = 0;
    if (n <= 0) return true;
    Builder B;
    B.opt = opt;
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
    std::vector<Prim> globals;
    while ((int)globals.size() < kBvhGlobals && (int)B.prims.size() > B.leaf_max + 1) {
        size_t big = 0;
        for (size_t i = 1; i < B.prims.size(); ++i)
            if (B.prims[i].box.area() > B.prims[big].box.area()) big = i;
        Box rest;
        for (size_t i = 0; i < B.prims.size(); ++i)
            if (i != big) rest.grow(B.prims[i].box);
        if (!(B.prims[big].box.area() >= kBvhGlobalRatio * rest.area())) break;
        globals.push_back(B.prims[big]);
        B.prims.erase(B.prims.begin() + (std::ptrdiff_t)big);
    }
    const int32_t nt = (int32_t)B.prims.size();
    if (nt <= B.leaf_max) return false;  // root must be an inner node
    B.bin.reserve((size_t)2 * nt);
    B.scratch.reserve((size_t)nt);
    B.nodes.reserve((size_t)nt);
    B.leaves.reserve((size_t)nt);
    B.geo.reserve((size_t)n);
    B.idx.reserve((size_t)n);
    const int root = B.build2(0, nt, 0);
    B.collapse(root, 0, s);
    std::sort(globals.begin(), globals.end(), [](const Prim& x, const Prim& y) { return x.index < y.index; });
    for (const Prim& g : globals) {  // the last slots, after every leaf's
        const tray_sphere& sp = s[g.index];
        B.geo.push_back(make_double4(sp.center[0], sp.center[1], sp.center[2], sp.radius * sp.radius));
        B.idx.push_back(g.index);
    }
    if ((int64_t)B.nodes.size() > kBvhMaxNodes || (int64_t)B.leaves.size() > kBvhMaxLeaves) return false;
    out->nodes.swap(B.nodes);
    out->leaves.swap(B.leaves);
    out->geo.swap(B.geo);
    out->idx.swap(B.idx);
    out->bound = m;
    out->stack_max = B.stack_max;
    out->leaf_max = B.leaf_max;
    out->n_global = (int32_t)globals.size();
    return true;
}

}  // namespace tray
