// Traversal-strategy simulator (development tool, host only): builds the
// kernel's BVH for a RichScene, path-traces a pixel sample with simplified
// shading to get a realistic segment distribution, and counts node visits,
// box tests and sphere tests per segment for several traversal orders.
//
//   hipcc -O2 -std=c++17 -x hip tools/bvh_sim.cpp tray_amd/csrc/tray_host.cpp \
//         tray_amd/csrc/tray_bvh.cpp -o tools/bvh_sim && tools/bvh_sim [seed] [half] [leafmax]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../include/tray.h"
#include "../tray_amd/csrc/bvh.hpp"

using namespace tray;

struct V {
    double x, y, z;
};
static V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V operator*(V a, double t) { return {a.x * t, a.y * t, a.z * t}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V unit(V a) { return a * (1.0 / sqrt(dot(a, a))); }
static double comp(V a, int k) { return k == 0 ? a.x : k == 1 ? a.y : a.z; }

static std::mt19937_64 rng(1);
static double U() { return std::uniform_real_distribution<double>(0, 1)(rng); }
static V rand_unit() {
    const double z = 1 - 2 * U(), r = sqrt(1 - z * z), p = 2 * M_PI * U();
    return {r * cos(p), r * sin(p), z};
}

static const tray_sphere* S;
static int N;

static double sphere_t(int i, V o, V d, double tmax) {
    const V c = {S[i].center[0], S[i].center[1], S[i].center[2]};
    const V oc = o - c;
    const double a = dot(d, d), h = dot(d, oc), cc = dot(oc, oc) - S[i].radius * S[i].radius;
    const double disc = h * h - a * cc;
    if (disc < 0) return INFINITY;
    const double sq = sqrt(disc);
    double t = (-h - sq) / a;
    if (!(t > 1e-6)) t = (-h + sq) / a;
    if (!(t > 1e-6) || t >= tmax) return INFINITY;
    return t;
}

struct Counts {
    double iters = 0, boxes = 0, spheres = 0, leaves = 0;
};

struct Tree {
    std::vector<BvhNode> nodes;
    std::vector<int32_t> idx;
    std::vector<int> left, right;  // children of inner nodes (DFS layout)
};

static bool box_hit(const BvhNode& n, V o, V d, double tmax, double& tn) {
    double t0 = 0, t1 = tmax;
    for (int k = 0; k < 3; ++k) {
        const double inv = 1.0 / comp(d, k);
        double a = (n.lo[k] - comp(o, k)) * inv, b = (n.hi[k] - comp(o, k)) * inv;
        if (a > b) std::swap(a, b);
        t0 = std::max(t0, a);
        t1 = std::min(t1, b);
    }
    tn = t0;
    return t0 <= t1;
}

static void test_leaf(const Tree& T, const BvhNode& n, V o, V d, double& closest, int& best, Counts& c) {
    const int slot = n.leaf >> 3, cnt = n.leaf & 7;
    c.leaves++;
    for (int k = 0; k < cnt; ++k) {
        c.spheres++;
        const int i = T.idx[slot + k];
        const double t = sphere_t(i, o, d, INFINITY);
        if (t < closest || (t == closest && i < best)) {
            closest = t;
            best = i;
        }
    }
}

// A: depth-first, fixed order, skip links (the current kernel).
static int trav_dfs(const Tree& T, V o, V d, Counts& c, int order) {
    double closest = INFINITY;
    int best = -1;
    // order 0: fixed; 1: near child first by child-centre projection (octant tables)
    std::vector<int> st;
    st.push_back(0);
    while (!st.empty()) {
        const int i = st.back();
        st.pop_back();
        const BvhNode& n = T.nodes[i];
        c.iters++;
        c.boxes++;
        double tn;
        if (!box_hit(n, o, d, closest, tn)) continue;
        if (n.leaf >= 0) {
            test_leaf(T, n, o, d, closest, best, c);
            continue;
        }
        int a = T.left[i], b = T.right[i];
        if (order == 1) {
            // split axis = largest separation of child box centres; near = along the ray's sign
            const BvhNode &A = T.nodes[a], &B = T.nodes[b];
            int ax = 0;
            double sep = -1;
            for (int k = 0; k < 3; ++k) {
                const double s = fabs((B.lo[k] + B.hi[k]) - (A.lo[k] + A.hi[k]));
                if (s > sep) sep = s, ax = k;
            }
            const bool b_first = ((B.lo[ax] + B.hi[ax]) - (A.lo[ax] + A.hi[ax])) * comp(d, ax) < 0;
            if (b_first) std::swap(a, b);
        }
        st.push_back(b);
        st.push_back(a);
    }
    return best;
}

// C: stack BVH2, both children tested at the parent, nearer entry first.
static int trav_pair(const Tree& T, V o, V d, Counts& c) {
    double closest = INFINITY;
    int best = -1;
    std::vector<std::pair<double, int>> st;
    c.boxes++;
    double tn;
    if (!box_hit(T.nodes[0], o, d, closest, tn)) return -1;
    if (T.nodes[0].leaf >= 0) {
        test_leaf(T, T.nodes[0], o, d, closest, best, c);
        return best;
    }
    st.push_back({0.0, 0});
    while (!st.empty()) {
        auto [t, i] = st.back();
        st.pop_back();
        if (t > closest) continue;
        c.iters++;
        const int ch[2] = {T.left[i], T.right[i]};
        double tt[2];
        bool h[2];
        for (int k = 0; k < 2; ++k) {
            c.boxes++;
            h[k] = box_hit(T.nodes[ch[k]], o, d, closest, tt[k]);
        }
        int order[2] = {0, 1};
        if (tt[1] < tt[0]) std::swap(order[0], order[1]);
        for (int r = 1; r >= 0; --r) {  // push far first so near pops first
            const int k = order[r];
            if (!h[k]) continue;
            if (T.nodes[ch[k]].leaf >= 0) {
                // leaf children are tested right away (nearest first)
                continue;
            }
            st.push_back({tt[k], ch[k]});
        }
        for (int r = 0; r < 2; ++r) {
            const int k = order[r];
            if (h[k] && T.nodes[ch[k]].leaf >= 0 && tt[k] <= closest) test_leaf(T, T.nodes[ch[k]], o, d, closest, best, c);
        }
    }
    return best;
}

// D: BVH4 by collapsing (children = grandchildren of inner children), stack, nearest first.
static void collect4(const Tree& T, int i, std::vector<int>& out) {
    const int a = T.left[i], b = T.right[i];
    for (int ch : {a, b}) {
        if (T.nodes[ch].leaf < 0) {
            out.push_back(T.left[ch]);
            out.push_back(T.right[ch]);
        } else {
            out.push_back(ch);
        }
    }
}
static int trav_wide(const Tree& T, V o, V d, Counts& c) {
    double closest = INFINITY;
    int best = -1;
    std::vector<std::pair<double, int>> st;
    st.push_back({0.0, 0});
    while (!st.empty()) {
        auto [t, i] = st.back();
        st.pop_back();
        if (t > closest) continue;
        if (T.nodes[i].leaf >= 0) {
            test_leaf(T, T.nodes[i], o, d, closest, best, c);
            continue;
        }
        c.iters++;
        std::vector<int> ch;
        collect4(T, i, ch);
        std::vector<std::pair<double, int>> hits;
        for (int k : ch) {
            c.boxes++;
            double tt;
            if (box_hit(T.nodes[k], o, d, closest, tt)) hits.push_back({tt, k});
        }
        std::sort(hits.begin(), hits.end(), [](auto& x, auto& y) { return x.first > y.first; });
        for (auto& h : hits) st.push_back(h);
    }
    return best;
}

// E: BVH4, the proposed kernel scheme: at each node all child boxes are tested;
// hit leaf children are tested right away, the nearest hit inner child is
// visited next and the other hit inner children are pushed far-to-near onto a
// stack of node indices (cull = drop popped entries whose entry distance is
// beyond the current closest hit; needs the distance stored).
static int max_stack = 0;
static int trav_e(const Tree& T, V o, V d, Counts& c, bool cull) {
    double closest = INFINITY;
    int best = -1;
    std::vector<std::pair<double, int>> st;
    int node = 0;
    double tn0;
    c.boxes++;
    if (!box_hit(T.nodes[0], o, d, closest, tn0)) return -1;
    if (T.nodes[0].leaf >= 0) {
        test_leaf(T, T.nodes[0], o, d, closest, best, c);
        return best;
    }
    while (true) {
        c.iters++;
        std::vector<int> ch;
        collect4(T, node, ch);
        std::vector<std::pair<double, int>> inner;
        std::vector<std::pair<double, int>> leaves;
        for (int k : ch) {
            c.boxes++;
            double tt;
            if (!box_hit(T.nodes[k], o, d, closest, tt)) continue;
            if (T.nodes[k].leaf >= 0) leaves.push_back({tt, k});
            else inner.push_back({tt, k});
        }
        for (auto& l : leaves) test_leaf(T, T.nodes[l.second], o, d, closest, best, c);
        std::sort(inner.begin(), inner.end(), [](auto& x, auto& y) { return x.first > y.first; });
        int next = -1;
        if (!inner.empty()) {
            next = inner.back().second;
            inner.pop_back();
            for (auto& h : inner) st.push_back(h);
        }
        max_stack = std::max(max_stack, (int)st.size());
        while (next < 0 && !st.empty()) {
            auto [t, i] = st.back();
            st.pop_back();
            if (cull && t > closest) continue;
            next = i;
        }
        if (next < 0) break;
        node = next;
    }
    return best;
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? atoll(argv[1]) : 2;
    const int half = argc > 2 ? atoi(argv[2]) : 11;
    std::vector<tray_sphere> sp(tray_rich_scene_capacity(half));
    int32_t n = 0;
    tray_rich_scene(seed, half, sp.data(), (int32_t)sp.size(), &n);
    S = sp.data();
    N = n;
    const int leaf_max = argc > 3 ? atoi(argv[3]) : kBvhLeafMax;
    Bvh bvh;
    build_bvh(sp.data(), n, &bvh, leaf_max);
    Tree T;
    T.nodes = bvh.nodes;
    T.idx = bvh.idx;
    T.left.assign(T.nodes.size(), -1);
    T.right.assign(T.nodes.size(), -1);
    for (size_t i = 0; i < T.nodes.size(); ++i)
        if (T.nodes[i].leaf < 0) {
            T.left[i] = (int)i + 1;
            T.right[i] = T.nodes[i + 1].skip;
        }
    tray_camera_setup cs;
    tray_rich_scene_camera(&cs);
    const int W = 1280, H = 720;
    tray_camera cam;
    tray_camera_initialize(&cs, W, H, &cam);
    const V pos = {cam.position[0], cam.position[1], cam.position[2]};
    const V p00 = {cam.pixel00[0], cam.pixel00[1], cam.pixel00[2]};
    const V px = {cam.pixel_x[0], cam.pixel_x[1], cam.pixel_x[2]};
    const V py = {cam.pixel_y[0], cam.pixel_y[1], cam.pixel_y[2]};
    Counts cA, cB, cC, cD, cE, cF;
    long segs = 0, mism = 0;
    for (int y = 0; y < H; y += 8)
        for (int x = 0; x < W; x += 8)
            for (int s = 0; s < 2; ++s) {
                V o = pos;
                V d = (p00 + px * (x + U() - 0.5) + py * (y + U() - 0.5)) - pos;
                for (int depth = 0; depth < 50; ++depth) {
                    ++segs;
                    const int best = trav_dfs(T, o, d, cA, 0);
                    const int b2 = trav_dfs(T, o, d, cB, 1);
                    const int b3 = trav_pair(T, o, d, cC);
                    const int b4 = trav_wide(T, o, d, cD);
                    const int b5 = trav_e(T, o, d, cE, true);
                    const int b6 = trav_e(T, o, d, cF, false);
                    mism += (b2 != best) + (b3 != best) + (b4 != best) + (b5 != best) + (b6 != best);
                    if (best < 0) break;
                    const double t = sphere_t(best, o, d, INFINITY);
                    const tray_sphere& q = S[best];
                    const V p = o + d * t;
                    V nrm = (p - V{q.center[0], q.center[1], q.center[2]}) * (1.0 / q.radius);
                    const bool front = dot(d, nrm) < 0;
                    if (!front) nrm = nrm * -1.0;
                    V nd;
                    if (q.material == TRAY_LAMBERTIAN) {
                        nd = nrm + rand_unit();
                    } else if (q.material == TRAY_METAL) {
                        const V u = unit(d);
                        nd = u - nrm * (2 * dot(u, nrm)) + rand_unit() * q.param;
                        if (dot(nd, nrm) <= 0) break;
                    } else {
                        const V u = unit(d);
                        const double ratio = front ? 1.0 / q.param : q.param;
                        const double ct = std::min(-dot(u, nrm), 1.0), st = sqrt(1 - ct * ct);
                        if (ratio * st > 1 || U() < 0.1) {
                            nd = u - nrm * (2 * dot(u, nrm));
                        } else {
                            const V perp = (u + nrm * ct) * ratio;
                            nd = perp + nrm * -sqrt(fabs(1 - dot(perp, perp)));
                        }
                    }
                    o = p;
                    d = nd;
                }
            }
    auto pr = [&](const char* name, const Counts& c) {
        printf("%-28s iters %6.2f boxes %6.2f spheres %5.2f leaves %5.2f\n", name, c.iters / segs, c.boxes / segs,
               c.spheres / segs, c.leaves / segs);
    };
    printf("spheres %d nodes %zu segments %ld mismatches %ld\n", n, T.nodes.size(), segs, mism);
    pr("A dfs fixed (kernel)", cA);
    pr("B dfs near-first", cB);
    pr("C bvh2 pair stack", cC);
    pr("D bvh4 stack", cD);
    pr("E bvh4 leaves-first cull", cE);
    pr("F bvh4 leaves-first nocull", cF);
    printf("max stack %d\n", max_stack);
    return 0;
}

namespace tray {
int fail(int code, const std::string& msg) {
    fprintf(stderr, "%s\n", msg.c_str());
    return code;
}
}  // namespace tray
