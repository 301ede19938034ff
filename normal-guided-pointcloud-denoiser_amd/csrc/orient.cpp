// Normal orientation (host, sequential by nature): GraphBuilder.flipNormals, Pointcloud/Modules/GraphBuilder.py:129-209.
//   calculateEdgeCost      cost_e = 1 - |n_a · n_b|                                   (:134-145)
//   calculateUndirectedMST Kruskal in ascending cost order (ties: edge order)          (:147-174)
//                          -> to_undirected (sorted by (row, col), deduplicated)
//   flipNormalsWithMST     DFS from argmax z (flip it if n_z < 0), visiting each node's tree neighbours in
//                          ascending index order; flip n_dst if n_src · n_dst < cos(7π/12)   (:176-209)
// The reference's O(E·N) group relabel and recursive DFS become union-find and an explicit stack; the visit
// order, and therefore every flip decision, is the same.
#include <algorithm>
#include <cmath>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/pcd.h"

namespace pcd {
int fail(int code, const std::string& msg);
}

namespace {
struct DSU {
    std::vector<int64_t> p;
    explicit DSU(int64_t n) : p(n) { std::iota(p.begin(), p.end(), 0); }
    int64_t find(int64_t x) {
        while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
        return x;
    }
};
inline float dotf(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
}  // namespace

extern "C" int pcd_orient_normals_mst(const float* pos, float* n, int64_t npts, const int64_t* a, const int64_t* b,
                                      int64_t e) {
    if (!pos || !n || (e > 0 && (!a || !b))) return pcd::fail(PCD_ERR_ARG, "pcd_orient_normals_mst: null argument");
    if (npts == 0) return PCD_OK;
    for (int64_t t = 0; t < e; ++t)
        if (a[t] < 0 || a[t] >= npts || b[t] < 0 || b[t] >= npts)
            return pcd::fail(PCD_ERR_ARG, "pcd_orient_normals_mst: edge index out of range");
    std::vector<float> cost(e);
    for (int64_t t = 0; t < e; ++t) cost[t] = 1.0f - std::fabs(dotf(n + 3 * a[t], n + 3 * b[t]));
    std::vector<int64_t> order(e);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return cost[x] < cost[y]; });
    DSU dsu(npts);
    std::vector<std::pair<int64_t, int64_t>> und;
    und.reserve(2 * (size_t)std::max<int64_t>(npts - 1, 0));
    for (int64_t t : order) {
        const int64_t ra = dsu.find(a[t]), rb = dsu.find(b[t]);
        if (ra != rb) {
            dsu.p[ra] = rb;
            und.emplace_back(a[t], b[t]);
            und.emplace_back(b[t], a[t]);
        }
    }
    std::sort(und.begin(), und.end());
    und.erase(std::unique(und.begin(), und.end()), und.end());
    std::vector<int64_t> off(npts + 1, 0);
    for (auto& pr : und) off[pr.first + 1]++;
    for (int64_t i = 0; i < npts; ++i) off[i + 1] += off[i];
    // und is sorted by (row, col): the CSR rows are already ascending
    const float thr = (float)std::cos(7.0 / 12.0 * M_PI);
    int64_t start = 0;
    for (int64_t i = 1; i < npts; ++i)
        if (pos[3 * i + 2] > pos[3 * start + 2]) start = i;
    if (n[3 * start + 2] < 0) { n[3 * start] *= -1; n[3 * start + 1] *= -1; n[3 * start + 2] *= -1; }
    std::vector<char> visited(npts, 0);
    std::vector<std::pair<int64_t, int64_t>> stack;  // (node, next edge slot)
    visited[start] = 1;
    stack.emplace_back(start, off[start]);
    while (!stack.empty()) {
        auto& top = stack.back();
        const int64_t src = top.first;
        if (top.second >= off[src + 1]) { stack.pop_back(); continue; }
        const int64_t dst = und[top.second].second;
        ++top.second;
        if (visited[dst]) continue;
        if (dotf(n + 3 * src, n + 3 * dst) < thr) { n[3 * dst] *= -1; n[3 * dst + 1] *= -1; n[3 * dst + 2] *= -1; }
        visited[dst] = 1;
        stack.emplace_back(dst, off[dst]);
    }
    return PCD_OK;
}
