// Normal orientation on the GPU: GraphBuilder.flipNormals (Pointcloud/Modules/GraphBuilder.py:129-209) without the
// host's sequential Kruskal and DFS, same result as pcd_orient_normals_mst (orient.cpp) bit for bit.
//
//   1. cost_e = 1 - |n_a . n_b| (:134-145); key_e = (cost bits << 32) | e.  Keys are distinct, so the minimum
//      spanning forest is unique and equals Kruskal's in ascending (cost, edge order) -- the host reference's order.
//   2. Borůvka: every component picks its minimum-key outgoing edge (atomicMin on the key), components hook along
//      them (mutual picks: the larger id hooks to the smaller), pointer jumping flattens the hooks; repeat until no
//      component has an outgoing edge (each round at least halves the component count).
//   3. Root the forest's tree that holds the start point (argmax z, first maximum, :206) with an Euler tour: the
//      tree edges in both directions, sorted by (source, destination); succ(u->v) = the edge after v->u in v's
//      circular adjacency list; Wyllie list ranking gives each directed edge its distance to the tour's end, and
//      u->v is the parent->child edge iff it comes before v->u.
//   4. Signs: the DFS flips dest when n_src(final) . n_dest < cos(7π/12) (:187-202).  With d = n_parent . n_child on
//      the ORIGINAL normals and s = the parent's final sign, the child's sign is f(s) with f = identity (d > -thr),
//      negation (d < thr), or constant +1 (|d| <= -thr): each node's map from the root's sign is the composition of
//      the maps on its root path, computed by pointer jumping.  The root itself is flipped when n_z < 0 (:207-208).
//      Nodes outside the root's tree keep their normals, as the reference's DFS never reaches them.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "pcd_device.h"
#include "pcd_host.h"

namespace pcd {
int fail(int code, const std::string& msg);

namespace {
constexpr unsigned long long kNoEdge = ~0ull;
constexpr int64_t kEnd = -1;

// float -> u32 with the float order (negative costs appear when |n_a . n_b| rounds above 1); -0 folds onto +0
__device__ __forceinline__ unsigned ordered_bits(float x) {
    unsigned u = __float_as_uint(x);
    if ((u & 0x7FFFFFFFu) == 0) u = 0;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct AsIndex {
    __device__ int64_t operator()(uint8_t x) const { return (int64_t)x; }
};

__global__ void k_check_edges(const int64_t* __restrict__ a, const int64_t* __restrict__ b, int64_t e, int64_t nv,
                              int* __restrict__ bad) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= e) return;
    if (a[t] < 0 || a[t] >= nv || b[t] < 0 || b[t] >= nv) *bad = 1;
}

__global__ void k_edge_keys(const float* __restrict__ n, const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                            int64_t e, unsigned long long* __restrict__ key) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= e) return;
    const float* p = n + 3 * a[t];
    const float* q = n + 3 * b[t];
    const float cost = 1.0f - fabsf((p[0] * q[0] + p[1] * q[1]) + p[2] * q[2]);
    key[t] = ((unsigned long long)ordered_bits(cost) << 32) | (unsigned long long)t;
}

__global__ void k_iota(int64_t* __restrict__ x, int64_t n) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < n) x[t] = t;
}

__global__ void k_fill_u64(unsigned long long* __restrict__ x, int64_t n, unsigned long long v) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < n) x[t] = v;
}

// Borůvka: cheapest outgoing edge per component (component ids are root vertices after pointer jumping)
__global__ void k_min_edge(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                           const unsigned long long* __restrict__ key, int64_t e, const int64_t* __restrict__ comp,
                           unsigned long long* __restrict__ best) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= e) return;
    const int64_t ca = comp[a[t]], cb = comp[b[t]];
    if (ca == cb) return;
    atomicMin(best + ca, key[t]);
    atomicMin(best + cb, key[t]);
}

__global__ void k_hook(const int64_t* __restrict__ a, const int64_t* __restrict__ b, int64_t nv,
                       const unsigned long long* __restrict__ best, const int64_t* __restrict__ comp,
                       int64_t* __restrict__ parent, uint8_t* __restrict__ in_tree, int* __restrict__ changed) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv || comp[v] != v) return;          // component roots only
    const unsigned long long k = best[v];
    if (k == kNoEdge) return;
    const int64_t e = (int64_t)(k & 0xFFFFFFFFull);
    const int64_t other = comp[a[e]] == v ? comp[b[e]] : comp[a[e]];
    in_tree[e] = 1;
    // mutual choice (the same edge from both sides): only the larger id hooks, so no 2-cycle forms
    if (best[other] == k && other > v) return;
    parent[v] = other;
    *changed = 1;
}

__global__ void k_jump(int64_t* __restrict__ comp, const int64_t* __restrict__ parent, int64_t nv,
                       int* __restrict__ changed) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const int64_t p = parent[comp[v]];
    const int64_t pp = comp[p];
    if (pp != comp[v]) { comp[v] = pp; *changed = 1; }
}

__global__ void k_flatten(int64_t* __restrict__ parent, int64_t nv, int* __restrict__ changed) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const int64_t p = parent[v], pp = parent[p];
    if (pp != p) { parent[v] = pp; *changed = 1; }
}

// directed tree edges: (src << 32 | dst) for both directions of every in-tree edge
__global__ void k_tree_dirs(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                            const uint8_t* __restrict__ in_tree, const int64_t* __restrict__ slot, int64_t e,
                            unsigned long long* __restrict__ dirs) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= e || !in_tree[t]) return;
    const int64_t s = slot[t];
    dirs[2 * s] = ((unsigned long long)a[t] << 32) | (unsigned long long)b[t];
    dirs[2 * s + 1] = ((unsigned long long)b[t] << 32) | (unsigned long long)a[t];
}

__global__ void k_row_counts(const unsigned long long* __restrict__ dirs, int64_t m, int64_t* __restrict__ off) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < m) atomicAdd(reinterpret_cast<unsigned long long*>(off) + (dirs[t] >> 32) + 1, 1ull);
}

// index of v->u in v's sorted row (binary search)
__device__ int64_t find_dir(const unsigned long long* __restrict__ dirs, const int64_t* __restrict__ off, int64_t v,
                            int64_t u) {
    int64_t lo = off[v], hi = off[v + 1] - 1;
    const unsigned long long want = ((unsigned long long)v << 32) | (unsigned long long)u;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (dirs[mid] < want) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void k_euler_succ(const unsigned long long* __restrict__ dirs, const int64_t* __restrict__ off, int64_t m,
                             int64_t root, const int64_t* __restrict__ comp, int64_t root_comp,
                             int64_t* __restrict__ succ, int64_t* __restrict__ twin, int64_t* __restrict__ rank) {
    const int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (d >= m) return;
    const int64_t u = (int64_t)(dirs[d] >> 32), v = (int64_t)(dirs[d] & 0xFFFFFFFFull);
    if (comp[u] != root_comp) { succ[d] = kEnd; rank[d] = 0; twin[d] = d; return; }   // other trees: not toured
    const int64_t t = find_dir(dirs, off, v, u);
    twin[d] = t;
    const int64_t nx = t + 1 < off[v + 1] ? t + 1 : off[v];
    const bool last = nx == off[root];            // closes the tour that starts at the root's first edge
    succ[d] = last ? kEnd : nx;
    rank[d] = last ? 0 : 1;
}

// Wyllie list ranking, double-buffered
__global__ void k_rank_step(const int64_t* __restrict__ succ_in, const int64_t* __restrict__ rank_in, int64_t m,
                            int64_t* __restrict__ succ_out, int64_t* __restrict__ rank_out, int* __restrict__ changed) {
    const int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (d >= m) return;
    const int64_t s = succ_in[d];
    if (s == kEnd) { succ_out[d] = kEnd; rank_out[d] = rank_in[d]; return; }
    rank_out[d] = rank_in[d] + rank_in[s];
    succ_out[d] = succ_in[s];
    *changed = 1;
}

// parent pointers + the child's sign map from its parent's sign (0 identity, 1 negate, 2 constant +1)
__global__ void k_parents(const unsigned long long* __restrict__ dirs, const int64_t* __restrict__ twin,
                          const int64_t* __restrict__ rank, const int64_t* __restrict__ comp, int64_t root_comp,
                          int64_t m, const float* __restrict__ n, float thr, int64_t* __restrict__ par,
                          uint8_t* __restrict__ fmap) {
    const int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (d >= m) return;
    const int64_t u = (int64_t)(dirs[d] >> 32), v = (int64_t)(dirs[d] & 0xFFFFFFFFull);
    if (comp[u] != root_comp) return;
    if (rank[d] <= rank[twin[d]]) return;         // v->u comes first in the tour: v is u's parent
    par[v] = u;
    const float* p = n + 3 * u;
    const float* q = n + 3 * v;
    const float dd = (p[0] * q[0] + p[1] * q[1]) + p[2] * q[2];
    // parent sign +1: flip iff dd < thr; parent sign -1: flip iff -dd < thr
    const bool flip_pos = dd < thr, flip_neg = -dd < thr;
    fmap[v] = (!flip_pos && flip_neg) ? 0 : (flip_pos && !flip_neg) ? 1 : (!flip_pos && !flip_neg) ? 2 : 3;
}

__device__ __forceinline__ int apply_map(uint8_t f, int s) {
    return f == 0 ? s : f == 1 ? -s : f == 2 ? 1 : -1;
}
// (g o f): apply f first, then g
__device__ __forceinline__ uint8_t compose(uint8_t g, uint8_t f) {
    const int p = apply_map(g, apply_map(f, 1)), q = apply_map(g, apply_map(f, -1));
    return (p == 1 && q == -1) ? 0 : (p == -1 && q == 1) ? 1 : (p == 1 && q == 1) ? 2 : 3;
}

// pointer jumping toward the root: map[v] := map[v] o map[anc[v]], anc[v] := anc[anc[v]] (double-buffered)
__global__ void k_sign_step(const int64_t* __restrict__ anc_in, const uint8_t* __restrict__ map_in, int64_t nv,
                            int64_t root, int64_t* __restrict__ anc_out, uint8_t* __restrict__ map_out,
                            int* __restrict__ changed) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const int64_t a = anc_in[v];
    if (a < 0 || a == root) { anc_out[v] = a; map_out[v] = map_in[v]; return; }
    map_out[v] = compose(map_in[v], map_in[a]);
    anc_out[v] = anc_in[a];
    *changed = 1;
}

__global__ void k_apply_signs(float* __restrict__ n, const int64_t* __restrict__ anc, const uint8_t* __restrict__ map,
                              int64_t nv, int64_t root, const int* __restrict__ root_sign) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv) return;
    int s;
    if (v == root) s = *root_sign;
    else if (anc[v] == root) s = apply_map(map[v], *root_sign);
    else return;                                   // outside the root's tree: untouched
    if (s < 0) { n[3 * v] *= -1.f; n[3 * v + 1] *= -1.f; n[3 * v + 2] *= -1.f; }
}

__global__ void k_argmax_z(const float* __restrict__ pos, int64_t nv, unsigned long long* __restrict__ best) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nv) return;
    // order-preserving key: larger z first, then SMALLER index (the first maximum, like torch.argmax); NaN never wins
    const float z = pos[3 * v + 2];
    if (z != z) return;
    atomicMax(best, ((unsigned long long)ordered_bits(z) << 32) | (0xFFFFFFFFull - (unsigned long long)v));
}

__global__ void k_root_sign(const float* __restrict__ n, const unsigned long long* __restrict__ best,
                            int64_t* __restrict__ root_out, int* __restrict__ sign_out) {
    if (threadIdx.x != 0) return;
    const int64_t r = (int64_t)(0xFFFFFFFFull - (*best & 0xFFFFFFFFull));
    *root_out = r;
    *sign_out = n[3 * r + 2] < 0.f ? -1 : 1;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

struct Scratch {
    std::vector<void*> ptrs;
    ~Scratch() { for (void* p : ptrs) (void)hipFree(p); }
    template <class T>
    T* alloc(int64_t count) {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<int64_t>(count, 1) * sizeof(T)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return static_cast<T*>(p);
    }
};

int read_flag(int* dflag, hipStream_t st, int& out) {
    PCD_HIP(hipMemcpyAsync(&out, dflag, sizeof(int), hipMemcpyDeviceToHost, st));
    PCD_HIP(hipStreamSynchronize(st));
    return PCD_OK;
}
}  // namespace
}  // namespace pcd

using namespace pcd;

extern "C" int pcd_orient_normals_mst_gpu(const float* pos, float* n, int64_t npts, const int64_t* a,
                                          const int64_t* b, int64_t e, void* stream) {
    PCD_CHECK_ARG(pos && n && (e == 0 || (a && b)), "pcd_orient_normals_mst_gpu: null argument");
    PCD_CHECK_ARG(e < (int64_t)UINT32_MAX && npts < (int64_t)UINT32_MAX, "more than 2^32 edges or points");
    if (npts == 0) return PCD_OK;
    hipStream_t st = as_stream(stream);
    Scratch sc;
    int* flag = sc.alloc<int>(1);
    int* root_sign = sc.alloc<int>(1);
    int64_t* root_dev = sc.alloc<int64_t>(1);
    unsigned long long* zbest = sc.alloc<unsigned long long>(1);
    unsigned long long* key = sc.alloc<unsigned long long>(e);
    int64_t* comp = sc.alloc<int64_t>(npts);
    int64_t* parent = sc.alloc<int64_t>(npts);
    unsigned long long* best = sc.alloc<unsigned long long>(npts);
    uint8_t* in_tree = sc.alloc<uint8_t>(e);
    if (!flag || !root_sign || !root_dev || !zbest || !key || !comp || !parent || !best || !in_tree)
        return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scratch");
    if (e > 0) {
        PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
        hipLaunchKernelGGL(k_check_edges, grid_for(e), dim3(256), 0, st, a, b, e, npts, flag);
        int bad = 0;
        if (read_flag(flag, st, bad) != PCD_OK) return PCD_ERR_HIP;
        if (bad) return fail(PCD_ERR_ARG, "pcd_orient_normals_mst_gpu: edge index out of range");
    }
    // root: argmax z (first maximum; point 0 when every z is NaN), flipped up
    const unsigned long long z0 = 0xFFFFFFFFull;                       // key of (lowest z, index 0)
    PCD_HIP(hipMemcpyAsync(zbest, &z0, sizeof(z0), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_argmax_z, grid_for(npts), dim3(256), 0, st, pos, npts, zbest);
    hipLaunchKernelGGL(k_root_sign, dim3(1), dim3(64), 0, st, n, zbest, root_dev, root_sign);
    // 1-2. Borůvka minimum spanning forest
    if (e > 0) hipLaunchKernelGGL(k_edge_keys, grid_for(e), dim3(256), 0, st, n, a, b, e, key);
    hipLaunchKernelGGL(k_iota, grid_for(npts), dim3(256), 0, st, comp, npts);
    hipLaunchKernelGGL(k_iota, grid_for(npts), dim3(256), 0, st, parent, npts);
    PCD_HIP(hipMemsetAsync(in_tree, 0, std::max<int64_t>(e, 1), st));
    for (int round = 0; round < 64 && e > 0; ++round) {
        hipLaunchKernelGGL(k_fill_u64, grid_for(npts), dim3(256), 0, st, best, npts, kNoEdge);
        hipLaunchKernelGGL(k_min_edge, grid_for(e), dim3(256), 0, st, a, b, key, e, comp, best);
        PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
        hipLaunchKernelGGL(k_hook, grid_for(npts), dim3(256), 0, st, a, b, npts, best, comp, parent, in_tree, flag);
        int hooked = 0;
        if (read_flag(flag, st, hooked) != PCD_OK) return PCD_ERR_HIP;
        if (!hooked) break;
        for (int j = 0; j < 64; ++j) {               // flatten the hook forest, then relabel every vertex
            PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
            hipLaunchKernelGGL(k_flatten, grid_for(npts), dim3(256), 0, st, parent, npts, flag);
            int ch = 0;
            if (read_flag(flag, st, ch) != PCD_OK) return PCD_ERR_HIP;
            if (!ch) break;
        }
        for (int j = 0; j < 64; ++j) {
            PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
            hipLaunchKernelGGL(k_jump, grid_for(npts), dim3(256), 0, st, comp, parent, npts, flag);
            int ch = 0;
            if (read_flag(flag, st, ch) != PCD_OK) return PCD_ERR_HIP;
            if (!ch) break;
        }
    }
    // 3. tree edges in both directions, sorted by (src, dst) -> CSR; Euler tour of the root's tree
    int64_t* slot = sc.alloc<int64_t>(e);
    if (!slot) return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scratch");
    int64_t ntree = 0;
    if (e > 0) {
        size_t bytes = 0;
        auto in_it = rocprim::make_transform_iterator(in_tree, AsIndex());
        (void)rocprim::exclusive_scan(nullptr, bytes, in_it, slot, (int64_t)0, (size_t)e, rocprim::plus<int64_t>(), st);
        void* tmp = sc.alloc<char>((int64_t)bytes);
        if (!tmp) return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scan temp");
        PCD_HIP(rocprim::exclusive_scan(tmp, bytes, in_it, slot, (int64_t)0, (size_t)e, rocprim::plus<int64_t>(), st));
        int64_t last_slot = 0;
        uint8_t last_in = 0;
        PCD_HIP(hipMemcpyAsync(&last_slot, slot + e - 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PCD_HIP(hipMemcpyAsync(&last_in, in_tree + e - 1, 1, hipMemcpyDeviceToHost, st));
        PCD_HIP(hipStreamSynchronize(st));
        ntree = last_slot + last_in;
    }
    int64_t root = 0;
    PCD_HIP(hipMemcpyAsync(&root, root_dev, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PCD_HIP(hipStreamSynchronize(st));
    const int64_t m = 2 * ntree;
    int64_t* anc = sc.alloc<int64_t>(npts);
    int64_t* anc2 = sc.alloc<int64_t>(npts);
    uint8_t* fmap = sc.alloc<uint8_t>(npts);
    uint8_t* fmap2 = sc.alloc<uint8_t>(npts);
    if (!anc || !anc2 || !fmap || !fmap2) return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scratch");
    PCD_HIP(hipMemsetAsync(anc, 0xFF, npts * sizeof(int64_t), st));     // -1: not in the root's tree
    PCD_HIP(hipMemsetAsync(fmap, 0, npts, st));
    if (m > 0) {
        unsigned long long* dirs = sc.alloc<unsigned long long>(m);
        unsigned long long* dirs_s = sc.alloc<unsigned long long>(m);
        int64_t* off = sc.alloc<int64_t>(npts + 1);
        int64_t* succ = sc.alloc<int64_t>(m);
        int64_t* succ2 = sc.alloc<int64_t>(m);
        int64_t* rank = sc.alloc<int64_t>(m);
        int64_t* rank2 = sc.alloc<int64_t>(m);
        int64_t* twin = sc.alloc<int64_t>(m);
        if (!dirs || !dirs_s || !off || !succ || !succ2 || !rank || !rank2 || !twin)
            return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scratch");
        hipLaunchKernelGGL(k_tree_dirs, grid_for(e), dim3(256), 0, st, a, b, in_tree, slot, e, dirs);
        size_t bytes = 0;
        (void)rocprim::radix_sort_keys(nullptr, bytes, dirs, dirs_s, (size_t)m, 0, 64, st);
        void* tmp = sc.alloc<char>((int64_t)bytes);
        if (!tmp) return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: sort temp");
        PCD_HIP(rocprim::radix_sort_keys(tmp, bytes, dirs, dirs_s, (size_t)m, 0, 64, st));
        PCD_HIP(hipMemsetAsync(off, 0, (npts + 1) * sizeof(int64_t), st));
        hipLaunchKernelGGL(k_row_counts, grid_for(m), dim3(256), 0, st, dirs_s, m, off);
        size_t sb = 0;
        (void)rocprim::inclusive_scan(nullptr, sb, off, off, (size_t)(npts + 1), rocprim::plus<int64_t>(), st);
        void* tmp2 = sc.alloc<char>((int64_t)sb);
        if (!tmp2) return fail(PCD_ERR_OOM, "pcd_orient_normals_mst_gpu: scan temp");
        PCD_HIP(rocprim::inclusive_scan(tmp2, sb, off, off, (size_t)(npts + 1), rocprim::plus<int64_t>(), st));
        int64_t r0 = 0, r1 = 0;
        PCD_HIP(hipMemcpyAsync(&r0, off + root, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PCD_HIP(hipMemcpyAsync(&r1, off + root + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PCD_HIP(hipStreamSynchronize(st));
        if (r1 > r0) {                                 // the root has tree edges: rank its tour
            int64_t root_comp = 0;
            PCD_HIP(hipMemcpyAsync(&root_comp, comp + root, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            PCD_HIP(hipStreamSynchronize(st));
            hipLaunchKernelGGL(k_euler_succ, grid_for(m), dim3(256), 0, st, dirs_s, off, m, root, comp, root_comp, succ,
                               twin, rank);
            for (int j = 0; j < 70; ++j) {
                PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
                hipLaunchKernelGGL(k_rank_step, grid_for(m), dim3(256), 0, st, succ, rank, m, succ2, rank2, flag);
                std::swap(succ, succ2);
                std::swap(rank, rank2);
                int ch = 0;
                if (read_flag(flag, st, ch) != PCD_OK) return PCD_ERR_HIP;
                if (!ch) break;
            }
            const float thr = (float)std::cos(7.0 / 12.0 * M_PI);
            hipLaunchKernelGGL(k_parents, grid_for(m), dim3(256), 0, st, dirs_s, twin, rank, comp, root_comp, m, n,
                               thr, anc, fmap);
            for (int j = 0; j < 70; ++j) {
                PCD_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
                hipLaunchKernelGGL(k_sign_step, grid_for(npts), dim3(256), 0, st, anc, fmap, npts, root, anc2, fmap2,
                                   flag);
                std::swap(anc, anc2);
                std::swap(fmap, fmap2);
                int ch = 0;
                if (read_flag(flag, st, ch) != PCD_OK) return PCD_ERR_HIP;
                if (!ch) break;
            }
        }
    }
    hipLaunchKernelGGL(k_apply_signs, grid_for(npts), dim3(256), 0, st, n, anc, fmap, npts, root, root_sign);
    PCD_HIP(hipStreamSynchronize(st));
    return PCD_OK;
}
