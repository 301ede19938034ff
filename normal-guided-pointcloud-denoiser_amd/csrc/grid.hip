// Frozen-snapshot index (H1) and kNN queries (H2, kNN-graph for H15, kNN-1 for H17).
//
// Reference: Selector.__init__ builds scipy KDTree(graph.pos) once and never rebuilds it
// (Pointcloud/Modules/Selector.py:138-141); getKNNSelection queries the CURRENT positions against that
// snapshot (Selector.py:235-246).  Here: bbox -> cell size -> Morton keys -> radix sort (rocPRIM) -> sorted
// float4 snapshot + bricked cell index (hash of occupied 4x4x4 bricks, dense per-brick cell ranges).  Build is
// one-time and synchronises the stream.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "pcd_knn.h"

namespace pcd {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// ------------------------------------------------------------------ build kernels
__global__ void k_bbox(const float* __restrict__ xyz, int64_t n, float* __restrict__ part) {
    float mn[3] = {3.0e38f, 3.0e38f, 3.0e38f}, mx[3] = {-3.0e38f, -3.0e38f, -3.0e38f};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = xyz[3 * i + a];
            mn[a] = fminf(mn[a], v);
            mx[a] = fmaxf(mx[a], v);
        }
    }
    __shared__ float s[6][256];
#pragma unroll
    for (int a = 0; a < 3; ++a) { s[a][threadIdx.x] = mn[a]; s[3 + a][threadIdx.x] = mx[a]; }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                s[a][threadIdx.x] = fminf(s[a][threadIdx.x], s[a][threadIdx.x + w]);
                s[3 + a][threadIdx.x] = fmaxf(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + w]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

__global__ void k_sample(const float* __restrict__ xyz, int64_t n, int64_t stride, int64_t s, float* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= s) return;
    const int64_t i = t * stride;
    out[3 * t] = xyz[3 * i];
    out[3 * t + 1] = xyz[3 * i + 1];
    out[3 * t + 2] = xyz[3 * i + 2];
}

// Sort keys: the Morton code of the cell, refined by `sub` bits per axis of the point's position inside its cell
// (kGridSub when every axis has at most 2^(21 - kGridSub) cells, else 0).  Morton order is hierarchical, so a cell's
// points stay one contiguous run (cell key = key >> 3 sub), and inside it they follow the same space-filling curve:
// rows that are neighbours in space are neighbours in memory at a finer grain than the search cell, which is what
// the row-order gathers of the fused loop (anchor sets, NVT windows) feed on, and it lets the search cell be coarse.
#ifndef PCD_GRID_SUB
#define PCD_GRID_SUB 2
#endif
static constexpr int kGridSub = PCD_GRID_SUB;
PCD_DEV int sub_coord(float p, float o, float inv_h, int c, int sub) {
    const float f = fminf(fmaxf((p - o) * inv_h, -1.0e9f), 1.0e9f);   // as cell_coord
    const float r = (f - (float)c) * (float)(1 << sub);                 // exact: f - floor(f), times a power of two
    return min(max((int)floorf(r), 0), (1 << sub) - 1);
}
__global__ void k_keys(const float* __restrict__ xyz, int64_t n, float ox, float oy, float oz, float inv_h, int sub,
                       unsigned long long* __restrict__ keys, int32_t* __restrict__ vals) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    const int cx = cell_coord(x, ox, inv_h), cy = cell_coord(y, oy, inv_h), cz = cell_coord(z, oz, inv_h);
    const int fx = cx < 0 ? 0 : (cx << sub) | sub_coord(x, ox, inv_h, cx, sub);
    const int fy = cy < 0 ? 0 : (cy << sub) | sub_coord(y, oy, inv_h, cy, sub);
    const int fz = cz < 0 ? 0 : (cz << sub) | sub_coord(z, oz, inv_h, cz, sub);
    keys[i] = morton3(fx, fy, fz);
    vals[i] = (int32_t)i;
}

// sorted fine keys -> cell keys
__global__ void k_key_shift(unsigned long long* __restrict__ keys, int64_t n, int shift) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) keys[i] >>= shift;
}

__global__ void k_gather_sorted(const float* __restrict__ xyz, const int32_t* __restrict__ perm, int64_t n,
                                float4* __restrict__ pts) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t i = perm[r];
    pts[r] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], __uint_as_float((uint32_t)i));
}

// pts[n]: a row at +inf, the stand-in for the unused slots of a partial anchor set (rank n): its distance to any
// finite query is +inf, so the anchor test needs no per-slot validity select
__global__ void k_sentinel(float4* __restrict__ p) {
    if (threadIdx.x == 0) *p = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
}

// number of distinct (key >> shift) values of a sorted key array
__global__ void k_count_starts(const unsigned long long* __restrict__ keys, int64_t n, int shift, unsigned long long* count) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const bool st = (r < n) && (r == 0 || (keys[r] >> shift) != (keys[r - 1] >> shift));
    const unsigned long long b = __ballot(st);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (unsigned long long)__popcll(b));
}

__global__ void k_brick_flags(const unsigned long long* __restrict__ keys, int64_t n, uint32_t* __restrict__ flag) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r < n) flag[r] = (r == 0 || (keys[r] >> 6) != (keys[r - 1] >> 6)) ? 1u : 0u;
}

// bidx = inclusive scan of the brick-start flags: row r lies in brick bidx[r] - 1 (bricks numbered in Morton order)
__global__ void k_insert(const unsigned long long* __restrict__ keys, const uint32_t* __restrict__ bidx, int64_t n,
                         HashSlot* table, int hbits, unsigned long long mask, uint2* __restrict__ cellr) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    const unsigned long long key = keys[r];
    if (r != 0 && keys[r - 1] == key) return;        // one thread per cell
    int64_t end = r + 1;
    while (end < n && keys[end] == key) ++end;
    const uint32_t b = bidx[r] - 1u;
    cellr[(uint64_t)b * 64 + (key & 63)] = make_uint2((uint32_t)r, (uint32_t)end);
    if (r != 0 && (keys[r - 1] >> 6) == (key >> 6)) return;   // one thread per brick inserts it
    const unsigned long long bkey = key >> 6;
    unsigned long long slot = hash_slot(bkey, hbits);
    for (;;) {
        unsigned long long prev = atomicCAS(&table[slot].key, kEmptyKey, bkey);
        if (prev == kEmptyKey || prev == bkey) break;
        slot = (slot + 1) & mask;
    }
    table[slot].brick = b;
}

// ------------------------------------------------------------------ query kernels
template <int K, bool ORIG>
__global__ __launch_bounds__(256) void k_knn(GridView g, const float* __restrict__ q, int64_t nq, int kq, int k,
                                              void* __restrict__ idx_out, int idx64, int exclude_self,
                                              float* __restrict__ d2_out, const int32_t* __restrict__ order) {
    const int64_t nb = gridDim.x;
    const int64_t b = xcd_block(blockIdx.x, nb);
    const int64_t t = b * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const int64_t i = order ? (int64_t)order[t] : t;   // spatial order: a wave's queries share cells and L2 lines
    const Vec3 qi = v3(q[3 * i], q[3 * i + 1], q[3 * i + 2]);
    TopK<K> tk;
    knn_search<K, ORIG>(g, qi, tk);
    int w = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int id = tk.idx(j);
        const bool take = (w < k) && (j < kq) && !(exclude_self && id == i);
        if (take) {
            if (idx64) reinterpret_cast<int64_t*>(idx_out)[i * k + w] = id;
            else reinterpret_cast<int32_t*>(idx_out)[i * k + w] = id;
            if (d2_out) d2_out[i * k + w] = tk.d2(j);
            ++w;
        }
    }
}

__global__ void k_nn1(GridView g, const float* __restrict__ q, int64_t nq, float* __restrict__ d2_out,
                      int64_t* __restrict__ idx_out, const int32_t* __restrict__ order) {
    const int64_t t = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const int64_t i = order ? (int64_t)order[t] : t;
    TopK<1> tk;
    knn_search<1, true>(g, v3(q[3 * i], q[3 * i + 1], q[3 * i + 2]), tk);
    if (d2_out) d2_out[i] = tk.d2(0);
    if (idx_out) idx_out[i] = tk.idx(0);
}

// ------------------------------------------------------------------ radius search (CPSD selection)
// Selector.getPointsInRangeSelectionVectorized (Pointcloud/Modules/Selector.py:214-230): scipy query_ball_point on the
// frozen f64 snapshot.  The membership test is scipy's own: ((dx² + dy²) + dz²) <= r² in float64 on the f32 inputs
// (exact conversions), so the sets are identical, not just within a tolerance.  FILL = false counts per query,
// FILL = true writes the members' ORIGINAL indices at out + off[q] (then sorted per query, scipy's order for
// multi-point queries).
template <bool FILL>
__global__ __launch_bounds__(256) void k_radius(GridView g, const float* __restrict__ q, int64_t nq,
                                                 const float* __restrict__ radii, int64_t* __restrict__ count,
                                                 const int64_t* __restrict__ off, int64_t* __restrict__ out) {
    const int64_t i = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
    const double r = (double)radii[i];
    const double r2 = r * r;
    int64_t n = 0, w = FILL ? off[i] : 0;
    if (r >= 0.0) {
        // cells overlapping [q - r, q + r]; the f32 box is widened by one ulp-scale margin, the test is exact f64
        const float rf = (float)(r * (1.0 + 1e-6)) + 1e-30f;
        const int lo[3] = {max(cell_coord(qx - rf, g.ox, g.inv_h), 0), max(cell_coord(qy - rf, g.oy, g.inv_h), 0),
                           max(cell_coord(qz - rf, g.oz, g.inv_h), 0)};
        const int hi[3] = {min(cell_coord(qx + rf, g.ox, g.inv_h), g.dx - 1), min(cell_coord(qy + rf, g.oy, g.inv_h), g.dy - 1),
                           min(cell_coord(qz + rf, g.oz, g.inv_h), g.dz - 1)};
        for (int cz = lo[2]; cz <= hi[2]; ++cz)
            for (int cy = lo[1]; cy <= hi[1]; ++cy)
                for (int cx = lo[0]; cx <= hi[0]; ++cx) {
                    uint32_t s, e;
                    if (!cell_range(g, cx, cy, cz, s, e)) continue;
                    for (uint32_t r0 = s; r0 < e; ++r0) {
                        const float4 p = g.pts[r0];
                        const double dx = (double)qx - (double)p.x, dy = (double)qy - (double)p.y,
                                     dz = (double)qz - (double)p.z;
                        const double d2 = __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
                        if (d2 <= r2) {
                            if (FILL) out[w++] = (int64_t)__float_as_uint(p.w);
                            ++n;
                        }
                    }
                }
    }
    if (!FILL) count[i] = n;
}

// K capacity ladder of the register top-k lists.
static const int kCaps[] = {1, 4, 8, 13, 16, 32, 64};
int knn_cap(int k) {
    for (int c : kCaps)
        if (k <= c) return c;
    return -1;
}

// Queries in the caller's order are spatially random (a moved cloud in its input order): every lane of a wave then
// reads its own cells and nothing is shared in L1/L2 (the 6 KB/query of the round-1 kNN(6) over 10M points).  Large
// query sets are processed in the Morton order of the grid's lattice instead: keys, a radix sort of (key, index),
// and the kernels read query order[t] and write row order[t].  Results are identical (per-query work only moves).
struct QueryOrder {
    int32_t* order = nullptr;
    void* mem = nullptr;
    hipStream_t st = nullptr;
    ~QueryOrder() { if (mem) (void)hipFreeAsync(mem, st); }   // stream-ordered: after the kernels that read it
};
static constexpr int64_t kOrderMinQueries = 32768;
static int query_order(const GridView& g, const float* q, int64_t nq, hipStream_t st, QueryOrder& qo) {
    if (nq < kOrderMinQueries || nq >= (int64_t)INT32_MAX) return PCD_OK;
    int maxd = std::max({g.dx, g.dy, g.dz, 2});
    int bits = 0;
    while ((1 << bits) < maxd) ++bits;
    const unsigned end_bit = (unsigned)std::min(63, 3 * bits);
    size_t tmp_bytes = 0;
    unsigned long long *keys = nullptr, *keys2 = nullptr;
    int32_t *vals = nullptr, *order = nullptr;
    (void)rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys, keys2, vals, order, (size_t)nq, 0u, end_bit, st);
    const size_t off_k2 = (size_t)nq * 8, off_v = 2 * off_k2, off_o = off_v + (size_t)nq * 4,
                 off_t = (off_o + (size_t)nq * 4 + 255) & ~(size_t)255;
    if (hipMallocAsync(&qo.mem, off_t + tmp_bytes, st) != hipSuccess) return fail(PCD_ERR_OOM, "query order scratch");
    qo.st = st;
    char* base = static_cast<char*>(qo.mem);
    keys = reinterpret_cast<unsigned long long*>(base);
    keys2 = reinterpret_cast<unsigned long long*>(base + off_k2);
    vals = reinterpret_cast<int32_t*>(base + off_v);
    order = reinterpret_cast<int32_t*>(base + off_o);
    hipLaunchKernelGGL(k_keys, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, st, q, nq, g.ox, g.oy, g.oz, g.inv_h, 0,
                       keys, vals);
    if (rocprim::radix_sort_pairs(base + off_t, tmp_bytes, keys, keys2, vals, order, (size_t)nq, 0u, end_bit, st) !=
        hipSuccess)
        return fail(PCD_ERR_HIP, "query order: rocprim::radix_sort_pairs failed");
    qo.order = order;
    return PCD_OK;
}

template <bool ORIG>
static int launch_knn(const GridView& g, const float* q, int64_t nq, int kq, int k, void* idx, int idx64,
                      int excl, float* d2, hipStream_t st) {
    QueryOrder qo;
    if (const int rc = query_order(g, q, nq, st, qo); rc != PCD_OK) return rc;
    const int cap = knn_cap(kq);
    const dim3 blk(256), grd((unsigned)cdiv(nq, 256));
#define PCD_KNN_CASE(C) \
    case C: hipLaunchKernelGGL((k_knn<C, ORIG>), grd, blk, 0, st, g, q, nq, kq, k, idx, idx64, excl, d2, qo.order); break;
    switch (cap) {
        PCD_KNN_CASE(1) PCD_KNN_CASE(4) PCD_KNN_CASE(8) PCD_KNN_CASE(13) PCD_KNN_CASE(16) PCD_KNN_CASE(32)
        PCD_KNN_CASE(64)
        default: return fail(PCD_ERR_ARG, "pcd_knn: k larger than pcd_max_k()");
    }
#undef PCD_KNN_CASE
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

// ------------------------------------------------------------------ host: cell size selection
// Surface-sampled clouds: mean occupancy of a non-empty cell grows like h^2, and a strided sample of S points at
// cell h_s*sqrt(N/S) has the same occupancy as the full cloud at h_s.  Aim for ~max(2, k_hint/2) points per
// occupied cell, so the 27-cell block usually holds the k nearest.  Only speed depends on this choice.
static float choose_cell(const std::vector<float>& smp, int64_t n, const float mn[3], const float mx[3], int k_hint) {
    const int64_t S = (int64_t)smp.size() / 3;
    const float target = std::max(2.0f, 0.5f * (float)k_hint);
    const double ext = std::max({(double)mx[0] - mn[0], (double)mx[1] - mn[1], (double)mx[2] - mn[2], 1e-30});
    double hs = ext * std::sqrt((double)target / std::max<int64_t>(S, 1));
    std::vector<unsigned long long> keys((size_t)S);
    for (int it = 0; it < 4; ++it) {
        for (int64_t i = 0; i < S; ++i) {
            unsigned long long c[3];
            for (int a = 0; a < 3; ++a) c[a] = (unsigned long long)std::floor((smp[3 * i + a] - mn[a]) / hs) & 0x1fffff;
            keys[i] = c[0] | (c[1] << 21) | (c[2] << 42);
        }
        std::sort(keys.begin(), keys.end());
        const int64_t u = std::unique(keys.begin(), keys.end()) - keys.begin();
        const double occ = (double)S / (double)std::max<int64_t>(u, 1);
        const double f = std::sqrt(target / occ);
        hs *= std::min(std::max(f, 0.25), 4.0);
        if (std::fabs(f - 1.0) < 0.05) break;
    }
    double h = hs * std::sqrt((double)S / (double)std::max<int64_t>(n, 1));
    // keep every axis within 2^21 cells
    h = std::max(h, ext / 2000000.0);
    if (!(h > 0) || !std::isfinite(h)) h = 1.0;
    return (float)h;
}

}  // namespace pcd

using namespace pcd;

extern "C" {

const char* pcd_last_error(void) { return g_last_error.c_str(); }
int pcd_version(void) { return 1; }
int pcd_max_k(void) { return 64; }
int pcd_denoise_params_size(void) { return (int)sizeof(pcd_denoise_params); }

// bbox + cell edge of a point set (the part of the build that fixes the cell lattice).
static int grid_lattice(const float* xyz, int64_t n, int k_hint, float cell, hipStream_t st, float mn[3], float mx[3],
                        float& h_out) {
    const int nbb = 512;
    float* part = nullptr;
    if (hipMalloc(&part, nbb * 6 * sizeof(float)) != hipSuccess) return fail(PCD_ERR_OOM, "bbox");
    hipLaunchKernelGGL(k_bbox, dim3(nbb), dim3(256), 0, st, xyz, n, part);
    std::vector<float> hp(nbb * 6);
    (void)hipMemcpyAsync(hp.data(), part, nbb * 6 * sizeof(float), hipMemcpyDeviceToHost, st);
    // strided sample for the cell-size heuristic
    const int64_t S = std::min<int64_t>(n, 65536);
    const int64_t stride = n / S;
    float* dsmp = nullptr;
    if (hipMalloc(&dsmp, S * 3 * sizeof(float)) != hipSuccess) { (void)hipFree(part); return fail(PCD_ERR_OOM, "sample"); }
    hipLaunchKernelGGL(k_sample, dim3((unsigned)cdiv(S, 256)), dim3(256), 0, st, xyz, n, stride, S, dsmp);
    std::vector<float> smp(S * 3);
    (void)hipMemcpyAsync(smp.data(), dsmp, S * 3 * sizeof(float), hipMemcpyDeviceToHost, st);
    hipError_t e = hipStreamSynchronize(st);
    (void)hipFree(part);
    (void)hipFree(dsmp);
    if (e != hipSuccess) return fail(PCD_ERR_HIP, std::string("grid bbox: ") + hipGetErrorString(e));
    for (int a = 0; a < 3; ++a) { mn[a] = 3.0e38f; mx[a] = -3.0e38f; }
    for (int b = 0; b < nbb; ++b)
        for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], hp[b * 6 + a]); mx[a] = std::max(mx[a], hp[b * 6 + 3 + a]); }
    for (int a = 0; a < 3; ++a)
        if (!std::isfinite(mn[a]) || !std::isfinite(mx[a])) return fail(PCD_ERR_ARG, "pcd_grid_build: non-finite coordinates");
    float h = cell > 0 ? cell : choose_cell(smp, n, mn, mx, k_hint);
    for (int a = 0; a < 3; ++a) {
        const double dimd = std::floor(((double)mx[a] - mn[a]) / h) + 1.0;
        if (dimd >= 2097151.0) h = (float)(((double)mx[a] - mn[a]) / 2000000.0);
    }
    h_out = h;
    return PCD_OK;
}

int pcd_grid_params(const float* xyz, int64_t n, int k_hint, float cell, float* origin3, float* cell_out, void* stream) {
    PCD_CHECK_ARG(xyz != nullptr && n > 0 && origin3 && cell_out, "null argument or empty point set");
    float mn[3], mx[3], h;
    const int rc = grid_lattice(xyz, n, k_hint, cell, as_stream(stream), mn, mx, h);
    if (rc != PCD_OK) return rc;
    for (int a = 0; a < 3; ++a) origin3[a] = mn[a];
    *cell_out = h;
    return PCD_OK;
}

int pcd_grid_build(const float* xyz, int64_t n, int k_hint, float cell, const float* origin3, void* stream,
                   pcd_grid** out) {
    PCD_CHECK_ARG(out != nullptr, "out is null");
    *out = nullptr;
    PCD_CHECK_ARG(xyz != nullptr && n > 0, "empty point set");
    PCD_CHECK_ARG(n < (int64_t)INT32_MAX, "more than 2^31-1 points in one grid");
    PCD_CHECK_ARG(!origin3 || cell > 0, "an explicit origin needs an explicit cell edge");
    hipStream_t st = as_stream(stream);
    float mn[3], mx[3], h;
    int rc = grid_lattice(xyz, n, k_hint, cell, st, mn, mx, h);
    if (rc != PCD_OK) return rc;
    if (origin3) {
        for (int a = 0; a < 3; ++a) {
            PCD_CHECK_ARG(std::isfinite(origin3[a]) && origin3[a] <= mn[a], "origin must lie below every point");
            mn[a] = origin3[a];
            PCD_CHECK_ARG(std::floor(((double)mx[a] - mn[a]) / h) + 1.0 < 2097151.0, "origin/cell give more than 2^21 cells per axis");
        }
    }
    pcd_grid* g = new pcd_grid();
    g->n = n;
    PCD_HIP(hipGetDevice(&g->device));
    auto cleanup = [&]() { pcd_grid_destroy(g); };
    hipError_t e;
    GridView& v = g->view;
    v.h = h;
    v.inv_h = 1.0f / h;
    v.ox = mn[0]; v.oy = mn[1]; v.oz = mn[2];
    v.dx = (int)std::floor(((double)mx[0] - mn[0]) * v.inv_h) + 2;
    v.dy = (int)std::floor(((double)mx[1] - mn[1]) * v.inv_h) + 2;
    v.dz = (int)std::floor(((double)mx[2] - mn[2]) * v.inv_h) + 2;
    v.n = n;

    // keys + sort
    unsigned long long *keys = nullptr, *keys2 = nullptr, *cnt = nullptr;
    int32_t* vals = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    auto free_tmp = [&]() { (void)hipFree(keys); (void)hipFree(keys2); (void)hipFree(vals); (void)hipFree(tmp); (void)hipFree(cnt); };
    if (hipMalloc(&keys, n * 8) != hipSuccess || hipMalloc(&keys2, n * 8) != hipSuccess ||
        hipMalloc(&vals, n * 4) != hipSuccess || hipMalloc(&g->perm, n * 4) != hipSuccess ||
        hipMalloc(&g->pts, (n + 1) * sizeof(float4)) != hipSuccess || hipMalloc(&cnt, 16) != hipSuccess) {
        free_tmp(); cleanup(); return fail(PCD_ERR_OOM, "pcd_grid_build: device allocation");
    }
    const dim3 blk(256), grd((unsigned)cdiv(n, 256));
    const int sub = std::max({v.dx, v.dy, v.dz}) <= (1 << (21 - kGridSub)) ? kGridSub : 0;
    hipLaunchKernelGGL(k_keys, grd, blk, 0, st, xyz, n, v.ox, v.oy, v.oz, v.inv_h, sub, keys, vals);
    (void)rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys, keys2, vals, g->perm, (size_t)n, 0u, 63u, st);
    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) { free_tmp(); cleanup(); return fail(PCD_ERR_OOM, "sort temp"); }
    if (rocprim::radix_sort_pairs(tmp, tmp_bytes, keys, keys2, vals, g->perm, (size_t)n, 0u, 63u, st) != hipSuccess) {
        free_tmp(); cleanup(); return fail(PCD_ERR_HIP, "rocprim::radix_sort_pairs failed");
    }
    if (sub) hipLaunchKernelGGL(k_key_shift, grd, blk, 0, st, keys2, n, 3 * sub);
    hipLaunchKernelGGL(k_gather_sorted, grd, blk, 0, st, xyz, g->perm, n, g->pts);
    hipLaunchKernelGGL(k_sentinel, dim3(1), dim3(64), 0, st, g->pts + n);
    (void)hipMemsetAsync(cnt, 0, 16, st);
    hipLaunchKernelGGL(k_count_starts, grd, blk, 0, st, keys2, n, 0, cnt);
    hipLaunchKernelGGL(k_count_starts, grd, blk, 0, st, keys2, n, 6, cnt + 1);
    unsigned long long counts[2] = {0, 0};
    (void)hipMemcpyAsync(counts, cnt, 16, hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) { free_tmp(); cleanup(); return fail(PCD_ERR_HIP, std::string("grid sort: ") + hipGetErrorString(e)); }
    g->cells = (int64_t)counts[0];
    g->bricks = (int64_t)counts[1];
    int hbits = 1;
    while ((1ll << hbits) < 2 * g->bricks) ++hbits;
    g->slots = 1ll << hbits;
    uint32_t* bflag = reinterpret_cast<uint32_t*>(vals);   // vals is free after the sort: reuse for the flags,
    uint32_t* bidx = reinterpret_cast<uint32_t*>(keys);    // keys (pre-sort) for their scan
    if (hipMalloc(&g->table, g->slots * sizeof(HashSlot)) != hipSuccess ||
        hipMalloc(&g->cellr, g->bricks * 64 * sizeof(uint2)) != hipSuccess) {
        free_tmp(); cleanup(); return fail(PCD_ERR_OOM, "brick table");
    }
    (void)hipMemsetAsync(g->table, 0xFF, g->slots * sizeof(HashSlot), st);
    (void)hipMemsetAsync(g->cellr, 0, g->bricks * 64 * sizeof(uint2), st);
    hipLaunchKernelGGL(k_brick_flags, grd, blk, 0, st, keys2, n, bflag);
    size_t scan_bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, scan_bytes, bflag, bidx, (size_t)n, rocprim::plus<uint32_t>(), st);
    if (scan_bytes > tmp_bytes) {
        (void)hipFree(tmp);
        tmp = nullptr;
        if (hipMalloc(&tmp, scan_bytes) != hipSuccess) { free_tmp(); cleanup(); return fail(PCD_ERR_OOM, "scan temp"); }
    }
    if (rocprim::inclusive_scan(tmp, scan_bytes, bflag, bidx, (size_t)n, rocprim::plus<uint32_t>(), st) != hipSuccess) {
        free_tmp(); cleanup(); return fail(PCD_ERR_HIP, "rocprim::inclusive_scan failed");
    }
    hipLaunchKernelGGL(k_insert, grd, blk, 0, st, keys2, bidx, n, g->table, hbits, (unsigned long long)(g->slots - 1),
                       g->cellr);
    e = hipStreamSynchronize(st);
    free_tmp();
    if (e != hipSuccess) { cleanup(); return fail(PCD_ERR_HIP, std::string("grid hash: ") + hipGetErrorString(e)); }
    v.pts = g->pts;
    v.table = g->table;
    v.cells = g->cellr;
    {
        // a row's key comes from fp32 (p - o) * inv_h: its true position can sit a few ulps of |p|, |o| and of the
        // cell coordinate (times h) outside the box its cell describes
        const double amax = std::max({std::fabs((double)mn[0]), std::fabs((double)mn[1]), std::fabs((double)mn[2]),
                                      std::fabs((double)mx[0]), std::fabs((double)mx[1]), std::fabs((double)mx[2])});
        const double dmax = std::max({v.dx, v.dy, v.dz});
        v.slack = (float)(8.0 * std::ldexp(1.0, -23) * (2.0 * amax + dmax * (double)h));
    }
    v.hbits = hbits;
    v.mask = (unsigned long long)(g->slots - 1);
    *out = g;
    return PCD_OK;
}

int pcd_grid_destroy(pcd_grid* g) {
    if (!g) return PCD_OK;
    (void)hipFree(g->pts);
    (void)hipFree(g->perm);
    (void)hipFree(g->table);
    (void)hipFree(g->cellr);

    delete g;
    return PCD_OK;
}

// the snapshot back in caller order (pts[r] -> xyz[perm[r]])
__global__ void k_unsort_xyz(const float4* __restrict__ pts, const int32_t* __restrict__ perm, int64_t n,
                             float* __restrict__ xyz) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float4 p = pts[r];
    const int64_t i = perm[r];
    xyz[3 * i] = p.x; xyz[3 * i + 1] = p.y; xyz[3 * i + 2] = p.z;
}

int pcd_grid_rebuild(const pcd_grid* src, int k_hint, float cell, void* stream, pcd_grid** out) {
    PCD_CHECK_ARG(src && out, "null argument");
    *out = nullptr;
    hipStream_t st = as_stream(stream);
    float* xyz = nullptr;
    if (hipMalloc(&xyz, src->n * 3 * sizeof(float)) != hipSuccess) return fail(PCD_ERR_OOM, "pcd_grid_rebuild: xyz");
    hipLaunchKernelGGL(k_unsort_xyz, dim3((unsigned)cdiv(src->n, 256)), dim3(256), 0, st, src->pts, src->perm, src->n, xyz);
    const int rc = pcd_grid_build(xyz, src->n, k_hint, cell, nullptr, stream, out);   // (synchronises st)
    (void)hipStreamSynchronize(st);
    (void)hipFree(xyz);
    return rc;
}

int pcd_grid_get_info(const pcd_grid* g, pcd_grid_info_t* out) {
    PCD_CHECK_ARG(g && out, "null argument");
    out->n = g->n;
    out->cells = g->cells;
    out->table_slots = g->slots;
    out->cell = g->view.h;
    out->origin[0] = g->view.ox; out->origin[1] = g->view.oy; out->origin[2] = g->view.oz;
    out->dims[0] = g->view.dx; out->dims[1] = g->view.dy; out->dims[2] = g->view.dz;
    return PCD_OK;
}

int pcd_grid_perm(const pcd_grid* g, int32_t* perm, void* stream) {
    PCD_CHECK_ARG(g && perm, "null argument");
    PCD_HIP(hipMemcpyAsync(perm, g->perm, g->n * sizeof(int32_t), hipMemcpyDeviceToDevice, as_stream(stream)));
    return PCD_OK;
}

int pcd_knn(const pcd_grid* g, const float* q, int64_t nq, int k, void* idx_out, int idx_bits, int sorted_ids,
            int exclude_self, float* d2_out, void* stream) {
    PCD_CHECK_ARG(g != nullptr, "grid is null");
    PCD_CHECK_ARG(k >= 1 && k <= pcd_max_k(), "k out of range [1, pcd_max_k()]");
    PCD_CHECK_ARG(idx_bits == 32 || idx_bits == 64, "idx_bits must be 32 or 64");
    const int kq = k + (exclude_self ? 1 : 0);
    PCD_CHECK_ARG(kq <= g->n, "k exceeds the number of snapshot points");
    PCD_CHECK_ARG(kq <= pcd_max_k(), "k (+1 for exclude_self) exceeds pcd_max_k()");
    if (nq == 0) return PCD_OK;
    PCD_CHECK_ARG(q && idx_out, "null query / output");
    PCD_CHECK_ARG(!(exclude_self && sorted_ids), "exclude_self requires original ids");
    hipStream_t st = as_stream(stream);
    return sorted_ids ? launch_knn<false>(g->view, q, nq, kq, k, idx_out, idx_bits == 64, exclude_self, d2_out, st)
                      : launch_knn<true>(g->view, q, nq, kq, k, idx_out, idx_bits == 64, exclude_self, d2_out, st);
}

int pcd_radius_count(const pcd_grid* g, const float* q, int64_t nq, const float* radii, int64_t* counts,
                     void* stream) {
    PCD_CHECK_ARG(g != nullptr, "grid is null");
    if (nq == 0) return PCD_OK;
    PCD_CHECK_ARG(q && radii && counts, "null argument");
    hipLaunchKernelGGL(k_radius<false>, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, as_stream(stream), g->view, q,
                       nq, radii, counts, nullptr, nullptr);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_radius_fill(const pcd_grid* g, const float* q, int64_t nq, const float* radii, const int64_t* offsets,
                    int64_t total, int64_t* idx_out, void* stream) {
    PCD_CHECK_ARG(g != nullptr, "grid is null");
    if (nq == 0 || total == 0) return PCD_OK;
    PCD_CHECK_ARG(q && radii && offsets && idx_out, "null argument");
    hipStream_t st = as_stream(stream);
    int64_t* tmp_keys = nullptr;
    void* tmp = nullptr;
    size_t bytes = 0;
    if (hipMalloc(&tmp_keys, total * sizeof(int64_t)) != hipSuccess) return fail(PCD_ERR_OOM, "radius fill temp");
    hipLaunchKernelGGL(k_radius<true>, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, st, g->view, q, nq, radii,
                       nullptr, offsets, tmp_keys);
    // ascending original index within each query (scipy sorts multi-point query_ball_point results)
    (void)rocprim::segmented_radix_sort_keys(nullptr, bytes, tmp_keys, idx_out, (unsigned int)total,
                                             (unsigned int)nq, offsets, offsets + 1, 0, 64, st);
    if (hipMalloc(&tmp, bytes) != hipSuccess) { (void)hipFree(tmp_keys); return fail(PCD_ERR_OOM, "radius sort temp"); }
    hipError_t e = rocprim::segmented_radix_sort_keys(tmp, bytes, tmp_keys, idx_out, (unsigned int)total,
                                                      (unsigned int)nq, offsets, offsets + 1, 0, 64, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(tmp);
    (void)hipFree(tmp_keys);
    if (e != hipSuccess) return fail(PCD_ERR_HIP, std::string("radius fill: ") + hipGetErrorString(e));
    return PCD_OK;
}

int pcd_nn_dist(const pcd_grid* g, const float* q, int64_t nq, float* d2_out, int64_t* idx_out, void* stream) {
    PCD_CHECK_ARG(g != nullptr, "grid is null");
    if (nq == 0) return PCD_OK;
    PCD_CHECK_ARG(q != nullptr, "null query");
    QueryOrder qo;
    if (const int rc = query_order(g->view, q, nq, as_stream(stream), qo); rc != PCD_OK) return rc;
    hipLaunchKernelGGL(k_nn1, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, as_stream(stream), g->view, q, nq,
                       d2_out, idx_out, qo.order);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

}  // extern "C"
