// Diagnostic build of the kNN search with per-query work counters (cells considered / probed / found, candidates
// scanned, sorted inserts (insertion) or drain merges (capped at the exact k-th key), extra rings).  Compiled into its own namespace so the counters never touch the
// production kernels.  Exported as pcd_knn_stats.
#define PCD_KNN_STATS 1
#include "pcd_knn.h"

namespace pcd {

template <int K, bool BATCHED>
__global__ void k_knn_stats(GridView g, const float* __restrict__ q, int64_t nq, unsigned long long* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    unsigned st[6] = {0, 0, 0, 0, 0, 0};
    if (i < nq) {
        TopK<K> tk;
        const Vec3 qi = v3(q[3 * i], q[3 * i + 1], q[3 * i + 2]);
        if constexpr (BATCHED) {  // capped search with the tightest valid cap: the exact k-th key + 1
            __shared__ uint32_t s_buf[48 * kCapStride];
            TopK<K> ex;
            knn_search<K, false>(g, qi, ex);
            knn_search_capped<K, 48>(g, qi, tk, ex.key[K - 1] + 1ull, s_buf + threadIdx.x);
        } else {
            knn_search<K, false>(g, qi, tk);
        }
        for (int s = 0; s < 6; ++s) st[s] = tk.stat[s];
    }
    for (int s = 0; s < 6; ++s) {
        unsigned long long v = st[s];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) atomicAdd(out + s, v);
    }
}

}  // namespace pcd

using namespace pcd;


extern "C" int pcd_knn_stats(const pcd_grid* g, const float* q, int64_t nq, int k, int variant,
                             unsigned long long* out6, void* stream) {
    PCD_CHECK_ARG(g && q && out6, "null argument");
    hipStream_t st = as_stream(stream);
    PCD_HIP(hipMemsetAsync(out6, 0, 6 * sizeof(unsigned long long), st));
    const dim3 grd((unsigned)cdiv(nq, 256)), blk(256);
    PCD_CHECK_ARG(variant == 0 || variant == 1, "variant must be 0 (insertion) or 1 (capped)");
    PCD_CHECK_ARG(variant == 0 || k > 8, "the capped variant is built for k 16 and 32");
    const int kc = k <= 8 ? 8 : k <= 16 ? 16 : 32;
#define PCD_KS(C, V) hipLaunchKernelGGL((k_knn_stats<C, V>), grd, blk, 0, st, g->view, q, nq, out6)
    if (variant == 0) {
        if (kc == 8) PCD_KS(8, false);
        else if (kc == 16) PCD_KS(16, false);
        else PCD_KS(32, false);
    } else {
        if (kc == 16) PCD_KS(16, true);
        else PCD_KS(32, true);
    }
#undef PCD_KS
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}
