// Diagnostic build of the kNN search with per-query work counters (cells considered / probed / found, candidates
// scanned, sorted inserts, extra rings).  Compiled into its own namespace so the counters never touch the
// production kernels.  Exported as pcd_knn_stats.
#define PCD_KNN_STATS 1
#include "pcd_knn.h"

namespace pcd {

template <int K>
__global__ void k_knn_stats(GridView g, const float* __restrict__ q, int64_t nq, unsigned long long* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    unsigned st[6] = {0, 0, 0, 0, 0, 0};
    if (i < nq) {
        TopK<K> tk;
        knn_search<K, false>(g, v3(q[3 * i], q[3 * i + 1], q[3 * i + 2]), tk);
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


extern "C" int pcd_knn_stats(const pcd_grid* g, const float* q, int64_t nq, int k, unsigned long long* out6,
                             void* stream) {
    PCD_CHECK_ARG(g && q && out6, "null argument");
    hipStream_t st = as_stream(stream);
    PCD_HIP(hipMemsetAsync(out6, 0, 6 * sizeof(unsigned long long), st));
    const dim3 grd((unsigned)cdiv(nq, 256)), blk(256);
    switch (k <= 8 ? 8 : k <= 16 ? 16 : 32) {
        case 8: hipLaunchKernelGGL(k_knn_stats<8>, grd, blk, 0, st, g->view, q, nq, out6); break;
        case 16: hipLaunchKernelGGL(k_knn_stats<16>, grd, blk, 0, st, g->view, q, nq, out6); break;
        default: hipLaunchKernelGGL(k_knn_stats<32>, grd, blk, 0, st, g->view, q, nq, out6); break;
    }
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}
