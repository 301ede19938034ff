// Mesh vertex update (H18): Mesh.updateVertices, PatchGeneration/Modules/Mesh.py:377-418 (= Vertex_updating.ipynb
// Algorithm 3; native twin MeshDenoisingBase::updateVertexPosition, src/GCNDenoiser/GCNDenoiser/
// MeshDenoisingBase.cpp:107-143).  One thread per vertex gathers its incident faces through the igl
// vertex->face CSR (VF, NI) instead of the reference's padded (V, max_degree, 3, 3) temporaries; fp64 like numpy;
// Jacobi sweeps (the reference adds the whole update after computing it for every vertex).
#include "pcd_host.h"

namespace pcd {

__global__ __launch_bounds__(256) void k_mesh_update(const double* __restrict__ vin, double* __restrict__ vout,
                                                      int64_t nv, const int64_t* __restrict__ f,
                                                      const double* __restrict__ fn, const int64_t* __restrict__ vf,
                                                      const int64_t* __restrict__ ni) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const double x = vin[3 * i], y = vin[3 * i + 1], z = vin[3 * i + 2];
    double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};   // [corner][axis], summed over faces first (numpy order)
    const int64_t s = ni[i], e = ni[i + 1];
    for (int64_t t = s; t < e; ++t) {
        const int64_t face = vf[t];
        const double n0 = fn[3 * face], n1 = fn[3 * face + 1], n2 = fn[3 * face + 2];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int64_t vc = f[3 * face + c];
            const double d0 = vin[3 * vc] - x, d1 = vin[3 * vc + 1] - y, d2 = vin[3 * vc + 2] - z;
            const double dot = __dadd_rn(__dadd_rn(__dmul_rn(n0, d0), __dmul_rn(n1, d1)), __dmul_rn(n2, d2));
            S[c][0] = __dadd_rn(S[c][0], __dmul_rn(dot, n0));
            S[c][1] = __dadd_rn(S[c][1], __dmul_rn(dot, n1));
            S[c][2] = __dadd_rn(S[c][2], __dmul_rn(dot, n2));
        }
    }
    const double deg3 = 3.0 * (double)(e - s);   // degree 0 -> 0/0 = NaN, as numpy
    vout[3 * i] = x + (S[0][0] + S[1][0] + S[2][0]) / deg3;
    vout[3 * i + 1] = y + (S[0][1] + S[1][1] + S[2][1]) / deg3;
    vout[3 * i + 2] = z + (S[0][2] + S[1][2] + S[2][2]) / deg3;
}

}  // namespace pcd

using namespace pcd;

extern "C" int pcd_mesh_update(double* v, int64_t nv, const int64_t* f, const double* fn, int64_t nf,
                               const int64_t* vf, const int64_t* ni, int k, void* stream) {
    PCD_CHECK_ARG(k >= 0, "k must be >= 0");
    if (nv == 0 || k == 0) return PCD_OK;
    PCD_CHECK_ARG(v && f && fn && vf && ni && nf > 0, "null argument");
    hipStream_t st = as_stream(stream);
    double* tmp = nullptr;
    PCD_HIP(hipMallocAsync((void**)&tmp, nv * 3 * sizeof(double), st));
    double* buf[2] = {v, tmp};
    int cur = 0;
    const dim3 grd((unsigned)cdiv(nv, 256)), blk(256);
    for (int it = 0; it < k; ++it) {
        hipLaunchKernelGGL(k_mesh_update, grd, blk, 0, st, buf[cur], buf[cur ^ 1], nv, f, fn, vf, ni);
        cur ^= 1;
    }
    PCD_LAUNCH_CHECK();
    if (cur != 0) PCD_HIP(hipMemcpyAsync(v, tmp, nv * 3 * sizeof(double), hipMemcpyDeviceToDevice, st));
    PCD_HIP(hipFreeAsync(tmp, st));
    return PCD_OK;
}
