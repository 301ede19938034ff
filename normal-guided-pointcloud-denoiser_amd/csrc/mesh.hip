// Mesh vertex update (H18): Mesh.updateVertices, PatchGeneration/Modules/Mesh.py:377-418 (= Vertex_updating.ipynb
// Algorithm 3; native twin MeshDenoisingBase::updateVertexPosition, src/GCNDenoiser/GCNDenoiser/
// MeshDenoisingBase.cpp:107-143).  One thread per vertex gathers its incident faces through the igl
// vertex->face CSR (VF, NI) instead of the reference's padded (V, max_degree, 3, 3) temporaries; fp64 like numpy;
// Jacobi sweeps (the reference adds the whole update after computing it for every vertex).
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "pcd_device.h"
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

// ---------------------------------------------------------------------------------------------- fp32 path
// The same update in fp32 on MI355X-shaped buffers: vertices and face normals as float4 rows (one 16-B load per
// gather), faces as int4 (three corner ids + pad), the vertex->face CSR in int32.  Algorithmic bytes per vertex per
// sweep: own v 12 + write 12 + NI 8 + per incident face (VF 4 + normal 12 + corners 12 + 3 corner
// rows 36) = 32 + 64 deg (416 B at deg 6).  Sums in the reference's order (per corner over faces, then corners).
__global__ __launch_bounds__(256) void k_mesh_update_f32(const float4* __restrict__ vin, float4* __restrict__ vout,
                                                          int64_t nv, const int4* __restrict__ f4,
                                                          const float4* __restrict__ fn4, const int32_t* __restrict__ vf,
                                                          const int32_t* __restrict__ ni) {
    const int64_t i = xcd_block(blockIdx.x, gridDim.x) * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const float4 p = vin[i];
    float S[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const int s = ni[i], e = ni[i + 1];
    for (int t = s; t < e; ++t) {
        const int face = vf[t];
        const float4 n = fn4[face];
        const int4 c = f4[face];
        const float4 q[3] = {vin[c.x], vin[c.y], vin[c.z]};   // the three corner rows in flight together
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float d0 = q[k].x - p.x, d1 = q[k].y - p.y, d2 = q[k].z - p.z;
            const float dot = (n.x * d0 + n.y * d1) + n.z * d2;
            S[k][0] += dot * n.x;
            S[k][1] += dot * n.y;
            S[k][2] += dot * n.z;
        }
    }
    const float deg3 = 3.f * (float)(e - s);
    vout[i] = make_float4(p.x + (S[0][0] + S[1][0] + S[2][0]) / deg3, p.y + (S[0][1] + S[1][1] + S[2][1]) / deg3,
                          p.z + (S[0][2] + S[1][2] + S[2][2]) / deg3, 0.f);
}
__global__ void k_rows3_to4(const float* __restrict__ a, int64_t n, float4* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float4(a[3 * i], a[3 * i + 1], a[3 * i + 2], 0.f);
}
__global__ void k_rows4_to3(const float4* __restrict__ a, int64_t n, float* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) { const float4 v = a[i]; out[3 * i] = v.x; out[3 * i + 1] = v.y; out[3 * i + 2] = v.z; }
}
template <class I>
__global__ void k_faces_to4(const I* __restrict__ f, int64_t nf, int4* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < nf) out[i] = make_int4((int)f[3 * i], (int)f[3 * i + 1], (int)f[3 * i + 2], 0);
}

// ---------------------------------------------------------------------------------------------- adjacency
// igl.vertex_triangle_adjacency on the device: corners (vertex id, corner index 3f + c) radix-sorted by vertex id
// (stable: each vertex's faces in increasing face order, igl's VF), VF = corner / 3, NI = first corner of each
// vertex in the sorted order (degree-0 vertices get empty ranges).
template <class I>
__global__ void k_vta_keys(const I* __restrict__ f, int64_t nc, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                           int* __restrict__ bad, int64_t nv) {
    const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (c >= nc) return;
    const int64_t v = (int64_t)f[c];
    if (v < 0 || v >= nv) atomicOr(bad, 1);
    keys[c] = (uint32_t)(v < 0 ? 0 : v >= nv ? nv - 1 : v);
    vals[c] = (uint32_t)c;
}
template <class I>
__global__ void k_vta_out(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals, int64_t nc,
                          int64_t nv, I* __restrict__ vf, I* __restrict__ ni) {
    const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (p > nc) return;
    if (p < nc) vf[p] = (I)(svals[p] / 3u);
    const int64_t prev = p == 0 ? -1 : (int64_t)skeys[p - 1];
    const int64_t cur = p == nc ? nv : (int64_t)skeys[p];
    for (int64_t v = prev + 1; v <= cur && v <= nv; ++v) ni[v] = (I)p;   // first corner of v (empty runs: same p)
    if (p == nc) ni[nv] = (I)nc;
}

}  // namespace pcd

using namespace pcd;

extern "C" int pcd_mesh_vta(const void* f, int f_bits, int64_t nf, int64_t nv, void* vf, void* ni, int out_bits,
                            void* stream) {
    PCD_CHECK_ARG((f_bits == 32 || f_bits == 64) && (out_bits == 32 || out_bits == 64), "bits must be 32 or 64");
    PCD_CHECK_ARG(nv >= 0 && nf >= 0 && 3 * nf < (1ll << 32) && nv < (1ll << 32), "mesh too large");
    PCD_CHECK_ARG(out_bits == 64 || 3 * nf < (1ll << 31), "int32 adjacency needs 3 nf < 2^31");
    hipStream_t st = as_stream(stream);
    if (nv == 0) return PCD_OK;
    PCD_CHECK_ARG(ni && (nf == 0 || (f && vf)), "null argument");
    const int64_t nc = 3 * nf;
    uint32_t *keys = nullptr, *vals = nullptr, *skeys = nullptr, *svals = nullptr;
    int* bad = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    const size_t n = (size_t)std::max<int64_t>(nc, 1);
    StreamTemps tt(st);                    // freed on every exit path
    PCD_HIP(tt.alloc(&keys, n * 4));
    PCD_HIP(tt.alloc(&vals, n * 4));
    PCD_HIP(tt.alloc(&skeys, n * 4));
    PCD_HIP(tt.alloc(&svals, n * 4));
    PCD_HIP(tt.alloc(&bad, sizeof(int)));
    PCD_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    const dim3 blk(256);
    if (nc > 0) {
        if (f_bits == 64) hipLaunchKernelGGL(k_vta_keys<int64_t>, dim3((unsigned)cdiv(nc, 256)), blk, 0, st, (const int64_t*)f, nc, keys, vals, bad, nv);
        else hipLaunchKernelGGL(k_vta_keys<int32_t>, dim3((unsigned)cdiv(nc, 256)), blk, 0, st, (const int32_t*)f, nc, keys, vals, bad, nv);
        unsigned end_bit = 1;
        while (end_bit < 32 && ((uint64_t)1 << end_bit) < (uint64_t)nv) ++end_bit;
        (void)rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys, skeys, vals, svals, (size_t)nc, 0u, end_bit, st);
        PCD_HIP(tt.alloc(&tmp, tmp_bytes));
        if (rocprim::radix_sort_pairs(tmp, tmp_bytes, keys, skeys, vals, svals, (size_t)nc, 0u, end_bit, st) != hipSuccess)
            return fail(PCD_ERR_HIP, "pcd_mesh_vta: rocprim::radix_sort_pairs failed");
    }
    const dim3 grd((unsigned)cdiv(nc + 1, 256));
    if (out_bits == 64) hipLaunchKernelGGL(k_vta_out<int64_t>, grd, blk, 0, st, skeys, svals, nc, nv, (int64_t*)vf, (int64_t*)ni);
    else hipLaunchKernelGGL(k_vta_out<int32_t>, grd, blk, 0, st, skeys, svals, nc, nv, (int32_t*)vf, (int32_t*)ni);
    PCD_LAUNCH_CHECK();
    int hbad = 0;
    PCD_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    PCD_HIP(tt.release());                 // (synchronises: hbad is valid)
    PCD_CHECK_ARG(hbad == 0, "face index out of range [0, nv)");
    return PCD_OK;
}

extern "C" int pcd_mesh_update_f32(float* v, int64_t nv, const int32_t* f, const float* fn, int64_t nf,
                                   const int32_t* vf, const int32_t* ni, int k, void* stream) {
    PCD_CHECK_ARG(k >= 0, "k must be >= 0");
    if (nv == 0 || k == 0) return PCD_OK;
    PCD_CHECK_ARG(v && f && fn && vf && ni && nf > 0, "null argument");
    PCD_CHECK_ARG(nv < (1ll << 31) && 3 * nf < (1ll << 31), "fp32 path: int32 indices");
    hipStream_t st = as_stream(stream);
    float4 *a = nullptr, *b = nullptr, *fn4 = nullptr;
    int4* f4 = nullptr;
    StreamTemps tt(st);                    // freed on every exit path
    PCD_HIP(tt.alloc(&a, nv * sizeof(float4)));
    PCD_HIP(tt.alloc(&b, nv * sizeof(float4)));
    PCD_HIP(tt.alloc(&fn4, nf * sizeof(float4)));
    PCD_HIP(tt.alloc(&f4, nf * sizeof(int4)));
    const dim3 blk(256);
    hipLaunchKernelGGL(k_rows3_to4, dim3((unsigned)cdiv(nv, 256)), blk, 0, st, v, nv, a);
    hipLaunchKernelGGL(k_rows3_to4, dim3((unsigned)cdiv(nf, 256)), blk, 0, st, fn, nf, fn4);
    hipLaunchKernelGGL(k_faces_to4<int32_t>, dim3((unsigned)cdiv(nf, 256)), blk, 0, st, f, nf, f4);
    float4* buf[2] = {a, b};
    int cur = 0;
    for (int it = 0; it < k; ++it) {
        hipLaunchKernelGGL(k_mesh_update_f32, dim3((unsigned)cdiv(nv, 256)), blk, 0, st, buf[cur], buf[cur ^ 1], nv,
                           f4, fn4, vf, ni);
        cur ^= 1;
    }
    hipLaunchKernelGGL(k_rows4_to3, dim3((unsigned)cdiv(nv, 256)), blk, 0, st, buf[cur], nv, v);
    PCD_LAUNCH_CHECK();
    PCD_HIP(tt.release(false));
    return PCD_OK;
}

extern "C" int pcd_mesh_update(double* v, int64_t nv, const int64_t* f, const double* fn, int64_t nf,
                               const int64_t* vf, const int64_t* ni, int k, void* stream) {
    PCD_CHECK_ARG(k >= 0, "k must be >= 0");
    if (nv == 0 || k == 0) return PCD_OK;
    PCD_CHECK_ARG(v && f && fn && vf && ni && nf > 0, "null argument");
    hipStream_t st = as_stream(stream);
    double* tmp = nullptr;
    StreamTemps tt(st);                    // freed on every exit path
    PCD_HIP(tt.alloc(&tmp, nv * 3 * sizeof(double)));
    double* buf[2] = {v, tmp};
    int cur = 0;
    const dim3 grd((unsigned)cdiv(nv, 256)), blk(256);
    for (int it = 0; it < k; ++it) {
        hipLaunchKernelGGL(k_mesh_update, grd, blk, 0, st, buf[cur], buf[cur ^ 1], nv, f, fn, vf, ni);
        cur ^= 1;
    }
    PCD_LAUNCH_CHECK();
    if (cur != 0) PCD_HIP(hipMemcpyAsync(v, tmp, nv * 3 * sizeof(double), hipMemcpyDeviceToDevice, st));
    PCD_HIP(tt.release(false));
    return PCD_OK;
}
