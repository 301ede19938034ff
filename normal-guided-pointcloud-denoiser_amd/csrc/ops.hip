// Public one-call-per-method kernels over caller-owned rows and CSR selections (the reference's
// Selection(i, j, slices), Pointcloud/Modules/Selector.py:41-134).  These back the drop-in Python classes when
// a notebook calls the operators one by one; the fused loop in denoise.hip is the throughput path.
#include "pcd_host.h"
#include "pcd_ops.h"

namespace pcd {

struct CsrNb {
    const int64_t* nbr;
    int64_t base;
    PCD_DEV int64_t operator()(int t) const { return nbr[base + t]; }
};
struct DenseNb64 {
    const int64_t* nbr;
    int64_t base;
    PCD_DEV int64_t operator()(int t) const { return nbr[base + t]; }
};

__global__ __launch_bounds__(256) void k_nvt_csr(Rows3 pos, Rows3 nrm, const int64_t* __restrict__ ci,
                                                  const int64_t* __restrict__ off, const int64_t* __restrict__ nbr,
                                                  int64_t m, float rho, float* __restrict__ eigval,
                                                  float* __restrict__ eigvec) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int64_t s = off[r], e = off[r + 1];
    const Vec3 vi = pos(ci[r]);
    const Sym3 T = nvt_tensor(pos, nrm, vi, (int)(e - s), CsrNb{nbr, s}, rho);
    float w[3], V[3][3];
    eigh3(T, w, V);
#pragma unroll
    for (int a = 0; a < 3; ++a) eigval[3 * r + a] = w[a];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) eigvec[9 * r + 3 * a + b] = V[a][b];
}

// The two device eigen-solvers on caller tensors (pcd_eigh3_batch): SOLVER 0 = eigh3 (the LAPACK ssyevd restatement
// NVT1 and the public ops run), 1 = eigh3_min (NVT2's fixed-sweep Jacobi on the hardware estimates, as k_nvt2
// compiles it).  t6 [m][6] = (a00, a01, a02, a11, a12, a22); vec: [m][3][3] columns (0) or the smallest's [m][3] (1).
template <int SOLVER>
__global__ __launch_bounds__(256) void k_eigh3_batch(const float* __restrict__ t6, int64_t m, float* __restrict__ w,
                                                      float* __restrict__ vec) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    const float* t = t6 + 6 * r;
    const Sym3 T{t[0], t[1], t[2], t[3], t[4], t[5]};
    float ww[3];
    if constexpr (SOLVER == 0) {
        float V[3][3];
        eigh3(T, ww, V);
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) vec[9 * r + 3 * a + b] = V[a][b];
    } else {
        Vec3 y;
        eigh3_min(T, ww, y);
        store3(vec, r, y);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) w[3 * r + a] = ww[a];
}

// CPSD tensors over a CSR selection (KIND 0: normal-filtered NVT, 1: normal-filtered PVT) + eigh.
template <int KIND>
__global__ __launch_bounds__(256) void k_cpsd_csr(Rows3 pos, Rows3 nrm, const int64_t* __restrict__ ci,
                                                   const int64_t* __restrict__ off, const int64_t* __restrict__ nbr,
                                                   int64_t m, float rho, float* __restrict__ eigval,
                                                   float* __restrict__ eigvec) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int64_t s = off[r], e = off[r + 1];
    const int64_t c = ci[r];
    const Sym3 T = KIND == 0 ? nvt_normal_tensor(nrm, nrm(c), (int)(e - s), CsrNb{nbr, s}, rho)
                             : pvt_normal_cov(pos, nrm, pos(c), nrm(c), (int)(e - s), CsrNb{nbr, s}, rho);
    float w[3], V[3][3];
    eigh3(T, w, V);
#pragma unroll
    for (int a = 0; a < 3; ++a) eigval[3 * r + a] = w[a];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) eigvec[9 * r + 3 * a + b] = V[a][b];
}

__global__ void k_vu_smooth(const float* __restrict__ eigval, const float* __restrict__ eigvec, Rows3 n, int64_t m,
                            float tau, float damp, float* __restrict__ out) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    float w[3], V[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a) w[a] = eigval[3 * r + a];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) V[a][b] = eigvec[9 * r + 3 * a + b];
    store3(out, r, vu_smooth(w, V, n(r), tau, damp));
}

__global__ void k_classify(const float* __restrict__ eigval, int64_t m, float scale, float* __restrict__ feat,
                           int64_t* __restrict__ cls) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    const float w[3] = {eigval[3 * r], eigval[3 * r + 1], eigval[3 * r + 2]};
    float f[3];
    const int c = classify(w, scale, f);
    if (feat) { feat[3 * r] = f[0]; feat[3 * r + 1] = f[1]; feat[3 * r + 2] = f[2]; }
    if (cls) cls[r] = c;
}

__global__ __launch_bounds__(256) void k_pca_dense(Rows3 pos, int64_t n, const int64_t* __restrict__ nbr, int k,
                                                    float* __restrict__ eigval, float* __restrict__ eigvec) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Sym3 C = pca_cov(pos, k, DenseNb64{nbr, i * k});
    float w[3], V[3][3];
    eigh3(C, w, V);
    if (eigval) {
#pragma unroll
        for (int a = 0; a < 3; ++a) eigval[3 * i + a] = w[a];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) eigvec[9 * i + 3 * a + b] = V[a][b];
}

// ---------------------------------------------------------------- global reductions for flat/new steps
// centre = mean over every row's v_j; delta = max ||v_j - centre||   (Denoiser.py:106-107, :138)
struct Red { double sx, sy, sz, cnt; };

__global__ void k_rows_sum(Rows3 pos, const int64_t* __restrict__ nbr, int64_t e, Red* __restrict__ part) {
    double sx = 0, sy = 0, sz = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < e; t += (int64_t)gridDim.x * blockDim.x) {
        const Vec3 v = pos(nbr[t]);
        sx += v.x; sy += v.y; sz += v.z;
    }
    __shared__ double s[3][256];
    s[0][threadIdx.x] = sx; s[1][threadIdx.x] = sy; s[2][threadIdx.x] = sz;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int a = 0; a < 3; ++a) s[a][threadIdx.x] += s[a][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = Red{s[0][0], s[1][0], s[2][0], 0.0};
}

// one block: reduce partials -> centre (fp32) at g[0..2], zero the delta slot g[3]
__global__ void k_finish_centre(const Red* __restrict__ part, int np, double count, float* __restrict__ g) {
    __shared__ double s[3][256];
    double a0 = 0, a1 = 0, a2 = 0;
    for (int b = threadIdx.x; b < np; b += blockDim.x) { a0 += part[b].sx; a1 += part[b].sy; a2 += part[b].sz; }
    s[0][threadIdx.x] = a0; s[1][threadIdx.x] = a1; s[2][threadIdx.x] = a2;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int a = 0; a < 3; ++a) s[a][threadIdx.x] += s[a][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        g[0] = (float)(s[0][0] / count);
        g[1] = (float)(s[1][0] / count);
        g[2] = (float)(s[2][0] / count);
        reinterpret_cast<unsigned int*>(g)[3] = 0u;
    }
}

__global__ void k_rows_maxdist(Rows3 pos, const int64_t* __restrict__ nbr, int64_t e, float* __restrict__ g) {
    const Vec3 c = v3(g[0], g[1], g[2]);
    float mx = 0.f;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < e; t += (int64_t)gridDim.x * blockDim.x)
        mx = fmaxf(mx, norm3(pos(nbr[t]) - c));
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(g) + 3, __float_as_uint(mx));
}

template <int KIND>
__global__ __launch_bounds__(256) void k_step_csr(Rows3 pos, Rows3 nrm, Rows3 ev, const int64_t* __restrict__ ci,
                                                   const int64_t* __restrict__ off, const int64_t* __restrict__ nbr,
                                                   int64_t m, const float* __restrict__ g, float d, float alpha,
                                                   float* __restrict__ out) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int64_t c = ci[r];
    const int64_t s = off[r];
    const int cnt = (int)(off[r + 1] - s);
    const Vec3 vi = pos(c);
    const CsrNb nb{nbr, s};
    Vec3 o;
    if (KIND == PCD_STEP_FLAT) o = step_flat(pos, nrm, vi, nrm(c), cnt, nb, __uint_as_float(((const unsigned*)g)[3]), d, alpha);
    else if (KIND == PCD_STEP_EDGE) o = step_edge(pos, nrm, vi, ev(c), cnt, nb, d, alpha);
    else if (KIND == PCD_STEP_FEATURE) o = step_feature<false>(pos, nrm, vi, nrm(c), cnt, nb, 1.f, d, alpha);
    else if (KIND == PCD_STEP_NEW) o = step_feature<true>(pos, nrm, vi, nrm(c), cnt, nb, __uint_as_float(((const unsigned*)g)[3]), d, alpha);
    else if (KIND == PCD_STEP_CORNER) o = step_corner(pos, nrm, vi, cnt, nb, d, alpha);
    else o = vi;
    store3(out, r, o);
}

__global__ void k_edge_len(Rows3 pos, const int64_t* __restrict__ a, const int64_t* __restrict__ b, int64_t e,
                           double* __restrict__ sum) {
    double acc = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < e; t += (int64_t)gridDim.x * blockDim.x)
        acc += (double)norm3(pos(b[t]) - pos(a[t]));
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

}  // namespace pcd

using namespace pcd;

extern "C" {

int pcd_nvt_csr(const float* pos, const float* n, int64_t npts, const int64_t* ci, const int64_t* off,
                const int64_t* nbr, int64_t m, float rho, float* eigval, float* eigvec, void* stream) {
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(pos && n && ci && off && nbr && eigval && eigvec, "null argument");
    PCD_CHECK_ARG(npts > 0, "empty point set");
    hipLaunchKernelGGL(k_nvt_csr, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, as_stream(stream), Rows3{pos},
                       Rows3{n}, ci, off, nbr, m, rho, eigval, eigvec);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_eigh3_batch(const float* t6, int64_t m, int solver, float* w, float* vec, void* stream) {
    PCD_CHECK_ARG(solver == 0 || solver == 1, "solver must be 0 (LAPACK restatement) or 1 (NVT2 Jacobi)");
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(t6 && w && vec, "null argument");
    const dim3 grd((unsigned)cdiv(m, 256)), blk(256);
    if (solver == 0) hipLaunchKernelGGL(k_eigh3_batch<0>, grd, blk, 0, as_stream(stream), t6, m, w, vec);
    else hipLaunchKernelGGL(k_eigh3_batch<1>, grd, blk, 0, as_stream(stream), t6, m, w, vec);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_nvt_normal_csr(const float* n, int64_t npts, const int64_t* ci, const int64_t* off, const int64_t* nbr,
                       int64_t m, float rho, float* eigval, float* eigvec, void* stream) {
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(n && ci && off && nbr && eigval && eigvec, "null argument");
    PCD_CHECK_ARG(npts > 0, "empty point set");
    hipLaunchKernelGGL(k_cpsd_csr<0>, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, as_stream(stream), Rows3{n},
                       Rows3{n}, ci, off, nbr, m, rho, eigval, eigvec);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_pvt_normal_csr(const float* pos, const float* n, int64_t npts, const int64_t* ci, const int64_t* off,
                       const int64_t* nbr, int64_t m, float rho, float* eigval, float* eigvec, void* stream) {
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(pos && n && ci && off && nbr && eigval && eigvec, "null argument");
    PCD_CHECK_ARG(npts > 0, "empty point set");
    hipLaunchKernelGGL(k_cpsd_csr<1>, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, as_stream(stream), Rows3{pos},
                       Rows3{n}, ci, off, nbr, m, rho, eigval, eigvec);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_vu_smooth(const float* eigval, const float* eigvec, const float* n, int64_t m, float tau, float damp,
                  float* out, void* stream) {
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(eigval && eigvec && n && out, "null argument");
    hipLaunchKernelGGL(k_vu_smooth, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, as_stream(stream), eigval, eigvec,
                       Rows3{n}, m, tau, damp, out);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_classify(const float* eigval, int64_t m, float scale, float* features, int64_t* classes, void* stream) {
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(eigval != nullptr, "null eigval");
    hipLaunchKernelGGL(k_classify, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, as_stream(stream), eigval, m, scale,
                       features, classes);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_pca_dense(const float* pos, int64_t n, const int64_t* nbr, int k, float* eigval, float* eigvec,
                  void* stream) {
    if (n == 0) return PCD_OK;
    PCD_CHECK_ARG(pos && nbr && eigvec && k > 0, "bad argument");
    hipLaunchKernelGGL(k_pca_dense, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream), Rows3{pos}, n,
                       nbr, k, eigval, eigvec);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_step_csr(int kind, const float* pos, const float* n, const float* edge_vectors, int64_t npts,
                 const int64_t* ci, const int64_t* off, const int64_t* nbr, int64_t m, float d, float alpha,
                 float* out, void* stream) {
    PCD_CHECK_ARG(kind >= PCD_STEP_FLAT && kind <= PCD_STEP_DUMMY, "unknown step kind");
    if (m == 0) return PCD_OK;
    PCD_CHECK_ARG(pos && n && ci && off && nbr && out, "null argument");
    PCD_CHECK_ARG(kind != PCD_STEP_EDGE || edge_vectors, "edge_step needs edge_vectors");
    hipStream_t st = as_stream(stream);
    float* g = nullptr;
    Red* part = nullptr;
    const int np = 512;
    if (kind == PCD_STEP_FLAT || kind == PCD_STEP_NEW) {
        int64_t e = 0;
        PCD_HIP(hipMemcpyAsync(&e, off + m, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PCD_HIP(hipStreamSynchronize(st));
        PCD_HIP(hipMallocAsync((void**)&g, 16, st));
        PCD_HIP(hipMallocAsync((void**)&part, np * sizeof(Red), st));
        // rows of the selection are nbr[off[0] .. off[m]); off[0] == 0 by the Selection contract
        hipLaunchKernelGGL(k_rows_sum, dim3(np), dim3(256), 0, st, Rows3{pos}, nbr, e, part);
        hipLaunchKernelGGL(k_finish_centre, dim3(1), dim3(256), 0, st, part, np, (double)e, g);
        hipLaunchKernelGGL(k_rows_maxdist, dim3(np), dim3(256), 0, st, Rows3{pos}, nbr, e, g);
    }
    const dim3 grd((unsigned)cdiv(m, 256)), blk(256);
    const Rows3 P{pos}, N{n}, E{edge_vectors};
    switch (kind) {
        case PCD_STEP_FLAT: hipLaunchKernelGGL(k_step_csr<PCD_STEP_FLAT>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
        case PCD_STEP_EDGE: hipLaunchKernelGGL(k_step_csr<PCD_STEP_EDGE>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
        case PCD_STEP_FEATURE: hipLaunchKernelGGL(k_step_csr<PCD_STEP_FEATURE>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
        case PCD_STEP_CORNER: hipLaunchKernelGGL(k_step_csr<PCD_STEP_CORNER>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
        case PCD_STEP_NEW: hipLaunchKernelGGL(k_step_csr<PCD_STEP_NEW>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
        default: hipLaunchKernelGGL(k_step_csr<PCD_STEP_DUMMY>, grd, blk, 0, st, P, N, E, ci, off, nbr, m, g, d, alpha, out); break;
    }
    PCD_LAUNCH_CHECK();
    if (g) { PCD_HIP(hipFreeAsync(g, st)); PCD_HIP(hipFreeAsync(part, st)); }
    return PCD_OK;
}

int pcd_edge_length_sum(const float* pos, const int64_t* a, const int64_t* b, int64_t e, double* sum_out,
                        void* stream) {
    PCD_CHECK_ARG(sum_out != nullptr, "null output");
    hipStream_t st = as_stream(stream);
    PCD_HIP(hipMemsetAsync(sum_out, 0, sizeof(double), st));
    if (e == 0) return PCD_OK;
    PCD_CHECK_ARG(pos && a && b, "null argument");
    hipLaunchKernelGGL(k_edge_len, dim3(512), dim3(256), 0, st, Rows3{pos}, a, b, e, sum_out);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

}  // extern "C"
