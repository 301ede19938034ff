// Host builds of the per-point math (the same __host__ __device__ source the kernels use), exported so the CPU
// test-suite can check eigen-decomposition signs, VU smoothing and the 3x3 solve without a GPU.
#include "pcd_host.h"
#include "pcd_ops.h"

using namespace pcd;

namespace {
struct HostCsrNb {
    const int64_t* nbr;
    int64_t base;
    int64_t operator()(int t) const { return nbr[base + t]; }
};
}  // namespace

extern "C" {

int pcd_host_eigh3(const float* t6, int64_t m, float* w, float* v) {
    PCD_CHECK_ARG(t6 && w && v, "null argument");
    for (int64_t i = 0; i < m; ++i) {
        const float* a = t6 + 6 * i;
        float ww[3], V[3][3];
        eigh3(Sym3{a[0], a[1], a[2], a[3], a[4], a[5]}, ww, V);
        for (int r = 0; r < 3; ++r) {
            w[3 * i + r] = ww[r];
            for (int c = 0; c < 3; ++c) v[9 * i + 3 * r + c] = V[r][c];
        }
    }
    return PCD_OK;
}

int pcd_host_vu_smooth(const float* w, const float* v, const float* n, int64_t m, float tau, float damp, float* out) {
    PCD_CHECK_ARG(w && v && n && out, "null argument");
    for (int64_t i = 0; i < m; ++i) {
        float V[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) V[r][c] = v[9 * i + 3 * r + c];
        const Vec3 f = vu_smooth(w + 3 * i, V, v3(n[3 * i], n[3 * i + 1], n[3 * i + 2]), tau, damp);
        out[3 * i] = f.x; out[3 * i + 1] = f.y; out[3 * i + 2] = f.z;
    }
    return PCD_OK;
}

int pcd_host_solve3(const float* a9, const float* b3, int64_t m, float* x3, int32_t* ok) {
    PCD_CHECK_ARG(a9 && b3 && x3 && ok, "null argument");
    for (int64_t i = 0; i < m; ++i) {
        float A[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) A[r][c] = a9[9 * i + 3 * r + c];
        Vec3 x = v3(0.f, 0.f, 0.f);
        ok[i] = solve3(A, v3(b3[3 * i], b3[3 * i + 1], b3[3 * i + 2]), x) ? 1 : 0;
        x3[3 * i] = x.x; x3[3 * i + 1] = x.y; x3[3 * i + 2] = x.z;
    }
    return PCD_OK;
}

int pcd_host_inv3(const float* a9, int64_t m, float* inv9, int32_t* ok) {
    PCD_CHECK_ARG(a9 && inv9 && ok, "null argument");
    for (int64_t i = 0; i < m; ++i) {
        float A[3][3], X[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) A[r][c] = a9[9 * i + 3 * r + c];
        ok[i] = inv3_ref(A, X) ? 1 : 0;
        if (!ok[i])
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) X[r][c] = 0.f;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) inv9[9 * i + 3 * r + c] = X[r][c];
    }
    return PCD_OK;
}

int pcd_host_step_csr(int kind, const float* pos, const float* n, const float* edge_vectors, const int64_t* ci,
                      const int64_t* off, const int64_t* nbr, int64_t m, float delta, float d, float alpha, float* out) {
    PCD_CHECK_ARG(pos && n && ci && off && (m == 0 || nbr) && out, "null argument");
    PCD_CHECK_ARG(kind != PCD_STEP_EDGE || edge_vectors, "edge_step needs edge vectors");
    const Rows3 P{pos}, N{n};
    for (int64_t r = 0; r < m; ++r) {
        const int64_t c = ci[r];
        const int cnt = (int)(off[r + 1] - off[r]);
        const HostCsrNb nb{nbr, off[r]};
        const Vec3 vi = P(c);
        Vec3 o;
        switch (kind) {
            case PCD_STEP_FLAT: o = step_flat(P, N, vi, N(c), cnt, nb, delta, d, alpha); break;
            case PCD_STEP_EDGE: o = step_edge(P, N, vi, Rows3{edge_vectors}(c), cnt, nb, d, alpha); break;
            case PCD_STEP_FEATURE: o = step_feature<false>(P, N, vi, N(c), cnt, nb, 1.f, d, alpha); break;
            case PCD_STEP_NEW: o = step_feature<true>(P, N, vi, N(c), cnt, nb, delta, d, alpha); break;
            case PCD_STEP_CORNER: o = step_corner(P, N, vi, cnt, nb, d, alpha); break;
            default: o = vi; break;
        }
        out[3 * r] = o.x; out[3 * r + 1] = o.y; out[3 * r + 2] = o.z;
    }
    return PCD_OK;
}

int pcd_host_nvt_tensor(const float* pos, const float* n, const int64_t* ci, const int64_t* off, const int64_t* nbr,
                        int64_t m, float rho, float* t6) {
    PCD_CHECK_ARG(pos && n && ci && off && (m == 0 || nbr) && t6, "null argument");
    for (int64_t r = 0; r < m; ++r) {
        const Sym3 T = nvt_tensor(Rows3{pos}, Rows3{n}, Rows3{pos}(ci[r]), (int)(off[r + 1] - off[r]),
                                  HostCsrNb{nbr, off[r]}, rho);
        float* o = t6 + 6 * r;
        o[0] = T.a00; o[1] = T.a01; o[2] = T.a02; o[3] = T.a11; o[4] = T.a12; o[5] = T.a22;
    }
    return PCD_OK;
}

}  // extern "C"
