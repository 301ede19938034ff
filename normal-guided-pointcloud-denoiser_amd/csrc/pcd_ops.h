// Per-point math of the reference's tensor-voting and position-update operators, written once as device
// functions over an abstract neighbour list (nb(t) -> point index) so that the public CSR kernels (one call per
// reference method) and the fused denoise kernels (dense column-major kNN lists) share one implementation.
#pragma once
#include "pcd_device.h"

namespace pcd {

#ifndef PCD_NB_BATCH
#define PCD_NB_BATCH 8
#endif
static constexpr int kNbBatch = PCD_NB_BATCH;   // neighbours gathered together (every load of a batch in flight)

// Neighbour loop of a fused kernel: M = compile-time bound on cnt (list cap).  The list entries are read first, then
// the neighbours' (v_j, n_j) in batches of kNbBatch whose loads are all issued before any is consumed; f(vj, nj) runs
// for t < cnt in list order, so every sum keeps the reference's summation order.  M = 0: plain runtime loop.
// A list accessor with `static constexpr bool kClamped = true` already repeats entry cnt-1 past cnt, so it is read at
// compile-time slots (a register list needs no run-time index).
template <class Nb, class = void> struct nb_clamped { static constexpr bool value = false; };
template <class Nb> struct nb_clamped<Nb, decltype((void)Nb::kClamped)> { static constexpr bool value = Nb::kClamped; };
template <int M, int BATCH = kNbBatch, class P, class Nr, class Nb, class F>
PCD_DEV void for_neighbours(P pos, Nr nrm, int cnt, Nb nb, F&& f) {
    if constexpr (M > 0) {
        int32_t jj[M];
#pragma unroll
        for (int t = 0; t < M; ++t) jj[t] = (int32_t)(nb_clamped<Nb>::value ? nb(t) : nb(t < cnt ? t : cnt - 1));
#pragma unroll
        for (int b = 0; b < M; b += BATCH) {
            constexpr int B = M < BATCH ? M : BATCH;
            Vec3 vb[B], nv[B];
#pragma unroll
            for (int u = 0; u < B; ++u) { vb[u] = pos(jj[b + u]); nv[u] = nrm(jj[b + u]); }
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (b + u < cnt) f(vb[u], nv[u]);
        }
    } else {
        for (int t = 0; t < cnt; ++t) {
            const int64_t j = nb(t);
            f(pos(j), nrm(j));
        }
    }
}

// ----------------------------------------------------------------- H5: Decompositionor.getBetterFilteredNVT
// w_ij = acos(|clamp(normalize(v_j - v_i) . n_j, -1, 1)|) > rho       (Decompositionor.py:290; F.normalize eps 1e-12)
// T_i  = Σ w n_j n_jᵀ / Σ w,  all w := 1 when Σ w = 0                 (Decompositionor.py:291-299)
// UNROLL > 0: the neighbour loop is fully unrolled to UNROLL (>= cnt) so register-resident neighbour lists stay
// in registers and every gather of the list can be issued before the first is consumed.
//
// The binary vote is decided without sqrt, divisions or acos whenever that is safe: with e = dv . n_j and
// sq = |dv|², the reference's |c| < cos(rho) is e² < cos²(rho)·sq (cos(rho) > 0; for rho >= π/2 no pair votes, and
// cos² is taken as -1 so that none does).  Only pairs with |e² - cos²(rho)·sq| <= 4e-6·(1 + |n_j|₁)²·sq, or with
// sq outside [1e-24, 1e30] (where F.normalize's eps or over/underflow matter), evaluate the reference expression
// exactly; sq = 0 (the row's own entry: the snapshot point of a row is its current point's neighbour) has the
// constant vote acos(0) > rho.  The margin covers the estimate's error: |c_est - c_ref| ~ 1e-6 and cos(rho) vs acos's own rounding
// < 1e-6 give |c_est - cos(rho)| > 4e-6·(1 + |n_j|₁) whenever the squared test clears its margin, since
// |c| + cos(rho) <= 1 + |n_j|₁; e² and cos²(rho)·sq are themselves within ~1e-7 of that scale.
// Sums: the voting neighbours' n_j n_jᵀ in list order (the weight folded into one factor: w·n_j, exact).  The
// all-ones fallback (no vote) re-reads the rows and sums every n_j n_jᵀ in list order -- a rare row.
// nbf: the same list for the rare fallback pass (a memory-backed accessor, so register-resident lists need not
// stay live across the vote loop).
// NORM = false: the sums without the division by Σ w (a positive scale: for callers that only need the
// eigenvectors and scale-free ratios of the eigenvalues, NVT2's classes and edge vector).
// UNIT = true: every n_j is a unit vector to rounding (|n_j| <= 1 + 1e-6, the kernels' own normalised f_n), so
// (1 + |n_j|₁)² <= (1 + √3 (1 + 1e-6))² < 7.47 and the margin is the constant kUnitMargin·sq.
static constexpr float kVoteEps = 4e-6f;
static constexpr float kUnitMargin = kVoteEps * 7.47f;
// wsum_out (nullable): Σ w after the fallback (the divisor of NORM; the NVT2 probe reports it).
template <int UNROLL = 0, bool NORM = true, bool UNIT = false, int BATCH = kNbBatch, class P, class Nr, class Nb,
          class NbF>
PCD_DEV Sym3 nvt_tensor(P pos, Nr nrm, Vec3 vi, int cnt, Nb nb, float rho, NbF nbf, int* wsum_out = nullptr) {
    float w00 = 0.f, w01 = 0.f, w02 = 0.f, w11 = 0.f, w12 = 0.f, w22 = 0.f;
    int wsum = 0;
    const float cthr = cosf(rho);
    const float cthr2 = cthr > 0.f ? cthr * cthr : -1.f;
    const bool w_self = acosf(0.f) > rho;   // the vote of a coincident neighbour (every row lists itself)
    // Packed fp32 (v_pk_mul / v_pk_add on gfx950: two lanes of a register pair per instruction) for the pairs of
    // products and sums; every component is the same IEEE multiply / add in the same order as the scalar code.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 vixy = {vi.x, vi.y};
    f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f}, acc2 = {0.f, 0.f};   // (w00, w01), (w02, w11), (w12, w22)
    auto body2 = [&](const Vec3 vj, const Vec3 nj) {
        const f2 dxy = f2{vj.x, vj.y} - vixy;
        const float dz = vj.z - vi.z;
        const f2 sxy = dxy * dxy;
        const float sq = (sxy.x + sxy.y) + dz * dz;
        const f2 exy = dxy * f2{nj.x, nj.y};
        const float e = (exy.x + exy.y) + dz * nj.z;
        const float lhs = e * e, rhs = cthr2 * sq;
        float m;
        if constexpr (UNIT) {
            m = kUnitMargin * sq;
        } else {
            const float n1 = 1.f + fabsf(nj.x) + fabsf(nj.y) + fabsf(nj.z);
            m = kVoteEps * n1 * n1 * sq;
        }
        // one rarely taken branch per neighbour: the pairs within the margin (or outside the safe range of sq)
        // evaluate the reference expression; sq = 0 (the row itself) has the constant vote and is never "near"
        const bool near = sq != 0.f && (!(fabsf(lhs - rhs) > m) || !(sq >= 1e-24f && sq < 1e30f));
        bool w = sq == 0.f ? w_self : lhs < rhs;
        if (near) {
            const float den = fmaxf(norm3(v3(dxy.x, dxy.y, dz)), 1e-12f);
            const Vec3 dn = v3(dxy.x / den, dxy.y / den, dz / den);
            float c = dot3(dn, nj);
            c = fabsf(fminf(fmaxf(c, -1.f), 1.f));
            w = acosf(c) > rho;
        }
        const Vec3 nw = sel3(w, nj, v3(0.f, 0.f, 0.f));
        acc0 += f2{nw.x, nw.x} * f2{nj.x, nj.y};
        acc1 += f2{nw.x, nw.y} * f2{nj.z, nj.y};
        acc2 += f2{nw.y, nw.z} * f2{nj.z, nj.z};
        wsum += w ? 1 : 0;
    };
    for_neighbours<UNROLL, BATCH>(pos, nrm, cnt, nb, body2);
    w00 = acc0.x; w01 = acc0.y; w02 = acc1.x; w11 = acc1.y; w12 = acc2.x; w22 = acc2.y;
    if (wsum == 0) {
        w00 = w01 = w02 = w11 = w12 = w22 = 0.f;
#pragma unroll 1
        for (int t = 0; t < cnt; ++t) {
            const Vec3 nj = nrm(nbf(t));
            w00 += nj.x * nj.x; w01 += nj.x * nj.y; w02 += nj.x * nj.z;
            w11 += nj.y * nj.y; w12 += nj.y * nj.z; w22 += nj.z * nj.z;
        }
        wsum = cnt;
    }
    if (wsum_out) *wsum_out = wsum;
    if (!NORM) return Sym3{w00, w01, w02, w11, w12, w22};
    const float c = (float)wsum;
    return Sym3{w00 / c, w01 / c, w02 / c, w11 / c, w12 / c, w22 / c};
}
template <int UNROLL = 0, class P, class Nr, class Nb>
PCD_DEV Sym3 nvt_tensor(P pos, Nr nrm, Vec3 vi, int cnt, Nb nb, float rho) {
    return nvt_tensor<UNROLL>(pos, nrm, vi, cnt, nb, rho, nb);
}

// ----------------------------------------------------------------- CPSD: Decompositionor.getNormalFilteredNVT
// w_ij = acos(clamp(n_i . n_j, -1, 1)) <= rho (no abs, <=; Decompositionor.py:269); T_i = Σ w n_j n_jᵀ / Σ w;
// a row where no neighbour votes gets n_i n_iᵀ (:273-275).  Sums in list order, like scatter_add.
// The vote: acos is decreasing, so acos(c) <= rho is c >= cos(rho) -- decided that way when c is more than 1e-6
// from cos(rho) (acosf's and cosf's roundings are ~1e-7 in c there), else by the reference's own acosf(c) <= rho.
PCD_DEV bool normal_vote(float c, float rho, float crho) {
    if (c - crho > 1e-6f) return true;
    if (crho - c > 1e-6f) return false;
    return acosf(c) <= rho;
}
template <class Nr, class Nb>
PCD_DEV Sym3 nvt_normal_tensor(Nr nrm, Vec3 ni, int cnt, Nb nb, float rho) {
    float w00 = 0.f, w01 = 0.f, w02 = 0.f, w11 = 0.f, w12 = 0.f, w22 = 0.f;
    int wsum = 0;
    const float crho = cosf(rho);
    constexpr int B = 8;            // members in batches: every list entry, then every normal, in flight together
    for (int t0 = 0; t0 < cnt; t0 += B) {
        Vec3 nv[B];
        {
            int64_t j[B];
#pragma unroll
            for (int u = 0; u < B; ++u) j[u] = nb(min(t0 + u, cnt - 1));
#pragma unroll
            for (int u = 0; u < B; ++u) nv[u] = nrm(j[u]);
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            if (t0 + u >= cnt) break;
            const Vec3 nj = nv[u];
            const float c = fminf(fmaxf(dot3(ni, nj), -1.f), 1.f);
            if (normal_vote(c, rho, crho)) {
                w00 += nj.x * nj.x; w01 += nj.x * nj.y; w02 += nj.x * nj.z;
                w11 += nj.y * nj.y; w12 += nj.y * nj.z; w22 += nj.z * nj.z;
                ++wsum;
            }
        }
    }
    if (wsum == 0) return Sym3{ni.x * ni.x, ni.x * ni.y, ni.x * ni.z, ni.y * ni.y, ni.y * ni.z, ni.z * ni.z};
    const float c = (float)wsum;
    return Sym3{w00 / c, w01 / c, w02 / c, w11 / c, w12 / c, w22 / c};
}

// ----------------------------------------------------------------- CPSD: Decompositionor.getNormalFilteredPVT
// Same vote; if none votes every w := 1 (:188-192).  c = Σ w v_j / Σ w, C = Σ w (v_j - c)(v_j - c)ᵀ / Σ w
// (:194-200); an EMPTY neighbourhood gets Σ s sᵀ over s = ±(n × v), ±(n × (n × v)) (:201-208).
PCD_DEV Vec3 cross3(Vec3 a, Vec3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
template <class P, class Nr, class Nb>
PCD_DEV Sym3 pvt_normal_cov(P pos, Nr nrm, Vec3 vi, Vec3 ni, int cnt, Nb nb, float rho) {
    if (cnt == 0) {
        const Vec3 s1 = cross3(ni, vi), s2 = cross3(ni, s1);
        const Vec3 sm[4] = {s1, -1.f * s1, s2, -1.f * s2};
        float a[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // samples[:, :, None] * samples[..., None] summed over the 4 samples
            a[0] += sm[u].x * sm[u].x; a[1] += sm[u].y * sm[u].x; a[2] += sm[u].z * sm[u].x;
            a[3] += sm[u].y * sm[u].y; a[4] += sm[u].z * sm[u].y; a[5] += sm[u].z * sm[u].z;
        }
        return Sym3{a[0], a[1], a[2], a[3], a[4], a[5]};
    }
    // members in batches of 8 (every list entry, then every gathered row of a batch in flight together); the votes
    // of the first 64 members are kept as bits, so the centroid and covariance passes re-gather positions only.  Sums
    // run over the voters in list order, as the reference's scatter.
    constexpr int B = 8;
    int wsum = 0;
    unsigned long long vbits = 0ull;
    const float crho = cosf(rho);
    for (int t0 = 0; t0 < cnt; t0 += B) {
        int64_t j[B];
        Vec3 nj[B];
#pragma unroll
        for (int u = 0; u < B; ++u) j[u] = nb(min(t0 + u, cnt - 1));
#pragma unroll
        for (int u = 0; u < B; ++u) nj[u] = nrm(j[u]);
#pragma unroll
        for (int u = 0; u < B; ++u) {
            if (t0 + u >= cnt) break;
            const float c = fminf(fmaxf(dot3(ni, nj[u]), -1.f), 1.f);
            const bool v = normal_vote(c, rho, crho);
            wsum += v ? 1 : 0;
            if (v && t0 + u < 64) vbits |= 1ull << (t0 + u);
        }
    }
    const bool all = wsum == 0;
    if (all) wsum = cnt;
    auto vote = [&](int t, int64_t j) {
        if (all) return true;
        if (t < 64) return ((vbits >> t) & 1ull) != 0ull;
        const float c = fminf(fmaxf(dot3(ni, nrm(j)), -1.f), 1.f);
        return normal_vote(c, rho, crho);
    };
    // voters' positions of members t0 .. t0+B-1 -> f(vj) in list order
    auto for_voters = [&](auto&& f) {
        for (int t0 = 0; t0 < cnt; t0 += B) {
            int64_t j[B];
            Vec3 vj[B];
#pragma unroll
            for (int u = 0; u < B; ++u) j[u] = nb(min(t0 + u, cnt - 1));
#pragma unroll
            for (int u = 0; u < B; ++u) vj[u] = pos(j[u]);
#pragma unroll
            for (int u = 0; u < B; ++u) {
                if (t0 + u >= cnt) break;
                if (vote(t0 + u, j[u])) f(vj[u]);
            }
        }
    };
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for_voters([&](Vec3 vj) { sx += vj.x; sy += vj.y; sz += vj.z; });
    const float c = (float)wsum;
    const Vec3 ctr = v3(sx / c, sy / c, sz / c);
    float a00 = 0.f, a01 = 0.f, a02 = 0.f, a11 = 0.f, a12 = 0.f, a22 = 0.f;
    for_voters([&](Vec3 vj) {
        const Vec3 d = vj - ctr;   // T[a][b] = dv[b] * dv[a] (wij[...,None] * dv[:,None] * dv[...,None])
        a00 += d.x * d.x; a01 += d.y * d.x; a02 += d.z * d.x;
        a11 += d.y * d.y; a12 += d.z * d.y; a22 += d.z * d.z;
    });
    return Sym3{a00 / c, a01 / c, a02 / c, a11 / c, a12 / c, a22 / c};
}

// ----------------------------------------------------------------- H15: GraphBuilder.getPVTDecompositionWithKNN
// C_i = Σ_j (v_j - v̄)(v_j - v̄)ᵀ with v̄ the mean of the k neighbours (GraphBuilder.py:105-110), in torch's CPU
// reduction order for vj.mean(dim=1) and (...).sum(dim=1) over the neighbour axis: four interleaved accumulators
// (neighbour t into accumulator t mod 4), combined in order, the mean a division by k -- bit-identical to the
// reference's covariances at its k = 12 (tests/test_capi.py)
template <class P, class Nb>
PCD_DEV Sym3 pca_cov(P pos, int cnt, Nb nb) {
    Vec3 s4[4] = {v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f)};
    for (int t = 0; t < cnt; ++t) {
        const Vec3 v = pos(nb(t));
        Vec3& a = s4[t & 3];
        a = t < 4 ? v : a + v;
    }
    Vec3 sum = s4[0];
    for (int l = 1; l < 4 && l < cnt; ++l) sum = sum + s4[l];
    const float c = (float)cnt;
    const Vec3 m = v3(sum.x / c, sum.y / c, sum.z / c);
    float C4[4][6];
    for (int t = 0; t < cnt; ++t) {
        const Vec3 d = pos(nb(t)) - m;
        const float o[6] = {d.x * d.x, d.y * d.x, d.z * d.x, d.y * d.y, d.z * d.y, d.z * d.z};
        float* a = C4[t & 3];
#pragma unroll
        for (int q = 0; q < 6; ++q) a[q] = t < 4 ? o[q] : a[q] + o[q];
    }
    float r[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) r[q] = cnt > 0 ? C4[0][q] : 0.f;
    for (int l = 1; l < 4 && l < cnt; ++l)
#pragma unroll
        for (int q = 0; q < 6; ++q) r[q] = r[q] + C4[l][q];
    return Sym3{r[0], r[1], r[2], r[3], r[4], r[5]};
}

// ----------------------------------------------------------------- helpers for the position updates
PCD_DEV Vec3 outer_mul(Vec3 a, Vec3 v) {  // (a aᵀ) v, einsum("nij,nj->ni") row order
    return v3((a.x * a.x) * v.x + (a.x * a.y) * v.y + (a.x * a.z) * v.z,
              (a.y * a.x) * v.x + (a.y * a.y) * v.y + (a.y * a.z) * v.z,
              (a.z * a.x) * v.x + (a.z * a.y) * v.y + (a.z * a.z) * v.z);
}
PCD_DEV void add_outer(float A[3][3], Vec3 a, float s = 1.f) {
    const float c[3] = {a.x, a.y, a.z};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) A[r][q] += s * (c[r] * c[q]);
}
// di = α(x - v_i); accept if ||di|| < d (strict; flat_step uses <=)
PCD_DEV Vec3 clamp_step(Vec3 vi, Vec3 x, float alpha, float d) {
    const Vec3 di = v3((x.x - vi.x) * alpha, (x.y - vi.y) * alpha, (x.z - vi.z) * alpha);
    const float nrm = norm3(di);
    return sel3(nrm < d, vi + di, vi);
}

// ----------------------------------------------------------------- H9: Denoiser.flat_step (Denoiser.py:90-119)
// delta is the GLOBAL max ||v_j - centre|| over every row of the selection (computed by the caller).
template <int M = 0, class P, class Nr, class Nb>
PCD_DEV Vec3 step_flat(P pos, Nr nrm, Vec3 vi, Vec3 ni, int cnt, Nb nb, float delta, float d, float alpha) {
    const float dd = delta * delta;
    float sx = 0.f, sy = 0.f, sz = 0.f, ws = 0.f;
    for_neighbours<M>(pos, nrm, cnt, nb, [&](const Vec3 vj, const Vec3 nj) {
        const Vec3 dist = vj - vi;
        const float sim = expf((-16.f * sq3(ni - nj)) / dd);
        const float clo = expf((-4.f * sq3(dist)) / dd);
        const float W = sim * clo;
        const float wd = W * dot3(nj, dist);
        sx += wd * ni.x; sy += wd * ni.y; sz += wd * ni.z;
        ws += W;
    });
    const Vec3 di = v3(sx / ws * alpha, sy / ws * alpha, sz / ws * alpha);
    const float nrm2 = norm3(di);
    return sel3(nrm2 <= d, vi + di, vi);   // NaN (Σ W = 0) -> no move, as di[~mask] = 0
}

// ----------------------------------------------------------------- H10: Denoiser.edge_step (Denoiser.py:53-88)
template <int M = 0, int BATCH = kNbBatch, class P, class Nr, class Nb>
PCD_DEV Vec3 step_edge(P pos, Nr nrm, Vec3 vi, Vec3 y, int cnt, Nb nb, float d, float alpha) {
    float A[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    Vec3 b = v3(0.f, 0.f, 0.f);
    const Vec3 yyvi = outer_mul(y, vi);
    const float yc[3] = {y.x, y.y, y.z};
    for_neighbours<M, BATCH>(pos, nrm, cnt, nb, [&](const Vec3 vj, const Vec3 nj) {
        const Vec3 vjp = vj - dot3(vj - vi, y) * y;
        const Vec3 njp = nj - dot3(nj, y) * y;
        const float nc[3] = {njp.x, njp.y, njp.z};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) A[r][q] += nc[r] * nc[q] + yc[r] * yc[q];
        b = b + (outer_mul(njp, vjp) + yyvi);
    });
    Vec3 x;
    if (!solve3(A, b, x)) x = vi;
    return clamp_step(vi, x, alpha, d);
}

// ----------------------------------------------------------------- H11: Denoiser.feature_step (Denoiser.py:174-219)
//                                 and H12: Denoiser.new_step (Denoiser.py:121-172; WEIGHTED=true)
template <bool WEIGHTED, int M = 0, int BATCH = kNbBatch, class P, class Nr, class Nb>
PCD_DEV Vec3 step_feature(P pos, Nr nrm, Vec3 vi, Vec3 ni, int cnt, Nb nb, float delta, float d, float alpha) {
    float S[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};  // Σ w nj njᵀ
    Vec3 svj = v3(0.f, 0.f, 0.f);                                       // Σ w vj
    Vec3 snv = v3(0.f, 0.f, 0.f);                                       // Σ w (nj njᵀ) vj
    const float dd = delta * delta;
    for_neighbours<M, BATCH>(pos, nrm, cnt, nb, [&](const Vec3 vj, const Vec3 nj) {
        float w = 1.f;
        if (WEIGHTED) {
            const float dt = dot3(nj, vj - vi);
            w = expf((-9.f * (dt * dt)) / dd);
        }
        const float nc[3] = {nj.x, nj.y, nj.z};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) S[r][q] += WEIGHTED ? w * (nc[r] * nc[q]) : (nc[r] * nc[q]);
        svj = svj + (WEIGHTED ? w * vj : vj);
        const Vec3 nv = outer_mul(nj, vj);
        snv = snv + (WEIGHTED ? w * nv : nv);
    });
    const float nc[3] = {ni.x, ni.y, ni.z};
    const float card = (float)cnt;
    float A[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const float no = nc[r] * nc[q];
            A[r][q] = (((r == q ? 1.f : 0.f) + no) + S[r][q]) + card * no;
        }
    const Vec3 b = ((vi + outer_mul(ni, vi)) + outer_mul(ni, svj)) + snv;
    Vec3 x;
    // optimal_pos[mask] = optimal_pos[mask] + (new_pos[mask] - optimal_pos[mask])  (Denoiser.py:167, 214)
    if (solve3(A, b, x)) x = vi + (x - vi);
    else x = vi;
    return clamp_step(vi, x, alpha, d);
}

// ----------------------------------------------------------------- H12: Denoiser.corner_step (Denoiser.py:26-51)
template <int M = 0, int BATCH = kNbBatch, class P, class Nr, class Nb>
PCD_DEV Vec3 step_corner(P pos, Nr nrm, Vec3 vi, int cnt, Nb nb, float d, float alpha) {
    float A[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    Vec3 b = v3(0.f, 0.f, 0.f);
    for_neighbours<M, BATCH>(pos, nrm, cnt, nb, [&](const Vec3 vj, const Vec3 nj) {
        add_outer(A, nj);
        b = b + outer_mul(nj, vj);
    });
    Vec3 x;
    if (!solve3(A, b, x)) x = vi;
    return clamp_step(vi, x, alpha, d);
}

}  // namespace pcd
