// Device-side building blocks shared by every pcd kernel (gfx950 / CDNA4, wave64).
//
//  * small fixed-size linear algebra: 3x3 symmetric eigen-decomposition following LAPACK ssyevd step by step
//    (replaces the reference's batched torch.linalg.eigh, Decompositionor.py:300), 3x3 LU with partial pivoting +
//    exact-zero-pivot detection (replaces torch.linalg.inv_ex's info mask, Denoiser.py:43-46,80-83,210-214)
//  * everything is __host__ __device__: libpcd exports host entry points (pcd_host_*) so the exact per-point math
//    is unit-tested on the CPU as well
//  * point accessors: the public API hands over caller-owned [n,3] fp32 rows (stride 3), the fused
//    denoise path keeps float4 rows in HBM (one 16-B load per gathered neighbour)
//  * XCD-aware block remap: consecutive logical blocks (spatially adjacent points after the Morton
//    sort) land on the same XCD so neighbour gathers hit that XCD's L2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PCD_DEV __host__ __device__ __forceinline__

namespace pcd {

struct Vec3 { float x, y, z; };

PCD_DEV Vec3 v3(float x, float y, float z) { return Vec3{x, y, z}; }
PCD_DEV Vec3 operator+(Vec3 a, Vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PCD_DEV Vec3 operator-(Vec3 a, Vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PCD_DEV Vec3 operator*(float s, Vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
// dot in the reference's summation order: (x*x' + y*y') + z*z'  ((a*b).sum(dim=1))
PCD_DEV float dot3(Vec3 a, Vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }  // built with -ffp-contract=off
PCD_DEV float sq3(Vec3 a) { return dot3(a, a); }
// Tensor.norm(dim=1) / F.normalize as torch computes them on the CPU: the squares accumulated with fmas (x² first),
// then one IEEE sqrt -- every ||.|| the reference compares against a threshold (the step clamps, the global clamp,
// flat_step's delta, the vote's normalize) rounds this way (pinned in oracle.norm3 against torch)
PCD_DEV float nsq3(Vec3 a) { return fmaf(a.z, a.z, fmaf(a.y, a.y, a.x * a.x)); }   // the sum under norm3's root
PCD_DEV float norm3(Vec3 a) { return sqrtf(nsq3(a)); }
// c ? a : b component by component (a select of the structs themselves can leave them in scratch memory)
PCD_DEV Vec3 sel3(bool c, Vec3 a, Vec3 b) { return v3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

// ---------------------------------------------------------------- point accessors
// Packed caller rows: float[n*3]
struct Rows3 {
    const float* p;
    PCD_DEV Vec3 operator()(int64_t i) const { const float* q = p + 3 * i; return v3(q[0], q[1], q[2]); }
};
// Internal padded rows: float4[n] (w unused / carries an index for the snapshot)
struct Rows4 {
    const float4* p;
    PCD_DEV Vec3 operator()(int64_t i) const { float4 q = p[i]; return v3(q.x, q.y, q.z); }
};

PCD_DEV void store3(float* out, int64_t i, Vec3 v) { float* q = out + 3 * i; q[0] = v.x; q[1] = v.y; q[2] = v.z; }
PCD_DEV void store4(float4* out, int64_t i, Vec3 v) { out[i] = make_float4(v.x, v.y, v.z, 0.f); }

// ---------------------------------------------------------------- XCD-aware block mapping
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md "Workgroup dispatch"). Remap so
// that XCD x processes the x-th contiguous slice of logical blocks (speed only, never correctness).
PCD_DEV int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t per = (nb + 7) / 8;
    const int64_t x = b % 8, w = b / 8;
    const int64_t full = nb - 8 * (per - 1);  // XCDs 0..full-1 own `per` blocks, the rest per-1
    int64_t base = (x < full) ? x * per : full * per + (x - full) * (per - 1);
    return base + w;
}

// Active-row view: thread t works on row rows[t] (sorted order), or on row t when rows is null.
struct RowMap {
    const int32_t* rows;
    int64_t nq;
    PCD_DEV int64_t operator()(int64_t t) const { return rows ? (int64_t)rows[t] : t; }
};

// ---------------------------------------------------------------- symmetric 3x3 eigen-decomposition
// A restatement of what torch.linalg.eigh does on the reference's CPU path for one 3x3 fp32 matrix: LAPACK ssyevd
// (JOBZ='V', UPLO='L') = ssytd2 Householder tridiagonalisation, ssteqr implicit QL/QR with Wilkinson shifts
// (compz='I', slaev2 for 2x2 blocks, pre-3.10 slartg sign convention), selection sort, back-transformation by the
// reflector.  The reference's VU smoothing is NOT invariant to eigenvector signs (Decompositionor.py:101-105 uses
// Eᵀ·M·E), so the signs must be LAPACK's.  tests/test_capi.py::test_host_eigh_matches_torch checks this code
// (through pcd_host_eigh3) against MKL's torch.linalg.eigh on the CPU: eigenvalues and every eigenvector sign.
// Output: ascending eigenvalues w[0] <= w[1] <= w[2]; V[r][k] = component r of eigenvector k.
struct Sym3 { float a00, a01, a02, a11, a12, a22; };

namespace lapack {
// LAPACK's IEEE division and square root (the hardware estimates flip eigenvector signs on 0.2-0.4 % of the fandisk
// points: measured)
PCD_DEV float ldiv(float a, float b) { return a / b; }
PCD_DEV float lsqrt(float x) { return sqrtf(x); }
static constexpr float kEps = 5.9604644775390625e-08f;      // slamch('E') = 2^-24
static constexpr float kSafmin = 1.17549435e-38f;          // slamch('S')
static constexpr float kSafmn2 = 4.4408920985006262e-16f;  // 2^-51 (slartg scaling bounds)
static constexpr float kSafmx2 = 2.2517998136852480e+15f;
// ssteqr's block scaling bounds: ssfmax = sqrt(1 / safmin) / 3, ssfmin = sqrt(safmin) / eps² = 2^-15.  A block whose
// largest |d|, |e| lies outside them is scaled to the bound (slascl: one multiplication by bound / anorm) before its
// QL/QR iteration and scaled back after it -- covariance-like tensors (PCA normals, the CPSD position voting) of
// small point spacings land below ssfmin
static constexpr float kSsfmax = 3.07445734e+18f;
static constexpr float kSsfmin = 3.0517578125e-05f;
// the scale factor of a block (1 when none applies) and its inverse, both as slascl forms them (cto / cfrom)
PCD_DEV float block_scale(float anorm) {
    return anorm > kSsfmax ? ldiv(kSsfmax, anorm) : (anorm < kSsfmin ? ldiv(kSsfmin, anorm) : 1.f);
}
PCD_DEV float block_unscale(float anorm) {
    return anorm > kSsfmax ? ldiv(anorm, kSsfmax) : (anorm < kSsfmin ? ldiv(anorm, kSsfmin) : 1.f);
}

PCD_DEV float fsign(float a, float b) { return b >= 0.f ? fabsf(a) : -fabsf(a); }
PCD_DEV float slapy2(float x, float y) {
    const float xa = fabsf(x), ya = fabsf(y);
    const float w = fmaxf(xa, ya), z = fminf(xa, ya);
    if (z == 0.f || w > 3.4028235e38f) return w;
    const float q = ldiv(z, w);
    return w * lsqrt(1.f + q * q);
}
// LAPACK <= 3.9 slartg: r = ±sqrt(f²+g²), c made positive only when |f| > |g|
PCD_DEV void slartg(float f, float g, float& c, float& s, float& r) {
    if (g == 0.f) { c = 1.f; s = 0.f; r = f; return; }
    if (f == 0.f) { c = 0.f; s = 1.f; r = g; return; }
    float f1 = f, g1 = g;
    const float scale = fmaxf(fabsf(f1), fabsf(g1));
    int count = 0;
    if (scale >= kSafmx2) {
        do { f1 *= kSafmn2; g1 *= kSafmn2; ++count; } while (fmaxf(fabsf(f1), fabsf(g1)) >= kSafmx2 && count < 20);
        r = lsqrt(f1 * f1 + g1 * g1);
        c = ldiv(f1, r); s = ldiv(g1, r);
        for (int i = 0; i < count; ++i) r *= kSafmx2;
    } else if (scale <= kSafmn2) {
        do { f1 *= kSafmx2; g1 *= kSafmx2; ++count; } while (fmaxf(fabsf(f1), fabsf(g1)) <= kSafmn2 && count < 20);
        r = lsqrt(f1 * f1 + g1 * g1);
        c = ldiv(f1, r); s = ldiv(g1, r);
        for (int i = 0; i < count; ++i) r *= kSafmn2;
    } else {
        r = lsqrt(f1 * f1 + g1 * g1);
        c = ldiv(f1, r); s = ldiv(g1, r);
    }
    if (fabsf(f) > fabsf(g) && c < 0.f) { c = -c; s = -s; r = -r; }
}
// eigensystem of [[a, b], [b, c]]: rt1 (larger |.|), rt2, (cs1, sn1) eigenvector of rt1
PCD_DEV void slaev2(float a, float b, float c, float& rt1, float& rt2, float& cs1, float& sn1) {
    const float sm = a + c, df = a - c, adf = fabsf(df), tb = b + b, ab = fabsf(tb);
    float acmx, acmn;
    if (fabsf(a) > fabsf(c)) { acmx = a; acmn = c; } else { acmx = c; acmn = a; }
    float rt;
    if (adf > ab) { const float q = ldiv(ab, adf); rt = adf * lsqrt(1.f + q * q); }
    else if (adf < ab) { const float q = ldiv(adf, ab); rt = ab * lsqrt(1.f + q * q); }
    else rt = ab * 1.41421356237309515f;
    int sgn1, sgn2;
    if (sm < 0.f) { rt1 = 0.5f * (sm - rt); sgn1 = -1; rt2 = ldiv(acmx, rt1) * acmn - ldiv(b, rt1) * b; }
    else if (sm > 0.f) { rt1 = 0.5f * (sm + rt); sgn1 = 1; rt2 = ldiv(acmx, rt1) * acmn - ldiv(b, rt1) * b; }
    else { rt1 = 0.5f * rt; rt2 = -0.5f * rt; sgn1 = 1; }
    float cs;
    if (df >= 0.f) { cs = df + rt; sgn2 = 1; } else { cs = df - rt; sgn2 = -1; }
    if (fabsf(cs) > ab) {
        const float ct = ldiv(-tb, cs);
        sn1 = ldiv(1.f, lsqrt(1.f + ct * ct));
        cs1 = ct * sn1;
    } else if (ab == 0.f) {
        cs1 = 1.f; sn1 = 0.f;
    } else {
        const float tn = ldiv(-cs, tb);
        cs1 = ldiv(1.f, lsqrt(1.f + tn * tn));
        sn1 = tn * cs1;
    }
    if (sgn1 == sgn2) { const float tn = cs1; cs1 = -sn1; sn1 = tn; }
}
// slasr('R', 'V', dir): rotation j acts on columns (j, j+1) of Z, for j in [j0, j0+cnt-1)
// MKL's slasr fuses each update into one fma around the second product (measured against mkl_lapack_ssteqr, 100 % bitwise):
//   z_{j+1} = fma(c, t, -(s z_j)),  z_j = fma(s, t, c z_j)
PCD_DEV void rot_cols(float Z[3][3], int j, float ct, float st) {
    if (ct == 1.f && st == 0.f) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float t = Z[i][j + 1], z = Z[i][j];
        Z[i][j + 1] = fmaf(ct, t, -(st * z));
        Z[i][j] = fmaf(st, t, ct * z);
    }
}

// ssteqr(compz='I') for n = 3: d[3] diagonal, e[2] off-diagonal -> eigenvalues (ascending) in d, vectors in Z.
// LAPACK's loop specialised to n = 3 so that every array index is a compile-time constant: the only blocks are
// [0,1] / [1,2] (one slaev2 or a deflation) and [0,2] (implicit QL or QR sweeps over both rotations, then a
// 2x2 tail).  Same operations in the same order as the general loop (ssteqr3_generic), so the results are
// bit-identical (tools/eigh_equiv.cpp); on the GPU it avoids the select chains of runtime-indexed registers.
PCD_DEV void rot_cols_c(float Z[3][3], int j, float ct, float st) {   // rot_cols, branch-free (j constant)
    const bool id = (ct == 1.f && st == 0.f);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float t = Z[i][j + 1], z = Z[i][j];
        const float n1 = fmaf(ct, t, -(st * z)), n0 = fmaf(st, t, ct * z);   // rot_cols' fma pattern
        Z[i][j + 1] = id ? t : n1;
        Z[i][j] = id ? z : n0;
    }
}
// QL deflation test of e[m] between d[m], d[m+1]; QR test of e[m] between d[m+1], d[m]
PCD_DEV bool ql_small(float e, float dm, float dm1) {
    return fabsf(e) * fabsf(e) <= (kEps * kEps * fabsf(dm)) * fabsf(dm1) + kSafmin;
}
// slaev2 on rows/cols (J, J+1) -> Z columns J, J+1
template <int J>
PCD_DEV void tail2(float d[3], float e[2], float Z[3][3]) {
    float rt1, rt2, c, s;
    slaev2(d[J], e[J], d[J + 1], rt1, rt2, c, s);
    rot_cols_c(Z, J, c, s);
    d[J] = rt1; d[J + 1] = rt2; e[J] = 0.f;
}
// tail2<0> / tail2<1> with the block chosen at run time (J1: [1,2]): one slaev2 for a wave whose lanes differ
PCD_DEV void tail2r(bool J1, float d[3], float e[2], float Z[3][3]) {
    float rt1, rt2, c, s;
    slaev2(J1 ? d[1] : d[0], J1 ? e[1] : e[0], J1 ? d[2] : d[1], rt1, rt2, c, s);
    const bool id = (c == 1.f && s == 0.f);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float t = J1 ? Z[i][2] : Z[i][1], z = J1 ? Z[i][1] : Z[i][0];
        const float n1 = id ? t : fmaf(c, t, -(s * z)), n0 = id ? z : fmaf(s, t, c * z);
        if (J1) { Z[i][2] = n1; Z[i][1] = n0; } else { Z[i][1] = n1; Z[i][0] = n0; }
    }
    if (J1) { d[1] = rt1; d[2] = rt2; e[1] = 0.f; } else { d[0] = rt1; d[1] = rt2; e[0] = 0.f; }
}
// rot_cols_c in a lane's own frame: in the mirrored (QR) frame the pair (j, j+1) holds the original columns
// (j'+1, j') and the original rotation's sine is -st, so the fused product falls on the other column -- the same
// two fmas as the original-frame rotation, operands exchanged (bit-identical to LAPACK's QR sweep under MKL's fmas)
PCD_DEV void rot_cols_m(float Z[3][3], int j, float ct, float st, bool mir) {
    const bool id = (ct == 1.f && st == 0.f);
    const float ss = mir ? -st : st;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a = Z[i][j], b = Z[i][j + 1];
        const float x = mir ? a : b, y = mir ? b : a;
        const float first = fmaf(ct, x, -(ss * y)), second = fmaf(ss, x, ct * y);
        Z[i][j + 1] = id ? b : (mir ? second : first);
        Z[i][j] = id ? a : (mir ? first : second);
    }
}
PCD_DEV void ql_sweep3(float d[3], float e[2], float Z[3][3], bool mir) {   // l = 0, m = 2 (mir: the QR frame)
    float p = d[0];
    float g = ldiv(d[1] - p, 2.f * e[0]);
    float r = slapy2(g, 1.f);
    g = d[2] - p + ldiv(e[0], g + fsign(r, g));
    float s = 1.f, c = 1.f;
    p = 0.f;
    float f = s * e[1], b = c * e[1];
    slartg(g, f, c, s, r);
    g = d[2] - p;
    r = (d[1] - g) * s + 2.f * c * b;
    p = s * r;
    d[2] = g + p;
    g = c * r - b;
    const float c1 = c, s1 = -s;
    f = s * e[0]; b = c * e[0];
    slartg(g, f, c, s, r);
    e[1] = r;
    g = d[1] - p;
    r = (d[0] - g) * s + 2.f * c * b;
    p = s * r;
    d[1] = g + p;
    g = c * r - b;
    rot_cols_m(Z, 1, c1, s1, mir);
    rot_cols_m(Z, 0, c, -s, mir);
    d[0] = d[0] - p;
    e[0] = g;
}
// a 2x2 block [J, J+1] in the outer loop: deflate or slaev2 (direction only changes the deflation test's order)
template <int J>
PCD_DEV void block2(float d[3], float e[2], float Z[3][3]) {
    const float anorm = fmaxf(fmaxf(fmaxf(0.f, fabsf(d[J])), fabsf(d[J + 1])), fabsf(e[J]));   // NaNs drop out, as in LAPACK's loop
    if (anorm == 0.f) return;
    const float sc = block_scale(anorm);
    if (sc != 1.f) { d[J] *= sc; d[J + 1] *= sc; e[J] *= sc; }
    const bool qr = fabsf(d[J + 1]) < fabsf(d[J]);
    const bool small = qr ? ql_small(e[J], d[J + 1], d[J]) : ql_small(e[J], d[J], d[J + 1]);
    if (small) e[J] = 0.f;
    else tail2<J>(d, e, Z);
    if (sc != 1.f) { const float us = block_unscale(anorm); d[J] *= us; d[J + 1] *= us; e[J] *= us; }
}
PCD_DEV void ssteqr3(float d[3], float e[2], float Z[3][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) Z[i][j] = (i == j) ? 1.f : 0.f;
    const int nmaxit = 3 * 30;
    auto split = [&](int mm) {
        const float tst = fabsf(e[mm]);
        if (tst == 0.f) return true;
        if (tst <= (lsqrt(fabsf(d[mm])) * lsqrt(fabsf(d[mm + 1]))) * kEps) { e[mm] = 0.f; return true; }
        return false;
    };
    if (split(0)) {                       // blocks [0,0] [1,...]
        e[0] = 0.f;
        if (split(1)) e[1] = 0.f;         // [1,1] [2,2]
        else block2<1>(d, e, Z);          // [1,2]
    } else if (split(1)) {                // [0,1] [2,2]
        block2<0>(d, e, Z);
        e[1] = 0.f;
    } else {                              // [0,2]
        float anorm = fmaxf(fmaxf(fmaxf(0.f, fabsf(d[0])), fabsf(d[1])), fabsf(d[2]));
        anorm = fmaxf(fmaxf(anorm, fabsf(e[0])), fabsf(e[1]));
        if (anorm != 0.f) {
            const float sc = block_scale(anorm);
            if (sc != 1.f) {
#pragma unroll
                for (int i = 0; i < 3; ++i) d[i] *= sc;
                e[0] *= sc; e[1] *= sc;
            }
            // LAPACK picks QL from the top, or QR from the bottom when |d[2]| < |d[0]|.  QR on (d, e, Z) is QL on the
            // reversed problem (d0 <-> d2, e0 <-> e1, Z's columns reversed) operation for operation -- the same
            // deflation tests on the same operands, the same sweep arithmetic (the rotations' sign conventions
            // mirror), so every lane runs ONE loop in its own frame instead of a wave running both loops.  Only the
            // 2x2 tail (slaev2's operand order) is frame-specific: it runs after the way back.
            const bool qr = fabsf(d[2]) < fabsf(d[0]);
            float fd[3] = {qr ? d[2] : d[0], d[1], qr ? d[0] : d[2]};
            float fe[2] = {qr ? e[1] : e[0], qr ? e[0] : e[1]};
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) Z[i][j] = (qr ? (i + j == 2) : (i == j)) ? 1.f : 0.f;   // Z J or Z
            int tail = 0;                     // 1: the frame's block [1,2] needs slaev2, 2: its block [0,1]
            int jtot = 0, l = 0;
            for (;;) {
                if (l == 0) {
                    if (ql_small(fe[0], fd[0], fd[1])) { fe[0] = 0.f; l = 1; continue; }
                    if (ql_small(fe[1], fd[1], fd[2])) { fe[1] = 0.f; tail = 2; break; }
                    if (jtot == nmaxit) break;
                    ++jtot;
                    ql_sweep3(fd, fe, Z, qr);
                } else {                      // l == 1: the frame's block [1,2]
                    if (ql_small(fe[1], fd[1], fd[2])) fe[1] = 0.f;
                    else tail = 1;
                    break;
                }
            }
            d[0] = qr ? fd[2] : fd[0]; d[1] = fd[1]; d[2] = qr ? fd[0] : fd[2];
            e[0] = qr ? fe[1] : fe[0]; e[1] = qr ? fe[0] : fe[1];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float z0 = Z[i][0], z2 = Z[i][2];
                Z[i][0] = qr ? z2 : z0;
                Z[i][2] = qr ? z0 : z2;
            }
            // the frame's [1,2] is the original [1,2] (QL) or [0,1] (QR); its [0,1] the original [0,1] or [1,2]
            if (tail != 0) tail2r((tail == 1) != qr, d, e, Z);
            if (sc != 1.f) {
                const float us = block_unscale(anorm);
#pragma unroll
                for (int i = 0; i < 3; ++i) d[i] *= us;
                e[0] *= us; e[1] *= us;
            }
        }
    }
    // selection sort, ascending (swaps columns of Z)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int k = i;
        float p = d[i];
#pragma unroll
        for (int j = i + 1; j < 3; ++j)
            if (d[j] < p) { k = j; p = d[j]; }
#pragma unroll
        for (int kk = i + 1; kk < 3; ++kk) {
            if (k == kk) {
                d[kk] = d[i]; d[i] = p;
#pragma unroll
                for (int r = 0; r < 3; ++r) { const float t = Z[r][i]; Z[r][i] = Z[r][kk]; Z[r][kk] = t; }
            }
        }
    }
}
}  // namespace lapack

PCD_DEV void eigh3(Sym3 A, float w[3], float V[3][3]) {
    using namespace lapack;
    // ssyevd's scaling: a matrix whose largest entry lies outside [rmin, rmax] is scaled into range first (slascl: one
    // multiplication by sigma for every sigma reachable here) and the eigenvalues are scaled back by 1/sigma
    const float anrm = fmaxf(fmaxf(fmaxf(fabsf(A.a00), fabsf(A.a01)), fmaxf(fabsf(A.a02), fabsf(A.a11))),
                             fmaxf(fabsf(A.a12), fabsf(A.a22)));
    constexpr float kRmin = 3.14018491736755e-16f;   // sqrt(slamch('S') / slamch('P')) = 2^-51.5
    constexpr float kRmax = 3.18452583626389e+15f;   // sqrt(1 / (slamch('S') / slamch('P')))
    float sigma = 1.f;
    if (anrm > 0.f && anrm < kRmin) sigma = ldiv(kRmin, anrm);
    else if (anrm > kRmax) sigma = ldiv(kRmax, anrm);
    if (sigma != 1.f) {
        A.a00 *= sigma; A.a01 *= sigma; A.a02 *= sigma; A.a11 *= sigma; A.a12 *= sigma; A.a22 *= sigma;
    }
    float a22 = A.a11, a32 = A.a12, a33 = A.a22;
    const float a21 = A.a01, a31 = A.a02;
    // ssytd2 (UPLO='L'), i = 1: slarfg(2, a21, a31) -> H(1) = I - tau v vᵀ, v = (1, v2) on rows/cols 2..3
    float tau = 0.f, v2 = 0.f, e1 = a21;
    if (fabsf(a31) != 0.f) {
        const float beta = -fsign(slapy2(a21, fabsf(a31)), a21);
        tau = ldiv(beta - a21, beta);
        v2 = a31 * ldiv(1.f, a21 - beta);
        e1 = beta;
        // x = tau * A22 * v (ssymv, lower), w = x - tau/2 (xᵀv) v, A22 -= v wᵀ + w vᵀ (ssyr2), with the fma
        // placement of MKL's kernels (fitted against mkl_lapack_ssytd2, 100 % bitwise): ssymv fuses the second column's
        // term, the dot product does not fuse, saxpy and ssyr2 fuse every update of the trailing column
        float y1 = fmaf(tau, a32 * v2, tau * a22);
        float y2 = fmaf(tau * v2, a33, tau * a32);
        const float alpha = -0.5f * tau * (y1 + y2 * v2);
        y1 = y1 + alpha;
        y2 = fmaf(alpha, v2, y2);
        a22 = (a22 - y1) - y1;
        a32 = fmaf(v2, -y1, a32) - y2;
        a33 = fmaf(y2, -v2, fmaf(v2, -y2, a33));
    }
    float d[3] = {A.a00, a22, a33};
    float e[2] = {e1, a32};
    float Z[3][3];
    ssteqr3(d, e, Z);
    // sormtr: Z := H(1) Z on rows 2..3 (slarf: w = Zᵀv unfused, then Z -= tau v wᵀ fused, as mkl_lapack_sormtr)
    if (tau != 0.f) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float s = Z[1][j] + v2 * Z[2][j];
            Z[1][j] = fmaf(-tau, s, Z[1][j]);
            Z[2][j] = fmaf(-(tau * s), v2, Z[2][j]);
        }
    }
    if (sigma != 1.f) {
        const float rs = ldiv(1.f, sigma);
        d[0] *= rs; d[1] *= rs; d[2] *= rs;
    }
    w[0] = d[0]; w[1] = d[1]; w[2] = d[2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) V[r][k] = Z[r][k];
}

// ---------------------------------------------------------------- 3x3 inverse, then A^-1 b (the reference's order)
// The position steps call torch.linalg.inv_ex(A) and then einsum("nij,nj->ni", A^-1, b) (Denoiser.py:43-46, 80-83,
// 163-166, 210-213).  inv_ex is linalg_solve_ex(A, I); for a row-major A torch factors the column-major view A^T
// (LAPACK sgetrf) and solves with trans = 'T' (sgetrs).  The arithmetic below restates what MKL (2024.2, AVX-512
// path, the library the golden fixtures were generated with) does for n = 3, operation for operation -- bit-identical
// to torch.linalg.inv_ex on 400k random and SPD-like matrices (tests/test_capi.py::test_host_inv3_matches_torch):
//   getrf(M = A^T): pivot = first max |m_r0|; l_r0 = m_r0 * (1 / m_00) (reciprocal, then multiply); trailing updates
//                   fused (fma); second column: pivot, l_21 = m_21 / m_11 (a division); m_22 = fma(-l_21, m_12, m_22)
//   info != 0 iff some U_ii is exactly zero (the reference's `mask_inversable`)
//   U^T Y = I  forward, unfused, each row times the reciprocal of its diagonal
//   L^T Z = Y  Z1 = fma(-l21, Z2, Y1); Z0 = Y0 - fma(l10, Z1, l20 * Z2)
//   X = P^T Z  (rows back through the interchanges)
// The product A^-1 b is then (a_0 b_0 + a_1 b_1) + a_2 b_2 per row, unfused, as torch's small-bmm loop sums.
PCD_DEV bool inv3_ref(const float A[3][3], float X[3][3]) {
    // M = A^T, rows r of M: (A[0][r], A[1][r], A[2][r]); perm tracks the original row of each pivoted row
    float m00 = A[0][0], m01 = A[1][0], m02 = A[2][0];
    float m10 = A[0][1], m11 = A[1][1], m12 = A[2][1];
    float m20 = A[0][2], m21 = A[1][2], m22 = A[2][2];
    int p0 = 0, p1 = 1, p2 = 2;
    auto swp = [](float& a, float& b) { const float t = a; a = b; b = t; };
    auto swpi = [](int& a, int& b) { const int t = a; a = b; b = t; };
    // column 0: first max |m_r0|
    {
        const float a0 = fabsf(m00), a1 = fabsf(m10), a2 = fabsf(m20);
        int piv = 0;
        float best = a0;
        if (a1 > best) { best = a1; piv = 1; }
        if (a2 > best) { piv = 2; }
        if (piv == 1) { swp(m00, m10); swp(m01, m11); swp(m02, m12); swpi(p0, p1); }
        if (piv == 2) { swp(m00, m20); swp(m01, m21); swp(m02, m22); swpi(p0, p2); }
    }
    bool ok = m00 != 0.f;
    float l10 = m10, l20 = m20;
    if (ok) {
        const float r0 = 1.f / m00;
        l10 = m10 * r0;
        l20 = m20 * r0;
    }
    m11 = __builtin_fmaf(-l10, m01, m11);
    m12 = __builtin_fmaf(-l10, m02, m12);
    m21 = __builtin_fmaf(-l20, m01, m21);
    m22 = __builtin_fmaf(-l20, m02, m22);
    // column 1
    if (fabsf(m21) > fabsf(m11)) { swp(l10, l20); swp(m11, m21); swp(m12, m22); swpi(p1, p2); }
    ok = ok && m11 != 0.f;
    float l21 = m21;
    if (m11 != 0.f) l21 = m21 / m11;
    m22 = __builtin_fmaf(-l21, m12, m22);
    ok = ok && m22 != 0.f;
    if (!ok) return false;
    // U = [[m00, m01, m02], [0, m11, m12], [0, 0, m22]]; solve U^T Y = e_j, then L^T Z = Y, column by column
    const float r00 = 1.f / m00, r11 = 1.f / m11, r22 = 1.f / m22;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float e0 = j == 0 ? 1.f : 0.f, e1 = j == 1 ? 1.f : 0.f, e2 = j == 2 ? 1.f : 0.f;
        const float y0 = e0 * r00;
        const float y1 = (e1 - m01 * y0) * r11;
        const float y2 = ((e2 - m02 * y0) - m12 * y1) * r22;
        const float z2 = y2;
        const float z1 = __builtin_fmaf(-l21, z2, y1);
        const float z0 = y0 - __builtin_fmaf(l10, z1, l20 * z2);
        // X[p_k][j] = z_k (static selects: no dynamic register index)
#pragma unroll
        for (int r = 0; r < 3; ++r) X[r][j] = r == p0 ? z0 : r == p1 ? z1 : z2;
    }
    return true;
}
PCD_DEV Vec3 matvec3(const float X[3][3], Vec3 b) {
    return v3((X[0][0] * b.x + X[0][1] * b.y) + X[0][2] * b.z, (X[1][0] * b.x + X[1][1] * b.y) + X[1][2] * b.z,
              (X[2][0] * b.x + X[2][1] * b.y) + X[2][2] * b.z);
}
// x = A^-1 b as the reference computes it; false iff inv_ex reports info != 0 (the caller keeps v_i).
PCD_DEV bool solve3(const float A[3][3], Vec3 b, Vec3& x) {
    float X[3][3];
    if (!inv3_ref(A, X)) return false;
    x = matvec3(X, b);
    return true;
}

// ---------------------------------------------------------------- NVT epilogues
// Decomposition.getVUSmoothedNormals(n, tau, d)  (Decompositionor.py:92-106), exactly as written there:
//   E[r][k] = r-th component of the k-th eigenvector in DESCENDING eigenvalue order (stable sort),
//   M = diag([λ_(r) > τ]) indexed by that same rank r,
//   f_n = normalize(d·n + Eᵀ M E n)                (normalisation without epsilon)
// (Eᵀ M E is not the projector E M Eᵀ; with M = I both are the identity.)
PCD_DEV Vec3 vu_smooth(const float w[3], const float V[3][3], Vec3 n, float tau, float damp) {
    // stable descending order of the ascending eigenvalues w[0..2]
    int o[3] = {2, 1, 0};
    // insertion sort by value descending, ties keep ascending index order
    int idx[3] = {0, 1, 2};
#pragma unroll
    for (int a = 1; a < 3; ++a) {
#pragma unroll
        for (int b = a; b > 0; --b) {
            if (w[idx[b]] > w[idx[b - 1]]) { const int t = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = t; }
        }
    }
    o[0] = idx[0]; o[1] = idx[1]; o[2] = idx[2];
    const float nv[3] = {n.x, n.y, n.z};
    float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float Er[3] = {V[r][o[0]], V[r][o[1]], V[r][o[2]]};
        const float u = (Er[0] * nv[0] + Er[1] * nv[1]) + Er[2] * nv[2];
        const float m = (w[o[r]] > tau) ? 1.f : 0.f;
        const float mu = m * u;
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] = acc[c] + mu * Er[c];
    }
    const Vec3 nn = v3(damp * n.x + acc[0], damp * n.y + acc[1], damp * n.z + acc[2]);
    // Tensor.norm(dim=1) on the CPU accumulates the squares with fmas (x² first), then one IEEE sqrt
    const float len = sqrtf(fmaf(nn.z, nn.z, fmaf(nn.y, nn.y, nn.x * nn.x)));
    return v3(nn.x / len, nn.y / len, nn.z / len);
}

// ---------------------------------------------------------------- NVT2: eigenvalues + smallest eigenvector
// NVT2's outputs are the classes (eigenvalues only) and the edge vector (the smallest eigenvalue's eigenvector,
// used only through y·yᵀ and (x·y)·y in edge_step, Denoiser.py:53-88 -- sign-invariant).  Unlike NVT1's VU smoothing
// (Eᵀ·M·E, Decompositionor.py:101-105), nothing here depends on LAPACK's eigenvector signs or degenerate bases, so
// a cyclic Jacobi solve replaces the ssytd2 + ssteqr port: 3 fixed sweeps of the 3 plane rotations (fp32 Jacobi
// converges quadratically; after 3 sweeps the off-diagonal is at rounding level), no data-dependent loop, no
// divergence.  Eigenvalue error ~1e-7 of the trace (the tests' bound for eigenvalues is 2e-6).
// On the device the rotation is built from the hardware reciprocal / square-root estimates (~1 ulp): any (c, s)
// with c² + s² = 1 to rounding keeps the similarity orthogonal, and the off-diagonal still vanishes to rounding
// after the fixed sweeps, so only the last bits of the eigenvalues change (the host build: the IEEE operations).
PCD_DEV float jrcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.f / x;
#endif
}
PCD_DEV float jsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
PCD_DEV float jrsq(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rsqf(x);
#else
    return 1.f / sqrtf(x);
#endif
}
template <int P, int Q, int R>
PCD_DEV void jacobi_rot(float (&a)[3][3], float (&V)[3][3]) {
    const float apq = a[P][Q];
    const float theta = (a[Q][Q] - a[P][P]) * (0.5f * jrcp(apq));
    float t = jrcp(fabsf(theta) + jsqrt(theta * theta + 1.f));
    t = theta < 0.f ? -t : t;
    t = apq == 0.f ? 0.f : t;                      // nothing to rotate (theta would be +-inf or NaN)
    t = t == t ? t : 0.f;                          // theta² overflowed to inf - inf: a negligible apq
    const float c = jrsq(t * t + 1.f), s = t * c;
    a[P][P] = a[P][P] - t * apq;
    a[Q][Q] = a[Q][Q] + t * apq;
    a[P][Q] = a[Q][P] = 0.f;
    const float arp = a[R][P], arq = a[R][Q];
    a[R][P] = a[P][R] = c * arp - s * arq;
    a[R][Q] = a[Q][R] = s * arp + c * arq;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float vp = V[i][P], vq = V[i][Q];
        V[i][P] = c * vp - s * vq;
        V[i][Q] = s * vp + c * vq;
    }
}
// Ascending eigenvalues w of T and the eigenvector y of w[0] (unit length, arbitrary sign).
static constexpr int kJacobiSweeps = 3;   // (4 measured: NVT2 +0.014 ms, same classes in every parity test)
PCD_DEV void eigh3_min(const Sym3& T, float w[3], Vec3& y) {
    float a[3][3] = {{T.a00, T.a01, T.a02}, {T.a01, T.a11, T.a12}, {T.a02, T.a12, T.a22}};
    float V[3][3] = {{1.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, {0.f, 0.f, 1.f}};
#pragma unroll
    for (int sweep = 0; sweep < kJacobiSweeps; ++sweep) {
        jacobi_rot<0, 1, 2>(a, V);
        jacobi_rot<0, 2, 1>(a, V);
        jacobi_rot<1, 2, 0>(a, V);
    }
    const float d0 = a[0][0], d1 = a[1][1], d2 = a[2][2];
    // ascending order (3 compare-exchanges on (value, column)); the smallest picks its column of V
    float e[3] = {d0, d1, d2};
    int c[3] = {0, 1, 2};
    auto cx = [&](int i, int j) {
        const bool sw = e[j] < e[i];
        const float ev = sw ? e[j] : e[i]; e[j] = sw ? e[i] : e[j]; e[i] = ev;
        const int cv = sw ? c[j] : c[i]; c[j] = sw ? c[i] : c[j]; c[i] = cv;
    };
    cx(0, 1); cx(1, 2); cx(0, 1);
    w[0] = e[0]; w[1] = e[1]; w[2] = e[2];
    y = c[0] == 0 ? v3(V[0][0], V[1][0], V[2][0]) : c[0] == 1 ? v3(V[0][1], V[1][1], V[2][1]) : v3(V[0][2], V[1][2], V[2][2]);
    // The rotation-accumulated vector carries the sweeps' leftover off-diagonal over the gap (~1e-6 / gap rad,
    // tests/test_gpu_stages.py); the null vector of T - λ0 I as the largest cross product of two of its rows is
    // accurate to rounding over the gap (λ0 itself is second-order accurate), as LAPACK's is.  Used where the gap
    // to λ1 is not degenerate (|cross|² >= (1e-3 λmax²)²: every edge point); else the Jacobi vector stays.
    {
        const float l = e[0];
        const float r0[3] = {T.a00 - l, T.a01, T.a02}, r1[3] = {T.a01, T.a11 - l, T.a12}, r2[3] = {T.a02, T.a12, T.a22 - l};
        auto cr = [](const float a[3], const float b[3]) {
            return v3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
        };
        const Vec3 x0 = cr(r0, r1), x1 = cr(r0, r2), x2 = cr(r1, r2);
        const float n0 = sq3(x0), n1 = sq3(x1), n2 = sq3(x2);
        Vec3 x = x0;
        float nn = n0;
        if (n1 > nn) { x = x1; nn = n1; }
        if (n2 > nn) { x = x2; nn = n2; }
        const float lm = fmaxf(fabsf(e[2]), fabsf(e[0]));
        const float thr = 1e-3f * lm * lm;
        if (nn >= thr * thr && nn < 3.0e38f) {
            const float inv = jrsq(nn);
            y = v3(x.x * inv, x.y * inv, x.z * inv);
        }
    }
    if (!(d0 == d0 && d1 == d1 && d2 == d2)) { w[0] = w[1] = w[2] = NAN; }
}

// Decomposition.getNVTFeatures + getClasses(scale)  (Decompositionor.py:57-69)
// argmax(scale*planarity, linearity, sphericity); first index wins ties, NaN propagates as in torch.
PCD_DEV int classify(const float w[3], float scale, float* feat /*nullable, 3*/) {
    const float l1 = w[2], l2 = w[1], l3 = w[0];
    const float lin = (l2 - l3) / l1;
    const float pla = (l1 - l2) / l1;
    const float sph = l3 / l1;
    if (feat) { feat[0] = pla; feat[1] = lin; feat[2] = sph; }
    const float f0 = pla * scale;
    // torch.argmax treats NaN as the maximum (first NaN wins)
    if (f0 != f0) return 0;
    if (lin != lin) return 1;
    if (sph != sph) return 2;
    int best = 0; float bv = f0;
    if (lin > bv) { best = 1; bv = lin; }
    if (sph > bv) { best = 2; }
    return best;
}

}  // namespace pcd
