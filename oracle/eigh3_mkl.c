/* CPU ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/pcd_oracle.py's header): imported through ctypes by
 * oracle/pcd_oracle.py alone, never by the product library.
 *
 * torch.linalg.eigh on CPU float32 for batches of 3x3 symmetric matrices -- the reference's own call in
 * Decompositionor.getBetterFilteredNVT / getNormalFilteredNVT / getNormalFilteredPVT (Decompositionor.py:211, 276,
 * 300) and GraphBuilder.getPVTDecompositionWithKNN (GraphBuilder.py:111) -- restated as LAPACK's ssyevd(JOBZ='V',
 * UPLO='L') written as LAPACK's own general loops (ssytd2, ssteqr, sormtr), with the rounding of MKL 2024.2's AVX-512
 * code path: the fused multiply-adds sit where MKL's kernels put them (listed at each routine).  MKL takes other code
 * paths on other CPUs (the GPU boxes' EPYC hosts round ~15 % of NVT neighbourhoods differently), so the oracle does not
 * call torch's eigh live; tests/test_oracle_golden.py pins this file bit for bit against tests/golden/eigh.npz (MKL's
 * outputs saved by tests/golden/make_eigh_golden.py) and against the reference's own NVT decompositions.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: every fma below is an explicit fmaf, nothing else contracts).
 */
#include <math.h>
#include <stdint.h>

#define EPS 5.9604644775390625e-08f       /* slamch('E') = 2^-24 */
#define SAFMIN 1.17549435e-38f             /* slamch('S') */
#define SAFMN2 4.4408920985006262e-16f     /* slartg's scaling bounds 2^-51 and 2^51 */
#define SAFMX2 2.2517998136852480e+15f
#define SSFMAX 3.07445734e+18f             /* ssteqr: sqrt(1 / safmin) / 3 */
#define SSFMIN 3.0517578125e-05f           /* ssteqr: sqrt(safmin) / eps^2 */
#define RMIN 3.14018491736755e-16f         /* ssyevd: sqrt(safmin / (eps * base)) */
#define RMAX 3.18452583626389e+15f

static float sgn(float a, float b) { return b >= 0.f ? fabsf(a) : -fabsf(a); }

static float slapy2(float x, float y) {
    float xa = fabsf(x), ya = fabsf(y);
    float w = xa > ya ? xa : ya, z = xa > ya ? ya : xa;
    if (z == 0.f || w > 3.4028235e38f) return w;
    return w * sqrtf(1.f + (z / w) * (z / w));
}

/* slartg as in LAPACK <= 3.9 (the version MKL's ssteqr follows): c > 0 forced only when |f| > |g| */
static void slartg(float f, float g, float *c, float *s, float *r) {
    if (g == 0.f) { *c = 1.f; *s = 0.f; *r = f; return; }
    if (f == 0.f) { *c = 0.f; *s = 1.f; *r = g; return; }
    float f1 = f, g1 = g, scale = fabsf(f1) > fabsf(g1) ? fabsf(f1) : fabsf(g1);
    int count = 0, i;
    if (scale >= SAFMX2) {
        do { f1 *= SAFMN2; g1 *= SAFMN2; ++count; scale = fabsf(f1) > fabsf(g1) ? fabsf(f1) : fabsf(g1); }
        while (scale >= SAFMX2 && count < 20);
        *r = sqrtf(f1 * f1 + g1 * g1); *c = f1 / *r; *s = g1 / *r;
        for (i = 0; i < count; ++i) *r *= SAFMX2;
    } else if (scale <= SAFMN2) {
        do { f1 *= SAFMX2; g1 *= SAFMX2; ++count; scale = fabsf(f1) > fabsf(g1) ? fabsf(f1) : fabsf(g1); }
        while (scale <= SAFMN2 && count < 20);
        *r = sqrtf(f1 * f1 + g1 * g1); *c = f1 / *r; *s = g1 / *r;
        for (i = 0; i < count; ++i) *r *= SAFMN2;
    } else {
        *r = sqrtf(f1 * f1 + g1 * g1); *c = f1 / *r; *s = g1 / *r;
    }
    if (fabsf(f) > fabsf(g) && *c < 0.f) { *c = -*c; *s = -*s; *r = -*r; }
}

/* slaev2: eigensystem of [[a, b], [b, c]] -- rt1 of larger absolute value, (cs1, sn1) its eigenvector */
static void slaev2(float a, float b, float c, float *rt1, float *rt2, float *cs1, float *sn1) {
    float sm = a + c, df = a - c, adf = fabsf(df), tb = b + b, ab = fabsf(tb), acmx, acmn, rt, cs, ct, tn;
    int sgn1, sgn2;
    if (fabsf(a) > fabsf(c)) { acmx = a; acmn = c; } else { acmx = c; acmn = a; }
    if (adf > ab) rt = adf * sqrtf(1.f + (ab / adf) * (ab / adf));
    else if (adf < ab) rt = ab * sqrtf(1.f + (adf / ab) * (adf / ab));
    else rt = ab * 1.41421356237309515f;
    if (sm < 0.f) { *rt1 = 0.5f * (sm - rt); sgn1 = -1; *rt2 = (acmx / *rt1) * acmn - (b / *rt1) * b; }
    else if (sm > 0.f) { *rt1 = 0.5f * (sm + rt); sgn1 = 1; *rt2 = (acmx / *rt1) * acmn - (b / *rt1) * b; }
    else { *rt1 = 0.5f * rt; *rt2 = -0.5f * rt; sgn1 = 1; }
    if (df >= 0.f) { cs = df + rt; sgn2 = 1; } else { cs = df - rt; sgn2 = -1; }
    if (fabsf(cs) > ab) { ct = -tb / cs; *sn1 = 1.f / sqrtf(1.f + ct * ct); *cs1 = ct * *sn1; }
    else if (ab == 0.f) { *cs1 = 1.f; *sn1 = 0.f; }
    else { tn = -cs / tb; *cs1 = 1.f / sqrtf(1.f + tn * tn); *sn1 = tn * *cs1; }
    if (sgn1 == sgn2) { tn = *cs1; *cs1 = -*sn1; *sn1 = tn; }
}

/* slasr(SIDE='R', PIVOT='V'): plane rotation (c, s) on columns j, j+1 of the 3x3 Z (row-major z[3*i + col]).
 * MKL's kernel fuses each update around its second product: z_{j+1} = fma(c, t, -(s z_j)), z_j = fma(s, t, c z_j). */
static void slasr_col(float *z, int j, float c, float s) {
    int i;
    if (c == 1.f && s == 0.f) return;
    for (i = 0; i < 3; ++i) {
        float t = z[3 * i + j + 1], zj = z[3 * i + j];
        z[3 * i + j + 1] = fmaf(c, t, -(s * zj));
        z[3 * i + j] = fmaf(s, t, c * zj);
    }
}

/* slascl over d[l..lend], e[l..lend-1] by cto / cfrom (the bounds reachable here take one multiplication) */
static void scale_block(float *d, float *e, int l, int lend, float f) {
    int i;
    for (i = l; i <= lend; ++i) d[i] *= f;
    for (i = l; i < lend; ++i) e[i] *= f;
}

/* ssteqr(COMPZ='I'), n = 3, LAPACK's loop: split into unreduced blocks, QL from the top or QR from the bottom
 * (whichever end is larger), Wilkinson shift, slaev2 for 2x2 blocks, 30n iterations at most, selection sort. */
static void ssteqr(float *d, float *e, float *z) {
    const int n = 3, nmaxit = 3 * 30;
    int i, j, jtot = 0, l1 = 0, m, mm, l, lsv, lend, lendsv, ii, k;
    float anorm, fac, p, g, r, s, c, f, b, rt1, rt2, wc[2], ws[2], tst;
    for (i = 0; i < 9; ++i) z[i] = (i % 4 == 0) ? 1.f : 0.f;
    while (l1 < n) {
        if (l1 > 0) e[l1 - 1] = 0.f;
        m = n - 1;
        for (mm = l1; mm < n - 1; ++mm) {
            tst = fabsf(e[mm]);
            if (tst == 0.f) { m = mm; break; }
            if (tst <= (sqrtf(fabsf(d[mm])) * sqrtf(fabsf(d[mm + 1]))) * EPS) { e[mm] = 0.f; m = mm; break; }
        }
        l = l1; lsv = l; lend = m; lendsv = lend; l1 = m + 1;
        if (lend == l) continue;
        anorm = 0.f;
        for (i = l; i <= lend; ++i) if (fabsf(d[i]) > anorm) anorm = fabsf(d[i]);
        for (i = l; i < lend; ++i) if (fabsf(e[i]) > anorm) anorm = fabsf(e[i]);
        if (anorm == 0.f) continue;
        fac = anorm > SSFMAX ? SSFMAX / anorm : (anorm < SSFMIN ? SSFMIN / anorm : 1.f);
        if (fac != 1.f) scale_block(d, e, l, lend, fac);
        if (fabsf(d[lend]) < fabsf(d[l])) { lend = lsv; l = lendsv; }
        if (lend > l) {                                   /* QL */
            for (;;) {
                m = lend;
                for (mm = l; mm < lend; ++mm) {
                    tst = fabsf(e[mm]) * fabsf(e[mm]);
                    if (tst <= (EPS * EPS * fabsf(d[mm])) * fabsf(d[mm + 1]) + SAFMIN) { m = mm; break; }
                }
                if (m < lend) e[m] = 0.f;
                p = d[l];
                if (m == l) { ++l; if (l <= lend) continue; break; }
                if (m == l + 1) {
                    slaev2(d[l], e[l], d[l + 1], &rt1, &rt2, &c, &s);
                    slasr_col(z, l, c, s);
                    d[l] = rt1; d[l + 1] = rt2; e[l] = 0.f; l += 2;
                    if (l <= lend) continue;
                    break;
                }
                if (jtot == nmaxit) break;
                ++jtot;
                g = (d[l + 1] - p) / (2.f * e[l]);
                r = slapy2(g, 1.f);
                g = d[m] - p + (e[l] / (g + sgn(r, g)));
                s = 1.f; c = 1.f; p = 0.f;
                for (i = m - 1; i >= l; --i) {
                    f = s * e[i]; b = c * e[i];
                    slartg(g, f, &c, &s, &r);
                    if (i != m - 1) e[i + 1] = r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * s + 2.f * c * b;
                    p = s * r;
                    d[i + 1] = g + p;
                    g = c * r - b;
                    wc[i - l] = c; ws[i - l] = -s;
                }
                for (j = m - 1; j >= l; --j) slasr_col(z, j, wc[j - l], ws[j - l]);    /* slasr DIRECT='B' */
                d[l] = d[l] - p;
                e[l] = g;
            }
        } else {                                          /* QR */
            for (;;) {
                m = lend;
                for (mm = l; mm > lend; --mm) {
                    tst = fabsf(e[mm - 1]) * fabsf(e[mm - 1]);
                    if (tst <= (EPS * EPS * fabsf(d[mm])) * fabsf(d[mm - 1]) + SAFMIN) { m = mm; break; }
                }
                if (m > lend) e[m - 1] = 0.f;
                p = d[l];
                if (m == l) { --l; if (l >= lend) continue; break; }
                if (m == l - 1) {
                    slaev2(d[l - 1], e[l - 1], d[l], &rt1, &rt2, &c, &s);
                    slasr_col(z, l - 1, c, s);
                    d[l - 1] = rt1; d[l] = rt2; e[l - 1] = 0.f; l -= 2;
                    if (l >= lend) continue;
                    break;
                }
                if (jtot == nmaxit) break;
                ++jtot;
                g = (d[l - 1] - p) / (2.f * e[l - 1]);
                r = slapy2(g, 1.f);
                g = d[m] - p + (e[l - 1] / (g + sgn(r, g)));
                s = 1.f; c = 1.f; p = 0.f;
                for (i = m; i <= l - 1; ++i) {
                    f = s * e[i]; b = c * e[i];
                    slartg(g, f, &c, &s, &r);
                    if (i != m) e[i - 1] = r;
                    g = d[i] - p;
                    r = (d[i + 1] - g) * s + 2.f * c * b;
                    p = s * r;
                    d[i] = g + p;
                    g = c * r - b;
                    wc[i - m] = c; ws[i - m] = s;
                }
                for (j = m; j <= l - 1; ++j) slasr_col(z, j, wc[j - m], ws[j - m]);    /* slasr DIRECT='F' */
                d[l] = d[l] - p;
                e[l - 1] = g;
            }
        }
        if (fac != 1.f) scale_block(d, e, lsv, lendsv, anorm > SSFMAX ? anorm / SSFMAX : anorm / SSFMIN);
        if (jtot >= nmaxit) break;
    }
    for (ii = 1; ii < n; ++ii) {                          /* selection sort, ascending */
        i = ii - 1; k = i; p = d[i];
        for (j = ii; j < n; ++j) if (d[j] < p) { k = j; p = d[j]; }
        if (k != i) {
            d[k] = d[i]; d[i] = p;
            for (j = 0; j < 3; ++j) { float t = z[3 * j + i]; z[3 * j + i] = z[3 * j + k]; z[3 * j + k] = t; }
        }
    }
}

/* ssyevd for one matrix a (row-major 3x3, lower triangle read): w ascending, v row-major (v[3r + k] = component r of
 * eigenvector k) */
static void ssyevd3(const float *a, float *w, float *v) {
    float a11 = a[0], a21 = a[3], a31 = a[6], a22 = a[4], a32 = a[7], a33 = a[8];
    float anrm = 0.f, sigma = 1.f, tau = 0.f, v2 = 0.f, e1, beta, y1, y2, alpha, d[3], e[2], s;
    const float lo[6] = {a11, a21, a31, a22, a32, a33};
    int i, j;
    for (i = 0; i < 6; ++i) if (fabsf(lo[i]) > anrm) anrm = fabsf(lo[i]);
    if (anrm > 0.f && anrm < RMIN) sigma = RMIN / anrm;
    else if (anrm > RMAX) sigma = RMAX / anrm;
    if (sigma != 1.f) { a11 *= sigma; a21 *= sigma; a31 *= sigma; a22 *= sigma; a32 *= sigma; a33 *= sigma; }
    /* ssytd2 (UPLO='L'): column 1's reflector H = I - tau (1, v2)(1, v2)^T from slarfg(2, a21, a31); column 2's
     * reflector is the identity (n - i = 1) */
    e1 = a21;
    if (a31 != 0.f) {
        beta = -sgn(slapy2(a21, fabsf(a31)), a21);
        tau = (beta - a21) / beta;
        v2 = a31 * (1.f / (a21 - beta));
        e1 = beta;
        /* ssymv y = tau A22 (1, v2) (MKL fuses the second column's term), alpha = -tau/2 y.v (unfused dot),
         * y += alpha v (saxpy, fused), A22 -= v y^T + y v^T (ssyr2, every trailing update fused) */
        y1 = fmaf(tau, a32 * v2, tau * a22);
        y2 = fmaf(tau * v2, a33, tau * a32);
        alpha = -0.5f * tau * (y1 + y2 * v2);
        y1 = y1 + alpha;
        y2 = fmaf(alpha, v2, y2);
        a22 = (a22 - y1) - y1;
        a32 = fmaf(v2, -y1, a32) - y2;
        a33 = fmaf(y2, -v2, fmaf(v2, -y2, a33));
    }
    d[0] = a11; d[1] = a22; d[2] = a33; e[0] = e1; e[1] = a32;
    ssteqr(d, e, v);
    /* sormtr: Z := H Z on rows 2..3 (slarf: s = Z^T (1, v2) unfused, then the rank-1 update fused) */
    if (tau != 0.f)
        for (j = 0; j < 3; ++j) {
            s = v[3 + j] + v2 * v[6 + j];
            v[3 + j] = fmaf(-tau, s, v[3 + j]);
            v[6 + j] = fmaf(-(tau * s), v2, v[6 + j]);
        }
    if (sigma != 1.f) { float rs = 1.f / sigma; d[0] *= rs; d[1] *= rs; d[2] *= rs; }
    w[0] = d[0]; w[1] = d[1]; w[2] = d[2];
}

/* batched entry point: t (m, 3, 3) float32 row-major -> w (m, 3), v (m, 3, 3) */
int oracle_eigh3(const float *t, int64_t m, float *w, float *v) {
    int64_t i;
    for (i = 0; i < m; ++i) ssyevd3(t + 9 * i, w + 3 * i, v + 9 * i);
    return 0;
}
