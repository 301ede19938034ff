// The CPSD ("Martin") comparison driver fused on the device: PostProcessing.ipynb:1041-1062, the
// thesis' 50-iteration baseline, as one library call.  Included once at the end of denoise.hip (it drives the fused
// loop's static stages).
//
// Per iteration, every step on the stream, no host synchronisation:
//   kNN(k_u) of the current positions            the fused loop's anchored kNN, lists only (Selector.py:235-246)
//   k_cpsd_nvt  radius selection r of the current positions over the frozen snapshot (Selector.py:214-233: scipy's
//               f64 membership, members in ascending ORIGINAL index), normal-filtered NVT (Decompositionor.py:260-276),
//               LAPACK-restated eigh, VU smoothing (:92-106) -> f_n
//   k_cpsd_pvt  normal-filtered PVT on f_n over the same members (:172-211), eigh, VU features (eigval < tau).sum % 3
//               (:84-85) -> classes, smallest eigenvector -> edge vectors
//   phases      flat_step (global centre / delta) / edge_step / corner_step with alphas, Jacobi across classes
//               (temp_pos = pos.clone()), per-step clamp d * 20000, global clamp ||temp_pos - original_pos|| < d
//               (the fused loop's jacobi + clamp_global phases, Denoiser.py:26-119)
//   n := f_n
// Radius members are collected as their ORIGINAL indices (the sort key) -- the first 32 in the lane's LDS slots, any
// further ones in the row's own slots of the member-row buffer -- insertion-sorted there, and mapped back to snapshot
// rows through the inverse permutation; the rows are stored slot-major, [cap][nq] (a wave's lanes read one slot
// together: whole lines).  A row with more than cap members raises a device flag; the call checks it once at the end
// (its only host sync) and, if set, restores the state it started from, doubles cap and runs again -- results never
// depend on cap.

namespace pcd {

static constexpr int kCpsdBS = 128;
#ifndef PCD_CPSD_CELLS
#define PCD_CPSD_CELLS 4
#endif
static constexpr int kCpsdCells = PCD_CPSD_CELLS;   // box cells looked up together by a lane
#ifndef PCD_CPSD_ROWS
#define PCD_CPSD_ROWS 8
#endif
static constexpr int kCpsdRows = PCD_CPSD_ROWS;     // candidate rows a lane has in flight

struct RowNb {              // slot-major member rows: slot t at L[t * stride]
    const int32_t* L;
    int64_t stride;
    PCD_DEV int64_t operator()(int t) const { return L[t * stride]; }
};

// A lane's member slots: slot t < L in LDS (slot-major across the block: conflict-free), past that the row's own
// slots of the member-row buffer (rows[t][nq], the row's column t0).
template <int L>
struct CpsdSlots {
    uint32_t* lds;              // this lane's slot 0; slot t at lds[t * BS]
    int bs;
    uint32_t* glb;              // rows + t0; slot t at glb[t * nq]
    int64_t nq;
    PCD_DEV uint32_t get(int t) const { return t < L ? lds[t * bs] : glb[t * nq]; }
    PCD_DEV void set(int t, uint32_t v) const {
        if (t < L) lds[t * bs] = v; else glb[t * nq] = v;
    }
};

// Radius selection + normal-filtered NVT + VU smoothing of each active row.  Members are collected as their original
// indices (scipy's order key) in the lane's slots, insertion-sorted there, mapped to snapshot rows through inv
// (original index -> row), stored slot-major for the PVT pass and summed in that order.  CAP: the call's slots (L of
// them in LDS: 32 x 4 B a lane keeps 5 waves/SIMD).
template <int L, int BS>
__global__ __launch_bounds__(BS) void k_cpsd_nvt(GridView g, const float4* __restrict__ pos,
                                                 const float4* __restrict__ nrm, int64_t N, RowMap rm, float r,
                                                 float rho, float tau, float damp, int32_t* __restrict__ rows,
                                                 int32_t* __restrict__ cnt, float4* __restrict__ fn,
                                                 int* __restrict__ ovf, const int32_t* __restrict__ inv, int cap) {
    __shared__ uint32_t s_k[L * BS];
    const int64_t t0 = xcd_block(blockIdx.x, gridDim.x) * BS + threadIdx.x;
    if (t0 >= rm.nq) return;
    const int64_t i = rm(t0);
    const float4 q4 = pos[i];
    const float qx = q4.x, qy = q4.y, qz = q4.z;
    const CpsdSlots<L> S{s_k + threadIdx.x, BS, reinterpret_cast<uint32_t*>(rows) + t0, rm.nq};
    int m = 0;
    const double rd = (double)r, r2 = rd * rd;
    if (rd >= 0.0) {
        // the cells overlapping [q - r, q + r] (an f32 box widened by a ulp-scale margin); membership is scipy's f64
        // ((dx² + dy²) + dz²) <= r² on the exact f32 inputs (k_radius, pcd_radius_count / _fill)
        const float rf = (float)(rd * (1.0 + 1e-6)) + 1e-30f;
        const int lo[3] = {max(cell_coord(qx - rf, g.ox, g.inv_h), 0), max(cell_coord(qy - rf, g.oy, g.inv_h), 0),
                           max(cell_coord(qz - rf, g.oz, g.inv_h), 0)};
        const int hi[3] = {min(cell_coord(qx + rf, g.ox, g.inv_h), g.dx - 1),
                           min(cell_coord(qy + rf, g.oy, g.inv_h), g.dy - 1),
                           min(cell_coord(qz + rf, g.oz, g.inv_h), g.dz - 1)};
        // f32 pre-test: a candidate clearly inside or outside (relative margin 1e-5, far above fp32 rounding of d²)
        // is decided without the f64 arithmetic; the rest take scipy's exact test
        const float r2f = (float)r2, r2lo = r2f * (1.f - 1e-5f), r2hi = r2f * (1.f + 1e-5f);
        // the box's cells in chunks of kCpsdCells, every lookup of a chunk in flight together: cells whose box
        // (widened by the grid's key slack) lies beyond r are skipped, then the chunk's brick probes, then its row
        // ranges, then its rows (4 in flight)
        const float h = g.h, sl = g.slack, r2c = r2f * (1.f + 1e-5f) + 1e-30f;
        int cx = lo[0], cy = lo[1], cz = lo[2];
        bool more = lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2];
        while (more) {
            int ccx[kCpsdCells], ccy[kCpsdCells], ccz[kCpsdCells];
            bool on[kCpsdCells];
#pragma unroll
            for (int u = 0; u < kCpsdCells; ++u) {
                on[u] = more;
                ccx[u] = cx; ccy[u] = cy; ccz[u] = cz;
                if (more && ++cx > hi[0]) {
                    cx = lo[0];
                    if (++cy > hi[1]) { cy = lo[1]; if (++cz > hi[2]) more = false; }
                }
                if (on[u]) {
                    const float lx = g.ox + ccx[u] * h, ly = g.oy + ccy[u] * h, lz = g.oz + ccz[u] * h;
                    const float gx = axis_gap(qx, lx - sl, lx + h + sl), gy = axis_gap(qy, ly - sl, ly + h + sl),
                                gz = axis_gap(qz, lz - sl, lz + h + sl);
                    on[u] = gx * gx + gy * gy + gz * gz <= r2c;
                }
            }
            unsigned long long bkey[kCpsdCells];
            uint32_t sidx[kCpsdCells], loc6[kCpsdCells];
            uint4 e[kCpsdCells];
#pragma unroll
            for (int u = 0; u < kCpsdCells; ++u) {
                bkey[u] = kEmptyKey; sidx[u] = 0; loc6[u] = 0;
                if (on[u]) {
                    const unsigned long long key = morton3(ccx[u], ccy[u], ccz[u]);
                    bkey[u] = key >> 6;
                    loc6[u] = (uint32_t)(key & 63);
                    sidx[u] = (uint32_t)hash_slot(bkey[u], g.hbits);
                }
            }
#pragma unroll
            for (int u = 0; u < kCpsdCells; ++u)
                e[u] = on[u] ? *reinterpret_cast<const uint4*>(g.table + sidx[u]) : make_uint4(~0u, ~0u, 0u, 0u);
            uint2 cr[kCpsdCells];
#pragma unroll
            for (int u = 0; u < kCpsdCells; ++u) {
                uint32_t brick = ~0u;
                if (on[u]) {
                    for (;;) {
                        const unsigned long long k2 = (unsigned long long)e[u].x | ((unsigned long long)e[u].y << 32);
                        if (k2 == bkey[u]) { brick = e[u].z; break; }
                        if (k2 == kEmptyKey) break;
                        sidx[u] = (uint32_t)((sidx[u] + 1) & g.mask);
                        e[u] = *reinterpret_cast<const uint4*>(g.table + sidx[u]);
                    }
                }
                cr[u] = make_uint2(0u, 0u);
                if (brick != ~0u) cr[u] = g.cells[(uint64_t)brick * 64 + loc6[u]];
            }
            // the chunk's rows as one stream across its cells (kCpsdRows loads in flight, whatever the cells' sizes)
            uint32_t pre[kCpsdCells + 1];
            pre[0] = 0;
#pragma unroll
            for (int u = 0; u < kCpsdCells; ++u) pre[u + 1] = pre[u] + (cr[u].y > cr[u].x ? cr[u].y - cr[u].x : 0u);
            const uint32_t total = pre[kCpsdCells];
            for (uint32_t b0 = 0; b0 < total; b0 += kCpsdRows) {
                float4 p[kCpsdRows];
#pragma unroll
                for (int w = 0; w < kCpsdRows; ++w) {
                    const uint32_t j = min(b0 + (uint32_t)w, total - 1u);
                    uint32_t row = 0;
#pragma unroll
                    for (int u = 0; u < kCpsdCells; ++u)
                        if (j >= pre[u] && j < pre[u + 1]) row = cr[u].x + (j - pre[u]);
                    p[w] = g.pts[row];
                }
#pragma unroll
                for (int w = 0; w < kCpsdRows; ++w) {
                    if (b0 + (uint32_t)w >= total) break;
                    const float fx = qx - p[w].x, fy = qy - p[w].y, fz = qz - p[w].z;
                    const float d2f = (fx * fx + fy * fy) + fz * fz;
                    bool in = d2f < r2lo;
                    if (!in && !(d2f > r2hi)) {
                        const double dx = (double)qx - (double)p[w].x, dy = (double)qy - (double)p[w].y,
                                     dz = (double)qz - (double)p[w].z;
                        const double d2 =
                            __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
                        in = d2 <= r2;
                    }
                    if (in) {
                        if (m < cap) S.set(m, __float_as_uint(p[w].w));   // (the snapshot's w: original index)
                        ++m;
                    }
                }
            }
        }
    }
    cnt[i] = m;
    if (m > cap) {          // (the call replays with more slots; this row's result is discarded)
        atomicOr(ovf, 1);
        m = cap;
    }
    // ascending original index: scipy's per-query order, the order the reference's scatter sums in
    {
    // the LDS slots by a fixed network in registers (no chain of dependent LDS round trips; unused slots padded with
    // the largest key), then the few overflow members (past L) inserted one by one (an LDS insertion sort over every
    // member: 601 -> 429 us at 1M points)
    {
        const int m0 = min(m, L);
        uint32_t v[L];
#pragma unroll
        for (int t = 0; t < L; ++t) v[t] = t < m0 ? S.lds[t * S.bs] : 0xFFFFFFFFu;
        oddeven_sort<L>(v);
#pragma unroll
        for (int t = 0; t < L; ++t)
            if (t < m0) S.lds[t * S.bs] = v[t];
    }
    for (int a = L; a < m; ++a) {
        const uint32_t k = S.get(a);
        int b = a - 1;
        for (; b >= 0; --b) {
            const uint32_t kb = S.get(b);
            if (kb <= k) break;
            S.set(b + 1, kb);
        }
        S.set(b + 1, k);
    }
    }
    // original index -> snapshot row, into the row's slots of the member-row buffer (in place past L)
    for (int t = 0; t < m; ++t) S.glb[t * rm.nq] = (uint32_t)inv[S.get(t)];
    const float4 n4 = nrm[i];
    const Vec3 ni = v3(n4.x, n4.y, n4.z);
    const Sym3 T = nvt_normal_tensor(Rows4{nrm}, ni, m, RowNb{rows + t0, rm.nq}, rho);
    float w[3], V[3][3];
    eigh3(T, w, V);
    const Vec3 f = vu_smooth(w, V, ni, tau, damp);
    fn[i] = make_float4(f.x, f.y, f.z, 0.f);
}

// Normal-filtered PVT on f_n over the same members, eigh, VU features + edge vector of each active row.
__global__ __launch_bounds__(kCpsdBS) void k_cpsd_pvt(const float4* __restrict__ pos, const float4* __restrict__ fn,
                                                      int64_t N, RowMap rm, float rho, float tau,
                                                      const int32_t* __restrict__ rows, int cap,
                                                      const int32_t* __restrict__ cnt, uint8_t* __restrict__ cls,
                                                      float4* __restrict__ edge) {
    const int64_t t0 = xcd_block(blockIdx.x, gridDim.x) * kCpsdBS + threadIdx.x;
    if (t0 >= rm.nq) return;
    const int64_t i = rm(t0);
    const int m = min(cnt[i], cap);
    const float4 p4 = pos[i], f4 = fn[i];
    const Sym3 C = pvt_normal_cov(Rows4{pos}, Rows4{fn}, v3(p4.x, p4.y, p4.z), v3(f4.x, f4.y, f4.z), m,
                                  RowNb{rows + t0, rm.nq}, rho);
    float w[3], V[3][3];
    eigh3(C, w, V);
    // getVUFeatures(tau) = (eigval < tau).sum(dim=1) % 3 (Decompositionor.py:84-85); NaN compares false
    const int below = (w[0] < tau ? 1 : 0) + (w[1] < tau ? 1 : 0) + (w[2] < tau ? 1 : 0);
    cls[i] = (uint8_t)(below % 3);
    edge[i] = make_float4(V[0][0], V[1][0], V[2][0], 0.f);   // eigvec[..., 0] (Processor's edge_vectors)
}

__global__ void k_cpsd_maxcnt(const int32_t* __restrict__ cnt, RowMap rm, int* __restrict__ mx) {
    int v = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < rm.nq; t += (int64_t)gridDim.x * blockDim.x)
        v = max(v, cnt[rm(t)]);
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) atomicMax(mx, v);
}

}  // namespace pcd

static constexpr int kCpsdLdsSlots = 32;   // member slots a lane keeps in LDS (4 B each; the rest in the row buffer)

namespace pcd {
__global__ void k_inv_perm(const int32_t* __restrict__ perm, int64_t n, int32_t* __restrict__ inv) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r < n) inv[perm[r]] = (int32_t)r;
}
}  // namespace pcd

static void destroy_cpsd_state(pcd_denoiser* dn) {
    (void)hipFree(dn->ckeys); (void)hipFree(dn->ccnt); (void)hipFree(dn->covf);
    (void)hipFree(dn->csave_pos); (void)hipFree(dn->csave_nrm); (void)hipFree(dn->cinv);
    dn->ckeys = nullptr; dn->ccnt = nullptr; dn->covf = nullptr; dn->cinv = nullptr;
    dn->csave_pos = dn->csave_nrm = nullptr;
    dn->cpsd_cap = 0;
    dn->cpsd_elems = 0;
}

// Every buffer the selected k_cpsd_nvt<L> / k_cpsd_pvt launch dereferences, sized for what it indexes: the member
// slots past L (and every slot k_cpsd_pvt reads) live in ckeys at [t][nq] for t < cap, so ckeys must hold cap x nq;
// counts, the inverse permutation and the save buffers hold N rows.  (Round 4's fault: a launch selector that sent
// cap > 16 at nq > 2^18 to a variant keeping its slots in a buffer allocated only past 128 slots -- a null ckeys.)
static bool cpsd_buffers_ok(const pcd_denoiser* dn, int L, int cap, int64_t nq) {
    return dn->ckeys && dn->ccnt && dn->covf && dn->cinv && dn->csave_pos && dn->csave_nrm && cap == dn->cpsd_cap &&
           L <= kCpsdLdsSlots && (cap <= 16 ? L == 16 : L == kCpsdLdsSlots && cap >= L) && nq <= dn->n &&
           dn->cpsd_elems >= (int64_t)cap * nq;
}

static int cpsd_alloc(pcd_denoiser* dn, int cap) {
    const int64_t N = dn->n;
    (void)hipFree(dn->ckeys);
    dn->ckeys = nullptr;
    dn->cpsd_cap = 0;
    dn->cpsd_elems = 0;
    if (hipMalloc(&dn->ckeys, (size_t)N * (size_t)cap * sizeof(int32_t)) != hipSuccess)
        return fail(PCD_ERR_OOM, "pcd_cpsd_iterate: radius lists");
    dn->cpsd_elems = N * (int64_t)cap;
    if (!dn->ccnt && (hipMalloc(&dn->ccnt, N * sizeof(int32_t)) != hipSuccess ||
                      hipMalloc(&dn->covf, sizeof(int)) != hipSuccess ||
                      hipMalloc(&dn->csave_pos, N * sizeof(float4)) != hipSuccess ||
                      hipMalloc(&dn->csave_nrm, N * sizeof(float4)) != hipSuccess ||
                      hipMalloc(&dn->cinv, N * sizeof(int32_t)) != hipSuccess))
        return fail(PCD_ERR_OOM, "pcd_cpsd_iterate: buffers");
    dn->cpsd_cap = cap;
    return PCD_OK;
}

extern "C" {

int pcd_cpsd_iterate(pcd_denoiser* dn, const pcd_cpsd_params* cp, int iterations, void* stream) {
    PCD_CHECK_ARG(dn && cp, "null argument");
    PCD_CHECK_ARG(dn->loaded, "pcd_denoiser_load must be called first");
    PCD_CHECK_ARG(iterations >= 0, "iterations must be >= 0");
    PCD_CHECK_ARG(cp->k_update >= 1 && cp->k_update <= dn->kcap && cp->k_update <= dn->n, "k_update out of range");
    PCD_CHECK_ARG(!(cp->r < 0.f) && !(cp->d < 0.f) && !(cp->step_clamp < 0.f), "r, d, step_clamp must be >= 0");
    hipStream_t st = as_stream(stream);
    int rc = settle(dn, st);
    if (rc != PCD_OK) return rc;
    // the fused loop's parameters for the kNN lists and the phases: Jacobi across classes with the global clamp
    pcd_denoise_params p{};
    p.k = p.k_update = cp->k_update;
    p.rho = cp->rho; p.tau = cp->tau; p.damp = cp->damp; p.class_scale = 0.2f;
    p.d = cp->step_clamp;
    p.nphases = 3;
    const int kinds[3] = {PCD_STEP_FLAT, PCD_STEP_EDGE, PCD_STEP_CORNER};
    for (int ph = 0; ph < 3; ++ph) { p.phase_class[ph] = ph; p.phase_kind[ph] = kinds[ph]; p.phase_alpha[ph] = cp->alpha[ph]; }
    p.jacobi = 1;
    p.clamp_global = cp->d;
    if ((rc = check_params(dn, &p)) != PCD_OK) return rc;
    if (dn->cpsd_cap == 0 && (rc = cpsd_alloc(dn, 16)) != PCD_OK) return rc;
    const int64_t N = dn->n;
    const RowMap rm = dn->rowmap();
    PCD_CHECK_ARG(dn->g && dn->g->n == N, "the denoiser's grid does not index its rows");
    // original index -> snapshot row (the sort key back to the row the member lists hold)
    hipLaunchKernelGGL(k_inv_perm, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, st, dn->g->perm, N, dn->cinv);
    // the state this call starts from (a replay after a radius-list overflow restarts from it)
    PCD_HIP(hipMemcpyAsync(dn->csave_pos, dn->pos[dn->cur], N * sizeof(float4), hipMemcpyDeviceToDevice, st));
    PCD_HIP(hipMemcpyAsync(dn->csave_nrm, dn->nrm, N * sizeof(float4), hipMemcpyDeviceToDevice, st));
    const int cur0 = dn->cur;
    const bool unit0 = dn->unit_nrm;
    for (;;) {
        PCD_HIP(hipMemsetAsync(dn->covf, 0, sizeof(int), st));
        dn->nvt1_on = false;
        for (int it = 0; it < iterations && rc == PCD_OK; ++it) {
            rc = stage_k1(dn, &p, st);                         // kNN(k_u) lists of the current positions
            if (rc != PCD_OK) break;
            const GridView gv = dn->g->view;
            const dim3 grd((unsigned)cdiv(rm.nq, kCpsdBS)), blk(kCpsdBS);
            if (rm.nq > 0) {
                const int cap = dn->cpsd_cap;
                const int L = cap <= 16 ? 16 : kCpsdLdsSlots;
                if (!cpsd_buffers_ok(dn, L, cap, rm.nq)) {
                    rc = fail(PCD_ERR_STATE, "pcd_cpsd_iterate: buffers do not cover the selected kernel variant");
                    break;
                }
#define PCD_CPSD_NVT(C, B)                                                                                             \
    hipLaunchKernelGGL((k_cpsd_nvt<C, B>), dim3((unsigned)cdiv(rm.nq, B)), dim3(B), 0, st, gv, dn->pos[dn->cur], dn->nrm, \
                       N, rm, cp->r, cp->rho, cp->tau, cp->damp, dn->ckeys, dn->ccnt, dn->fn, dn->covf, dn->cinv, cap)
                if (cap <= 16) PCD_CPSD_NVT(16, kCpsdBS);
                else PCD_CPSD_NVT(kCpsdLdsSlots, kCpsdBS);
#undef PCD_CPSD_NVT
                hipLaunchKernelGGL(k_cpsd_pvt, grd, blk, 0, st, dn->pos[dn->cur], dn->fn, N, rm, cp->rho, cp->tau,
                                   dn->ckeys, cap, dn->ccnt, dn->cls, dn->edge);
                if (hipGetLastError() != hipSuccess) { rc = fail(PCD_ERR_HIP, "pcd_cpsd_iterate: launch"); break; }
            }
            for (int ph = 0; ph < 3 && rc == PCD_OK; ++ph) {
                if (phase_is_global(&p, ph)) {
                    double* red4 = dn->red + 4 * ph;
                    if ((rc = stage_sum(dn, &p, ph, red4, st)) != PCD_OK) break;
                    if ((rc = stage_centre(dn, ph, red4, st)) != PCD_OK) break;
                    if ((rc = stage_maxdist(dn, &p, ph, nullptr, st)) != PCD_OK) break;
                }
                rc = stage_apply(dn, &p, ph, nullptr, st);
            }
            if (rc == PCD_OK) stage_finish(dn, &p);
        }
        dn->nvt1_on = true;
        if (rc != PCD_OK) return rc;
        int ovf = 0;
        PCD_HIP(hipMemcpyAsync(&ovf, dn->covf, sizeof(int), hipMemcpyDeviceToHost, st));
        PCD_HIP(hipStreamSynchronize(st));
        if (!ovf || iterations == 0) {
            // slots for the next call with headroom: the largest selection of the last iteration above 3/4 of the
            // slots doubles them now, so a later call does not replay when the points drift into denser spots
            if (iterations > 0 && rm.nq > 0) {
                int* mx = dn->covf;                       // (reused as the max-count cell)
                PCD_HIP(hipMemsetAsync(mx, 0, sizeof(int), st));
                hipLaunchKernelGGL(k_cpsd_maxcnt, dim3((unsigned)std::min<int64_t>(cdiv(rm.nq, 256), 1024)), dim3(256),
                                   0, st, dn->ccnt, rm, mx);
                int h = 0;
                PCD_HIP(hipMemcpyAsync(&h, mx, sizeof(int), hipMemcpyDeviceToHost, st));
                PCD_HIP(hipStreamSynchronize(st));
                if (4 * h > 3 * dn->cpsd_cap) {
                    int cap = dn->cpsd_cap;
                    while (4 * h > 3 * cap) cap *= 2;
                    if ((rc = cpsd_alloc(dn, cap)) != PCD_OK) return rc;
                }
            }
            break;
        }
        // a radius selection had more members than the list slots: back to the saved state first (so an error below
        // leaves the state the call started from), then slots for the largest selection of the last pass -- the
        // counts are exact past the slots -- and at least twice the old ones, and replay
        dn->cur = cur0;
        PCD_HIP(hipMemcpyAsync(dn->pos[dn->cur], dn->csave_pos, N * sizeof(float4), hipMemcpyDeviceToDevice, st));
        PCD_HIP(hipMemcpyAsync(dn->nrm, dn->csave_nrm, N * sizeof(float4), hipMemcpyDeviceToDevice, st));
        dn->unit_nrm = unit0;
        int h = 0;
        {
            int* mx = dn->covf;
            PCD_HIP(hipMemsetAsync(mx, 0, sizeof(int), st));
            hipLaunchKernelGGL(k_cpsd_maxcnt, dim3((unsigned)std::min<int64_t>(cdiv(rm.nq, 256), 1024)), dim3(256), 0,
                               st, dn->ccnt, rm, mx);
            PCD_HIP(hipMemcpyAsync(&h, mx, sizeof(int), hipMemcpyDeviceToHost, st));
            PCD_HIP(hipStreamSynchronize(st));
        }
        int64_t cap = (int64_t)dn->cpsd_cap * 2;
        while (cap < h) cap *= 2;
        PCD_CHECK_ARG(cap <= (1 << 20), "a radius selection holds more than 2^20 points");
        if ((rc = cpsd_alloc(dn, (int)cap)) != PCD_OK) return rc;
    }
    return PCD_OK;
}

}  // extern "C"
