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
// Radius members are collected and sorted in LDS (cap slots a lane, 16 / 32 / 64 / 128; past 128 in a global
// slot-major key buffer, the same code) and stored slot-major, [cap][nq] rows (a wave's lanes read one slot
// together: whole lines).  A row with more than cap members raises a
// device flag; the call checks it once at the end (its only host sync) and, if set, restores the state it started
// from, doubles cap and runs again -- results never depend on cap.

namespace pcd {

static constexpr int kCpsdBS = 128;

// Members of a row's list in ascending original index (the keys' row halves), read from the lane's LDS slots.
struct LdsKeyNb {
    const unsigned long long* L;    // this lane's slot 0; slot t at L[t * bs]
    int64_t bs;
    PCD_DEV int64_t operator()(int t) const { return (int64_t)(uint32_t)(L[t * bs] & 0xFFFFFFFFull); }
};
struct RowNb {              // slot-major member rows: slot t at L[t * stride]
    const int32_t* L;
    int64_t stride;
    PCD_DEV int64_t operator()(int t) const { return L[t * stride]; }
};

// Radius selection + normal-filtered NVT + VU smoothing of each active row.  The members are collected as
// (original index << 32 | row) keys in the lane's CAP LDS slots (slot-major: conflict-free), insertion-sorted there
// (a few dozen LDS round trips, not global ones), summed in that order, and their rows stored for the PVT pass.
// CAP = 0: the slots are gcap global ones, gk[slot][nq] (selections past the LDS budget; the same code).
template <int CAP, int BS>
__global__ __launch_bounds__(BS) void k_cpsd_nvt(GridView g, const float4* __restrict__ pos,
                                                 const float4* __restrict__ nrm, int64_t N, RowMap rm, float r,
                                                 float rho, float tau, float damp, int32_t* __restrict__ rows,
                                                 int32_t* __restrict__ cnt, float4* __restrict__ fn,
                                                 int* __restrict__ ovf, unsigned long long* __restrict__ gk, int gcap) {
    __shared__ unsigned long long s_k[CAP > 0 ? CAP * BS : 1];
    const int64_t t0 = xcd_block(blockIdx.x, gridDim.x) * BS + threadIdx.x;
    if (t0 >= rm.nq) return;
    const int64_t i = rm(t0);
    const float4 q4 = pos[i];
    const float qx = q4.x, qy = q4.y, qz = q4.z;
    const int64_t BSt = CAP > 0 ? (int64_t)BS : rm.nq;     // slot stride
    const int cap = CAP > 0 ? CAP : gcap;
    unsigned long long* L = CAP > 0 ? s_k + threadIdx.x : gk + t0;
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
        unsigned long long last_bkey = ~0ull;
        uint32_t last_brick = 0u;
        bool last_ok = false;
        for (int cz = lo[2]; cz <= hi[2]; ++cz)
            for (int cy = lo[1]; cy <= hi[1]; ++cy)
                for (int cx = lo[0]; cx <= hi[0]; ++cx) {
                    // the cell's brick (4x4x4 cells) from the hash, reused while the scan stays inside it
                    const unsigned long long key = morton3(cx, cy, cz), bkey = key >> 6;
                    if (bkey != last_bkey) {
                        last_bkey = bkey;
                        last_ok = false;
                        unsigned long long slot = hash_slot(bkey, g.hbits);
                        for (;;) {
                            const uint4 sl = *reinterpret_cast<const uint4*>(g.table + slot);
                            const unsigned long long k2 = (unsigned long long)sl.x | ((unsigned long long)sl.y << 32);
                            if (k2 == bkey) { last_brick = sl.z; last_ok = true; break; }
                            if (k2 == kEmptyKey) break;
                            slot = (slot + 1) & g.mask;
                        }
                    }
                    if (!last_ok) continue;
                    const uint2 ce = g.cells[(uint64_t)last_brick * 64 + (key & 63)];
                    for (uint32_t r0 = ce.x; r0 < ce.y; r0 += 4) {
                        float4 p[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) p[u] = g.pts[min(r0 + (uint32_t)u, ce.y - 1u)];   // 4 rows in flight
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (r0 + (uint32_t)u >= ce.y) break;
                            const float fx = qx - p[u].x, fy = qy - p[u].y, fz = qz - p[u].z;
                            const float d2f = (fx * fx + fy * fy) + fz * fz;
                            bool in = d2f < r2lo;
                            if (!in && !(d2f > r2hi)) {
                                const double dx = (double)qx - (double)p[u].x, dy = (double)qy - (double)p[u].y,
                                             dz = (double)qz - (double)p[u].z;
                                const double d2 =
                                    __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
                                in = d2 <= r2;
                            }
                            if (in) {
                                if (m < cap) L[m * BSt] = ((unsigned long long)__float_as_uint(p[u].w) << 32) | (r0 + u);
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
    for (int a = 1; a < m; ++a) {
        const unsigned long long k = L[a * BSt];
        int b = a - 1;
        for (; b >= 0; --b) {
            const unsigned long long kb = L[b * BSt];
            if (kb <= k) break;
            L[(b + 1) * BSt] = kb;
        }
        L[(b + 1) * BSt] = k;
    }
    int32_t* R = rows + t0;
    for (int t = 0; t < m; ++t) R[t * rm.nq] = (int32_t)(uint32_t)(L[t * BSt] & 0xFFFFFFFFull);
    const float4 n4 = nrm[i];
    const Vec3 ni = v3(n4.x, n4.y, n4.z);
    const Sym3 T = nvt_normal_tensor(Rows4{nrm}, ni, m, LdsKeyNb{L, BSt}, rho);
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

#ifndef PCD_CPSD_LDS_MAX
#define PCD_CPSD_LDS_MAX 128
#endif
static constexpr int kCpsdLdsCap = PCD_CPSD_LDS_MAX;   // larger caps keep their slots in global memory (cgkeys)

static void destroy_cpsd_state(pcd_denoiser* dn) {
    (void)hipFree(dn->ckeys); (void)hipFree(dn->ccnt); (void)hipFree(dn->covf);
    (void)hipFree(dn->csave_pos); (void)hipFree(dn->csave_nrm); (void)hipFree(dn->cgkeys);
    dn->ckeys = nullptr; dn->ccnt = nullptr; dn->covf = nullptr; dn->cgkeys = nullptr;
    dn->csave_pos = dn->csave_nrm = nullptr;
    dn->cpsd_cap = 0;
}

static int cpsd_alloc(pcd_denoiser* dn, int cap) {
    const int64_t N = dn->n;
    (void)hipFree(dn->ckeys);
    (void)hipFree(dn->cgkeys);
    dn->ckeys = nullptr;
    dn->cgkeys = nullptr;
    dn->cpsd_cap = 0;
    if (hipMalloc(&dn->ckeys, (size_t)N * (size_t)cap * sizeof(int32_t)) != hipSuccess)
        return fail(PCD_ERR_OOM, "pcd_cpsd_iterate: radius lists");
    if (cap > kCpsdLdsCap && hipMalloc(&dn->cgkeys, (size_t)N * (size_t)cap * sizeof(unsigned long long)) != hipSuccess)
        return fail(PCD_ERR_OOM, "pcd_cpsd_iterate: radius list slots");
    if (!dn->ccnt && (hipMalloc(&dn->ccnt, N * sizeof(int32_t)) != hipSuccess ||
                      hipMalloc(&dn->covf, sizeof(int)) != hipSuccess ||
                      hipMalloc(&dn->csave_pos, N * sizeof(float4)) != hipSuccess ||
                      hipMalloc(&dn->csave_nrm, N * sizeof(float4)) != hipSuccess))
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
#define PCD_CPSD_NVT(C, B)                                                                                             \
    hipLaunchKernelGGL((k_cpsd_nvt<C, B>), dim3((unsigned)cdiv(rm.nq, B)), dim3(B), 0, st, gv, dn->pos[dn->cur], dn->nrm, \
                       N, rm, cp->r, cp->rho, cp->tau, cp->damp, dn->ckeys, dn->ccnt, dn->fn, dn->covf, dn->cgkeys, cap)
                // LDS slots cost occupancy (cap x 8 B a lane): past 16 slots they pay only on a launch too small to
                // fill the chip anyway (A/B: 50k points 0.23 LDS vs 0.29 ms global; 1M at 64 slots 1.79 vs 1.42 ms)
                const bool lds = cap <= 16 || (cap <= kCpsdLdsCap && rm.nq <= (int64_t)1 << 18);
                if (!lds) PCD_CPSD_NVT(0, 128);
                else if (cap == 16) PCD_CPSD_NVT(16, 128);
                else if (cap == 32) PCD_CPSD_NVT(32, 128);
                else if (cap == 64) PCD_CPSD_NVT(64, 64);
                else PCD_CPSD_NVT(128, 64);
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
        // a radius selection had more members than the list slots: restart from the saved state with twice the slots
        const int cap = dn->cpsd_cap * 2;
        PCD_CHECK_ARG(cap <= (1 << 20), "a radius selection holds more than 2^20 points");
        if ((rc = cpsd_alloc(dn, cap)) != PCD_OK) return rc;
        dn->cur = cur0;
        PCD_HIP(hipMemcpyAsync(dn->pos[dn->cur], dn->csave_pos, N * sizeof(float4), hipMemcpyDeviceToDevice, st));
        PCD_HIP(hipMemcpyAsync(dn->nrm, dn->csave_nrm, N * sizeof(float4), hipMemcpyDeviceToDevice, st));
        dn->unit_nrm = unit0;
    }
    return PCD_OK;
}

}  // extern "C"
