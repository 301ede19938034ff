// Fused denoise loop (H8 + H13/H14): the body of Processor.denoise (Pointcloud/Modules/Processor.py:119-139) on
// persistent device buffers in the grid's spatial (Morton) order.
//
// Per iteration:
//   K1 knn_nvt1   kNN(k) of the current positions against the frozen snapshot, fused with the first tensor vote
//                 (Decompositionor.getBetterFilteredNVT on n) and VU smoothing -> f_n; writes the kNN list
//                 in 8-column row-major blocks (pcd_lists.h: whole 32-B sectors per row and block)
//   K2 nvt2       second vote on f_n -> class (argmax of scaled features) + edge vector (smallest eigenvector)
//   per phase (Gauss-Seidel across phases, Jacobi within, reference order flat -> edge -> corner):
//     [flat/new]  rows_sum -> finish_centre -> rows_maxdist   (GLOBAL centre / delta, Denoiser.py:106-107)
//     K3 phase    class points update from the ping buffer into the pong buffer, the others copy through
//   n := f_n (pointer swap)
// The update kNN list (k_u = 8) is the first k_u columns of the k list: same query positions, same snapshot.
//
// Spatial slabs (multi-GPU): the grid holds a rank's own points plus a halo of other ranks' snapshot points.  Only
// the ACTIVE rows (pcd_denoiser_set_rows) are queried and updated; the halo rows' state is written by the caller's
// exchange between stages (pcd_denoiser_pack/unpack), and the global flat centre / delta reductions are exposed as
// separate stages so the caller can all-reduce them (pcd_denoiser_stage).  pcd_denoiser_iterate is the same stage
// sequence with no exchange.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pcd_knn.h"
#include "pcd_lists.h"
#include "pcd_ops.h"
#include "pcd_qknn.h"

namespace pcd {
int knn_cap(int k);

// Element i of a column whose base is uniform: a 32-bit byte offset (i * sizeof(T) < 4 GiB, checked on the host:
// N < 2^27, pcd_denoiser_create: the blocked lists take 32 B x N) lets the load take the base in SGPRs and one offset VGPR (global_load ... saddr),
// where 64-bit per-lane addresses cost a multiply-add and moves per column.
template <class T>
PCD_DEV const T* at32(const T* base, int64_t i) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (uint32_t)((uint32_t)i * (uint32_t)sizeof(T)));
}
template <class T>
PCD_DEV T* at32(T* base, int64_t i) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (uint32_t)((uint32_t)i * (uint32_t)sizeof(T)));
}

// Column t of row i of a stored list (blocked layout, pcd_lists.h), read from memory.
PCD_DEV const int32_t* lelem(const int32_t* idx, int64_t n, int64_t i, int t) {
    const char* b = reinterpret_cast<const char*>(idx + (int64_t)(t >> 3) * n * 8);
    return reinterpret_cast<const int32_t*>(b + (uint32_t)((uint32_t)i * 32u + (uint32_t)(t & 7) * 4u));
}
struct BlkNb {
    const int32_t* idx;
    int64_t n, i;
    PCD_DEV int64_t operator()(int t) const { return *lelem(idx, n, i, t); }
};
// A stored list re-read from memory with out-of-range entries mapped to the row itself (the fallback pass of
// nvt_tensor; an invalid entry is already reported by the kernel's own check).
struct BlkNbSafe {
    const int32_t* idx;
    int64_t n, i;
    PCD_DEV int64_t operator()(int t) const {
        const int64_t j = *lelem(idx, n, i, t);
        return (uint64_t)j < (uint64_t)n ? j : i;
    }
};
typedef float v4f __attribute__((ext_vector_type(4)));

// LDS window of per-point rows.  The rows are in spatial order, so the neighbours of a block's 256 consecutive rows
// mostly lie within a few hundred rows of them (~90 % within +-256 on scanned surfaces): the block stages that
// window of two row arrays into LDS with coalesced loads, and each neighbour gather reads LDS when it falls inside
// (one ds_read_b128) and global memory otherwise (a global load for those lanes only).  A wave's divergent 16-B
// gathers cost the texture-address unit ~1 cycle per distinct cache line, ~35 cycles per instruction -- the
// measured limiter of the NVT kernels (TA busy 65-77 %); LDS serves them in a few.
// Rows staged on either side of the block's own rows, per kernel (A/B'd at 10M with tools/ab_bench.sh: NVT2 gains
// 0.16 ms from 512, the flat phase loses 0.06 ms from it and gains 0.01 ms from 128).
#ifndef PCD_NVT1_HALO
#define PCD_NVT1_HALO 256
#endif
static constexpr int kWinHalo = PCD_NVT1_HALO;          // NVT1
#ifndef PCD_NVT2_HALO
#define PCD_NVT2_HALO 256   // (A/B at 10M after the round-3 changes: 256 0.870 ms, 384 0.882, 512 0.889)
#endif
#ifndef PCD_PHASE_HALO
#define PCD_PHASE_HALO 128
#endif
static constexpr int kWinHaloNvt2 = PCD_NVT2_HALO;
static constexpr int kWinHaloPhase = PCD_PHASE_HALO;
template <int H, int BS = 256> struct WinSize { static constexpr int rows = BS + 2 * H; };
#ifndef PCD_NVT_BS
#define PCD_NVT_BS 256
#endif
static constexpr int kNvtBS = PCD_NVT_BS;   // threads per NVT block (512 measured: fewer blocks fit the LDS, NVT2 0.92 -> 1.23 ms)
static constexpr int kWinRows = WinSize<kWinHalo, kNvtBS>::rows;
template <int H = kWinHalo, int BS = kNvtBS>
struct WinRows {
    const float4* g;
    const float4* s;
    int64_t lo;
    PCD_DEV Vec3 operator()(int64_t j) const {
        // one 64-bit base select and one scaled add (32-bit row arithmetic: rows < 2^31): the LDS base is biased by
        // -lo rows so that base + 16 j addresses s[j - lo] through the flat aperture.  (Measured against a ds_read for
        // the lanes inside + a masked global load for the others: that split is slower, NVT1 1.20 -> 1.25 ms.)
        const uint32_t j32 = (uint32_t)j;
        const bool in = j32 - (uint32_t)lo < (uint32_t)WinSize<H, BS>::rows;
        const uint64_t sb = (uint64_t)(uintptr_t)s - (uint64_t)(uint32_t)lo * 16u;
        const uint64_t base = in ? sb : (uint64_t)(uintptr_t)g;
        const float4 q = *reinterpret_cast<const float4*>(base + (uint64_t)j32 * 16u);
        return v3(q.x, q.y, q.z);
    }
};
// Stage rows [lo, lo + kWinRows) of a and b (clipped to [0, N)) for the block whose first active row is i_first.
// on == 0 (pcd_denoiser_set_windows, block-uniform): nothing is staged and every row is read from global memory --
// the reference path the windowed reads are checked against bitwise.
static constexpr int64_t kNoWindow = -(1ll << 60) + (1ll << 31);   // (low 32 bits 2^31: no row is inside)
template <int H = kWinHalo, int BS = kNvtBS>
PCD_DEV int64_t stage_window(const float4* __restrict__ a, const float4* __restrict__ b, int64_t N, int64_t i_first,
                             float4* sa, float4* sb, int on) {
    if (!on) return kNoWindow;
    int64_t lo = i_first - H;
    lo = lo < 0 ? 0 : lo;
    for (int r = threadIdx.x; r < WinSize<H, BS>::rows; r += blockDim.x) {
        const int64_t j = lo + r;
        if (j < N) { sa[r] = a[j]; sb[r] = b[j]; }
    }
    __syncthreads();
    return lo;
}
struct RegNb32 {
    const int* l;
    PCD_DEV int64_t operator()(int t) const { return l[t]; }
};

__global__ void k_load(const float* __restrict__ pos, const float* __restrict__ n, const int32_t* __restrict__ perm,
                       int64_t N, float4* __restrict__ pos_s, float4* __restrict__ n_s, float4* __restrict__ orig) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= N) return;
    const int64_t i = perm[r];
    pos_s[r] = make_float4(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2], 0.f);
    orig[r] = pos_s[r];
    n_s[r] = make_float4(n[3 * i], n[3 * i + 1], n[3 * i + 2], 0.f);
}

__global__ void k_gather_f32(const float* __restrict__ in, const int32_t* __restrict__ perm, int64_t N,
                             float* __restrict__ out) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r < N) out[r] = in[perm[r]];
}

__global__ void k_store(const float4* __restrict__ pos_s, const float4* __restrict__ n_s,
                        const uint8_t* __restrict__ cls_s, const float4* __restrict__ edge_s,
                        const int32_t* __restrict__ perm, int64_t N, float* __restrict__ pos, float* __restrict__ n,
                        int64_t* __restrict__ cls, float* __restrict__ edge) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= N) return;
    const int64_t i = perm[r];
    if (pos) { const float4 p = pos_s[r]; pos[3 * i] = p.x; pos[3 * i + 1] = p.y; pos[3 * i + 2] = p.z; }
    if (n) { const float4 p = n_s[r]; n[3 * i] = p.x; n[3 * i + 1] = p.y; n[3 * i + 2] = p.z; }
    if (cls) cls[i] = cls_s[r];
    if (edge) { const float4 p = edge_s[r]; edge[3 * i] = p.x; edge[3 * i + 1] = p.y; edge[3 * i + 2] = p.z; }
}

// Local snapshot coverage: the kNN of a query is exact when its k-ball lies inside this box (spatial slabs:
// the slab widened by the halo).  Disabled when lo > hi on axis 0.
struct Cover {
    float lo[3], hi[3];
    // spatial slabs: rows whose snapshot ball the local snapshot holds beyond the box (a sparse point near a cut:
    // every snapshot point within xr[i] of its load-time position org[i] is local; 0 = none)
    const float* xr = nullptr;
    const float4* org = nullptr;
    PCD_DEV bool enabled() const { return !(lo[0] > hi[0]); }
    PCD_DEV bool holds(Vec3 q, float d2) const {
        if (lo[0] > hi[0]) return true;
        const float r = sqrtf(d2) * 1.000001f + 1e-30f;
        return q.x - r >= lo[0] && q.x + r <= hi[0] && q.y - r >= lo[1] && q.y + r <= hi[1] && q.z - r >= lo[2] &&
               q.z + r <= hi[2];
    }
    // row i's k-ball (centre q, squared radius d2) lies inside the box, or inside the row's own sphere
    PCD_DEV bool holds_row(int64_t i, Vec3 q, float d2) const {
        if (holds(q, d2)) return true;
        if (!xr) return false;
        const float R = xr[i];
        if (!(R > 0.f)) return false;
        const float4 o = org[i];
        const float m = sqrtf(sq3(q - v3(o.x, o.y, o.z))) * 1.000001f + sqrtf(d2) * 1.000001f + 1e-30f;
        return m <= R * (1.f - 1e-6f);
    }
    // the coverage check of row i: on a failure, err[0] |= 2 and what failed -- bit 4: a row without a sphere (the
    // band; err[1] = atomic max of how far its ball reaches past the box, float bits), bit 8: a sphere row (err[2] =
    // atomic max of (|q - centre| + d_k) / R) -- so a re-plan grows only what failed, by what it lacked
    PCD_DEV void check_row(int* err, int64_t i, Vec3 q, float d2) const {
        if (holds_row(i, q, d2)) return;
        const float r = sqrtf(d2) * 1.000001f + 1e-30f;
        const float R = xr ? xr[i] : 0.f;
        if (R > 0.f) {
            const float4 o = org[i];
            const float m = sqrtf(sq3(q - v3(o.x, o.y, o.z))) * 1.000001f + r;
            atomicOr(err, 2 | 8);
            atomicMax(err + 2, __float_as_int(m / R));
        } else {
            const float ex = fmaxf(fmaxf(fmaxf(lo[0] - (q.x - r), (q.x + r) - hi[0]), fmaxf(lo[1] - (q.y - r), (q.y + r) - hi[1])),
                                   fmaxf(lo[2] - (q.z - r), (q.z + r) - hi[2]));
            atomicOr(err, 2 | 4);
            atomicMax(err + 1, __float_as_int(fmaxf(ex, 0.f)));   // (non-negative floats order as their bits)
        }
    }
};

// Spatial slabs: the rank's OWN slab (the points it owns, no halo).  K1 marks every active row whose k-ball is not
// strictly inside it: only those rows can list a halo row (every snapshot point strictly inside the owned slab on
// the cut axis is owned -- slabs are contiguous ranges of the sorted axis key), so the NVT2 / phase passes of the
// other rows need no halo data and run while the halo exchange is in flight (pcd_slab_iterate).  flag null: off.
struct Band {
    Cover box;
    uint8_t* flag;    // [active rows]: 1 = may read a halo row
    PCD_DEV void mark(int64_t t, Vec3 q, float d2) const { if (flag) flag[t] = box.holds(q, d2) ? 0 : 1; }
};
// Row selection of a pass: flag null -> every active row; else the active rows t with flag[t] == want.
struct RowSel {
    const uint8_t* flag;
    int want;
    PCD_DEV bool take(int64_t t) const { return !flag || (int)flag[t] == want; }
};

// K1 epilogue (every kNN variant): store the list (blocked layout), check it, NVT1 + eigh + VU smoothing -> f_n.
// dk = d² of the kstore-th neighbour.
template <int K>
PCD_DEV void k1_epilogue(const float4* __restrict__ pos, const float4* __restrict__ nrm, int64_t N, int64_t i,
                         Vec3 vi, int (&l)[K], float dk, int k, int kstore, float rho, float tau, float damp,
                         const Cover& cov, int32_t* __restrict__ idx, float4* __restrict__ fn, int* __restrict__ err,
                         const Band& band, int64_t t0) {
    bool bad = false;
#pragma unroll
    for (int t = 0; t < K; ++t) {
        // a list entry that is not a point would be an internal error: record it, never fault on it
        if (t < kstore && (uint32_t)l[t] >= (uint32_t)N) { bad = true; l[t] = (int)i; }
    }
    store_list<K, true>(idx, N, i, kstore, l);   // streamed: keep L2 for the gathers
    if (bad) atomicOr(err, 1);
    cov.check_row(err, i, vi, dk);
    band.mark(t0, vi, dk);
    const Sym3 T = nvt_tensor<K>(Rows4{pos}, Rows4{nrm}, vi, k, RegNb32{l}, rho, BlkNbSafe{idx, N, i});
    const float4 n4 = nrm[i];
    float w[3], V[3][3];
    eigh3(T, w, V);
    const Vec3 f = vu_smooth(w, V, v3(n4.x, n4.y, n4.z), tau, damp);
    __builtin_nontemporal_store(v4f{f.x, f.y, f.z, 0.f}, reinterpret_cast<v4f*>(fn + i));
}

// K1: kNN + NVT1 + VU smoothing.
// SEED (iterations after the first): the largest key of last iteration's list (kstore distinct snapshot points),
// re-keyed at the current position, caps the acceptance threshold from the first candidate on, and the capped
// search (LDS append + one sorted drain) replaces per-candidate inserts.
// err bits: 1 = invalid list entry (internal error), 2 = a k-ball leaves the local snapshot's coverage box.
static constexpr int kCapRows = 48;  // LDS rows per lane: 48 KB per 256-thread block
template <int K, bool SEED>
__global__ __launch_bounds__(256) void k_knn_nvt1(GridView g, const float4* __restrict__ pos,
                                                   const float4* __restrict__ nrm, int64_t N, RowMap rm, int k,
                                                   int kstore, float rho, float tau, float damp, Cover cov,
                                                   int32_t* __restrict__ idx, float4* __restrict__ fn,
                                                   int* __restrict__ err, Band band) {
    const int64_t t0 = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (t0 >= rm.nq) return;
    const int64_t i = rm(t0);
    const float4 p4 = pos[i];
    const Vec3 vi = v3(p4.x, p4.y, p4.z);
    TopK<K> tk;
    unsigned long long cap = kInfKey;
    if constexpr (SEED) {           // max key of last iteration's list >= this iteration's kstore-th key
        // all list rows first (K loads in flight), then their points; columns >= kstore re-read column 0
        int sl[K];
        load_list<K, true>(idx, N, i, kstore, sl);
        uint32_t sd[K];
#pragma unroll
        for (int t = 0; t < K; ++t) sd[t] = (uint32_t)(t < kstore ? sl[t] : sl[0]);
        cap = 0ull;
#pragma unroll
        for (int t = 0; t < K; ++t) {
            const unsigned long long c = cand_key<false>(vi, g.pts[sd[t]], sd[t]);
            cap = c > cap ? c : cap;
        }
        cap += 1ull;                 // acceptance is `key < cap`: keep the seed list's own largest key
    }
    if constexpr (SEED && K <= 32) {
        __shared__ uint32_t s_buf[kCapRows * kCapStride];
        knn_search_capped<K, kCapRows>(g, vi, tk, cap, s_buf + threadIdx.x);
    } else if constexpr (SEED) {
        knn_search<K, false>(g, vi, tk, cap);
    } else {
        knn_search<K, false>(g, vi, tk);
    }
    int l[K];
    float dk = 0.f;                  // d² of the kstore-th neighbour (static select: no dynamic register index)
#pragma unroll
    for (int t = 0; t < K; ++t) {
        l[t] = tk.idx(t);
        if (t == kstore - 1) dk = tk.d2(t);
    }
    k1_epilogue<K>(pos, nrm, N, i, vi, l, dk, k, kstore, rho, tau, damp, cov, idx, fn, err, band, t0);
}

// ------------------------------------------------------------------ anchored kNN (seeded iterations, K <= 32)
// Every point keeps an ANCHOR: a position a it was searched at, the exact KA = 2K nearest snapshot points S of a
// (alist, blocked [KA/8][N][8], pcd_lists.h) and D = the KA-th distance there (anc[i].w; < 0: none yet).  Every snapshot point
// outside S is >= D from a, hence >= D - |q - a| from the current position q.  So when the kstore-th distance of q
// over S is below D - |q - a| (with rounding margins), the kstore nearest of q over the WHOLE snapshot are the
// kstore nearest over S, in the same (d², index) key order -- exact, with KA gathers and one sorting network
// instead of a grid search.  Points move a few % of their k-th distance per iteration, so 1-3 % of the queries per
// iteration fail the test (measured at 1M and 10M, tools/anchor_probe.py); they are appended to a redo list and
// re-anchored at q by a full grid search (k_knn_redo_nvt1).  Anchors depend only on the snapshot, so they stay
// valid across load() calls.
static constexpr float kAnchorEps = 4e-6f;   // relative slack for the fp32 distances (each is within ~2 ulp)

PCD_DEV bool anchor_holds(float d2k, Vec3 q, float4 a) {
    const float dq = sqrtf(d2k) * (1.f + kAnchorEps);
    const float delta = sqrtf(sq3(q - v3(a.x, a.y, a.z))) * (1.f + kAnchorEps);
    return a.w >= 0.f && dq + delta < a.w * (1.f - kAnchorEps);
}

// The anchor test for every active row; certified rows get their kstore-column list, the others go to the redo
// list.  (NVT1 runs afterwards over all rows, k_nvt1.)
// VALU-lean ordering: the KA candidates are ranked by 32-bit keys (fixed-point d² << 6 | list slot), so a
// compare-exchange is one min + one max instead of a 64-bit compare and four selects; the slot -> snapshot rank
// map sits in LDS (slot-major [KA][BS]: bank = lane for any slot, conflict-free).  Fixed point
// floor(d² · 2^26 / R²) with R >= every candidate's distance is monotone in d², so where the first kstore + 1
// sorted keys differ in their fixed parts the order and set are exactly those of the (d², rank) keys; any tie there
// (an exact d² tie included, which the rank would break) sends the row to the redo search instead.  The
// certificate counts candidates below the squared anchor bound, a rounding-safe restatement of anchor_holds.
// Rows that fail take the exact redo path, so the stored lists are bit-identical to the 64-bit-key ordering.
#ifndef PCD_ANCHOR_BS
#define PCD_ANCHOR_BS 128
#endif
static constexpr int kAnchorBS = PCD_ANCHOR_BS;
#ifndef PCD_ANCHOR_OCC
#define PCD_ANCHOR_OCC 1
#endif
// (measured and dropped, DESIGN.md §3 tried table: a 24-bit LDS slot map at 3 waves/SIMD, four 16-slot quarters,
// smaller gather batches, anchor sets reloaded after the first half's sort)
template <int K, int KA>
__global__ __launch_bounds__(kAnchorBS, PCD_ANCHOR_OCC) void k_knn_anchor(GridView g, const float4* __restrict__ pos, int64_t N,
                                                          RowMap rm, int kstore, const float4* __restrict__ anc,
                                                          const int32_t* __restrict__ alist,
                                                          int32_t* __restrict__ idx, uint8_t* __restrict__ fail) {
    static_assert(KA == 2 * K && KA <= 64, "anchor lists hold twice the list cap; 6 slot bits");
    __shared__ uint32_t s_r[KA * kAnchorBS];
    const int64_t t0 = xcd_block(blockIdx.x, gridDim.x) * kAnchorBS + threadIdx.x;
    bool failed = false;
    if (t0 < rm.nq) {
        const int64_t i = rm(t0);
        // every block of the anchor set issued with the row's own loads (they depend on the row only): the second
        // half's ranks are not fetched after the first half's keys, one HBM round trip off the critical path
        // (anchor test 1.306 -> 1.29 ms, 211 -> 181 VGPRs)
        v4i pre[KA / 4];
#pragma unroll
        for (int g8 = 0; g8 < KA / 8; ++g8) {
            const v4i* lp = lblock(alist, N, i, g8);
            pre[2 * g8] = __builtin_nontemporal_load(lp);
            pre[2 * g8 + 1] = __builtin_nontemporal_load(lp + 1);
        }
        const float4 p4 = pos[i];
        const Vec3 vi = v3(p4.x, p4.y, p4.z);
        const float4 a = anc[i];
        const float delta = sqrtf(sq3(vi - v3(a.x, a.y, a.z)));
        // anchor_holds(d²_k) <=> sqrt(d²_k)(1+e) + delta(1+e) < D(1-e); squared, with 1e-6 for the rounding of the square
        const float rhs = a.w * (1.f - kAnchorEps) - delta * (1.f + kAnchorEps);
        if (!(rhs > 0.f)) {
            failed = true;                            // no anchor (NaN radius) or moved too far
        } else {
            const float bnd = rhs / (1.f + kAnchorEps);
            const float T = bnd * bnd * (1.f - 1e-6f);
            // every list point is within D of the anchor, hence within D + delta of q
            const float R = (a.w + delta) * (1.f + 1e-5f);
            const float S = 67108864.f / fmaxf(R * R, 1e-30f);
            uint32_t c[KA];
            int below = 0;
            // slot t -> snapshot rank rt into the LDS map
            auto map_store = [&](int t, uint32_t rt) { s_r[t * kAnchorBS + threadIdx.x] = rt; };
            if constexpr (KA == 64) {
            // two halves of 32 slots: the second half's gathers are in flight while the first half's keys sort; the
            // sorted halves merge by a half-cleaner (its low side: the 32 smallest, bitonic; its high side's minimum:
            // the 33rd) and a 32-wide bitonic merge -- the same first kstore + 1 keys as the 64-key network
            // (anchor test 1.29 -> 1.26 ms)
            uint32_t ca[32], cb[32];
            auto half = [&](int h, uint32_t (&cc)[32], auto&& between) {
                uint32_t r[32];
#pragma unroll
                for (int g8 = 0; g8 < 4; ++g8) {
                    const v4i x = pre[2 * (4 * h + g8)], y = pre[2 * (4 * h + g8) + 1];
                    r[8 * g8 + 0] = (uint32_t)x.x; r[8 * g8 + 1] = (uint32_t)x.y; r[8 * g8 + 2] = (uint32_t)x.z;
                    r[8 * g8 + 3] = (uint32_t)x.w; r[8 * g8 + 4] = (uint32_t)y.x; r[8 * g8 + 5] = (uint32_t)y.y;
                    r[8 * g8 + 6] = (uint32_t)y.z; r[8 * g8 + 7] = (uint32_t)y.w;
                }
                float4 pj[32];
#pragma unroll
                for (int u = 0; u < 32; ++u) {
                    const uint32_t rt = min(r[u], (uint32_t)N);
                    map_store(32 * h + u, rt);
                    pj[u] = *at32(g.pts, rt);
                }
                between();
#pragma unroll
                for (int u = 0; u < 32; ++u) {
                    const float d2 = dist2(vi, pj[u]);
                    below += d2 < T ? 1 : 0;
                    cc[u] = ((uint32_t)fminf(d2 * S, 67108860.f) << 6) | (uint32_t)(32 * h + u);
                }
            };
            half(0, ca, [] {});
            half(1, cb, [&] { oddeven_sort<32>(ca); });
            oddeven_sort<32>(cb);
            uint32_t c33 = 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < 32; ++u) {
                const uint32_t lo = min(ca[u], cb[31 - u]), hi = max(ca[u], cb[31 - u]);
                ca[u] = lo;
                c33 = min(c33, hi);
            }
#pragma unroll
            for (int d = 16; d > 0; d >>= 1)
#pragma unroll
                for (int u = 0; u < 32; ++u)
                    if ((u & d) == 0) cswap(ca[u], ca[u + d]);
#pragma unroll
            for (int u = 0; u < 32; ++u) c[u] = ca[u];
            c[32] = c33;
            } else {
            // K <= 16: every gather of the set in flight at once, then one KA-key network
            uint32_t r[KA];
#pragma unroll
            for (int g8 = 0; g8 < KA / 8; ++g8) {
                const v4i* lp = lblock(alist, N, i, g8);
                const v4i x = __builtin_nontemporal_load(lp), y = __builtin_nontemporal_load(lp + 1);
                r[8 * g8 + 0] = (uint32_t)x.x; r[8 * g8 + 1] = (uint32_t)x.y; r[8 * g8 + 2] = (uint32_t)x.z;
                r[8 * g8 + 3] = (uint32_t)x.w; r[8 * g8 + 4] = (uint32_t)y.x; r[8 * g8 + 5] = (uint32_t)y.y;
                r[8 * g8 + 6] = (uint32_t)y.z; r[8 * g8 + 7] = (uint32_t)y.w;
            }
#pragma unroll
            for (int t = 0; t < KA; ++t) {
                // an unused slot of a partial anchor set holds N: the snapshot's +inf sentinel row (the min keeps
                // any entry inside the allocation)
                const uint32_t rt = min(r[t], (uint32_t)N);
                map_store(t, rt);
                const float d2 = dist2(vi, *at32(g.pts, rt));   // unconditional load: every gather in flight
                below += d2 < T ? 1 : 0;
                // clamp below 2^26 in fp32 (2^26 - 1 rounds UP to 2^26, which would wrap to 0 after the shift);
                // only the sentinel's infinite distance reaches it
                c[t] = ((uint32_t)fminf(d2 * S, 67108860.f) << 6) | (uint32_t)t;
            }
            oddeven_sort<KA>(c);
            }
            bool ok = below >= kstore;
#pragma unroll
            for (int t = 0; t < K; ++t)
                if (t < kstore) ok = ok && (c[t] >> 6) < (c[t + 1] >> 6);
            failed = !ok;
            if (ok) {
                int out[K];
#pragma unroll
                for (int t = 0; t < K; ++t) out[t] = (int32_t)s_r[(c[t] & 63u) * kAnchorBS + threadIdx.x];
                store_list<K, true>(idx, N, i, kstore, out);
            }
        }
    }
    if (t0 < rm.nq) fail[t0] = failed ? 1 : 0;   // -> the redo list (k_compact_fail)
}

// The anchor test's failed rows -> the redo list: each block takes 4,096 consecutive flags (16 per thread, one 16-B
// load), writes its failed rows in row order at a base it takes with ONE atomic -- blocks start roughly in order, so
// the list stays spatially coherent for the re-anchoring waves (what rocprim::select's strict order bought, at a
// tenth of its time: 10 MB of flags).
static constexpr int kCompactBS = 256, kCompactPer = 16;
__global__ __launch_bounds__(kCompactBS) void k_compact_fail(const uint8_t* __restrict__ fail, RowMap rm,
                                                             int32_t* __restrict__ list, unsigned* __restrict__ cnt) {
    __shared__ uint32_t s_w[kCompactBS / 64];
    __shared__ uint32_t s_base;
    const int64_t f0 = ((int64_t)blockIdx.x * kCompactBS + threadIdx.x) * kCompactPer;
    uint32_t bits = 0;
    if (f0 + kCompactPer <= rm.nq) {
        const uint4 v = *reinterpret_cast<const uint4*>(fail + f0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int b = 0; b < 4; ++b) bits |= ((w[q] >> (8 * b)) & 0xFFu) ? 1u << (4 * q + b) : 0u;
    } else {
        for (int k = 0; k < kCompactPer; ++k)
            if (f0 + k < rm.nq && fail[f0 + k]) bits |= 1u << k;
    }
    const uint32_t n = (uint32_t)__popc(bits);
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const uint32_t incl = lane_scan_incl<64>(n);
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kCompactBS / 64; ++w) { before += w < wv ? s_w[w] : 0u; total += s_w[w]; }
    if (threadIdx.x == 0) s_base = total ? atomicAdd(cnt, total) : 0u;
    __syncthreads();
    uint32_t o = s_base + before + incl - n;
    while (bits) {
        const int k = __ffs(bits) - 1;
        bits &= bits - 1;
        list[o++] = (int32_t)rm(f0 + k);
    }
}

// NVT1 + eigh + VU smoothing over the stored lists (lane per row); checks every list entry and, for spatial slabs,
// that the kstore-ball stays inside the local snapshot.
template <int K, bool UNIT, class P, class Nr>
__device__ __forceinline__ void nvt1_row(const GridView& g, const float4* __restrict__ pos, const float4* __restrict__ nrm,
                      const int32_t* __restrict__ idx, int64_t N, int64_t i, int k, int kstore, float rho, float tau,
                      float damp, const Cover& cov, float4* __restrict__ fn, int* __restrict__ err, P rp, Nr rn,
                      const Band& band = Band{Cover{{1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, nullptr}, int64_t t0 = 0) {
    const float4 p4 = pos[i];
    const Vec3 vi = v3(p4.x, p4.y, p4.z);
    int l[K];
    bool bad = false;
    load_list<K>(idx, N, i, kstore, l);
#pragma unroll
    for (int t = 0; t < K; ++t) {
        l[t] = t < kstore ? l[t] : (int)i;
        if ((uint32_t)l[t] >= (uint32_t)N) { bad = true; l[t] = (int)i; }
    }
    if (bad) atomicOr(err, 1);
    if (cov.enabled() || band.flag) {
        float dk = 0.f;
#pragma unroll
        for (int t = 0; t < K; ++t)
            if (t == kstore - 1) dk = dist2(vi, g.pts[l[t]]);
        cov.check_row(err, i, vi, dk);
        band.mark(t0, vi, dk);
    }
    // 4 neighbours in flight per batch (8 measured 0.06 ms slower at 10M: the VGPRs of 8 rows in flight)
    const Sym3 T = nvt_tensor<K, true, UNIT, 4>(rp, rn, vi, k, RegNb32{l}, rho, BlkNbSafe{idx, N, i});
    float w[3], V[3][3];
    eigh3(T, w, V);
    const float4 n4 = nrm[i];
    const Vec3 f = vu_smooth(w, V, v3(n4.x, n4.y, n4.z), tau, damp);
    __builtin_nontemporal_store(v4f{f.x, f.y, f.z, 0.f}, reinterpret_cast<v4f*>(fn + i));
}

// Every active row, its neighbours read through the block's LDS row window (without it: 1.38 ms instead of 1.01).
// UNIT: the normals are the loop's own normalised f_n (every iteration after the first since load): the vote's
// margin is a constant (nvt_tensor).
#ifndef PCD_NVT1_OCC
#define PCD_NVT1_OCC 1
#endif
template <int K, bool UNIT>
__global__ __launch_bounds__(kNvtBS, PCD_NVT1_OCC) void k_nvt1(GridView g, const float4* __restrict__ pos, const float4* __restrict__ nrm,
                                               const int32_t* __restrict__ idx, int64_t N, RowMap rm, int k,
                                               int kstore, float rho, float tau, float damp, Cover cov,
                                               float4* __restrict__ fn, int* __restrict__ err, int win, Band band,
                                               RowSel sel) {
    __shared__ float4 s_pos[kWinRows], s_nrm[kWinRows];
    const int64_t b0 = xcd_block(blockIdx.x, gridDim.x) * blockDim.x;
    const int64_t lo = stage_window(pos, nrm, N, rm(b0), s_pos, s_nrm, win);
    const int64_t t0 = b0 + threadIdx.x;
    if (t0 >= rm.nq || !sel.take(t0)) return;
    nvt1_row<K, UNIT>(g, pos, nrm, idx, N, rm(t0), k, kstore, rho, tau, damp, cov, fn, err, WinRows<>{pos, s_pos, lo},
                WinRows<>{nrm, s_nrm, lo}, band, t0);
}

// Re-anchor: the exact KA nearest at the current position, one query per WAVE (pcd_wknn.h), capped by the old
// anchor list re-keyed here when there is one (KA distinct points: its largest key bounds the new KA-th key).
// Writes the anchor, its list and the kstore-column kNN list.
// DENSE: every active row (no anchors yet); else the rows on the redo list.  Grid-stride over waves.
#ifndef PCD_REDO_OCC
#define PCD_REDO_OCC 4
#endif
#ifndef PCD_REDO_GRID
#define PCD_REDO_GRID 2048
#endif
template <int KA, bool DENSE>
__global__ __launch_bounds__(256, PCD_REDO_OCC) void k_knn_redo_wave(GridView g, const float4* __restrict__ pos, int64_t N, RowMap rm,
                                                        int kstore, float4* __restrict__ anc,
                                                        int32_t* __restrict__ alist, int32_t* __restrict__ idx,
                                                        const int32_t* __restrict__ redo,
                                                        const unsigned* __restrict__ redo_cnt, int* __restrict__ err) {
    __shared__ unsigned long long s_buf[4][kWaveSurv];
    __shared__ WaveCells s_cells[4];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const int64_t cnt = DENSE ? rm.nq : (int64_t)*redo_cnt;
    // consecutive redo rows (spatial neighbours) -> consecutive logical blocks -> the same XCD's L2
    const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
    for (int64_t t0 = lb * 4 + wv; t0 < cnt; t0 += (int64_t)gridDim.x * 4) {
        const int64_t i = DENSE ? rm(t0) : (int64_t)redo[t0];
        const float4 p4 = pos[i];
        const Vec3 q = v3(p4.x, p4.y, p4.z);
        unsigned long long cap = kInfKey;
        if (!DENSE) {
            const float4 a = anc[i];
            // (D + |q - a|)² bounds the KA-th key at q only for a FULL anchor set (KA points within D of a); a partial
            // set (fewer points within its radius, unused slots = N, the +inf sentinel row) gives no such bound
            if (a.w >= 0.f && (uint32_t)alist[lpos(N, i, KA - 1)] < (uint32_t)N) cap = anchor_cap(q, a);
        }
        const unsigned long long top = wave_knn<KA>(g, q, cap, s_buf[wv], &s_cells[wv], lane);
        // a slot without a finite candidate (non-finite query, fewer than KA points) is never stored as an index:
        // the row itself stands in, the error word reports it, and the anchor is dropped (NaN radius)
        const uint32_t r32 = (uint32_t)(top & 0xFFFFFFFFull);
        const bool valid = (uint32_t)(top >> 32) < 0x7F800000u && r32 < (uint64_t)N;
        const int32_t r = valid ? (int32_t)r32 : (int32_t)i;
        const bool all_valid = !__any(lane < KA && !valid);
        if (!all_valid && lane == 0) atomicOr(err, 1);
        if (lane < kstore) idx[lpos(N, i, lane)] = r;   // (whole 32-B sectors, pcd_lists.h)
        {   // the anchor set in rank order (a consistent order for the anchor test's gathers, like the re-anchoring
            // search's scan order, rq_finish), unused slots last
            uint32_t v[1] = {lane < KA ? (uint32_t)r : 0xFFFFFFFFu};
            grp_bitonic_sort32<64, 1>(v, lane);
            if (lane < KA) alist[lpos(N, i, lane)] = (int32_t)v[0];
        }
        // D: the KA-th distance (every other snapshot point is at least this far from the anchor)
        if (lane == KA - 1)
            anc[i] = make_float4(q.x, q.y, q.z, all_valid ? sqrtf(__uint_as_float((unsigned)(top >> 32))) : __int_as_float(0x7FC00000));
    }
}

// K2: NVT2 on f_n -> classes + edge vectors.
#ifndef PCD_NVT2_OCC
#define PCD_NVT2_OCC 1
#endif
template <int K>
__global__ __launch_bounds__(kNvtBS, PCD_NVT2_OCC) void k_nvt2(const float4* __restrict__ pos, const float4* __restrict__ fn,
                                               const int32_t* __restrict__ idx, int64_t N, RowMap rm, int k,
                                               float rho, float scale, uint8_t* __restrict__ cls,
                                               float4* __restrict__ edge, int win, float4* __restrict__ probe,
                                               RowSel sel) {
    __shared__ float4 s_pos[WinSize<kWinHaloNvt2, kNvtBS>::rows], s_fn[WinSize<kWinHaloNvt2, kNvtBS>::rows];
    const int64_t b0 = xcd_block(blockIdx.x, gridDim.x) * blockDim.x;
    const int64_t t0 = b0 + threadIdx.x;
    const bool mine = t0 < rm.nq && sel.take(t0);
    if (sel.flag && !__syncthreads_or(mine)) return;     // (block-uniform: a pass skips the blocks it has no row in)
    const int64_t lo = stage_window<kWinHaloNvt2, kNvtBS>(pos, fn, N, rm(b0), s_pos, s_fn, win);
    if (!mine) return;
    const int64_t i = rm(t0);
    const float4 p4 = pos[i];
    // classes and the edge vector are invariant to the positive scale 1/Σw (ratios of eigenvalues, a unit
    // eigenvector): the tensor is left unnormalised.  f_n is NVT1's normalised output: the vote margin is constant.
    int wsum = 0;
    int l[K];
    load_list<K, true>(idx, N, i, k, l);   // read once: streamed past L2 so the neighbour gathers keep it
    const Sym3 T = nvt_tensor<K, false, true>(WinRows<kWinHaloNvt2, kNvtBS>{pos, s_pos, lo}, WinRows<kWinHaloNvt2, kNvtBS>{fn, s_fn, lo},
                                                v3(p4.x, p4.y, p4.z), k, RegNb32{l}, rho, BlkNbSafe{idx, N, i},
                                                &wsum);   // (unconditional: a selected pointer would keep wsum in scratch)
    float w[3];
    Vec3 y;
    eigh3_min(T, w, y);
    cls[i] = (uint8_t)classify(w, scale, nullptr);
    store4(edge, i, y);
    // parity probe (pcd_denoiser_set_probe): the eigenvalues of the reference's normalised tensor T / Σw
    // (Decompositionor.py:299-300) as this kernel computes them, and Σw
    if (probe) {
        const float c = (float)wsum;
        probe[i] = make_float4(w[0] / c, w[1] / c, w[2] / c, (float)wsum);
    }
}

// One flat-reduction block's partial: f64 sums and count of its rows, the box of those rows (for the pruned max
// distance pass), and whether that pass must scan the block (set by k_centre).
struct RedC { double sx, sy, sz, cnt; float lo[3], hi[3]; int scan, pad; };

// The k_u neighbour rows of point i, all loads in flight together (KU = compile-time bound on ku).
template <int KU>
PCD_DEV void gather_rows(const float4* __restrict__ pos, const int32_t* __restrict__ idx, int64_t N, int64_t i, int ku,
                         float4 (&v)[KU]) {
    int j[KU];
    load_list_clamped<KU>(idx, N, i, ku, j);   // (block 0: two 16-B loads per lane)
#pragma unroll
    for (int u = 0; u < KU; ++u) v[u] = pos[j[u]];
}

// Flat-phase centre, pass 1: per-block f64 partial sums of the k_u neighbour rows of the class-c points.
// Each thread walks rows t, t+G, t+2G, ... (G = grid threads) kRowsInFlight at a time: all their list and point loads
// are issued together, then accumulated in the same row order as a one-row loop (bit-identical sums).
#ifndef PCD_ROWS_IN_FLIGHT
#define PCD_ROWS_IN_FLIGHT 2
#endif
static constexpr int kRowsInFlight = PCD_ROWS_IN_FLIGHT;
template <int KU>
PCD_DEV void gather_rows_batch(const float4* __restrict__ pos, const int32_t* __restrict__ idx, int64_t N, RowMap rm,
                               const uint8_t* __restrict__ cls, int c, int ku, int64_t t, int64_t G, int64_t end,
                               bool (&on)[kRowsInFlight], float4 (&v)[kRowsInFlight][KU]) {
    int64_t ii[kRowsInFlight];
#pragma unroll
    for (int r = 0; r < kRowsInFlight; ++r) {
        const int64_t tt = t + r * G;
        ii[r] = tt < end ? rm(tt) : 0;
        on[r] = tt < end;
    }
#pragma unroll
    for (int r = 0; r < kRowsInFlight; ++r) on[r] = on[r] && cls[ii[r]] == c;
#pragma unroll
    for (int r = 0; r < kRowsInFlight; ++r) gather_rows<KU>(pos, idx, N, on[r] ? ii[r] : 0, ku, v[r]);
}

// Block b of the flat reductions owns the CONTIGUOUS active rows [b R, (b + 1) R), R = ceil(nq / blocks): rows are
// in spatial order, so the box of a block's rows is small and the max-distance pass can skip the blocks whose box
// provably holds no farther row than another block's nearest bound (k_centre).
PCD_DEV void part_range(int64_t nq, int64_t& beg, int64_t& end) {
    const int64_t R = (nq + gridDim.x - 1) / gridDim.x;
    beg = (int64_t)blockIdx.x * R;
    end = beg + R < nq ? beg + R : nq;
}

template <int KU>
__global__ __launch_bounds__(256) void k_class_rows_sum(const float4* __restrict__ pos, const int32_t* __restrict__ idx, int64_t N, RowMap rm,
                                 int ku, const uint8_t* __restrict__ cls, int c, RedC* __restrict__ part) {
    double sx = 0, sy = 0, sz = 0, cnt = 0;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int64_t beg, end;
    part_range(rm.nq, beg, end);
    for (int64_t t = beg + threadIdx.x; t < end; t += kRowsInFlight * 256) {
        bool on[kRowsInFlight];
        float4 v[kRowsInFlight][KU];
        gather_rows_batch<KU>(pos, idx, N, rm, cls, c, ku, t, 256, end, on, v);
#pragma unroll
        for (int r = 0; r < kRowsInFlight; ++r) {
            if (!on[r]) continue;
#pragma unroll
            for (int u = 0; u < KU; ++u)
                if (u < ku) {
                    sx += v[r][u].x; sy += v[r][u].y; sz += v[r][u].z;
                    lo[0] = fminf(lo[0], v[r][u].x); lo[1] = fminf(lo[1], v[r][u].y); lo[2] = fminf(lo[2], v[r][u].z);
                    hi[0] = fmaxf(hi[0], v[r][u].x); hi[1] = fmaxf(hi[1], v[r][u].y); hi[2] = fmaxf(hi[2], v[r][u].z);
                }
            cnt += ku;
        }
    }
    __shared__ double s[4][256];
    __shared__ float sb[6][256];
    s[0][threadIdx.x] = sx; s[1][threadIdx.x] = sy; s[2][threadIdx.x] = sz; s[3][threadIdx.x] = cnt;
    for (int a = 0; a < 3; ++a) { sb[a][threadIdx.x] = lo[a]; sb[3 + a][threadIdx.x] = hi[a]; }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            for (int a = 0; a < 4; ++a) s[a][threadIdx.x] += s[a][threadIdx.x + w];
            for (int a = 0; a < 3; ++a) {
                sb[a][threadIdx.x] = fminf(sb[a][threadIdx.x], sb[a][threadIdx.x + w]);
                sb[3 + a][threadIdx.x] = fmaxf(sb[3 + a][threadIdx.x], sb[3 + a][threadIdx.x + w]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        part[blockIdx.x] = RedC{s[0][0], s[1][0], s[2][0], s[3][0], {sb[0][0], sb[1][0], sb[2][0]},
                                {sb[3][0], sb[4][0], sb[5][0]}, 1, 0};
}

// pass 2: the partials -> (Σx, Σy, Σz, count) in f64 (what a multi-rank caller all-reduces).
__global__ void k_part_reduce(const RedC* __restrict__ part, int np, double* __restrict__ red) {
    __shared__ double s[4][256];
    double a[4] = {0, 0, 0, 0};
    for (int b = threadIdx.x; b < np; b += blockDim.x) { a[0] += part[b].sx; a[1] += part[b].sy; a[2] += part[b].sz; a[3] += part[b].cnt; }
    for (int q = 0; q < 4; ++q) s[q][threadIdx.x] = a[q];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) for (int q = 0; q < 4; ++q) red[q] = s[q][0];
}

// pass 3: centre = Σ / count (the reference's f32 mean over all E rows, Denoiser.py:106), delta reset, and the blocks
// pass 4 must scan: with d_b = max over axes of the farther of |hi_a - c_a|, |c_a - lo_a| (a row attains each face
// of the box, so some row of block b lies at least d_b from the centre) and U_b = the distance to the farthest box
// corner (no row of b lies farther), every block with U_b below max_b d_b is skipped: it cannot hold the maximum.
// Bounds in f64 with a relative margin far above the fp32 rounding of pass 4's squared distances.
__global__ void k_centre(const double* __restrict__ red, float* __restrict__ g, RedC* __restrict__ part, int np) {
    __shared__ float s_c[3];
    __shared__ double s_lb[256];
    if (threadIdx.x == 0) {
        const double c = red[3];
        g[0] = (float)(red[0] / c);
        g[1] = (float)(red[1] / c);
        g[2] = (float)(red[2] / c);
        reinterpret_cast<unsigned int*>(g)[3] = 0u;
        s_c[0] = g[0]; s_c[1] = g[1]; s_c[2] = g[2];
    }
    __syncthreads();
    if (!part) return;
    auto bounds = [&](const RedC& p, double& lb2, double& ub2) {
        lb2 = 0.0; ub2 = 0.0;
        for (int a = 0; a < 3; ++a) {
            const double f = fmax((double)p.hi[a] - (double)s_c[a], (double)s_c[a] - (double)p.lo[a]);
            lb2 = fmax(lb2, f * f);
            ub2 += f * f;
        }
    };
    double lb = 0.0;
    for (int b = threadIdx.x; b < np; b += blockDim.x) {
        if (!(part[b].cnt > 0)) continue;
        double l, u;
        bounds(part[b], l, u);
        lb = fmax(lb, l);
    }
    s_lb[threadIdx.x] = lb;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s_lb[threadIdx.x] = fmax(s_lb[threadIdx.x], s_lb[threadIdx.x + w]);
        __syncthreads();
    }
    const double LB = s_lb[0] * (1.0 - 1e-4);
    for (int b = threadIdx.x; b < np; b += blockDim.x) {
        double l, u;
        bounds(part[b], l, u);
        part[b].scan = part[b].cnt > 0 && !(u * (1.0 + 1e-4) < LB) ? 1 : 0;
    }
}

// pass 4: delta = max ||v_j - centre|| over the same rows (Denoiser.py:107), atomicMax on the f32 bits.  The max is
// taken over d² and rooted once (sqrt is monotone); rows kRowsInFlight at a time as in pass 1, only in the blocks
// k_centre left to scan.
template <int KU>
__global__ __launch_bounds__(256) void k_class_rows_maxdist(const float4* __restrict__ pos, const int32_t* __restrict__ idx, int64_t N,
                                     RowMap rm, int ku, const uint8_t* __restrict__ cls, int c, float* __restrict__ g,
                                     const RedC* __restrict__ part) {
    if (part && !part[blockIdx.x].scan) return;       // (block-uniform)
    const Vec3 ctr = v3(g[0], g[1], g[2]);
    float mx2 = 0.f;
    int64_t beg, end;
    part_range(rm.nq, beg, end);
    for (int64_t t = beg + threadIdx.x; t < end; t += kRowsInFlight * 256) {
        bool on[kRowsInFlight];
        float4 v[kRowsInFlight][KU];
        gather_rows_batch<KU>(pos, idx, N, rm, cls, c, ku, t, 256, end, on, v);
#pragma unroll
        for (int r = 0; r < kRowsInFlight; ++r) {
            if (!on[r]) continue;
#pragma unroll
            for (int u = 0; u < KU; ++u)
                if (u < ku) mx2 = fmaxf(mx2, nsq3(v3(v[r][u].x, v[r][u].y, v[r][u].z) - ctr));
        }
    }
    float mx = sqrtf(mx2);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(g) + 3, __float_as_uint(mx));
}

__global__ void k_copy_delta(const float* __restrict__ from, float* __restrict__ to) {
    if (threadIdx.x == 0) *to = *from;
}

// K3: one Gauss-Seidel phase: active points of class c move (reading pin), other active points copy through.
// SPLIT (the fused loop's three Gauss-Seidel phases over every row, one class each): no phase copies the rows it
// does not move.  Every phase reads pin and writes its own class's rows to pout, so after phase ph a row's current
// position is in pout if its class was moved by an earlier phase (bit cls of `moved`) and in pin otherwise; after the
// last phase every row is in pout.  Same arithmetic on the same inputs as the copying phases (the parity tests
// compare the two paths bitwise: test_gpu_slab's world-1 slab runs the copying stages).
struct SplitRows {
    const float4* a;             // positions before this iteration's phases
    const float4* b;             // rows moved by the earlier phases of this iteration
    const uint8_t* cls;
    uint32_t moved;
    PCD_DEV Vec3 operator()(int64_t j) const {
        const float4 q = ((moved >> cls[j]) & 1u) ? b[j] : a[j];
        return v3(q.x, q.y, q.z);
    }
};

#ifndef PCD_PHASE_OCC
#define PCD_PHASE_OCC 1
#endif
template <int KIND, int KU>
__global__ __launch_bounds__(256, PCD_PHASE_OCC) void k_phase(const float4* __restrict__ pin, float4* __restrict__ pout,
                                                const float4* __restrict__ fn, const float4* __restrict__ edge,
                                                const int32_t* __restrict__ idx, int64_t N, RowMap rm, int ku,
                                                const uint8_t* __restrict__ cls, int c, const float* __restrict__ g,
                                                float d, float alpha, int win, int copy_others,
                                                const float4* __restrict__ orig, float clampg, uint32_t moved,
                                                RowSel sel) {
    // the flat phase moves most rows: its neighbour rows come from an LDS window of pin / fn around the block
    constexpr bool WIN = KIND == PCD_STEP_FLAT;
    __shared__ float4 s_pos[WIN ? WinSize<kWinHaloPhase, 256>::rows : 1], s_fn[WIN ? WinSize<kWinHaloPhase, 256>::rows : 1];
    const int64_t b0 = xcd_block(blockIdx.x, gridDim.x) * blockDim.x;
    const int64_t t0 = b0 + threadIdx.x;
    const bool mine = t0 < rm.nq && sel.take(t0);
    if (sel.flag && !__syncthreads_or(mine)) return;     // (block-uniform)
    int64_t lo = 0;
    if constexpr (WIN) lo = stage_window<kWinHaloPhase, 256>(pin, fn, N, rm(b0 < rm.nq ? b0 : rm.nq - 1), s_pos, s_fn, win);
    if (!mine) return;
    const int64_t i = rm(t0);
    if (cls[i] != c) {                  // Gauss-Seidel: every phase copies the others; Jacobi / SPLIT: only the first
        if (copy_others) pout[i] = pin[i];
        return;
    }
    const float4 p4 = pin[i];
    const Vec3 vi = v3(p4.x, p4.y, p4.z);
    const Rows4 P{pin}, F{fn};
    const SplitRows PS{pin, pout, cls, moved};
    // the update list: block 0 (pcd_lists.h), 16-B loads (8-B in the windowed flat phase: load_list_clamped8)
    RegNbC<KU> nb;
    if constexpr (WIN) load_list_clamped8<KU>(idx, N, i, ku, nb.l);
    else load_list_clamped<KU>(idx, N, i, ku, nb.l);
    Vec3 o;
    if constexpr (WIN)
        o = step_flat<KU>(WinRows<kWinHaloPhase, 256>{pin, s_pos, lo}, WinRows<kWinHaloPhase, 256>{fn, s_fn, lo}, vi, F(i), ku,
                          nb, __uint_as_float(((const unsigned*)g)[3]), d, alpha);
    else if (KIND == PCD_STEP_FLAT) o = step_flat<KU>(P, F, vi, F(i), ku, nb, __uint_as_float(((const unsigned*)g)[3]), d, alpha);
    else if (moved && KIND == PCD_STEP_EDGE) o = step_edge<KU, 4>(PS, F, vi, Rows4{edge}(i), ku, nb, d, alpha);
    else if (moved && KIND == PCD_STEP_FEATURE) o = step_feature<false, KU, 4>(PS, F, vi, F(i), ku, nb, 1.f, d, alpha);
    else if (moved && KIND == PCD_STEP_CORNER) o = step_corner<KU, 4>(PS, F, vi, ku, nb, d, alpha);
    else if (KIND == PCD_STEP_EDGE) o = step_edge<KU, 4>(P, F, vi, Rows4{edge}(i), ku, nb, d, alpha);
    else if (KIND == PCD_STEP_FEATURE) o = step_feature<false, KU, 4>(P, F, vi, F(i), ku, nb, 1.f, d, alpha);
    else if (KIND == PCD_STEP_NEW) o = step_feature<true, KU>(P, F, vi, F(i), ku, nb, __uint_as_float(((const unsigned*)g)[3]), d, alpha);
    else if (KIND == PCD_STEP_CORNER) o = step_corner<KU, 4>(P, F, vi, ku, nb, d, alpha);
    else o = vi;
    if (clampg > 0.f) {                 // global clamp against the loaded positions (PostProcessing.ipynb:1088-1089)
        const float4 o4 = orig[i];
        const bool keep = norm3(o - v3(o4.x, o4.y, o4.z)) < clampg;
        o = sel3(keep, o, vi);
    }
    store4(pout, i, o);
}

// sorted-order float4 rows -> caller order (the probe)
__global__ void k_scatter4(const float4* __restrict__ src, const int32_t* __restrict__ perm, int64_t N,
                           float4* __restrict__ out) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r < N) out[perm[r]] = src[r];
}

// pcd_denoiser_lists: blocked sorted-order lists -> caller rows of original indices
__global__ void k_lists(const int32_t* __restrict__ idx, const int32_t* __restrict__ perm, int64_t N, int cols,
                        int64_t* __restrict__ out) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= N) return;
    const int64_t i = perm[r];
    for (int t = 0; t < cols; ++t) {
        const int32_t j = idx[lpos(N, r, t)];
        out[i * cols + t] = (uint32_t)j < (uint64_t)N ? (int64_t)perm[j] : -1;
    }
}

// One exchanged field of the spatial slabs (pcd_slab.h): pack reads row r from b if its class was moved by an
// earlier phase of this iteration (the copy-free phases' two buffers), else from a; unpack writes the received row to
// da and (non-null) db.
struct XField {
    const float4* a;
    const float4* b;
    const uint8_t* cls;
    uint32_t moved;
    float4* da;
    float4* db;
};

// halo exchange: rows of one state field <-> a packed float4 buffer
__global__ void k_pack(const float4* __restrict__ f, const int32_t* __restrict__ rows, int64_t n, float4* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < n) out[t] = f[rows[t]];
}
__global__ void k_unpack(float4* __restrict__ f, const int32_t* __restrict__ rows, int64_t n, const float4* __restrict__ in) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < n) f[rows[t]] = in[t];
}

}  // namespace pcd

using namespace pcd;

struct pcd_denoiser {
    const pcd_grid* g = nullptr;
    int64_t n = 0;
    int kcap = 0;                 // columns of the stored kNN list
    float4 *pos[2] = {nullptr, nullptr}, *nrm = nullptr, *fn = nullptr, *edge = nullptr;
    float4* orig = nullptr;       // positions at load(): the global clamp's reference (pcd_denoise_params)
    float* xrad = nullptr;        // spatial slabs: per-row coverage sphere radius (Cover::xr), null: none
    int cur = 0;                  // pos[cur] holds the current positions
    int32_t* idx = nullptr;
    uint8_t* cls = nullptr;
    RedC* part = nullptr;
    int part_ph = -1;             // phase whose rows the flat-reduction partials (boxes) describe, -1: none
    int scan_ph = -1;             // phase whose max-distance block flags k_centre set, -1: none
    double* red = nullptr;        // 4 doubles per phase: (Σx, Σy, Σz, count) of the global reductions
    float* gscal = nullptr;       // 4 floats per phase: centre xyz, delta bits
    int* err = nullptr;           // device error word (see k_knn_nvt1), checked by store() / check()
    const int32_t* rows = nullptr;  // active rows (sorted order), or null = all rows
    int64_t n_rows = 0;
    Cover cov{{1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};  // disabled
    int seed_cols = 0;            // columns of idx holding a valid kNN list of the snapshot (0: none yet)
    int list_cols = 0;            // columns the last K1 stage stored (pcd_denoiser_lists)
    bool seeding = true;          // use the stored list as an acceptance cap (pcd_denoiser_set_seeding)
    // anchored kNN (list cap <= 32): anchors + their 2K-lists, the redo list of queries that failed the test
    float4* anc = nullptr;
    int32_t* alist = nullptr;
    int32_t* redo = nullptr;      // rows that failed the anchor test (redo list)
    int32_t* spill = nullptr;     // rows the re-anchoring search hands to the exact-key wave search
    RqStats* rqs = nullptr;       // lengths of the redo and spill lists (pcd_qknn.h)
    uint8_t* fail = nullptr;      // per active row: anchor test failed
    int anchor_ka = 0;            // KA of the stored anchors (0: none)
    int64_t last_dense = -1;      // rows of the last anchored stage when it re-anchored every row, else -1
    bool anchoring = true;        // anchored kNN for seeded searches (pcd_denoiser_set_anchoring)
    bool unit_nrm = false;        // nrm holds the loop's own normalised f_n (set by finish, cleared by load / writes)
    int windows = 1;              // LDS row windows in NVT1 / NVT2 / the flat phase (pcd_denoiser_set_windows)
    float4* probe = nullptr;      // NVT2 parity probe (pcd_denoiser_set_probe): normalised eigenvalues + Σw per row
    bool loaded = false, iterated = false;
    bool timing = false;
    bool timing_k1 = false;       // level 2: only the K1 stage's two events (the bench's timed region)
    std::vector<hipEvent_t> ev;   // kTimingSets sets of kTimingEvents events, one set per timed iteration
    int ev_used = 0;              // sets recorded since set_timing / the last get_timing
    // spatial slabs (pcd_slab.h): halo routes, band flags, the exchange stream and the exchange in flight
    int npeers = 0;
    std::vector<int> peers;
    std::vector<int64_t> soff{0}, roff{0};   // per-peer offsets into the send / receive row lists
    int32_t *srows = nullptr, *rrows = nullptr;
    float4 *sbuf = nullptr, *rbuf = nullptr;  // device staging of the packed rows
    float4 *hs = nullptr, *hr = nullptr;      // pinned host staging (host transport)
    uint8_t* bflag = nullptr;     // per active row: its k-ball leaves the owned slab (it may read a halo row)
    Cover own{{1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    hipStream_t xst = nullptr;    // exchange stream
    hipEvent_t xev_in = nullptr, xev_out = nullptr;
    bool xpending = false;        // xev_out marks an exchange the state's next reader must wait for
    bool xbegun = false;          // host transport: packed, callback not yet run
    XField xfield{};
    // read-set exchange (pcd_slab.h): each iteration moves only the halo rows some own row's list reads
    bool readset = true;          // on by default (PCD_SLAB_READSET=0: every halo row, every exchange)
    bool use_sel = false;         // the exchanges of this iteration use the selected routes
    int32_t* rpos = nullptr;      // local row -> its index in rrows, -1: not a halo row
    uint8_t* rmark = nullptr;     // per receive-route row: read by some own row's list
    uint32_t *rwords = nullptr, *swords = nullptr, *wpopc = nullptr, *wscan = nullptr;
    int32_t *sel_srows = nullptr, *sel_rrows = nullptr;
    int64_t* xoff_d = nullptr;    // device: roff, soff, rwoff, swoff (npeers + 1 each)
    int64_t* seloff_d = nullptr;  // device: selected receive / send offsets (npeers + 1 each)
    int64_t* seloff_h = nullptr;  // pinned host copy
    std::vector<int64_t> rwoff{0}, swoff{0}, sel_soff{0}, sel_roff{0};
    hipEvent_t rs_ev = nullptr;
    int64_t rs_iters = 0, rs_send_rows = 0, rs_recv_rows = 0;   // read-set iterations and their summed row counts
    // CPSD driver (pcd_cpsd.h): radius member rows, member counts, overflow flag
    bool nvt1_on = true;          // K1 runs NVT1 after the kNN (off: the lists only)
    int32_t* ckeys = nullptr;                            // [cpsd_cap][nq] member rows (slot-major), ascending original index
    int32_t* ccnt = nullptr;
    int32_t* cinv = nullptr;                             // original index -> snapshot row (the grid's perm inverted)
    int* covf = nullptr;
    int cpsd_cap = 0;
    int64_t cpsd_elems = 0;                              // ckeys' allocated entries (N x cpsd_cap)
    float4 *csave_pos = nullptr, *csave_nrm = nullptr;   // the state at the call's start (a replay after overflow)
    RowMap rowmap() const { return RowMap{rows, rows ? n_rows : n}; }
};
static int settle(pcd_denoiser* dn, hipStream_t st);   // (pcd_slab.h)
static void destroy_slab_state(pcd_denoiser* dn);
static void destroy_cpsd_state(pcd_denoiser* dn);       // (pcd_cpsd.h)

#ifndef PCD_NUM_PART
#define PCD_NUM_PART 2048
#endif
static const int kNumPart = PCD_NUM_PART;   // blocks of the flat reductions (grid-stride), = their partials
// Timing events per iteration: start, after the anchor test (+ redo-list select), after the re-anchoring search,
// after the exact-key spill search, after NVT1 (= end of K1), after NVT2, after each of 3 phases, after finish, end.
static const int kTimingSets = 256, kTimingEvents = 11;

static int check_params(const pcd_denoiser* dn, const pcd_denoise_params* p) {
    PCD_CHECK_ARG(dn && p, "null argument");
    PCD_CHECK_ARG(dn->loaded, "pcd_denoiser_load must be called first");
    PCD_CHECK_ARG(p->k >= 1 && p->k_update >= 1, "k, k_update must be >= 1");
    PCD_CHECK_ARG(std::max(p->k, p->k_update) <= dn->kcap, "k / k_update exceed the k_max given at create");
    PCD_CHECK_ARG(std::max(p->k, p->k_update) <= dn->n, "k exceeds the number of points");
    PCD_CHECK_ARG(p->nphases >= 0 && p->nphases <= 3, "nphases must be 0..3");
    PCD_CHECK_ARG(p->jacobi == 0 || p->jacobi == 1, "jacobi must be 0 or 1");
    PCD_CHECK_ARG(!(p->clamp_global < 0.f), "clamp_global must be >= 0");
    for (int ph = 0; ph < p->nphases; ++ph) {
        PCD_CHECK_ARG(p->phase_class[ph] >= 0 && p->phase_class[ph] <= 2, "phase class must be 0, 1 or 2");
        PCD_CHECK_ARG(p->phase_kind[ph] >= PCD_STEP_FLAT && p->phase_kind[ph] <= PCD_STEP_DUMMY, "bad phase kind");
    }
    return PCD_OK;
}

static int list_cap(const pcd_denoise_params* p) {
    const int kstore = std::max(p->k, p->k_update);
    return kstore <= 8 ? 8 : kstore <= 16 ? 16 : kstore <= 32 ? 32 : 64;
}

static bool phase_is_global(const pcd_denoise_params* p, int ph) {
    return p->phase_kind[ph] == PCD_STEP_FLAT || p->phase_kind[ph] == PCD_STEP_NEW;
}

// Anchored K1 (seeded, list cap K <= 32, KA = 2K): the anchor test for every active row, then the re-anchoring
// search (pcd_qknn.h) of the rows that failed it -- or of every row when there are no anchors (of this KA) yet --
// and the exact-key wave search (pcd_wknn.h) for the few rows it spills.
#ifndef PCD_RQ_RDENSE
#define PCD_RQ_RDENSE 1.1f   // first iteration at 10M: 1.45 35.3 ms, 1.3 31.7, 1.2 29.7 (16-point cells); 1.2 26.0-26.7, 1.1 24.3 (32-point cells)
#endif
#ifndef PCD_RQ_GRID
#define PCD_RQ_GRID 8192     // steady re-anchoring blocks (A/B at 10M: 4096 / 8192 / 16384 -> requery 1.23 / 1.18 / 1.17 ms)
#endif
static const Band kNoBand{Cover{{1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, nullptr};
static int stage_k1_anchored(pcd_denoiser* dn, const pcd_denoise_params* p, int K, hipStream_t st,
                             hipEvent_t* ev, const Band& band, hipEvent_t before_nvt1, bool lists_only) {
    const int64_t N = dn->n;
    const RowMap rm = dn->rowmap();
    const int kstore = std::max(p->k, p->k_update);
    const int KA = 2 * K;
    if (!dn->anc) {
        if (hipMalloc(&dn->anc, N * sizeof(float4)) != hipSuccess ||
            hipMalloc(&dn->alist, (int64_t)2 * knn_cap(dn->kcap) * N * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->redo, N * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->spill, N * sizeof(int32_t)) != hipSuccess || hipMalloc(&dn->fail, N) != hipSuccess ||
            hipMalloc(&dn->rqs, sizeof(RqStats)) != hipSuccess)
            return fail(PCD_ERR_OOM, "pcd_denoiser: anchor buffers");
        dn->anchor_ka = 0;
    }
    const bool dense = dn->anchor_ka != KA;
    dn->last_dense = dense ? rm.nq : -1;
    if (dense) PCD_HIP(hipMemsetAsync(dn->anc, 0xFF, N * sizeof(float4), st));   // NaN radius: no anchor
    PCD_HIP(hipMemsetAsync(dn->rqs, 0, sizeof(RqStats), st));
    const GridView gv = dn->g->view;
    float4* P = dn->pos[dn->cur];
    unsigned* redo_cnt = &dn->rqs->redo_cnt;
    unsigned* spill_cnt = &dn->rqs->spill_cnt;
    const dim3 blk(256), grd((unsigned)cdiv(rm.nq, 256));
    const dim3 grd_rq((unsigned)std::min<int64_t>(cdiv(rm.nq, 4), PCD_RQ_GRID));
    const dim3 grd_wave((unsigned)std::min<int64_t>(cdiv(rm.nq, 4), PCD_REDO_GRID));
    const dim3 grd_dq((unsigned)std::min<int64_t>(cdiv(rm.nq, 4 * PCD_DENSE_Q), 16384));
    const dim3 grd_anc((unsigned)cdiv(rm.nq, kAnchorBS)), grd_cmp((unsigned)cdiv(rm.nq, kCompactBS * kCompactPer));
    // Dense (no anchors): every row is re-anchored (PCD_DENSE_Q queries per wave sharing one scan), then NVT1 runs
    // over all rows.  Seeded: the anchor test, the redo list of its failures, their re-anchoring search, then NVT1
    // over all rows.  (A side-stream NVT1 of the certified rows beside the search, and two steady queries per wave,
    // were measured slower: DESIGN.md §3 tried table.)
    const dim3 blk_nvt(kNvtBS), grd_nvt((unsigned)cdiv(rm.nq, kNvtBS));
#define PCD_K1A(C)                                                                                                     \
    case C:                                                                                                            \
        if (dense) {                                                                                                   \
            if (ev) PCD_HIP(hipEventRecord(ev[1], st));                                                                \
            /* the radii by a lane-per-row pass (k_dense_radius), into the redo list (idle until the steady */      \
            /* iterations), and the query boxes into f_n (rewritten by NVT1 after the search; not when K1 runs */     \
            /* lists only): first iteration 21.1 -> 19.6 -> 19.1 ms at 10M */                                       \
            float* rpre = reinterpret_cast<float*>(dn->redo);                                                          \
            uint4* bpre = !rm.rows && dn->nvt1_on ? reinterpret_cast<uint4*>(dn->fn) : nullptr;                        \
            hipLaunchKernelGGL(k_dense_radius, grd, blk, 0, st, gv, P, rm, PCD_RQ_RDENSE, rpre, bpre);                 \
            hipLaunchKernelGGL((k_knn_dense_q<2 * C, PCD_DENSE_Q>), grd_dq, blk, 0, st, gv, P, N, rm, kstore,          \
                               dn->anc, dn->alist, dn->idx, dn->spill, spill_cnt, rpre, bpre);                         \
        } else {                                                                                                       \
            hipLaunchKernelGGL((k_knn_anchor<C, 2 * C>), grd_anc, dim3(kAnchorBS), 0, st, gv, P, N, rm, kstore,        \
                               dn->anc, dn->alist, dn->idx, dn->fail);                                                 \
            hipLaunchKernelGGL(k_compact_fail, grd_cmp, dim3(kCompactBS), 0, st, dn->fail, rm, dn->redo, redo_cnt);    \
            if (ev) PCD_HIP(hipEventRecord(ev[1], st));                                                                \
            hipLaunchKernelGGL((k_knn_requery<2 * C>), grd_rq, blk, 0, st, gv, P, N, rm, kstore, dn->anc,              \
                               dn->alist, dn->idx, dn->redo, redo_cnt, dn->spill, spill_cnt);                          \
        }                                                                                                              \
        if (ev) PCD_HIP(hipEventRecord(ev[2], st));                                                                    \
        hipLaunchKernelGGL((k_knn_redo_wave<2 * C, false>), grd_wave, blk, 0, st, gv, P, N, rm, kstore, dn->anc,       \
                           dn->alist, dn->idx, dn->spill, spill_cnt, dn->err);                                         \
        if (ev) PCD_HIP(hipEventRecord(ev[3], st));                                                                    \
        if (before_nvt1) PCD_HIP(hipStreamWaitEvent(st, before_nvt1, 0));                                              \
        if (!dn->nvt1_on || lists_only) {                                                                              \
            /* the kNN lists only (the CPSD driver's update selection, pcd_cpsd.h; the slabs' read-set exchange) */   \
        } else if (dn->unit_nrm) {                                                                                     \
            hipLaunchKernelGGL((k_nvt1<C, true>), grd_nvt, blk_nvt, 0, st, gv, P, dn->nrm, dn->idx, N, rm, p->k, kstore,       \
                               p->rho, p->tau, p->damp, dn->cov, dn->fn, dn->err, dn->windows, band, RowSel{nullptr, 0});  \
        } else {                                                                                                       \
            hipLaunchKernelGGL((k_nvt1<C, false>), grd_nvt, blk_nvt, 0, st, gv, P, dn->nrm, dn->idx, N, rm, p->k, kstore,      \
                               p->rho, p->tau, p->damp, dn->cov, dn->fn, dn->err, dn->windows, band, RowSel{nullptr, 0});  \
        }                                                                                                              \
        break;
    switch (K) {
        PCD_K1A(8) PCD_K1A(16) PCD_K1A(32)
        default: return fail(PCD_ERR_ARG, "unsupported k");
    }
#undef PCD_K1A
    PCD_LAUNCH_CHECK();
    dn->anchor_ka = KA;
    dn->seed_cols = dn->list_cols = kstore;
    return PCD_OK;
}

// K1 takes the anchored path (its kNN and NVT1 are separate launches)
static bool k1_anchored(const pcd_denoiser* dn, const pcd_denoise_params* p) {
    const int K = list_cap(p);
    return dn->rowmap().nq > 0 && dn->seeding && dn->anchoring && K <= 32 && dn->n >= 2 * K && knn_cap(dn->kcap) <= 32;
}

// band: spatial slabs, mark the rows that may read a halo row (pcd_slab_iterate); before_nvt1: an event the
// neighbour gathers must wait for (the previous iteration's position exchange; the kNN itself reads only the row's
// own position and the frozen snapshot).  lists_only (anchored path): the kNN lists, NVT1 left to stage_nvt1.
static int stage_k1(pcd_denoiser* dn, const pcd_denoise_params* p, hipStream_t st, hipEvent_t* ev = nullptr,
                    const Band& band = kNoBand, hipEvent_t before_nvt1 = nullptr, bool lists_only = false) {
    const int64_t N = dn->n;
    const RowMap rm = dn->rowmap();
    const int kstore = std::max(p->k, p->k_update);
    const int K = list_cap(p);
    if (k1_anchored(dn, p)) return stage_k1_anchored(dn, p, K, st, ev, band, before_nvt1, lists_only);
    if (lists_only) return fail(PCD_ERR_ARG, "stage_k1: lists only needs the anchored path");
    if (ev) for (int e = 1; e <= 3; ++e) PCD_HIP(hipEventRecord(ev[e], st));   // no anchored sub-stages
    if (before_nvt1) PCD_HIP(hipStreamWaitEvent(st, before_nvt1, 0));         // (the fused kernel gathers at once)
    if (rm.nq == 0) return PCD_OK;
    const dim3 blk(256), grd((unsigned)cdiv(rm.nq, 256));
    const GridView gv = dn->g->view;
    float4* P = dn->pos[dn->cur];
    const bool seed = dn->seeding && dn->seed_cols >= kstore;
#define PCD_K1(C)                                                                                                      \
    case C:                                                                                                            \
        if (seed) hipLaunchKernelGGL((k_knn_nvt1<C, true>), grd, blk, 0, st, gv, P, dn->nrm, N, rm, p->k, kstore, p->rho, p->tau, p->damp, dn->cov, dn->idx, dn->fn, dn->err, band); \
        else hipLaunchKernelGGL((k_knn_nvt1<C, false>), grd, blk, 0, st, gv, P, dn->nrm, N, rm, p->k, kstore, p->rho, p->tau, p->damp, dn->cov, dn->idx, dn->fn, dn->err, band); \
        break;
    switch (K) {
        PCD_K1(8) PCD_K1(16) PCD_K1(32) PCD_K1(64)
        default: return fail(PCD_ERR_ARG, "unsupported k");
    }
#undef PCD_K1
    PCD_LAUNCH_CHECK();
    dn->seed_cols = dn->list_cols = kstore;
    return PCD_OK;
}

// NVT1 + eigh + VU smoothing over the stored lists of the rows `sel` takes (after a lists-only K1)
static int stage_nvt1(pcd_denoiser* dn, const pcd_denoise_params* p, hipStream_t st, RowSel sel) {
    const RowMap rm = dn->rowmap();
    if (rm.nq == 0) return PCD_OK;
    const int64_t N = dn->n;
    const int kstore = std::max(p->k, p->k_update);
    const GridView gv = dn->g->view;
    float4* P = dn->pos[dn->cur];
    const dim3 blk_nvt(kNvtBS), grd_nvt((unsigned)cdiv(rm.nq, kNvtBS));
#define PCD_NV(C)                                                                                                      \
    case C:                                                                                                            \
        if (dn->unit_nrm)                                                                                              \
            hipLaunchKernelGGL((k_nvt1<C, true>), grd_nvt, blk_nvt, 0, st, gv, P, dn->nrm, dn->idx, N, rm, p->k, kstore, \
                               p->rho, p->tau, p->damp, dn->cov, dn->fn, dn->err, dn->windows, kNoBand, sel);          \
        else                                                                                                           \
            hipLaunchKernelGGL((k_nvt1<C, false>), grd_nvt, blk_nvt, 0, st, gv, P, dn->nrm, dn->idx, N, rm, p->k,      \
                               kstore, p->rho, p->tau, p->damp, dn->cov, dn->fn, dn->err, dn->windows, kNoBand, sel);  \
        break;
    switch (list_cap(p)) {
        PCD_NV(8) PCD_NV(16) PCD_NV(32)
        default: return fail(PCD_ERR_ARG, "unsupported k");
    }
#undef PCD_NV
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

static int stage_k2(pcd_denoiser* dn, const pcd_denoise_params* p, hipStream_t st, RowSel sel = RowSel{nullptr, 0}) {
    const RowMap rm = dn->rowmap();
    if (rm.nq == 0) return PCD_OK;
    const dim3 blk(kNvtBS), grd((unsigned)cdiv(rm.nq, kNvtBS));
    float4* P = dn->pos[dn->cur];
#define PCD_K2(C) \
    case C:                                                                                                            \
        hipLaunchKernelGGL((k_nvt2<C>), grd, blk, 0, st, P, dn->fn, dn->idx, dn->n, rm, p->k, p->rho, p->class_scale, dn->cls, dn->edge, dn->windows, dn->probe, sel); \
        break;
    switch (list_cap(p)) {
        PCD_K2(8) PCD_K2(16) PCD_K2(32) PCD_K2(64)
        default: return fail(PCD_ERR_ARG, "unsupported k");
    }
#undef PCD_K2
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

// local (Σx, Σy, Σz, count) of phase ph -> red4 (device)
static int stage_sum(pcd_denoiser* dn, const pcd_denoise_params* p, int ph, double* red4, hipStream_t st) {
    const int c = p->phase_class[ph];
#define PCD_RS(C) hipLaunchKernelGGL(k_class_rows_sum<C>, dim3(kNumPart), dim3(256), 0, st, dn->pos[dn->cur], dn->idx, \
                                     dn->n, dn->rowmap(), p->k_update, dn->cls, c, dn->part)
    switch (knn_cap(p->k_update)) {
        case 8: PCD_RS(8); break;
        case 16: PCD_RS(16); break;
        case 32: PCD_RS(32); break;
        default: PCD_RS(64); break;
    }
#undef PCD_RS
    hipLaunchKernelGGL(k_part_reduce, dim3(1), dim3(256), 0, st, dn->part, kNumPart, red4);
    PCD_LAUNCH_CHECK();
    dn->part_ph = ph;
    dn->scan_ph = -1;
    return PCD_OK;
}

static int stage_centre(pcd_denoiser* dn, int ph, const double* red4, hipStream_t st) {
    // (the pruning needs this phase's partials: stage_sum of the same phase on the same positions)
    const bool prune = dn->part_ph == ph;   // the max-distance pass skips the blocks that cannot hold the maximum
    hipLaunchKernelGGL(k_centre, dim3(1), dim3(256), 0, st, red4, dn->gscal + 4 * ph, prune ? dn->part : nullptr,
                       kNumPart);
    dn->scan_ph = prune ? ph : -1;
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

// local max distance of phase ph -> gscal delta (and *red1 when given)
static int stage_maxdist(pcd_denoiser* dn, const pcd_denoise_params* p, int ph, float* red1, hipStream_t st) {
    float* gs = dn->gscal + 4 * ph;
#define PCD_MD(C) hipLaunchKernelGGL(k_class_rows_maxdist<C>, dim3(kNumPart), dim3(256), 0, st, dn->pos[dn->cur], \
                                     dn->idx, dn->n, dn->rowmap(), p->k_update, dn->cls, p->phase_class[ph], gs,   \
                                     dn->scan_ph == ph ? dn->part : nullptr)
    switch (knn_cap(p->k_update)) {
        case 8: PCD_MD(8); break;
        case 16: PCD_MD(16); break;
        case 32: PCD_MD(32); break;
        default: PCD_MD(64); break;
    }
#undef PCD_MD
    if (red1) hipLaunchKernelGGL(k_copy_delta, dim3(1), dim3(64), 0, st, gs + 3, red1);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

// split: the fused loop's copy-free phases (k_phase SPLIT; pcd_denoiser_iterate decides), moved = the classes the
// earlier phases of this iteration moved into pos[cur ^ 1]; cur flips after the last phase only.
// sel: one pass of the rows (spatial slabs: the rows that read no halo row, then the others after the exchange);
// flip: this call completes the phase (the last pass), cur may flip.
static int stage_apply(pcd_denoiser* dn, const pcd_denoise_params* p, int ph, const float* red1, hipStream_t st,
                       bool split = false, uint32_t moved = 0, RowSel sel = RowSel{nullptr, 0}, bool flip = true) {
    const RowMap rm = dn->rowmap();
    dn->part_ph = dn->scan_ph = -1;     // positions change: the partials' boxes no longer describe them
    float* gs = dn->gscal + 4 * ph;
    if (red1) hipLaunchKernelGGL(k_copy_delta, dim3(1), dim3(64), 0, st, red1, gs + 3);
    const int kind = p->phase_kind[ph], c = p->phase_class[ph];
    const float a = p->phase_alpha[ph];
    float4* pin = dn->pos[dn->cur];
    float4* pout = dn->pos[dn->cur ^ 1];
    const int copy_others = split ? 0 : (!p->jacobi || ph == 0) ? 1 : 0;
    if (rm.nq > 0) {
        const dim3 blk(256), grd((unsigned)cdiv(rm.nq, 256));
#define PCD_PH2(KD, C) hipLaunchKernelGGL((k_phase<KD, C>), grd, blk, 0, st, pin, pout, dn->fn, dn->edge, dn->idx, dn->n, rm, p->k_update, dn->cls, c, gs, p->d, a, dn->windows, copy_others, dn->orig, p->clamp_global, moved, sel)
#define PCD_PH(KD)                                                                                                     \
    switch (knn_cap(p->k_update)) {                                                                                    \
        case 8: PCD_PH2(KD, 8); break;                                                                                 \
        case 16: PCD_PH2(KD, 16); break;                                                                               \
        case 32: PCD_PH2(KD, 32); break;                                                                               \
        default: PCD_PH2(KD, 64); break;                                                                               \
    }
        switch (kind) {
            case PCD_STEP_FLAT: PCD_PH(PCD_STEP_FLAT); break;
            case PCD_STEP_EDGE: PCD_PH(PCD_STEP_EDGE); break;
            case PCD_STEP_FEATURE: PCD_PH(PCD_STEP_FEATURE); break;
            case PCD_STEP_CORNER: PCD_PH(PCD_STEP_CORNER); break;
            case PCD_STEP_NEW: PCD_PH(PCD_STEP_NEW); break;
            default: PCD_PH(PCD_STEP_DUMMY); break;
        }
#undef PCD_PH
#undef PCD_PH2
        PCD_LAUNCH_CHECK();
    }
    if (flip && (split ? ph == p->nphases - 1 : !p->jacobi)) dn->cur ^= 1;   // Jacobi: the swap happens at finish
    return PCD_OK;
}

static void stage_finish(pcd_denoiser* dn, const pcd_denoise_params* p) {
    if (p->jacobi && p->nphases > 0) dn->cur ^= 1;
    std::swap(dn->nrm, dn->fn);   // graph.n = f_n  (Processor.py:139)
    dn->unit_nrm = true;
    dn->iterated = true;
}

static float4* field_ptr(pcd_denoiser* dn, int field) {
    switch (field) {
        case PCD_FIELD_POS: return dn->pos[dn->cur];
        case PCD_FIELD_NRM: return dn->nrm;
        case PCD_FIELD_FN: return dn->fn;
        case PCD_FIELD_EDGE: return dn->edge;
        default: return nullptr;
    }
}

extern "C" {

int pcd_denoiser_create(const pcd_grid* g, int k_max, pcd_denoiser** out) {
    PCD_CHECK_ARG(out != nullptr, "out is null");
    *out = nullptr;
    PCD_CHECK_ARG(g != nullptr, "grid is null");
    PCD_CHECK_ARG(k_max >= 1 && k_max <= pcd_max_k(), "k_max out of range");
    // the kernels address rows and list blocks by 32-bit byte offsets from uniform bases (at32, pcd_lists.h):
    // 32 B x N < 4 GiB
    PCD_CHECK_ARG(g->n < (1ll << 27), "more than 2^27 points per denoiser (split into spatial slabs)");
    pcd_denoiser* dn = new pcd_denoiser();
    dn->g = g;
    dn->n = g->n;
    dn->kcap = k_max;
    const int64_t N = g->n;
    bool ok = hipMalloc(&dn->pos[0], N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->pos[1], N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->nrm, N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->fn, N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->edge, N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->orig, N * sizeof(float4)) == hipSuccess &&
              hipMalloc(&dn->idx, (int64_t)knn_cap(k_max) * N * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dn->cls, N) == hipSuccess &&
              hipMalloc(&dn->part, kNumPart * sizeof(RedC)) == hipSuccess &&
              hipMalloc(&dn->red, 16 * sizeof(double)) == hipSuccess &&
              hipMalloc(&dn->gscal, 16 * sizeof(float)) == hipSuccess &&
              hipMalloc(&dn->err, 4 * sizeof(int)) == hipSuccess && hipMemset(dn->err, 0, 4 * sizeof(int)) == hipSuccess &&
              hipMemset(dn->cls, 0xFF, N) == hipSuccess;
    if (!ok) {
        pcd_denoiser_destroy(dn);
        return fail(PCD_ERR_OOM, "pcd_denoiser_create: device allocation");
    }
    *out = dn;
    return PCD_OK;
}

int pcd_denoiser_destroy(pcd_denoiser* dn) {
    if (!dn) return PCD_OK;
    destroy_slab_state(dn);
    destroy_cpsd_state(dn);
    (void)hipFree(dn->pos[0]); (void)hipFree(dn->pos[1]); (void)hipFree(dn->nrm); (void)hipFree(dn->fn);
    (void)hipFree(dn->xrad);
    (void)hipFree(dn->edge); (void)hipFree(dn->orig); (void)hipFree(dn->idx); (void)hipFree(dn->cls); (void)hipFree(dn->part);
    (void)hipFree(dn->red); (void)hipFree(dn->gscal); (void)hipFree(dn->err);
    (void)hipFree(dn->anc); (void)hipFree(dn->alist); (void)hipFree(dn->redo); (void)hipFree(dn->spill);
    (void)hipFree(dn->rqs); (void)hipFree(dn->fail); (void)hipFree(dn->probe);
    for (auto e : dn->ev) (void)hipEventDestroy(e);
    delete dn;
    return PCD_OK;
}

int pcd_denoiser_load(pcd_denoiser* dn, const float* pos, const float* n, void* stream) {
    PCD_CHECK_ARG(dn && pos && n, "null argument");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    hipLaunchKernelGGL(k_load, dim3((unsigned)cdiv(dn->n, 256)), dim3(256), 0, as_stream(stream), pos, n,
                       dn->g->perm, dn->n, dn->pos[0], dn->nrm, dn->orig);
    PCD_LAUNCH_CHECK();
    dn->cur = 0;
    dn->part_ph = dn->scan_ph = -1;
    dn->loaded = true;
    dn->iterated = false;
    dn->unit_nrm = false;         // the caller's normals: the general vote margin until the first finish
    dn->seed_cols = 0;
    return PCD_OK;
}

int pcd_denoiser_set_rows(pcd_denoiser* dn, const int32_t* rows, int64_t n_rows) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    PCD_CHECK_ARG(rows != nullptr || n_rows == 0, "rows is null");
    PCD_CHECK_ARG(n_rows >= 0 && n_rows <= dn->n, "n_rows out of range");
    dn->rows = rows;
    dn->n_rows = rows ? n_rows : 0;
    dn->part_ph = dn->scan_ph = -1;
    return PCD_OK;
}

int pcd_denoiser_set_coverage(pcd_denoiser* dn, const float* lo3, const float* hi3) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    if (!lo3 || !hi3) {
        dn->cov = Cover{{1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
        dn->cov.xr = dn->xrad;
        dn->cov.org = dn->orig;
        return PCD_OK;
    }
    for (int a = 0; a < 3; ++a) {
        PCD_CHECK_ARG(!(lo3[a] > hi3[a]), "coverage box has lo > hi");
        dn->cov.lo[a] = lo3[a];
        dn->cov.hi[a] = hi3[a];
    }
    dn->cov.xr = dn->xrad;
    dn->cov.org = dn->orig;
    return PCD_OK;
}

int pcd_denoiser_set_coverage_spheres(pcd_denoiser* dn, const float* radii, void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    hipStream_t st = as_stream(stream);
    if (!radii) {
        PCD_HIP(hipStreamSynchronize(st));
        (void)hipFree(dn->xrad);
        dn->xrad = nullptr;
        dn->cov.xr = nullptr;
        return PCD_OK;
    }
    if (!dn->xrad && hipMalloc(&dn->xrad, dn->n * sizeof(float)) != hipSuccess)
        return fail(PCD_ERR_OOM, "pcd_denoiser_set_coverage_spheres");
    // caller order -> the denoiser's sorted rows (the load permutation)
    hipLaunchKernelGGL(k_gather_f32, dim3((unsigned)cdiv(dn->n, 256)), dim3(256), 0, st, radii, dn->g->perm, dn->n,
                       dn->xrad);
    PCD_LAUNCH_CHECK();
    dn->cov.xr = dn->xrad;
    dn->cov.org = dn->orig;
    return PCD_OK;
}

int pcd_denoiser_pack(pcd_denoiser* dn, int field, const int32_t* rows, int64_t n, float* out4, void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    float4* f = field_ptr(dn, field);
    PCD_CHECK_ARG(f != nullptr, "bad field");
    PCD_CHECK_ARG(n == 0 || (rows && out4), "null rows / buffer");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    if (n == 0) return PCD_OK;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream), f, rows, n,
                       reinterpret_cast<float4*>(out4));
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_denoiser_unpack(pcd_denoiser* dn, int field, const int32_t* rows, int64_t n, const float* in4, void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    float4* f = field_ptr(dn, field);
    PCD_CHECK_ARG(f != nullptr, "bad field");
    PCD_CHECK_ARG(n == 0 || (rows && in4), "null rows / buffer");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    if (n == 0) return PCD_OK;
    dn->part_ph = dn->scan_ph = -1;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream), f, rows, n,
                       reinterpret_cast<const float4*>(in4));
    PCD_LAUNCH_CHECK();
    if (field == PCD_FIELD_NRM) dn->unit_nrm = false;   // (FN rows must be another rank's NVT1 output: unit)
    return PCD_OK;
}

int pcd_denoiser_stage(pcd_denoiser* dn, const pcd_denoise_params* p, int stage, int phase, void* red,
                       void* stream) {
    const int rc = check_params(dn, p);
    if (rc != PCD_OK) return rc;
    PCD_CHECK_ARG(stage >= PCD_STAGE_KNN_NVT1 && stage <= PCD_STAGE_FINISH, "bad stage");
    const bool ph_stage = stage >= PCD_STAGE_PHASE_SUM && stage <= PCD_STAGE_PHASE_APPLY;
    PCD_CHECK_ARG(!ph_stage || (phase >= 0 && phase < p->nphases), "phase out of range");
    PCD_CHECK_ARG(!(stage == PCD_STAGE_PHASE_SUM || stage == PCD_STAGE_PHASE_CENTRE) || red, "red is null");
    hipStream_t st = as_stream(stream);
    if (settle(dn, st) != PCD_OK) return PCD_ERR_HIP;
    switch (stage) {
        case PCD_STAGE_KNN_NVT1: return stage_k1(dn, p, st);
        case PCD_STAGE_NVT2: return stage_k2(dn, p, st);
        case PCD_STAGE_PHASE_SUM: return stage_sum(dn, p, phase, static_cast<double*>(red), st);
        case PCD_STAGE_PHASE_CENTRE: return stage_centre(dn, phase, static_cast<const double*>(red), st);
        case PCD_STAGE_PHASE_MAXDIST: return stage_maxdist(dn, p, phase, static_cast<float*>(red), st);
        case PCD_STAGE_PHASE_APPLY: return stage_apply(dn, p, phase, static_cast<const float*>(red), st);
        default: stage_finish(dn, p); return PCD_OK;
    }
}

int pcd_denoiser_check(pcd_denoiser* dn, void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    int err = 0;
    PCD_HIP(hipMemcpyAsync(&err, dn->err, sizeof(int), hipMemcpyDeviceToHost, as_stream(stream)));
    PCD_HIP(hipStreamSynchronize(as_stream(stream)));
    if (err & 1) return fail(PCD_ERR_STATE, "pcd_denoiser: the kNN kernel produced an invalid neighbour index");
    if (err & 2)
        return fail(PCD_ERR_STATE, "pcd_denoiser: a k-neighbourhood reaches past the local snapshot (halo too thin)");
    return PCD_OK;
}

int pcd_denoiser_coverage_excess(pcd_denoiser* dn, float* band_excess, float* sphere_ratio, void* stream) {
    PCD_CHECK_ARG(dn && band_excess && sphere_ratio, "null argument");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    int w[4];
    PCD_HIP(hipMemcpyAsync(w, dn->err, sizeof w, hipMemcpyDeviceToHost, as_stream(stream)));
    PCD_HIP(hipStreamSynchronize(as_stream(stream)));
    *band_excess = (w[0] & 4) ? __builtin_bit_cast(float, w[1]) : 0.f;
    *sphere_ratio = (w[0] & 8) ? __builtin_bit_cast(float, w[2]) : 0.f;
    return PCD_OK;
}

int pcd_denoiser_status(pcd_denoiser* dn, int* bits, void* stream) {
    PCD_CHECK_ARG(dn && bits, "null argument");
    // (an exchange still in flight finishes first: a collective the caller issues next on its comm -- the slab
    // driver's coverage verdict -- then follows it in stream order rather than racing it on another stream)
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    PCD_HIP(hipMemcpyAsync(bits, dn->err, sizeof(int), hipMemcpyDeviceToHost, as_stream(stream)));
    PCD_HIP(hipStreamSynchronize(as_stream(stream)));
    return PCD_OK;
}

int pcd_denoiser_lists(pcd_denoiser* dn, int64_t* out, int cols, void* stream) {
    PCD_CHECK_ARG(dn && out, "null argument");
    PCD_CHECK_ARG(dn->iterated && cols >= 1 && cols <= dn->list_cols, "cols must be in [1, stored list length]");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    hipLaunchKernelGGL(k_lists, dim3((unsigned)cdiv(dn->n, 256)), dim3(256), 0, as_stream(stream), dn->idx,
                       dn->g->perm, dn->n, cols, out);
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_denoiser_reset_seed(pcd_denoiser* dn) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->seed_cols = 0;
    dn->anchor_ka = 0;
    return PCD_OK;
}

int pcd_denoiser_anchor_stats(pcd_denoiser* dn, int64_t* redo_rows, void* stream) {
    PCD_CHECK_ARG(dn && redo_rows, "null argument");
    int64_t v[4];
    const int rc = pcd_denoiser_tile_stats(dn, v, stream);
    *redo_rows = v[0];
    return rc;
}

int pcd_denoiser_tile_stats(pcd_denoiser* dn, int64_t* out4, void* stream) {
    PCD_CHECK_ARG(dn && out4, "null argument");
    for (int a = 0; a < 4; ++a) out4[a] = -1;
    if (!dn->rqs || dn->anchor_ka == 0) return PCD_OK;
    RqStats rs;
    PCD_HIP(hipMemcpyAsync(&rs, dn->rqs, sizeof rs, hipMemcpyDeviceToHost, as_stream(stream)));
    PCD_HIP(hipStreamSynchronize(as_stream(stream)));
    out4[0] = dn->last_dense >= 0 ? dn->last_dense : (int64_t)rs.redo_cnt;
    out4[1] = (int64_t)rs.spill_cnt;
    out4[2] = (int64_t)rs.spill_big;
    out4[3] = (int64_t)rs.spill_amb;
    return PCD_OK;
}

int pcd_denoiser_set_anchoring(pcd_denoiser* dn, int enable) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->anchoring = enable != 0;
    return PCD_OK;
}

int pcd_denoiser_set_windows(pcd_denoiser* dn, int enable) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->windows = enable != 0;
    return PCD_OK;
}

int pcd_denoiser_set_probe(pcd_denoiser* dn, int enable) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    if (!enable) {
        (void)hipFree(dn->probe);
        dn->probe = nullptr;
        return PCD_OK;
    }
    if (!dn->probe) {
        if (hipMalloc(&dn->probe, dn->n * sizeof(float4)) != hipSuccess) return fail(PCD_ERR_OOM, "pcd_denoiser: probe");
        PCD_HIP(hipMemset(dn->probe, 0xFF, dn->n * sizeof(float4)));   // NaN until an NVT2 stage writes a row
    }
    return PCD_OK;
}

int pcd_denoiser_probe_store(pcd_denoiser* dn, float* nvt2_eig4, void* stream) {
    PCD_CHECK_ARG(dn && nvt2_eig4, "null argument");
    PCD_CHECK_ARG(dn->probe != nullptr, "probe not enabled (pcd_denoiser_set_probe)");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    hipLaunchKernelGGL(k_scatter4, dim3((unsigned)cdiv(dn->n, 256)), dim3(256), 0, as_stream(stream), dn->probe,
                       dn->g->perm, dn->n, reinterpret_cast<float4*>(nvt2_eig4));
    PCD_LAUNCH_CHECK();
    return PCD_OK;
}

int pcd_denoiser_set_seeding(pcd_denoiser* dn, int enable) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->seeding = enable != 0;
    return PCD_OK;
}

int pcd_denoiser_set_timing(pcd_denoiser* dn, int enable) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->timing = enable != 0;
    dn->timing_k1 = enable == 2;
    dn->ev_used = 0;
    if (dn->timing && dn->ev.empty()) {
        dn->ev.resize((size_t)kTimingSets * kTimingEvents);
        for (auto& e : dn->ev) PCD_HIP(hipEventCreate(&e));
    }
    return PCD_OK;
}

int pcd_denoiser_get_timing(pcd_denoiser* dn, float* ms_out, int n_slots, int* n_written) {
    PCD_CHECK_ARG(dn && ms_out && n_written, "null argument");
    *n_written = 0;
    if (!dn->timing || dn->ev.empty() || dn->ev_used == 0) return PCD_OK;
    const int sets = dn->ev_used;
    int w = 0;
    if (dn->timing_k1) {                  // one slot: the K1 stage (events 0 and 4 of each set)
        PCD_HIP(hipEventSynchronize(dn->ev[(size_t)(sets - 1) * kTimingEvents + 4]));
        double acc = 0.0;
        for (int st = 0; st < sets && n_slots > 0; ++st) {
            float m = 0.f;
            hipEvent_t* e = &dn->ev[(size_t)st * kTimingEvents];
            PCD_HIP(hipEventElapsedTime(&m, e[0], e[4]));
            acc += m;
        }
        if (n_slots > 0) ms_out[w++] = (float)(acc / sets);
        *n_written = w;
        dn->ev_used = 0;
        return PCD_OK;
    }
    PCD_HIP(hipEventSynchronize(dn->ev[(size_t)(sets - 1) * kTimingEvents + kTimingEvents - 1]));
    for (int slot = 0; slot + 1 < kTimingEvents && w < n_slots; ++slot) {
        double acc = 0.0;
        for (int st = 0; st < sets; ++st) {
            float m = 0.f;
            hipEvent_t* e = &dn->ev[(size_t)st * kTimingEvents];
            PCD_HIP(hipEventElapsedTime(&m, e[slot], e[slot + 1]));
            acc += m;
        }
        ms_out[w++] = (float)(acc / sets);
    }
    *n_written = w;
    dn->ev_used = 0;
    return PCD_OK;
}

int pcd_denoiser_iterate(pcd_denoiser* dn, const pcd_denoise_params* p, int iterations, void* stream) {
    int rc = check_params(dn, p);
    if (rc != PCD_OK) return rc;
    hipStream_t st = as_stream(stream);
    if ((rc = settle(dn, st)) != PCD_OK) return rc;
    for (int it = 0; it < iterations; ++it) {
        hipEvent_t* ev = nullptr;     // this iteration's event set (timing on, and a set left)
        if (dn->timing && dn->ev_used < kTimingSets) ev = &dn->ev[(size_t)dn->ev_used++ * kTimingEvents];
        if (ev) PCD_HIP(hipEventRecord(ev[0], st));
        if ((rc = stage_k1(dn, p, st, dn->timing_k1 ? nullptr : ev)) != PCD_OK) return rc;
        if (ev) PCD_HIP(hipEventRecord(ev[4], st));
        if (dn->timing_k1) ev = nullptr;   // (level 2: K1 only)
        if ((rc = stage_k2(dn, p, st)) != PCD_OK) return rc;
        if (ev) PCD_HIP(hipEventRecord(ev[5], st));
        // copy-free phases when three Gauss-Seidel phases move the three classes of every row once each and only the
        // first phase reduces globally (its reductions read the positions before any phase)
        const bool split = !p->jacobi && !dn->rows && p->nphases == 3 &&
                           ((1u << p->phase_class[0]) | (1u << p->phase_class[1]) | (1u << p->phase_class[2])) == 7u &&
                           !phase_is_global(p, 1) && !phase_is_global(p, 2);
        uint32_t moved = 0;
        for (int ph = 0; ph < p->nphases; ++ph) {
            if (phase_is_global(p, ph)) {
                double* red4 = dn->red + 4 * ph;
                if ((rc = stage_sum(dn, p, ph, red4, st)) != PCD_OK) return rc;
                if ((rc = stage_centre(dn, ph, red4, st)) != PCD_OK) return rc;
                if ((rc = stage_maxdist(dn, p, ph, nullptr, st)) != PCD_OK) return rc;
            }
            if ((rc = stage_apply(dn, p, ph, nullptr, st, split, split ? moved : 0u)) != PCD_OK) return rc;
            moved |= 1u << p->phase_class[ph];
            if (ev) PCD_HIP(hipEventRecord(ev[6 + ph], st));
        }
        if (ev)
            for (int ph = p->nphases; ph < 3; ++ph) PCD_HIP(hipEventRecord(ev[6 + ph], st));
        stage_finish(dn, p);
        if (ev) PCD_HIP(hipEventRecord(ev[9], st));
        if (ev) PCD_HIP(hipEventRecord(ev[10], st));
    }
    return PCD_OK;
}

int pcd_denoiser_store(pcd_denoiser* dn, float* pos, float* n, int64_t* classes, float* edge_vectors,
                       void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    PCD_CHECK_ARG(dn->loaded, "nothing loaded");
    PCD_CHECK_ARG(dn->iterated || (!classes && !edge_vectors), "classes/edge vectors need one iteration");
    if (settle(dn, as_stream(stream)) != PCD_OK) return PCD_ERR_HIP;
    hipLaunchKernelGGL(k_store, dim3((unsigned)cdiv(dn->n, 256)), dim3(256), 0, as_stream(stream), dn->pos[dn->cur],
                       dn->nrm, dn->cls, dn->edge, dn->g->perm, dn->n, pos, n, classes, edge_vectors);
    PCD_LAUNCH_CHECK();
    return pcd_denoiser_check(dn, stream);
}

}  // extern "C"

#include "pcd_slab.h"
#include "pcd_cpsd.h"
