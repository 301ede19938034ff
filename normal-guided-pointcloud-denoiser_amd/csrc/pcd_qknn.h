// Re-anchoring search of the anchored kNN (denoise.hip): the exact KA nearest snapshot points of a moved query,
// one query per wave, lean enough for 8 waves per SIMD.
//
// The search is the one of pcd_wknn.h (cap box -> brick probes -> flattened candidate rows -> ballot-appended
// survivors below the acceptance cap), re-cut for occupancy and VALU:
//   * the query (row, position, anchor) is wave-uniform and lives in SGPRs (readfirstlane + scalar loads);
//   * the survivors stay exact 64-bit keys (d² bits << 32 | snapshot rank) in the wave's LDS buffer, but they are
//     ORDERED by 32-bit keys floor(d² · 2^24 / cap d²) << 8 | buffer slot: a compare-exchange is one min + one max
//     on one register and one cross-lane move, where the exact keys need two registers, two moves, a 64-bit compare
//     and four selects (the sort was ~65 % of the old kernel's VALU).  The quantised order is the exact order
//     wherever neighbouring quantised values differ; a query whose anchor set (first KA) or stored list (first
//     kstore + 1) has two equal quantised values at a decision point is SPILLED to the exact-key wave search
//     (k_knn_redo_wave), so the lists stay bit-identical to it;
//   * a full buffer is cut to the KA best the same way (the cap tightens to the largest kept exact key + 1).
// DENSE (no anchors yet): the cap radius is r_scale · h · (16 / n)^(1/3), n = occupancy of the query's cell; a
// query with fewer than KA points inside it is spilled (the wave search then grows its own box).
#pragma once
#include "pcd_wknn.h"

namespace pcd {

// Acceptance cap for re-anchoring at q: the KA anchor points are within D of a, hence within D + |q - a| of q, so
// the KA-th key at q is below this bound (rounding margin included).
PCD_DEV unsigned long long anchor_cap(Vec3 q, float4 a) {
    const float R = (a.w + sqrtf(sq3(q - v3(a.x, a.y, a.z)))) * (1.f + 1e-5f) + 1e-30f;
    const float R2 = R * R * (1.f + 1e-5f);
    return ((unsigned long long)__float_as_uint(R2) << 32) | 0xFFFFFFFFull;
}

// Ascending bitonic sort of the 64*M 32-bit keys v[s] (element e = s*64 + lane) across the wave.
template <int M>
PCD_DEV void wave_bitonic_sort32(uint32_t (&v)[M], int lane) {
    constexpr int NT = 64 * M;
#pragma unroll
    for (int size = 2; size <= NT; size <<= 1) {
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1) {
            if (stride >= 64) {
                const int ss = stride / 64;
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    if ((s & ss) == 0) {
                        const bool asc = ((s * 64 + lane) & size) == 0;
                        const uint32_t a = v[s], b = v[s + ss];
                        const uint32_t mn = min(a, b), mx = max(a, b);
                        v[s] = asc ? mn : mx;
                        v[s + ss] = asc ? mx : mn;
                    }
                }
            } else {
                const bool lower = (lane & stride) == 0;
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    const bool asc = ((s * 64 + lane) & size) == 0;
                    const uint32_t o = (uint32_t)__shfl_xor((int)v[s], stride);
                    v[s] = (lower == asc) ? min(o, v[s]) : max(o, v[s]);
                }
            }
        }
    }
}

// The survivors buf[0..cnt) ordered by quantised 32-bit keys (cnt <= kWaveSurv): lane t returns element t
// (0xFFFFFFFF past cnt) and the element after the last lane's (for the boundary checks of a full first slot).
PCD_DEV uint32_t wave_order32(const unsigned long long* buf, int cnt, float capd2, int lane, uint32_t& after63) {
    wave_sync();
    const float S = 16777216.f / fmaxf(capd2, 1e-30f);
    auto k32 = [&](int e) -> uint32_t {
        if (e >= cnt) return 0xFFFFFFFFu;
        const float d2 = __uint_as_float((uint32_t)(buf[e] >> 32));
        return ((uint32_t)fminf(d2 * S, 16777214.f) << 8) | (uint32_t)e;
    };
    uint32_t top;
    if (cnt <= 64) {
        uint32_t v[1] = {k32(lane)};
        wave_bitonic_sort32<1>(v, lane);
        top = v[0];
        after63 = 0xFFFFFFFFu;
    } else if (cnt <= 128) {
        uint32_t v[2] = {k32(lane), k32(64 + lane)};
        wave_bitonic_sort32<2>(v, lane);
        top = v[0];
        after63 = (uint32_t)__shfl((int)v[1], 0);
    } else {
        uint32_t v[4] = {k32(lane), k32(64 + lane), k32(128 + lane), k32(192 + lane)};
        wave_bitonic_sort32<4>(v, lane);
        top = v[0];
        after63 = (uint32_t)__shfl((int)v[1], 0);
    }
    return top;
}

// Do the first n elements of the quantised order hold their exact order and the set boundary after element
// n-1?  Exact iff every quantised value among elements 0..n (n+1 elements) is distinct, i.e. no two neighbours
// in 0..n share one (a pad compares larger than every real key).  n <= 64.
PCD_DEV bool order_exact(uint32_t k, uint32_t after63, int n, int lane) {
    const uint32_t nxt = lane == 63 ? after63 : (uint32_t)__shfl_down((int)k, 1);
    const bool tie = lane < n && (k >> 8) == (nxt >> 8) && k != 0xFFFFFFFFu;
    return !__any(tie);
}

PCD_DEV unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = shfl_xor_u64(v, o);
        v = w > v ? w : v;
    }
    return v;
}

PCD_DEV uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
PCD_DEV unsigned long long rfl64(unsigned long long v) {
    return (unsigned long long)rfl((uint32_t)v) | ((unsigned long long)rfl((uint32_t)(v >> 32)) << 32);
}

// Shrink a survivor set of more than 128 to at most 128 before ordering it (a 2-slot sort instead of 4): a few
// bisection steps on d² find a bound with KA <= count(d² <= bound) <= 128; the keys under it contain the KA best
// of the whole set (at least KA keys are under it), so the compaction never changes the result.
template <int KA>
PCD_DEV float rq_shrink(unsigned long long* buf, int& cnt, float capd2, int lane) {
    if (cnt <= 128) return -1.f;
    wave_sync();
    float d[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int e = s * 64 + lane;
        d[s] = e < cnt ? __uint_as_float((uint32_t)(buf[e] >> 32)) : 3.0e38f;
    }
    auto count_le = [&](float t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < 4; ++s) c += __popcll(__ballot(d[s] <= t));
        return c;
    };
    float lo = 0.f, hi = capd2, bound = -1.f;
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
        const float mid = 0.5f * (lo + hi);
        const int c = count_le(mid);
        if (c < KA) lo = mid;
        else if (c > 128) hi = mid;
        else { bound = mid; break; }
    }
    if (bound < 0.f) return -1.f;                     // no such bound found quickly: order the full set
    unsigned long long keep[4];
    int base = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) keep[s] = (s * 64 + lane) < cnt ? buf[s * 64 + lane] : 0ull;
    wave_sync();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const bool in = d[s] <= bound;
        const unsigned long long m = __ballot(in);
        if (in) buf[base + __popcll(m & ((1ull << lane) - 1ull))] = keep[s];
        base += __popcll(m);
    }
    cnt = base;
    return bound;
}

// Cut the survivors to the K best (quantised order): false when the cut is ambiguous (the query must spill).
template <int K>
PCD_DEV bool rq_cut(unsigned long long* buf, int& cnt, unsigned long long& cap, int lane) {
    {
        const float bound = rq_shrink<K>(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), lane);
        if (bound >= 0.f) {                           // >= K keys have d² <= bound: a valid, tighter cap
            const unsigned long long c2 = ((unsigned long long)__float_as_uint(bound) << 32) | 0xFFFFFFFFull;
            if (c2 < cap) cap = c2;
            return true;
        }
    }
    uint32_t after;
    const uint32_t k = wave_order32(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), lane, after);
    const uint32_t kK = K < 64 ? (uint32_t)__shfl((int)k, K < 64 ? K : 0) : after;
    const uint32_t kK1 = (uint32_t)__shfl((int)k, K - 1);
    if ((kK >> 8) == (kK1 >> 8)) return false;
    const unsigned long long mine = lane < K ? buf[k & 255u] : 0ull;
    wave_sync();
    if (lane < K) buf[lane] = mine;
    wave_sync();
    const unsigned long long mx = rfl64(wave_max_u64(lane < K ? mine : 0ull));
    if (mx + 1ull < cap) cap = mx + 1ull;
    cnt = K;
    return true;
}

// Scan the cells of box [lo, hi] (at most kRqMaxCells) appending keys < cap to buf: pcd_wknn.h wave_scan_box
// in 32-bit cell arithmetic, with the quantised buffer cut.  Returns false when a cut was ambiguous (spill).
static constexpr int kRqMaxCells = 4096;
#ifndef PCD_RQ_ROWS
#define PCD_RQ_ROWS 2
#endif
static constexpr int kRqRows = PCD_RQ_ROWS;   // candidate rows per lane per round (all loads in flight)
#ifndef PCD_RQ_CPL
#define PCD_RQ_CPL 1
#endif
static constexpr int kRqCPL = PCD_RQ_CPL;     // cells per lane per chunk
static constexpr int kRqChunk = 64 * kRqCPL;
static constexpr int kRqChunkLog2 = kRqCPL == 1 ? 6 : kRqCPL == 2 ? 7 : 8;
struct RqCells {            // per-wave LDS scratch for one chunk of cells
    uint32_t start[kRqChunk];
    uint32_t end_incl[kRqChunk];
};
template <int K>
PCD_DEV bool rq_scan_box(const GridView& g, Vec3 q, const int lo[3], const int hi[3], unsigned long long& cap,
                         unsigned long long* buf, int& cnt, RqCells* wc, int lane) {
    static_assert(K + 64 * kRqRows <= kWaveSurv, "a cut to K plus one round of appends must fit the buffer");
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1;
    const int nc = ex * ey * (hi[2] - lo[2] + 1);
    const uint32_t exy = (uint32_t)ex * (uint32_t)ey;
    for (int base = 0; base < nc; base += kRqChunk) {
        uint32_t slot[kRqCPL], loc6[kRqCPL];
        unsigned long long bkey[kRqCPL];
        const float kth = __uint_as_float((unsigned)(cap >> 32));
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u) {
            const uint32_t ci = (uint32_t)(base + lane * kRqCPL + u);
            slot[u] = ~0u; loc6[u] = 0; bkey[u] = kEmptyKey;
            if (ci < (uint32_t)nc) {
                const uint32_t zq = ci / exy, rem = ci - zq * exy, yq = rem / (uint32_t)ex;
                const int cx = lo[0] + (int)(rem - yq * (uint32_t)ex), cy = lo[1] + (int)yq, cz = lo[2] + (int)zq;
                const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
                const float gx = axis_gap(q.x, lx, lx + g.h), gy = axis_gap(q.y, ly, ly + g.h), gz = axis_gap(q.z, lz, lz + g.h);
                if (gx * gx + gy * gy + gz * gz <= kth * 1.00001f + 1e-30f) {
                    const unsigned long long key = morton3(cx, cy, cz);
                    bkey[u] = key >> 6;
                    loc6[u] = (uint32_t)(key & 63);
                    slot[u] = (uint32_t)hash_slot(bkey[u], g.hbits);
                }
            }
        }
        uint4 sl[kRqCPL];
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u)
            sl[u] = slot[u] != ~0u ? *reinterpret_cast<const uint4*>(g.table + slot[u]) : make_uint4(~0u, ~0u, 0u, 0u);
        uint32_t brick[kRqCPL];
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u) {
            brick[u] = ~0u;
            if (slot[u] == ~0u) continue;
            uint4 e = sl[u];
            uint32_t sidx = slot[u];
            for (;;) {
                const unsigned long long k2 = (unsigned long long)e.x | ((unsigned long long)e.y << 32);
                if (k2 == bkey[u]) { brick[u] = e.z; break; }
                if (k2 == kEmptyKey) break;
                sidx = (uint32_t)((sidx + 1) & g.mask);
                e = *reinterpret_cast<const uint4*>(g.table + sidx);
            }
        }
        uint2 cr[kRqCPL];
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u)
            cr[u] = brick[u] != ~0u ? g.cells[(uint64_t)brick[u] * 64 + loc6[u]] : make_uint2(0u, 0u);
        uint32_t loc[kRqCPL], run = 0;
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u) {
            run += cr[u].y > cr[u].x ? cr[u].y - cr[u].x : 0u;
            loc[u] = run;
        }
        uint32_t incl = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += t;
        }
        const uint32_t total = rfl((uint32_t)__shfl((int)incl, 63));
        if (total == 0) continue;
        const uint32_t excl = incl - run;
        wave_sync();
#pragma unroll
        for (int u = 0; u < kRqCPL; ++u) {
            wc->start[lane * kRqCPL + u] = cr[u].x;
            wc->end_incl[lane * kRqCPL + u] = excl + loc[u];
        }
        wave_sync();
        for (uint32_t j0 = 0; j0 < total; j0 += 64 * kRqRows) {
            // room for a whole round of appends (one cut site: the sort network is inlined once)
            if (cnt > kWaveSurv - 64 * kRqRows && !rq_cut<K>(buf, cnt, cap, lane)) return false;
            uint32_t r[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * 64 + lane);
                int a = 0, b = kRqChunk - 1;
#pragma unroll
                for (int it = 0; it < kRqChunkLog2; ++it) {
                    const int m = (a + b) >> 1;
                    if (wc->end_incl[m] > j) b = m; else a = m + 1;
                }
                r[u] = j < total ? wc->start[a] + (j - (a ? wc->end_incl[a - 1] : 0u)) : 0u;
            }
            float px[kRqRows], py[kRqRows], pz[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                if (j0 + (uint32_t)(u * 64) < total) {
                    const float* pp = reinterpret_cast<const float*>(g.pts + r[u]);
                    px[u] = pp[0]; py[u] = pp[1]; pz[u] = pp[2];
                }
            }
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * 64 + lane);
                if (j0 + (uint32_t)(u * 64) < total) {
                    const unsigned long long key2 =
                        ((unsigned long long)__float_as_uint(dist2(q, make_float4(px[u], py[u], pz[u], 0.f))) << 32) | r[u];
                    wave_append(j < total && key2 < cap, key2, buf, cnt, lane);
                }
            }
        }
        wave_sync();
    }
    return true;
}

// Per-stage counters of the anchored kNN (device): rows that failed the anchor test (= length of the redo list),
// rows spilled to the exact-key wave search (= length of the spill list).
struct RqStats { unsigned redo_cnt, spill_cnt, spill_big, spill_amb; };

#ifndef PCD_RQ_RSCALE
#define PCD_RQ_RSCALE 1.1f   // re-anchoring radius / the old anchor's D
#endif
#ifndef PCD_RQ_OCC
#define PCD_RQ_OCC 8
#endif
// One query per wave (grid-stride): DENSE = every active row (cap from the cell occupancy), else the rows of
// `list` (the anchor test's failures, cap from the anchor).  Spilled rows go to `spill` for k_knn_redo_wave.
template <int KA, bool DENSE>
__global__ __launch_bounds__(256, PCD_RQ_OCC) void k_knn_requery(GridView g, const float4* __restrict__ pos,
                                                                 int64_t N, RowMap rm, int kstore, float r_scale,
                                                                 float4* __restrict__ anc, int32_t* __restrict__ alist,
                                                                 int32_t* __restrict__ idx,
                                                                 const int32_t* __restrict__ list,
                                                                 const unsigned* __restrict__ list_cnt,
                                                                 int32_t* __restrict__ spill,
                                                                 unsigned* __restrict__ spill_cnt) {
    static_assert(KA <= 64, "one key per lane");
    __shared__ unsigned long long s_buf[4][kWaveSurv];
    __shared__ RqCells s_cells[4];
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t cnt_rows = DENSE ? rm.nq : (int64_t)*list_cnt;
    const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
    unsigned long long* buf = s_buf[wv];
    for (int64_t t0 = lb * 4 + wv; t0 < cnt_rows; t0 += (int64_t)gridDim.x * 4) {
        const int64_t i = __builtin_amdgcn_readfirstlane(DENSE ? (int)rm(t0) : list[t0]);
        const float4 p4 = pos[i];
        const Vec3 q = v3(p4.x, p4.y, p4.z);
        // The search radius r: DENSE from the occupancy of the query's cell, else from the old anchor's D (the local
        // KA-th distance; the cap (D + |q - a|)^2 that bounds the KA-th key at q is ~2x the area to scan).  The new
        // anchor set is the KA nearest within r, or -- when fewer than KA points lie within r -- ALL of them, with
        // D = r: every other snapshot point is then farther than r, which is all the anchor test needs.
        float r_s;
        if (DENSE) {
            const int cx = min(max(cell_coord(q.x, g.ox, g.inv_h), 0), g.dx - 1);
            const int cy = min(max(cell_coord(q.y, g.oy, g.inv_h), 0), g.dy - 1);
            const int cz = min(max(cell_coord(q.z, g.oz, g.inv_h), 0), g.dz - 1);
            uint32_t s = 0, e = 0;
            const int n = cell_range(g, cx, cy, cz, s, e) ? (int)(e - s) : 1;
            r_s = r_scale * g.h * cbrtf(16.f / (float)n);
        } else {
            const float4 a = anc[i];
            if (!(a.w > 0.f)) {                       // no anchor: the wave search grows its own box
                if (lane == 0) spill[atomicAdd(spill_cnt, 1u)] = (int32_t)i;
                continue;
            }
            r_s = a.w * PCD_RQ_RSCALE;
        }
        unsigned long long cap = 0;
        int cnt = 0;
        bool big = false, ok = false;
        // a radius holding at most kstore points is widened (x 1.6, twice) before the query spills
#pragma unroll 1
        for (int attempt = 0; attempt < 3; ++attempt) {
            if (attempt > 0) r_s *= 1.6f;
            cap = ((unsigned long long)__float_as_uint(r_s * r_s) << 32) | 0xFFFFFFFFull;
            const float rr = r_s * 1.0001f + 1e-30f;
            int lo[3], hi[3];
            cell_box(g, q, rr, lo, hi);
            cnt = 0;
            const int64_t nbox = (int64_t)(hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1);
            big = nbox > kRqMaxCells;
            if (big) break;
            const bool clean = rq_scan_box<KA>(g, q, lo, hi, cap, buf, cnt, &s_cells[wv], lane);
            ok = clean && cnt > kstore;
            if (ok || !clean) break;
            wave_sync();
        }
        const bool partial = cnt < KA;               // (after a buffer cut cnt == KA)
        uint32_t k = 0xFFFFFFFFu;
        if (ok) {
            uint32_t after;
            (void)rq_shrink<KA>(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), lane);
            k = wave_order32(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), lane, after);
            // exact order of the stored list (first kstore + its successor) and of the anchor set boundary
            ok = order_exact(k, after, kstore, lane);
            const uint32_t kK = KA < 64 ? (uint32_t)__shfl((int)k, KA < 64 ? KA : 0) : after;  // element KA
            const uint32_t kK1 = (uint32_t)__shfl((int)k, KA - 1);
            ok = ok && (cnt <= KA || (kK >> 8) != (kK1 >> 8));
        }
        if (!ok) {
            wave_sync();
            if (lane == 0) {
                spill[atomicAdd(spill_cnt, 1u)] = (int32_t)i;
                atomicAdd(big ? spill_cnt + 1 : spill_cnt + 2, 1u);   // RqStats::spill_big / spill_amb
            }
            continue;
        }
        const bool have = lane < KA && lane < cnt;
        const unsigned long long mine = have ? buf[k & 255u] : 0ull;
        // unused slots of a partial set hold -1 (the anchor test gives them an infinite distance)
        const int32_t r = have ? (int32_t)(uint32_t)(mine & 0xFFFFFFFFull) : -1;
#if defined(PCD_EXP_RQ_WRITE) && PCD_EXP_RQ_WRITE == 1      // timing experiment: no list writes (results wrong)
        if (r == -12345) alist[i] = r;
#elif defined(PCD_EXP_RQ_WRITE) && PCD_EXP_RQ_WRITE == 2    // timing experiment: contiguous writes (results wrong)
        if (lane < KA) alist[t0 * 64 + lane] = r;
#else
        if (lane < KA) alist[(int64_t)lane * N + i] = r;
        if (lane < kstore) idx[(int64_t)lane * N + i] = r;
#endif
        // D: the KA-th distance = the largest exact d² of the anchor set (quantised ties inside it are harmless); for
        // a partial set, r (rounded down: a point outside has fp32 d² > r², true distance > r (1 - 1e-7))
        const unsigned long long mx = wave_max_u64(mine);
        const float D = partial ? r_s * (1.f - 1e-6f) : sqrtf(__uint_as_float((unsigned)(mx >> 32)));
        if (lane == 0) anc[i] = make_float4(q.x, q.y, q.z, D);
        wave_sync();                                  // buf is free for the next query
    }
}

}  // namespace pcd
