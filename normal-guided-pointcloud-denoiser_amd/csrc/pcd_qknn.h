// Re-anchoring search of the anchored kNN (denoise.hip): the exact KA nearest snapshot points of a moved query
// within a radius, one query per group of W lanes (two per wave at W = 32), lean enough for 8 waves per SIMD.
//
// The search is the one of pcd_wknn.h (cap box -> brick probes -> flattened candidate rows -> ballot-appended
// survivors below the acceptance cap), re-cut for occupancy and VALU:
//   * the query (row, position, anchor) is wave-uniform and lives in SGPRs (readfirstlane + scalar loads);
//   * the survivors stay exact 64-bit keys (d² bits << 32 | snapshot rank) in the wave's LDS buffer, but they are
//     ORDERED by 32-bit keys floor(d² · 2^24 / cap d²) << 8 | buffer slot: a compare-exchange is one min + one max
//     on one register and one cross-lane move, where the exact keys need two registers, two moves, a 64-bit compare
//     and four selects (the sort was ~65 % of the old kernel's VALU).  The quantised order is the exact order
//     wherever neighbouring quantised values differ; a query whose stored list (first kstore + 1) has two equal
//     quantised values at a decision point is SPILLED to the exact-key wave search (k_knn_redo_wave), so the lists
//     stay bit-identical to it;
//   * the anchor set is not ordered: with more than KA survivors it is every survivor under an exact d² bound found
//     by a few ballot-counted interpolation steps (rq_bound), kept in the scan's order;
//   * a full buffer is cut to the KA best the same way (the cap tightens to the largest kept exact key + 1).
// The first iteration (no anchors yet, k_knn_dense_q): the radius is r_scale · h · (16 / n)^(1/3), n = occupancy of
// the query's cell; a query with too few points inside it is widened, then spilled (the wave search grows its own box).
#pragma once
#include "pcd_lists.h"
#include "pcd_wknn.h"

namespace pcd {

// Acceptance cap for re-anchoring at q: the KA anchor points are within D of a, hence within D + |q - a| of q, so
// the KA-th key at q is below this bound (rounding margin included).
PCD_DEV unsigned long long anchor_cap(Vec3 q, float4 a) {
    const float R = (a.w + sqrtf(sq3(q - v3(a.x, a.y, a.z)))) * (1.f + 1e-5f) + 1e-30f;
    const float R2 = R * R * (1.f + 1e-5f);
    return ((unsigned long long)__float_as_uint(R2) << 32) | 0xFFFFFFFFull;
}

// Lane groups: W = 64 (one query per wave) or W = 32 (two queries per wave, one per half).  The search is a chain
// of dependent memory round trips (query -> brick probes -> brick blocks -> candidate rows) with little VALU in
// between (12 % VALU-active, 68 % of wave cycles waiting at 8 waves/SIMD), so two queries per wave keep twice as many
// chains in flight for the same wave slots; the shuffles below stay inside a group (width-W shuffles) and the
// ballots are masked to the group's bits.
template <int W>
struct LaneGrp {
    int lane, hl, base;        // hl: lane inside the group; base: the group's first lane
    PCD_DEV LaneGrp(int l) : lane(l), hl(l & (W - 1)), base(l & ~(W - 1)) {}
    PCD_DEV unsigned long long bits(unsigned long long m) const {
        return W == 64 ? m : (m >> base) & 0xFFFFFFFFull;
    }
    PCD_DEV unsigned long long ballot(bool p) const { return bits(__ballot(p)); }
    PCD_DEV bool any(bool p) const { return ballot(p) != 0ull; }
    PCD_DEV int below() const { return hl; }
    PCD_DEV uint32_t bcast(uint32_t v, int src) const { return (uint32_t)__shfl((int)v, src, W); }
    PCD_DEV unsigned long long bcast64(unsigned long long v, int src) const {
        return (unsigned long long)bcast((uint32_t)v, src) | ((unsigned long long)bcast((uint32_t)(v >> 32), src) << 32);
    }
};

// Ascending bitonic sort of the W*M 32-bit keys v[s] (element e = s*W + hl) across the group.
template <int W, int M>
PCD_DEV void grp_bitonic_sort32(uint32_t (&v)[M], int hl) {
    constexpr int NT = W * M;
#pragma unroll
    for (int size = 2; size <= NT; size <<= 1) {
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1) {
            if (stride >= W) {
                const int ss = stride / W;
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    if ((s & ss) == 0) {
                        const bool asc = ((s * W + hl) & size) == 0;
                        const uint32_t a = v[s], b = v[s + ss];
                        const uint32_t mn = min(a, b), mx = max(a, b);
                        v[s] = asc ? mn : mx;
                        v[s + ss] = asc ? mx : mn;
                    }
                }
            } else {
                const bool lower = (hl & stride) == 0;
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    const bool asc = ((s * W + hl) & size) == 0;
                    const uint32_t o = lane_xor(v[s], stride);   // stride < W: stays inside the group
                    v[s] = (lower == asc) ? min(o, v[s]) : max(o, v[s]);
                }
            }
        }
    }
}

#ifndef PCD_RQ_ROWS
#define PCD_RQ_ROWS 2
#endif
static constexpr int kRqRows = PCD_RQ_ROWS;   // candidate rows per lane per round (all loads in flight)
// Survivors per group: room for 2W (W = 64; 4W at W = 32) before a cut plus one round of appends (W * kRqRows).
template <int W> struct RqSurv { static constexpr int n = W == 64 ? 64 * (2 + kRqRows) : 32 * (4 + kRqRows); };

// The quantised order of the survivors buf[0..cnt) (cnt <= RqSurv): element e lives in slot e / W of lane e % W;
// o.s0 / o.s1 = this lane's elements hl and W + hl (0xFFFFFFFF past cnt), o.at(e) broadcasts element e.
template <int W>
struct GrpOrder {
    uint32_t s0, s1, s2_0;     // slot 0, slot 1 of this lane; element 2W (slot 2, lane 0)
    const LaneGrp<W>* g;
    PCD_DEV uint32_t at(int e) const {   // e < 2W + 1
        if (e >= 2 * W) return s2_0;
        return e < W ? g->bcast(s0, e) : g->bcast(s1, e - W);
    }
};
// MS: the most slots a caller's set can fill (cnt <= MS * W; 1 or 2 drop the larger networks from the code)
template <int W, int MS = 4>
PCD_DEV GrpOrder<W> grp_order32(const unsigned long long* buf, int cnt, float capd2, const LaneGrp<W>& g) {
    wave_sync();
    const float S = 16777216.f / fmaxf(capd2, 1e-30f);
    auto k32 = [&](int e) -> uint32_t {
        if (e >= cnt) return 0xFFFFFFFFu;
        const float d2 = __uint_as_float((uint32_t)(buf[e] >> 32));
        return ((uint32_t)fminf(d2 * S, 16777214.f) << 8) | (uint32_t)e;
    };
    const int hl = g.hl;
    GrpOrder<W> o{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, &g};
    if (MS == 1 || cnt <= W) {
        uint32_t v[1] = {k32(hl)};
        grp_bitonic_sort32<W, 1>(v, hl);
        o.s0 = v[0];
    } else if (MS == 2 || cnt <= 2 * W) {
        uint32_t v[2] = {k32(hl), k32(W + hl)};
        grp_bitonic_sort32<W, 2>(v, hl);
        o.s0 = v[0]; o.s1 = v[1];
    } else {                                 // cnt <= 4W (callers spill a larger set that did not shrink)
        uint32_t v[4] = {k32(hl), k32(W + hl), k32(2 * W + hl), k32(3 * W + hl)};
        grp_bitonic_sort32<W, 4>(v, hl);
        o.s0 = v[0]; o.s1 = v[1]; o.s2_0 = g.bcast(v[2], 0);
    }
    return o;
}

// Do the first n elements of the quantised order hold their exact order and the set boundary after element
// n-1?  Exact iff every quantised value among elements 0..n (n+1 elements) is distinct, i.e. no two neighbours
// in 0..n share one (a pad compares larger than every real key).  n <= W.
template <int W>
PCD_DEV bool order_exact(const GrpOrder<W>& o, int n, const LaneGrp<W>& g) {
    const uint32_t k = o.s0;
    const uint32_t aw = o.at(W);                      // (a shuffle: every lane of the group executes it)
    const uint32_t dn = (uint32_t)__shfl_down((int)k, 1, W);
    const uint32_t nxt = g.hl == W - 1 ? aw : dn;
    const bool tie = g.hl < n && (k >> 8) == (nxt >> 8) && k != 0xFFFFFFFFu;
    return !g.any(tie);
}

template <int W>
PCD_DEV unsigned long long grp_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) {
        const unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
        const unsigned long long w = (unsigned long long)lane_xor(lo, o) | ((unsigned long long)lane_xor(hi, o) << 32);
        v = w > v ? w : v;
    }
    return v;
}

PCD_DEV uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// Shrink a survivor set of more than 128 to at most 128 before ordering it: a few bisection steps on d² find a
// bound with KA <= count(d² <= bound) <= 128; the keys under it contain the KA best of the whole set (at least KA
// keys are under it), so the compaction never changes the result.
template <int KA, int W>
PCD_DEV float rq_shrink(unsigned long long* buf, int& cnt, float capd2, const LaneGrp<W>& g) {
    constexpr int SL = RqSurv<W>::n / W;   // slots per lane
    if (cnt <= 128) return -1.f;
    wave_sync();
    float d[SL];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        const int e = s * W + g.hl;
        d[s] = e < cnt ? __uint_as_float((uint32_t)(buf[e] >> 32)) : 3.0e38f;
    }
    auto count_le = [&](float t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < SL; ++s) c += __popcll(g.ballot(d[s] <= t));
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
    unsigned long long keep[SL];
    int base = 0;
#pragma unroll
    for (int s = 0; s < SL; ++s) keep[s] = (s * W + g.hl) < cnt ? buf[s * W + g.hl] : 0ull;
    wave_sync();
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        const bool in = d[s] <= bound;
        const unsigned long long m = g.ballot(in);
        if (in) buf[base + __popcll(m & ((1ull << g.hl) - 1ull))] = keep[s];
        base += __popcll(m);
    }
    cnt = base;
    return bound;
}

// The anchor set of a query with more than KA survivors, without ordering them: the largest bound b (a d²) found with
// count(d² <= b) <= KA, by interpolation steps on [0, capd2) (survivor d² is near-uniform there: the count grows
// with the area of the ball).  buf is compacted to the members d² <= b, in buffer order, and cnt set to their
// count.  Every other snapshot point has fp32 d² > b, so sqrtf(b) is the set's D.  Returns false, buf untouched,
// when no bound holding `need`..KA members was found (equal distances crowding the boundary: the query spills).
template <int KA, int W>
PCD_DEV bool rq_bound(unsigned long long* buf, int& cnt, float capd2, int need, float& b, const LaneGrp<W>& g) {
    constexpr int SL = RqSurv<W>::n / W;   // slots per lane
    wave_sync();
    float d[SL];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        const int e = s * W + g.hl;
        d[s] = e < cnt ? __uint_as_float((uint32_t)(buf[e] >> 32)) : 3.0e38f;
    }
    auto count_le = [&](float t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < SL; ++s)
            if (s * W < cnt) c += __popcll(g.ballot(d[s] <= t));
        return c;
    };
    float lo = 0.f, hi = capd2;
    int clo = 0, chi = cnt, best = -1;   // (clo: a model value until lo is measured)
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        const float f = fminf(fmaxf(((float)KA + 0.5f - (float)clo) * __builtin_amdgcn_rcpf((float)max(chi - clo, 1)),
                                    0.0625f), 0.9375f);   // (a guess: the estimate reciprocal is enough)
        const float mid = lo + (hi - lo) * f;
        const int c = count_le(mid);
        if (c <= KA) {
            lo = mid; clo = c; best = c;
            if (c == KA) break;
        } else {
            hi = mid; chi = c;
        }
    }
    if (best < need) return false;
    b = lo;
    // in-place compaction, a slot at a time: slot s's members land below (s + 1) W, never on a later slot's keys,
    // and each slot's keys are in registers before its writes
    const unsigned long long below = (1ull << g.hl) - 1ull;
    int base = 0;
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        if (s * W >= cnt) break;
        const bool in = d[s] <= lo;
        const unsigned long long m = g.ballot(in);
        const unsigned long long key = in ? buf[s * W + g.hl] : 0ull;
        wave_sync();
        if (in) buf[base + __popcll(m & below)] = key;
        base += __popcll(m);
    }
    cnt = base;
    return true;
}

// Cut the survivors to the K best (quantised order; K <= 2W): false when the cut is ambiguous (the query spills).
template <int K, int W>
PCD_DEV bool rq_cut(unsigned long long* buf, int& cnt, unsigned long long& cap, const LaneGrp<W>& g) {
    static_assert(K <= 2 * W, "the K best fit two slots of the group");
    {
        const float bound = rq_shrink<K, W>(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), g);
        if (bound >= 0.f) {                           // >= K keys have d² <= bound: a valid, tighter cap
            const unsigned long long c2 = ((unsigned long long)__float_as_uint(bound) << 32) | 0xFFFFFFFFull;
            if (c2 < cap) cap = c2;
            return true;
        }
    }
    if (cnt > 4 * W) return false;                    // did not shrink (W = 32: more than 128 survivors)
    const GrpOrder<W> o = grp_order32<W>(buf, cnt, __uint_as_float((unsigned)(cap >> 32)), g);
    if ((o.at(K) >> 8) == (o.at(K - 1) >> 8)) return false;
    const bool h0 = g.hl < K, h1 = W + g.hl < K;
    const unsigned long long m0 = h0 ? buf[o.s0 & 255u] : 0ull;
    const unsigned long long m1 = h1 ? buf[o.s1 & 255u] : 0ull;
    wave_sync();
    if (h0) buf[g.hl] = m0;
    if (h1) buf[W + g.hl] = m1;
    wave_sync();
    const unsigned long long mx = grp_max_u64<W>(m0 > m1 ? m0 : m1);
    if (mx + 1ull < cap) cap = mx + 1ull;
    cnt = K;
    return true;
}

// Scan the cells of box [lo, hi] (at most kRqMaxCells) appending keys < cap to buf: pcd_wknn.h wave_scan_box
// in 32-bit cell arithmetic, with the quantised buffer cut, for one lane group.  Returns false when a cut was
// ambiguous (spill).
static constexpr int kRqMaxCells = 4096;
#ifndef PCD_RQ_CELLS
#define PCD_RQ_CELLS 64
#endif
static constexpr int kRqChunk = PCD_RQ_CELLS;  // cells per chunk (per group)
template <int W> struct RqCPL { static constexpr int n = kRqChunk / W; };   // cells per lane per chunk
static constexpr int kRqChunkLog2 = kRqChunk == 64 ? 6 : kRqChunk == 128 ? 7 : 8;
// A chunk's flattened candidate rows mapped to their snapshot rows in LDS, so a row costs one LDS read (round 6; it
// was the row's cell slot, a byte, then that cell's start and offset: three dependent reads).  A chunk with more
// flattened rows than the map holds finds each row's cell by a binary search over the chunk instead.
static constexpr int kRqRowMap = 512;
struct RqCells {            // per-group LDS scratch for one chunk of cells
    uint32_t start[kRqChunk];
    uint32_t end_incl[kRqChunk];
    uint32_t rowof[kRqRowMap];   // snapshot row of each flattened candidate row
};
PCD_DEV void fill_rowof(uint32_t* rowof, uint32_t b, uint32_t e, uint32_t s) {
    for (uint32_t k = b; k < e; ++k) rowof[k] = s + (k - b);
}
// Where a scan reads its cells and candidate rows from: GridSrc is the grid in global memory (brick hash probes,
// brick cell blocks, snapshot rows; a row's rank is its index).  A source only has to resolve a lane's cells to row
// ranges, load a row with its rank, and say whether it covers a cell box (an LDS-staged brick neighbourhood was
// measured this way: DESIGN §3).
struct GridSrc {
    const GridView* g;
    template <int CPL>
    PCD_DEV void ranges(const int (&cx)[CPL], const int (&cy)[CPL], const int (&cz)[CPL], const bool (&on)[CPL],
                        uint2 (&cr)[CPL]) const {
        uint32_t slot[CPL], loc6[CPL];
        unsigned long long bkey[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            slot[u] = ~0u; loc6[u] = 0; bkey[u] = kEmptyKey;
            if (on[u]) {
                const unsigned long long key = morton3(cx[u], cy[u], cz[u]);
                bkey[u] = key >> 6;
                loc6[u] = (uint32_t)(key & 63);
                slot[u] = (uint32_t)hash_slot(bkey[u], g->hbits);
            }
        }
        uint4 sl[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u)
            sl[u] = slot[u] != ~0u ? *reinterpret_cast<const uint4*>(g->table + slot[u]) : make_uint4(~0u, ~0u, 0u, 0u);
        uint32_t brick[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            brick[u] = ~0u;
            if (slot[u] == ~0u) continue;
            uint4 e = sl[u];
            uint32_t sidx = slot[u];
            for (;;) {
                const unsigned long long k2 = (unsigned long long)e.x | ((unsigned long long)e.y << 32);
                if (k2 == bkey[u]) { brick[u] = e.z; break; }
                if (k2 == kEmptyKey) break;
                sidx = (uint32_t)((sidx + 1) & g->mask);
                e = *reinterpret_cast<const uint4*>(g->table + sidx);
            }
        }
#pragma unroll
        for (int u = 0; u < CPL; ++u)
            cr[u] = brick[u] != ~0u ? g->cells[(uint64_t)brick[u] * 64 + loc6[u]] : make_uint2(0u, 0u);
    }
    PCD_DEV void row(uint32_t r, float& x, float& y, float& z, uint32_t& rank) const {
        const float* pp = reinterpret_cast<const float*>(g->pts + r);
        x = pp[0]; y = pp[1]; z = pp[2]; rank = r;
    }
    PCD_DEV bool covers(const int (&)[3], const int (&)[3]) const { return true; }
};

// Scan the cells of box [lo, hi] (at most kRqMaxCells) appending keys < cap to buf: pcd_wknn.h wave_scan_box
// in 32-bit cell arithmetic, with the quantised buffer cut, for one lane group.  Returns false when a cut was
// ambiguous (spill).
template <int K, int W, class Src>
PCD_DEV bool rq_scan_box(const GridView& g, const Src& src, Vec3 q, const int lo[3], const int hi[3],
                         unsigned long long& cap, unsigned long long* buf, int& cnt, RqCells* wc, const LaneGrp<W>& lg) {
    constexpr int CPL = RqCPL<W>::n;
    static_assert(CPL >= 1 && CPL * W == kRqChunk, "chunk = whole cells per lane");
    static_assert(K + W * kRqRows <= RqSurv<W>::n, "a cut to K plus one round of appends must fit the buffer");
    const int hl = lg.hl;
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1;
    const int nc = ex * ey * (hi[2] - lo[2] + 1);
    const uint32_t exy = (uint32_t)ex * (uint32_t)ey;
    for (int base = 0; base < nc; base += kRqChunk) {
        int cxs[CPL], cys[CPL], czs[CPL];
        bool on[CPL];
        const float kth = __uint_as_float((unsigned)(cap >> 32));
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const uint32_t ci = (uint32_t)(base + hl * CPL + u);
            on[u] = false; cxs[u] = cys[u] = czs[u] = 0;
            if (ci < (uint32_t)nc) {
                const uint32_t zq = ci / exy, rem = ci - zq * exy, yq = rem / (uint32_t)ex;
                const int cx = lo[0] + (int)(rem - yq * (uint32_t)ex), cy = lo[1] + (int)yq, cz = lo[2] + (int)zq;
                const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
                const float gx = axis_gap(q.x, lx, lx + g.h), gy = axis_gap(q.y, ly, ly + g.h), gz = axis_gap(q.z, lz, lz + g.h);
                on[u] = gx * gx + gy * gy + gz * gz <= kth * 1.00001f + 1e-30f;
                cxs[u] = cx; cys[u] = cy; czs[u] = cz;
            }
        }
        uint2 cr[CPL];
        src.template ranges<CPL>(cxs, cys, czs, on, cr);
        uint32_t loc[CPL], run = 0;
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            run += cr[u].y > cr[u].x ? cr[u].y - cr[u].x : 0u;
            loc[u] = run;
        }
        const uint32_t incl = lane_scan_incl<W>(run);
        const uint32_t total = lg.bcast(incl, W - 1);
        if (total == 0) continue;
        const uint32_t excl = incl - run;
        wave_sync();
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            wc->start[hl * CPL + u] = cr[u].x;
            wc->end_incl[hl * CPL + u] = excl + loc[u];
        }
        // the cell of every flattened row, so a row finds its cell with one LDS read instead of a binary search over
        // the chunk (~40 VALU per row): each lane fills the runs of its own cells
        const bool mapped = total <= (uint32_t)kRqRowMap;   // (group-uniform)
        if (mapped) {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
                fill_rowof(wc->rowof, excl + (u ? loc[u - 1] : 0u), excl + loc[u], cr[u].x);
        }
        wave_sync();
        for (uint32_t j0 = 0; j0 < total; j0 += W * kRqRows) {
            // room for a whole round of appends (one cut site: the sort network is inlined once)
            if (cnt > RqSurv<W>::n - W * kRqRows && !rq_cut<K, W>(buf, cnt, cap, lg)) return false;
            uint32_t r[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * W + hl);
                if (mapped) {
                    r[u] = j < total ? wc->rowof[j] : 0u;
                    continue;
                }
                int a = 0, b = kRqChunk - 1;
#pragma unroll
                for (int it = 0; it < kRqChunkLog2; ++it) {
                    const int m = (a + b) >> 1;
                    if (wc->end_incl[m] > j) b = m; else a = m + 1;
                }
                r[u] = j < total ? wc->start[a] + (j - (a ? wc->end_incl[a - 1] : 0u)) : 0u;
            }
            float px[kRqRows], py[kRqRows], pz[kRqRows];
            uint32_t rk[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                if (j0 + (uint32_t)(u * W) < total) src.row(r[u], px[u], py[u], pz[u], rk[u]);
            }
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * W + hl);
                if (j0 + (uint32_t)(u * W) < total) {
                    const unsigned long long key2 =
                        ((unsigned long long)__float_as_uint(dist2(q, make_float4(px[u], py[u], pz[u], 0.f))) << 32) | rk[u];
                    const bool pass = j < total && key2 < cap;
                    const unsigned long long m = lg.ballot(pass);
                    if (pass) buf[cnt + __popcll(m & ((1ull << hl) - 1ull))] = key2;
                    cnt += __popcll(m);
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
#define PCD_RQ_RSCALE 1.02f  // re-anchoring radius / the old anchor's D (A/B at 10M: 1.0 / 1.02 / 1.05 / 1.1 / 1.2 -> 5.35 / 5.35 / 5.38 / 5.44 / 5.58 ms per iteration; 1.0 loses on the long run)
#endif
#ifndef PCD_RQ_OCC
#define PCD_RQ_OCC 8
#endif
// The end of a re-anchoring query once its survivors are in buf[0..cnt) under cap: the exact order checks, then the
// stored list, the anchor set (scan order) and the anchor -- or the spill list when a check fails (ok = false on
// entry: the scan was ambiguous or found too few points).
template <int KA, int W>
PCD_DEV void rq_finish(int64_t i, Vec3 q, float r_s, int64_t N, int kstore, float4* __restrict__ anc,
                       int32_t* __restrict__ alist, int32_t* __restrict__ idx, int32_t* __restrict__ spill,
                       unsigned* __restrict__ spill_cnt, unsigned long long* buf, int cnt, unsigned long long cap,
                       bool ok, bool big, const LaneGrp<W>& lg) {
    const bool partial = cnt < KA;               // (after a buffer cut cnt == KA)
    GrpOrder<W> o{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, &lg};
    float capd2 = __uint_as_float((unsigned)(cap >> 32)), b = -1.f;
    const bool bounded = ok && cnt > KA;
    // more than KA survivors: the set is every survivor under a bound (rq_bound), so only the <= KA members are
    // ordered, for the stored list
    if (bounded) ok = rq_bound<KA, W>(buf, cnt, capd2, kstore + 1, b, lg);
    if (ok) {
        o = grp_order32<W, (KA + W - 1) / W>(buf, cnt, bounded ? b : capd2, lg);   // (cnt <= KA here)
        // exact order of the stored list (first kstore + its successor)
        ok = order_exact<W>(o, kstore, lg);
    }
    if (!ok) {
        wave_sync();
        if (lg.hl == 0) {
            spill[atomicAdd(spill_cnt, 1u)] = (int32_t)i;
            atomicAdd(big ? spill_cnt + 1 : spill_cnt + 2, 1u);   // RqStats::spill_big / spill_amb
        }
        return;
    }
    // the stored list: the first kstore of the order, whole 32-B sectors of the blocked list layout (pcd_lists.h):
    // lanes 8b .. 8b+7 fill block b of row i
    const int e0 = lg.hl, e1 = W + lg.hl;
    if (e0 < kstore) idx[lpos(N, i, e0)] = (int32_t)(uint32_t)(buf[o.s0 & 255u] & 0xFFFFFFFFull);
    if (e1 < kstore) idx[lpos(N, i, e1)] = (int32_t)(uint32_t)(buf[o.s1 & 255u] & 0xFFFFFFFFull);
    // the anchor set: every survivor left in buf (cnt <= KA), in BUFFER order, i.e. the scan's: cells in (z, y, x)
    // order of the box, ranks ascending inside a cell -- one global order, so neighbouring rows (neighbouring lanes
    // of the anchor test's waves) hold mostly the same snapshot rows at the same slot and gather the same cache
    // lines.  (It was rank order, by a 64-key sort here; the anchor test ranks the set by distance itself.)  Unused
    // slots of a partial set hold N, the snapshot's +inf sentinel row (the anchor test gives them an infinite
    // distance).
    const unsigned long long m0 = e0 < cnt ? buf[e0] : 0ull, m1 = e1 < cnt ? buf[e1] : 0ull;
    if (e0 < KA) alist[lpos(N, i, e0)] = e0 < cnt ? (int32_t)(uint32_t)(m0 & 0xFFFFFFFFull) : (int32_t)N;
    if (e1 < KA) alist[lpos(N, i, e1)] = e1 < cnt ? (int32_t)(uint32_t)(m1 & 0xFFFFFFFFull) : (int32_t)N;
    // D: every snapshot point outside the set is at least D from q.  Bounded set: sqrtf(b) (rq_bound); a partial
    // set: r (rounded down: a point outside has fp32 d² > r², true distance > r (1 - 1e-7)); exactly KA survivors
    // (a buffer cut's, or the ball's own): the largest exact d² of the set (an outside point's 64-bit key is larger)
    float D;
    if (bounded) D = sqrtf(b);
    else if (partial) D = r_s * (1.f - 1e-6f);
    else D = sqrtf(__uint_as_float((unsigned)(grp_max_u64<W>(m0 > m1 ? m0 : m1) >> 32)));
    if (lg.hl == 0) anc[i] = make_float4(q.x, q.y, q.z, D);
}

// One re-anchoring query (the rows of a lane group; q, i uniform in the group): the exact anchor set within radius
// r_s (widened x 1.6 up to twice while it holds at most kstore points), the stored list, the new anchor.  Spills an
// ambiguous or oversized query to the exact-key wave search.  Returns false, having written nothing, when a box
// leaves what `src` covers (StagedSrc: the caller hands the query to the global-memory pass).
template <int KA, int W, class Src>
PCD_DEV bool rq_query(const GridView& g, const Src& src, int64_t i, Vec3 q, float r_s, int64_t N, int kstore,
                      float4* __restrict__ anc, int32_t* __restrict__ alist, int32_t* __restrict__ idx,
                      int32_t* __restrict__ spill, unsigned* __restrict__ spill_cnt, unsigned long long* buf,
                      RqCells* wc, const LaneGrp<W>& lg) {
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
        if (!src.covers(lo, hi)) return false;    // (block-uniform per query: every lane of the group)
        const bool clean = rq_scan_box<KA, W>(g, src, q, lo, hi, cap, buf, cnt, wc, lg);
        ok = clean && cnt > kstore;
        if (ok || !clean) break;
        wave_sync();
    }
    rq_finish<KA, W>(i, q, r_s, N, kstore, anc, alist, idx, spill, spill_cnt, buf, cnt, cap, ok, big, lg);
    return true;
}

// The steady re-anchoring: one query per wave (grid-stride) over the rows of `list` (the anchor test's failures,
// radius from the old anchor).  Spilled rows go to `spill` for k_knn_redo_wave.  (Two queries per wave, in 32-lane
// groups or sharing one scan, measured equal or slower: DESIGN.md §3.)
template <int KA, int W = 64>
__global__ __launch_bounds__(256, PCD_RQ_OCC) void k_knn_requery(GridView g, const float4* __restrict__ pos,
                                                                 int64_t N, RowMap rm, int kstore,
                                                                 float4* __restrict__ anc, int32_t* __restrict__ alist,
                                                                 int32_t* __restrict__ idx,
                                                                 const int32_t* __restrict__ list,
                                                                 const unsigned* __restrict__ list_cnt,
                                                                 int32_t* __restrict__ spill,
                                                                 unsigned* __restrict__ spill_cnt) {
    static_assert(KA <= 2 * W && KA <= 64, "the anchor set fits two slots of the group");
    constexpr int G = 64 / W;                    // groups (queries in flight) per wave
    __shared__ unsigned long long s_buf[4 * G][RqSurv<W>::n];
    __shared__ RqCells s_cells[4 * G];
    const int lane = (int)(threadIdx.x & 63);
    const LaneGrp<W> lg(lane);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int gid = wv * G + lane / W;           // group in the block
    (void)rm;
    const int64_t cnt_rows = (int64_t)*list_cnt;
    const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
    unsigned long long* buf = s_buf[gid];
    for (int64_t t0 = lb * 4 * G + gid; t0 < cnt_rows; t0 += (int64_t)gridDim.x * 4 * G) {
        int64_t i = (int64_t)list[t0];
        if (W == 64) i = (int64_t)rfl((uint32_t)i);
        const float4 p4 = pos[i];
        const Vec3 q = v3(p4.x, p4.y, p4.z);
        // The search radius r from the old anchor's D (the local KA-th distance; the cap (D + |q - a|)^2 that bounds
        // the KA-th key at q is ~2x the area to scan).  The new anchor set is the KA nearest within r, or -- when
        // fewer than KA points lie within r -- ALL of them, with D = r: every other snapshot point is then farther
        // than r, which is all the anchor test needs.
        const float4 a = anc[i];
        if (!(a.w > 0.f)) {                           // no anchor: the wave search grows its own box
            if (lg.hl == 0) spill[atomicAdd(spill_cnt, 1u)] = (int32_t)i;
            continue;
        }
        const float r_s = a.w * PCD_RQ_RSCALE;
        const bool done = rq_query<KA, W>(g, GridSrc{&g}, i, q, r_s, N, kstore, anc, alist, idx, spill, spill_cnt, buf,
                                          &s_cells[gid], lg);
        (void)done;                                   // (GridSrc covers every box)
        wave_sync();                                  // buf is free for the next query
    }
}

// ------------------------------------------------------------------ dense anchoring, Q queries per wave
// The first iteration re-anchors EVERY row (no anchors yet).  Consecutive rows are spatial neighbours (Morton order),
// so Q of them share one scan: the union of their boxes is resolved once (cell phase: hash probes, row ranges, the
// flattened row map) and every candidate row is loaded once, then tested against each query's own cap and appended
// to that query's survivor buffer.  Each query then finishes exactly as a single one (rq_finish): same survivors under
// the same cap, same checks, same writes.  A query whose own box is oversized, whose cut was ambiguous, or whose
// radius holds at most kstore points re-runs alone (rq_query, wider radius) -- the stored lists are exact either way.
template <int K, int Q, class Src>
PCD_DEV void rq_scan_box_q(const GridView& g, const Src& src, const Vec3 (&q)[Q], const bool (&act)[Q],
                           const int lo[3], const int hi[3], unsigned long long (&cap)[Q],
                           unsigned long long* const (&buf)[Q], int (&cnt)[Q], bool (&clean)[Q], RqCells* wc,
                           const LaneGrp<64>& lg) {
    constexpr int W = 64;
    constexpr int CPL = RqCPL<W>::n;
    const int hl = lg.hl;
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1;
    const int nc = ex * ey * (hi[2] - lo[2] + 1);
    const uint32_t exy = (uint32_t)ex * (uint32_t)ey;
    for (int base = 0; base < nc; base += kRqChunk) {
        int cxs[CPL], cys[CPL], czs[CPL];
        bool on[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const uint32_t ci = (uint32_t)(base + hl * CPL + u);
            on[u] = false; cxs[u] = cys[u] = czs[u] = 0;
            if (ci < (uint32_t)nc) {
                const uint32_t zq = ci / exy, rem = ci - zq * exy, yq = rem / (uint32_t)ex;
                const int cx = lo[0] + (int)(rem - yq * (uint32_t)ex), cy = lo[1] + (int)yq, cz = lo[2] + (int)zq;
                const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
#pragma unroll
                for (int j = 0; j < Q; ++j) {
                    const float gx = axis_gap(q[j].x, lx, lx + g.h), gy = axis_gap(q[j].y, ly, ly + g.h),
                                gz = axis_gap(q[j].z, lz, lz + g.h);
                    const float kth = __uint_as_float((unsigned)(cap[j] >> 32));
                    on[u] = on[u] || (act[j] && clean[j] && gx * gx + gy * gy + gz * gz <= kth * 1.00001f + 1e-30f);
                }
                cxs[u] = cx; cys[u] = cy; czs[u] = cz;
            }
        }
        uint2 cr[CPL];
        src.template ranges<CPL>(cxs, cys, czs, on, cr);
        uint32_t loc[CPL], run = 0;
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            run += cr[u].y > cr[u].x ? cr[u].y - cr[u].x : 0u;
            loc[u] = run;
        }
        const uint32_t incl = lane_scan_incl<W>(run);
        const uint32_t total = lg.bcast(incl, W - 1);
        if (total == 0) continue;
        const uint32_t excl = incl - run;
        wave_sync();
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            wc->start[hl * CPL + u] = cr[u].x;
            wc->end_incl[hl * CPL + u] = excl + loc[u];
        }
        const bool mapped = total <= (uint32_t)kRqRowMap;   // (group-uniform)
        if (mapped) {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
                fill_rowof(wc->rowof, excl + (u ? loc[u - 1] : 0u), excl + loc[u], cr[u].x);
        }
        wave_sync();
        for (uint32_t j0 = 0; j0 < total; j0 += W * kRqRows) {
#pragma unroll
            for (int j = 0; j < Q; ++j)
                if (clean[j] && cnt[j] > RqSurv<W>::n - W * kRqRows && !rq_cut<K, W>(buf[j], cnt[j], cap[j], lg))
                    clean[j] = false;                 // (this query re-runs alone)
            uint32_t r[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t jj = j0 + (uint32_t)(u * W + hl);
                if (mapped) {
                    r[u] = jj < total ? wc->rowof[jj] : 0u;
                    continue;
                }
                int a = 0, b = kRqChunk - 1;
#pragma unroll
                for (int it = 0; it < kRqChunkLog2; ++it) {
                    const int m = (a + b) >> 1;
                    if (wc->end_incl[m] > jj) b = m; else a = m + 1;
                }
                r[u] = jj < total ? wc->start[a] + (jj - (a ? wc->end_incl[a - 1] : 0u)) : 0u;
            }
            float px[kRqRows], py[kRqRows], pz[kRqRows];
            uint32_t rk[kRqRows];
#pragma unroll
            for (int u = 0; u < kRqRows; ++u)
                if (j0 + (uint32_t)(u * W) < total) src.row(r[u], px[u], py[u], pz[u], rk[u]);
#pragma unroll
            for (int u = 0; u < kRqRows; ++u) {
                const uint32_t jj = j0 + (uint32_t)(u * W + hl);
                if (j0 + (uint32_t)(u * W) < total) {
                    const float4 c4 = make_float4(px[u], py[u], pz[u], 0.f);
#pragma unroll
                    for (int j = 0; j < Q; ++j) {
                        const unsigned long long key2 =
                            ((unsigned long long)__float_as_uint(dist2(q[j], c4)) << 32) | rk[u];
                        const bool pass = jj < total && act[j] && clean[j] && key2 < cap[j];
                        const unsigned long long m = lg.ballot(pass);
                        if (pass) buf[j][cnt[j] + __popcll(m & ((1ull << hl) - 1ull))] = key2;
                        cnt[j] += __popcll(m);
                    }
                }
            }
        }
        wave_sync();
    }
}

#ifndef PCD_DENSE_Q
#define PCD_DENSE_Q 2        // queries per wave of the dense first anchoring (A/B at 10M: first iteration 23.6 / 21.8 / 25.4 ms at 1 / 2 / 4)
#endif
#ifndef PCD_DQ_OCC
#define PCD_DQ_OCC 6          // A/B at 10M: first iteration 21.7 / 20.7 / 21.3 ms at 4 (5 by VGPRs) / 6 / 7 waves per SIMD
#endif
// The dense radius of every active row, r_scale h (16 / n)^(1/3) with n the occupancy of the row's cell, one lane a
// row: the hash probe and the cube root leave the waves of k_knn_dense_q, where every query paid them at full wave
// width before its box was known (same float arithmetic: the same radius).
__global__ void k_dense_radius(GridView g, const float4* __restrict__ pos, RowMap rm, float r_scale,
                               float* __restrict__ out, uint4* __restrict__ box = nullptr) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= rm.nq) return;
    const float4 p4 = pos[rm(t)];
    const int cx = min(max(cell_coord(p4.x, g.ox, g.inv_h), 0), g.dx - 1);
    const int cy = min(max(cell_coord(p4.y, g.oy, g.inv_h), 0), g.dy - 1);
    const int cz = min(max(cell_coord(p4.z, g.oz, g.inv_h), 0), g.dz - 1);
    uint32_t s = 0, e = 0;
    const int n = cell_range(g, cx, cy, cz, s, e) ? (int)(e - s) : 1;
    const float rs = r_scale * g.h * cbrtf(16.f / (float)n);
    out[t] = rs;
    if (box) {   // and the query's cell box (cell_box at rs * 1.0001), 16 bits a coordinate; w = 1: not representable
        int lo[3], hi[3];
        cell_box(g, v3(p4.x, p4.y, p4.z), rs * 1.0001f + 1e-30f, lo, hi);
        const bool fits = hi[0] < 65536 && hi[1] < 65536 && hi[2] < 65536;
        box[t] = make_uint4((uint32_t)lo[0] | ((uint32_t)lo[1] << 16), (uint32_t)lo[2] | ((uint32_t)hi[0] << 16),
                            (uint32_t)hi[1] | ((uint32_t)hi[2] << 16), fits ? 0u : 1u);
    }
}

// rpre: every active row's radius (k_dense_radius); bpre (optional): its query box, else computed here.
template <int KA, int Q>
__global__ __launch_bounds__(256, PCD_DQ_OCC) void k_knn_dense_q(GridView g, const float4* __restrict__ pos, int64_t N,
                                                                RowMap rm, int kstore, float4* __restrict__ anc,
                                                                int32_t* __restrict__ alist, int32_t* __restrict__ idx,
                                                                int32_t* __restrict__ spill,
                                                                unsigned* __restrict__ spill_cnt,
                                                                const float* __restrict__ rpre,
                                                                const uint4* __restrict__ bpre) {
    constexpr int W = 64;
    __shared__ unsigned long long s_buf[4][Q][RqSurv<W>::n];
    __shared__ RqCells s_cells[4];
    const int lane = (int)(threadIdx.x & 63);
    const LaneGrp<W> lg(lane);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
    const int64_t nrows = rm.nq;
    for (int64_t t0 = (lb * 4 + wv) * Q; t0 < nrows; t0 += (int64_t)gridDim.x * 4 * Q) {
        int64_t iq[Q];
        Vec3 q[Q];
        float rs[Q];
        bool act[Q], clean[Q];
        unsigned long long cap[Q];
        int cnt[Q];
        unsigned long long* bufs[Q];
        int lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
        bool any_big = false;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            act[j] = t0 + j < nrows;
            const int64_t tj = act[j] ? t0 + j : t0;
            iq[j] = (int64_t)rfl((uint32_t)rm(tj));
            const float4 p4 = pos[iq[j]];
            q[j] = v3(p4.x, p4.y, p4.z);
            rs[j] = rpre[tj];                           // (k_dense_radius)
            cap[j] = ((unsigned long long)__float_as_uint(rs[j] * rs[j]) << 32) | 0xFFFFFFFFull;
            int l3[3], h3[3];
            uint4 bx = make_uint4(0u, 0u, 0u, 1u);
            if (bpre) bx = bpre[tj];                    // (k_dense_radius)
            if (bx.w == 0u) {
                l3[0] = (int)(bx.x & 0xFFFFu); l3[1] = (int)(bx.x >> 16); l3[2] = (int)(bx.y & 0xFFFFu);
                h3[0] = (int)(bx.y >> 16); h3[1] = (int)(bx.z & 0xFFFFu); h3[2] = (int)(bx.z >> 16);
            } else {
                cell_box(g, q[j], rs[j] * 1.0001f + 1e-30f, l3, h3);
            }
            const int64_t nbox = (int64_t)(h3[0] - l3[0] + 1) * (h3[1] - l3[1] + 1) * (h3[2] - l3[2] + 1);
            clean[j] = nbox <= kRqMaxCells;           // (an oversized box runs alone and spills there)
            any_big = any_big || (act[j] && !clean[j]);
            if (act[j] && clean[j])
                for (int a = 0; a < 3; ++a) { lo[a] = min(lo[a], l3[a]); hi[a] = max(hi[a], h3[a]); }
            cnt[j] = 0;
            bufs[j] = s_buf[wv][j];
        }
        const int64_t ubox = lo[0] <= hi[0] ? (int64_t)(hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1) : 0;
        if (ubox > 0 && ubox <= kRqMaxCells)
            rq_scan_box_q<KA, Q>(g, GridSrc{&g}, q, act, lo, hi, cap, bufs, cnt, clean, &s_cells[wv], lg);
        else
            for (int j = 0; j < Q; ++j) clean[j] = false;   // (the union is too wide: every query alone)
        (void)any_big;
        // the finishes one query at a time through ONE copy of the finish and of the lone re-run (not unrolled: the
        // query's state is picked by wave-uniform selects; half the kernel's code, measured neutral in time)
#pragma unroll 1
        for (int j = 0; j < Q; ++j) {
            bool aj = act[0], cj = clean[0];
            int64_t ij = iq[0];
            Vec3 qj = q[0];
            float rj = rs[0];
            int nj = cnt[0];
            unsigned long long capj = cap[0];
#pragma unroll
            for (int u = 1; u < Q; ++u)
                if (j == u) { aj = act[u]; cj = clean[u]; ij = iq[u]; qj = q[u]; rj = rs[u]; nj = cnt[u]; capj = cap[u]; }
            if (!aj) continue;
            unsigned long long* bj = s_buf[wv][j];
            if (cj && nj > kstore) {
                rq_finish<KA, W>(ij, qj, rj, N, kstore, anc, alist, idx, spill, spill_cnt, bj, nj, capj, true, false, lg);
            } else {
                // alone: its own box (an oversized one spills in there), the radius widened when too few were found
                wave_sync();
                (void)rq_query<KA, W>(g, GridSrc{&g}, ij, qj, cj ? rj * 1.6f : rj, N, kstore, anc, alist, idx, spill,
                                      spill_cnt, bj, &s_cells[wv], lg);
            }
            wave_sync();
        }
    }
}

}  // namespace pcd
