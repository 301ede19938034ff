// Wave-cooperative exact kNN: ONE query per wave64 (the re-anchoring search of the anchored kNN, denoise.hip).
//
// The lane-per-query searches (pcd_knn.h) keep a sorted top-K in each lane's registers; at K = 64 that list is 128
// VGPRs and every accepted candidate runs a 64-step select chain, so a sparse set of queries (the 1-3 % that fail
// the anchor test) runs at 2 waves/SIMD on long serial chains.  Here the 64 lanes split one query's work instead:
//   1. the cells of the box [q - r, q + r] (r = sqrt of the acceptance cap) are dealt 4 per lane, pruned by
//      box distance and probed in the brick hash in parallel (all probes of a chunk in flight together);
//   2. the chunk's candidate rows are flattened (count scan in LDS, binary-searched per row) and dealt kWaveRows
//      per lane per round, all
//      loads of a round in flight together; a key (d² bits << 32 | rank) below the cap is appended to the wave's
//      LDS survivor buffer with one ballot compaction per row slot;
//   3. the survivors (a few more than K when the cap is tight) are bitonic-sorted across the wave in registers
//      (4 keys per lane, slot-major: key e lives in lane e % 64, slot e / 64), so lane t ends with the t-th key.
// A full buffer is reduced in place (sort, keep the K best, tighten the cap), so any cap >= the true K-th key is
// exact; without a finite cap the search first runs over growing Chebyshev blocks to find one.
// Keys and their order are bit-identical to the lane searches: same fp32 (q-c)² and the same tie-break by rank.
#pragma once
#include "pcd_knn.h"

namespace pcd {

static constexpr int kWaveSurv = 256;   // survivor slots per wave (4 per lane)

PCD_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Cross-lane exchange with lane ^ s for a constant s (the unrolled sort / reduction networks): DPP moves for s <= 8
// (quad_perm, row half-mirror / mirror compositions) and the CDNA4 permlane16/32 swaps for 16 / 32 -- VALU-native,
// where __shfl_xor compiles to ds_bpermute (an LDS-crossbar round trip on every stage of a dependent network).
//   s = 4: quad_perm[3,2,1,0] (l^3) then row_half_mirror (l^7) -> l^4;   s = 8: half_mirror (l^7) then row_mirror (l^15)
PCD_DEV uint32_t lane_xor(uint32_t v, int s) {
    switch (s) {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
        case 4: {
            const int t = __builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);
            return (uint32_t)__builtin_amdgcn_mov_dpp(t, 0x141, 0xF, 0xF, false);
        }
        case 8: {
            const int t = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
            return (uint32_t)__builtin_amdgcn_mov_dpp(t, 0x140, 0xF, 0xF, false);
        }
        case 16: {   // swap odd rows of the first operand with even rows of the second
            const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (__lane_id() & 16) ? p[0] : p[1];
        }
        case 32: {   // swap the upper half of the first operand with the lower half of the second
            const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (__lane_id() & 32) ? p[0] : p[1];
        }
        default: return (uint32_t)__shfl_xor((int)v, s);
    }
}
PCD_DEV unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    return (unsigned long long)lane_xor((uint32_t)v, m) | ((unsigned long long)lane_xor((uint32_t)(v >> 32), m) << 32);
}
// Inclusive prefix sum over groups of W = 32 or 64 lanes (DPP row shifts inside rows of 16, then the row broadcasts).
template <int W>
PCD_DEV uint32_t lane_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    if (W == 64) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Ascending bitonic sort of the 64*M keys v[s] (element e = s*64 + lane) across the wave.
template <int M>
PCD_DEV void wave_bitonic_sort(unsigned long long (&v)[M], int lane) {
    constexpr int NT = 64 * M;
#pragma unroll
    for (int size = 2; size <= NT; size <<= 1) {
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1) {
            if (stride >= 64) {              // partner in another slot of the same lane
                const int ss = stride / 64;
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    if ((s & ss) == 0) {
                        const int e = s * 64 + lane;
                        const bool asc = (e & size) == 0;
                        unsigned long long& a = v[s];
                        unsigned long long& b = v[s + ss];
                        const bool sw = asc ? (b < a) : (a < b);
                        const unsigned long long lo = sw ? b : a;
                        b = sw ? a : b;
                        a = lo;
                    }
                }
            } else {                         // partner lane ^ stride, same slot
#pragma unroll
                for (int s = 0; s < M; ++s) {
                    const int e = s * 64 + lane;
                    const bool asc = (e & size) == 0;
                    const bool lower = (lane & stride) == 0;
                    const unsigned long long o = shfl_xor_u64(v[s], stride);
                    const unsigned long long mn = o < v[s] ? o : v[s];
                    const unsigned long long mx = o < v[s] ? v[s] : o;
                    v[s] = (lower == asc) ? mn : mx;
                }
            }
        }
    }
}

// Sort the cnt (<= kWaveSurv) survivors of buf; on return lane t's `top` is the t-th smallest key (kInfKey pad).
// If keep > 0, the keep smallest are written back to buf[0..keep) and the count returned.
PCD_DEV unsigned long long wave_sort_survivors(unsigned long long* buf, int cnt, int lane, int keep, int& kept) {
    wave_sync();                             // every lane's appends are visible
    unsigned long long top;
    if (cnt <= 64) {
        unsigned long long v[1] = {lane < cnt ? buf[lane] : kInfKey};
        wave_bitonic_sort<1>(v, lane);
        top = v[0];
    } else if (cnt <= 128) {
        unsigned long long v[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) v[s] = s * 64 + lane < cnt ? buf[s * 64 + lane] : kInfKey;
        wave_bitonic_sort<2>(v, lane);
        top = v[0];
    } else {
        unsigned long long v[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = s * 64 + lane < cnt ? buf[s * 64 + lane] : kInfKey;
        wave_bitonic_sort<4>(v, lane);
        top = v[0];
    }
    kept = 0;
    if (keep > 0) {
        wave_sync();
        const int n = cnt < keep ? cnt : keep;
        if (lane < n) buf[lane] = top;
        kept = n;
        wave_sync();
    }
    return top;
}

#ifndef PCD_WAVE_CPL
#define PCD_WAVE_CPL 2
#endif
static constexpr int kCellsPerLane = PCD_WAVE_CPL;      // cells per lane per chunk
static constexpr int kChunkCells = 64 * kCellsPerLane;  // cells per chunk
static constexpr int kChunkLog2 = kCellsPerLane == 1 ? 6 : kCellsPerLane == 2 ? 7 : kCellsPerLane == 4 ? 8 : 9;
struct WaveCells {          // per-wave LDS scratch for one chunk of cells
    uint32_t start[kChunkCells];
    uint32_t end_incl[kChunkCells];  // inclusive scan of the counts: flattened candidate end of each cell
};

// Append the keys < cap of one candidate row per lane to the wave's survivor buffer (one ballot compaction).
PCD_DEV void wave_append(bool pass, unsigned long long key, unsigned long long* buf, int& cnt, int lane) {
    const unsigned long long m = __ballot(pass);
    if (pass) buf[cnt + __popcll(m & ((1ull << lane) - 1ull))] = key;
    cnt += __popcll(m);
}

// Steps 3+ of a chunk: this lane's kCellsPerLane cell row ranges cr -> flattened candidate rows -> keys < cap
// appended to buf (a full buffer is cut to the K best and the cap tightened).
#ifndef PCD_WAVE_ROWS
#define PCD_WAVE_ROWS 4
#endif
static constexpr int kWaveRows = PCD_WAVE_ROWS;
template <int K>
PCD_DEV void wave_scan_chunk(const GridView& g, Vec3 q, const uint2 (&cr)[kCellsPerLane], unsigned long long& cap,
                             unsigned long long* buf, int& cnt, WaveCells* wc, int lane) {
    uint32_t loc[kCellsPerLane], run = 0;
#pragma unroll
    for (int u = 0; u < kCellsPerLane; ++u) {
        run += cr[u].y > cr[u].x ? cr[u].y - cr[u].x : 0u;
        loc[u] = run;
    }
    const uint32_t incl = lane_scan_incl<64>(run);
    const uint32_t total = (uint32_t)__shfl((int)incl, 63);
    if (total == 0) return;
    const uint32_t excl = incl - run;
    wave_sync();                         // the previous chunk's readers are done with wc
#pragma unroll
    for (int u = 0; u < kCellsPerLane; ++u) {
        wc->start[lane * kCellsPerLane + u] = cr[u].x;
        wc->end_incl[lane * kCellsPerLane + u] = excl + loc[u];
    }
    wave_sync();
    for (uint32_t j0 = 0; j0 < total; j0 += 64 * kWaveRows) {
        uint32_t r[kWaveRows];
#pragma unroll
        for (int u = 0; u < kWaveRows; ++u) {
            const uint32_t j = j0 + (uint32_t)(u * 64 + lane);
            r[u] = 0u;
            if (j0 + (uint32_t)(u * 64) >= total) continue;   // wave-uniform: slot past the chunk
            int a = 0, b = kChunkCells - 1;   // first cell whose inclusive end exceeds j
#pragma unroll
            for (int it = 0; it < kChunkLog2; ++it) {
                const int m = (a + b) >> 1;
                if (wc->end_incl[m] > j) b = m; else a = m + 1;
            }
            r[u] = j < total ? wc->start[a] + (j - (a ? wc->end_incl[a - 1] : 0u)) : 0u;
        }
        float4 p[kWaveRows];
#pragma unroll
        for (int u = 0; u < kWaveRows; ++u)
            if (j0 + (uint32_t)(u * 64) < total) p[u] = g.pts[r[u]];
#pragma unroll
        for (int u = 0; u < kWaveRows; ++u) {
            const uint32_t j = j0 + (uint32_t)(u * 64 + lane);
            if (j0 + (uint32_t)(u * 64) < total) {
                if (cnt > kWaveSurv - 64) {  // make room: keep the K best, tighten the cap
                    int kept;
                    const unsigned long long top = wave_sort_survivors(buf, cnt, lane, K, kept);
                    const unsigned long long kth_key = __shfl(top, K - 1);
                    if (kept == K && kth_key + 1ull < cap) cap = kth_key + 1ull;
                    cnt = kept;
                }
                const unsigned long long key2 = cand_key<false>(q, p[u], r[u]);
                wave_append(j < total && key2 < cap, key2, buf, cnt, lane);
            }
        }
        wave_sync();
    }
}

PCD_DEV bool cell_near(const GridView& g, Vec3 q, int cx, int cy, int cz, float kth) {
    const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
    const float gx = axis_gap(q.x, lx, lx + g.h), gy = axis_gap(q.y, ly, ly + g.h), gz = axis_gap(q.z, lz, lz + g.h);
    return gx * gx + gy * gy + gz * gz <= kth * 1.00001f + 1e-30f;
}

// Boxes of more than kBrickModeCells cells (far outliers, sparse regions, the growing blocks of an anchorless query)
// are walked brick by brick: one lane probes one 4x4x4 brick (one hash lookup for 64 cells, pruned by its box
// distance), the occupied bricks are compacted in LDS, and each then yields its 64 cell ranges from its dense block
// with no further probes -- empty space costs one probe per 64 cells instead of one per cell.
static constexpr int64_t kBrickModeCells = 1024;
PCD_DEV void cell_of_brick(int l, int& dx, int& dy, int& dz) {   // Morton decode of the low 6 key bits
    dx = (l & 1) | ((l >> 2) & 2);
    dy = ((l >> 1) & 1) | ((l >> 3) & 2);
    dz = ((l >> 2) & 1) | ((l >> 4) & 2);
}
template <int K>
PCD_DEV void wave_scan_bricks(const GridView& g, Vec3 q, const int lo[3], const int hi[3], unsigned long long& cap,
                              unsigned long long* buf, int& cnt, WaveCells* wc, int lane) {
    static_assert(kCellsPerLane == 2, "two bricks per chunk: lane l takes cell l of each");
    const int blo[3] = {lo[0] >> 2, lo[1] >> 2, lo[2] >> 2}, bhi[3] = {hi[0] >> 2, hi[1] >> 2, hi[2] >> 2};
    const int ex = bhi[0] - blo[0] + 1, ey = bhi[1] - blo[1] + 1, ez = bhi[2] - blo[2] + 1;
    const int64_t nb = (int64_t)ex * ey * ez;
    // the found bricks of a probe round go to wc (brick id, bx, by, bz in four 64-entry quarters), then into
    // registers (wave_scan_chunk reuses wc)
    for (int64_t base = 0; base < nb; base += 64) {
        const int64_t bi = base + lane;
        uint32_t brick = ~0u;
        int bx = 0, by = 0, bz = 0;
        if (bi < nb) {
            bx = blo[0] + (int)(bi % ex); by = blo[1] + (int)((bi / ex) % ey); bz = blo[2] + (int)(bi / ((int64_t)ex * ey));
            // brick box distance
            const float lx = g.ox + (bx * 4) * g.h, ly = g.oy + (by * 4) * g.h, lz = g.oz + (bz * 4) * g.h;
            const float w = 4.f * g.h;
            const float gx = axis_gap(q.x, lx, lx + w), gy = axis_gap(q.y, ly, ly + w), gz = axis_gap(q.z, lz, lz + w);
            const float kth = __uint_as_float((unsigned)(cap >> 32));
            if (gx * gx + gy * gy + gz * gz <= kth * 1.00001f + 1e-30f) {
                const unsigned long long bkey = morton3(bx, by, bz);
                unsigned long long slot = hash_slot(bkey, g.hbits);
                for (;;) {
                    const uint4 e = *reinterpret_cast<const uint4*>(g.table + slot);
                    const unsigned long long k2 = (unsigned long long)e.x | ((unsigned long long)e.y << 32);
                    if (k2 == bkey) { brick = e.z; break; }
                    if (k2 == kEmptyKey) break;
                    slot = (slot + 1) & g.mask;
                }
            }
        }
        const unsigned long long found = __ballot(brick != ~0u);
        const int nf = __popcll(found);
        if (nf == 0) continue;
        // this lane's found brick -> position in the compacted list (registers: bid / packed coords by shuffle)
        const int pos = __popcll(found & ((1ull << lane) - 1ull));
        wave_sync();
        if (brick != ~0u) {
            wc->start[pos] = brick;
            wc->start[64 + pos] = (uint32_t)bx;
            wc->end_incl[pos] = (uint32_t)by;
            wc->end_incl[64 + pos] = (uint32_t)bz;
        }
        wave_sync();
        const uint32_t my_b = lane < nf ? wc->start[lane] : 0u, my_x = lane < nf ? wc->start[64 + lane] : 0u,
                       my_y = lane < nf ? wc->end_incl[lane] : 0u, my_z = lane < nf ? wc->end_incl[64 + lane] : 0u;
        wave_sync();
        for (int f = 0; f < nf; f += 2) {            // two bricks per chunk
            uint2 cr[kCellsPerLane];
            const float kth = __uint_as_float((unsigned)(cap >> 32));
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                cr[u] = make_uint2(0u, 0u);
                if (f + u >= nf) continue;          // wave-uniform
                const uint32_t b = (uint32_t)__shfl((int)my_b, f + u);
                int dx, dy, dz;
                cell_of_brick(lane, dx, dy, dz);
                const int cx = __shfl((int)my_x, f + u) * 4 + dx, cy = __shfl((int)my_y, f + u) * 4 + dy,
                          cz = __shfl((int)my_z, f + u) * 4 + dz;
                const bool inbox = cx >= lo[0] && cx <= hi[0] && cy >= lo[1] && cy <= hi[1] && cz >= lo[2] && cz <= hi[2];
                if (inbox && cell_near(g, q, cx, cy, cz, kth)) cr[u] = g.cells[(uint64_t)b * 64 + lane];
            }
            wave_scan_chunk<K>(g, q, cr, cap, buf, cnt, wc, lane);
        }
    }
}

// Scan the cells of box [lo, hi] (cell coords), appending keys < cap to buf.  cap may tighten (buffer reduce).
// Latency-shaped: a chunk is up to 256 cells (the whole cap box of a typical query), kCellsPerLane per lane, whose
// brick-hash probes, then brick-block loads, are each issued together (two memory round trips for the chunk);
// then the chunk's flattened candidate rows in rounds of kWaveRows per lane -- every row index first (binary search
// of the count scan in LDS), then all the point loads at once, then the keys.
template <int K>
PCD_DEV void wave_scan_box(const GridView& g, Vec3 q, const int lo[3], const int hi[3], unsigned long long& cap,
                           unsigned long long* buf, int& cnt, WaveCells* wc, int lane) {
    // box extents in cells: the caller's r keeps them far below 2^10 per axis except for a pathological query,
    // whose box is clamped to the grid; 64-bit only for the (rare) giant product
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1, ez = hi[2] - lo[2] + 1;
    const int64_t nc = (int64_t)ex * ey * ez;
    if (nc > kBrickModeCells) {
        wave_scan_bricks<K>(g, q, lo, hi, cap, buf, cnt, wc, lane);
        return;
    }
    const uint32_t exy = (uint32_t)ex * (uint32_t)ey;
    for (int64_t base = 0; base < nc; base += kChunkCells) {
        // 1. this lane's cells (lane-major: cells lane*CPL .. +CPL-1 of the chunk): prune, hash slot, probe
        unsigned long long key[kCellsPerLane], slot[kCellsPerLane];
        bool want[kCellsPerLane];
        uint4 sl[kCellsPerLane];
        const float kth = __uint_as_float((unsigned)(cap >> 32));
#pragma unroll
        for (int u = 0; u < kCellsPerLane; ++u) {
            const int64_t ci = base + lane * kCellsPerLane + u;
            want[u] = false;
            key[u] = 0; slot[u] = 0;
            if (ci < nc) {
                const uint32_t c32 = (uint32_t)ci, zq = c32 / exy, rem = c32 - zq * exy, yq = rem / (uint32_t)ex;
                const int cx = lo[0] + (int)(rem - yq * (uint32_t)ex), cy = lo[1] + (int)yq, cz = lo[2] + (int)zq;
                if (cell_near(g, q, cx, cy, cz, kth)) {
                    want[u] = true;
                    key[u] = morton3(cx, cy, cz);
                    slot[u] = hash_slot(key[u] >> 6, g.hbits);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kCellsPerLane; ++u)
            sl[u] = want[u] ? *reinterpret_cast<const uint4*>(g.table + slot[u]) : make_uint4(~0u, ~0u, 0u, 0u);
        // 2. resolve the probes (linear probing past a collision is rare), then the brick blocks, all in flight
        uint32_t brick[kCellsPerLane];
#pragma unroll
        for (int u = 0; u < kCellsPerLane; ++u) {
            brick[u] = ~0u;
            if (!want[u]) continue;
            const unsigned long long bkey = key[u] >> 6;
            uint4 e = sl[u];
            unsigned long long sidx = slot[u];
            for (;;) {
                const unsigned long long k2 = (unsigned long long)e.x | ((unsigned long long)e.y << 32);
                if (k2 == bkey) { brick[u] = e.z; break; }
                if (k2 == kEmptyKey) break;
                sidx = (sidx + 1) & g.mask;
                e = *reinterpret_cast<const uint4*>(g.table + sidx);
            }
        }
        uint2 cr[kCellsPerLane];
#pragma unroll
        for (int u = 0; u < kCellsPerLane; ++u)
            cr[u] = brick[u] != ~0u ? g.cells[(uint64_t)brick[u] * 64 + (key[u] & 63)] : make_uint2(0u, 0u);
        wave_scan_chunk<K>(g, q, cr, cap, buf, cnt, wc, lane);
    }
}

PCD_DEV void cell_box(const GridView& g, Vec3 q, float r, int lo[3], int hi[3]) {
    const float qa[3] = {q.x, q.y, q.z}, o[3] = {g.ox, g.oy, g.oz};
    const int dm[3] = {g.dx, g.dy, g.dz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = min(max(cell_coord(qa[a] - r, o[a], g.inv_h), 0), dm[a] - 1);
        hi[a] = min(max(cell_coord(qa[a] + r, o[a], g.inv_h), 0), dm[a] - 1);
    }
}

// Exact top-K (K <= 64) of the snapshot for q; returns lane t's key t.  cap: kInfKey or a bound > the true K-th
// key.  Requires K <= g.n.  buf: the wave's kWaveSurv-key LDS buffer; wc: its cell scratch.
template <int K>
PCD_DEV unsigned long long wave_knn(const GridView& g, Vec3 q, unsigned long long cap, unsigned long long* buf,
                                    WaveCells* wc, int lane) {
    static_assert(K <= 64, "one key per lane");
    int cnt = 0, lo[3], hi[3];
    const int c[3] = {min(max(cell_coord(q.x, g.ox, g.inv_h), 0), g.dx - 1),
                      min(max(cell_coord(q.y, g.oy, g.inv_h), 0), g.dy - 1),
                      min(max(cell_coord(q.z, g.oz, g.inv_h), 0), g.dz - 1)};
    if (cap == kInfKey) {
        // no bound yet: Chebyshev blocks of growing radius until they hold K points; their K-th key bounds it
        for (int R = 1;; R = R * 2) {
            const int dm[3] = {g.dx, g.dy, g.dz};
            bool all = true;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                lo[a] = max(c[a] - R, 0);
                hi[a] = min(c[a] + R, dm[a] - 1);
                all = all && lo[a] == 0 && hi[a] == dm[a] - 1;
            }
            cnt = 0;
            unsigned long long cp = kInfKey;
            wave_scan_box<K>(g, q, lo, hi, cp, buf, cnt, wc, lane);
            if (cnt >= K || all) {
                int kept;
                const unsigned long long top = wave_sort_survivors(buf, cnt, lane, 0, kept);
                const unsigned long long kth_key = __shfl(top, K - 1);
                if (all) return top;          // the whole grid was scanned: exact as it stands
                cap = kth_key + 1ull;
                break;
            }
        }
        cnt = 0;
    }
    const float r = sqrtf(__uint_as_float((unsigned)(cap >> 32))) * 1.0001f + 1e-30f;
    cell_box(g, q, r, lo, hi);
    wave_scan_box<K>(g, q, lo, hi, cap, buf, cnt, wc, lane);
    int kept;
    return wave_sort_survivors(buf, cnt, lane, 0, kept);
}

}  // namespace pcd
