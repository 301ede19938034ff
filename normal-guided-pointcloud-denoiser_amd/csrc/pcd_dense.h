// Dense first anchoring by cell tiles (denoise.hip): the re-anchoring of EVERY row when the denoiser has no anchors
// yet (after create / reset_seed), the first iteration of Processor.denoise's loop (Processor.py:123-139, the kNN of
// Selector.getKNNSelection, Selector.py:235-246).
//
// k_knn_dense_q (pcd_qknn.h) shares one scan between two consecutive rows; its cell phase (hash probes, row ranges,
// the flattened row -> cell map) is still paid once per two queries and was the largest VALU item of the pass.  Here a
// wave takes the rows of ONE snapshot cell at a time (up to 64; a cell of the fused loop's grid holds about one list
// cap of points), resolves the union of their search boxes ONCE -- the cells within reach of the rows' bounding box,
// their row ranges -- and stages every candidate row in LDS.  Each query of the tile then scans the staged rows (LDS
// reads, no address arithmetic), appends the keys under its own cap and finishes exactly as a lone query (rq_finish:
// same survivors under the same cap, same exactness checks, same writes).  A tile whose box or candidate set does not
// fit runs its queries alone (rq_query), as does a query whose radius held too few points (radius x 1.6).
//
// The candidate set of a tile is a superset of every query's own scan (cells whose box lies within the largest cap
// radius of the tile's bounding box; every per-query test is monotone in that box), and a survivor is a key below the
// query's cap wherever it came from, so the stored lists are the exact (d², rank) order either way.
#pragma once
#include "pcd_qknn.h"

namespace pcd {

#ifndef PCD_TILE_CAP
#define PCD_TILE_CAP 1024        // staged candidate rows per wave (16 B each)
#endif
#ifndef PCD_TILE_CELLS
#define PCD_TILE_CELLS 256       // largest union box (cells) a tile stages; a wider one runs its queries alone
#endif
#ifndef PCD_TILE_OCC
#define PCD_TILE_OCC 2
#endif
static constexpr int kTileCap = PCD_TILE_CAP;

PCD_DEV float wave_min_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
PCD_DEV float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Stage the rows of every cell of box [lo, hi] within sqrt(reach2) of the tile's query box [qlo, qhi] into cand
// (x, y, z, rank bits).  Returns the number staged, or -1 when they do not fit kTileCap.
PCD_DEV int tile_stage(const GridView& g, const int lo[3], const int hi[3], const float qlo[3], const float qhi[3],
                       float reach2, float4* cand, RqCells* wc, const LaneGrp<64>& lg) {
    constexpr int W = 64, CPL = RqCPL<W>::n;
    const int hl = lg.hl;
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1;
    const int nc = ex * ey * (hi[2] - lo[2] + 1);
    const uint32_t exy = (uint32_t)ex * (uint32_t)ey;
    const GridSrc src{&g};
    int C = 0;
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
                // the gap from the cell to the query BOX: below every query's own gap to the cell (monotone)
                const float gx = fmaxf(fmaxf(lx - qhi[0], qlo[0] - (lx + g.h)), 0.f);
                const float gy = fmaxf(fmaxf(ly - qhi[1], qlo[1] - (ly + g.h)), 0.f);
                const float gz = fmaxf(fmaxf(lz - qhi[2], qlo[2] - (lz + g.h)), 0.f);
                on[u] = gx * gx + gy * gy + gz * gz <= reach2;
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
        if (C + (int)total > kTileCap || total > (uint32_t)kRqMap) return -1;
        const uint32_t excl = incl - run;
        wave_sync();
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            wc->start[hl * CPL + u] = cr[u].x;
            wc->end_incl[hl * CPL + u] = excl + loc[u];
            fill_cellof(wc->cellof, excl + (u ? loc[u - 1] : 0u), excl + loc[u], (uint32_t)(hl * CPL + u));
        }
        wave_sync();
        // the flattened rows, four per lane in flight
        for (uint32_t j0 = 0; j0 < total; j0 += 4 * W) {
            uint32_t r[4];
            float4 p[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * W + hl);
                const int a = j < total ? (int)wc->cellof[j] : 0;
                r[u] = j < total ? wc->start[a] + (j - (a ? wc->end_incl[a - 1] : 0u)) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j0 + (uint32_t)(u * W + hl) < total) p[u] = g.pts[r[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t j = j0 + (uint32_t)(u * W + hl);
                if (j < total) cand[C + (int)j] = make_float4(p[u].x, p[u].y, p[u].z, __uint_as_float(r[u]));
            }
        }
        C += (int)total;
        wave_sync();
    }
    return C;
}

// One wave per brick of the snapshot grid (all rows active: rm.rows == null); the rows of each occupied cell of the
// brick in tiles of at most 64.
template <int KA>
__global__ __launch_bounds__(64, PCD_TILE_OCC) void k_knn_dense_tile(GridView g, const float4* __restrict__ pos,
                                                                      int64_t N, int64_t bricks, int kstore,
                                                                      float r_scale, float4* __restrict__ anc,
                                                                      int32_t* __restrict__ alist,
                                                                      int32_t* __restrict__ idx,
                                                                      int32_t* __restrict__ spill,
                                                                      unsigned* __restrict__ spill_cnt) {
    constexpr int W = 64;
    __shared__ float4 s_cand[kTileCap];
    __shared__ unsigned long long s_buf[RqSurv<W>::n];
    __shared__ RqCells s_cells;
    const int lane = (int)(threadIdx.x & 63);
    const LaneGrp<W> lg(lane);
    for (int64_t b = xcd_block(blockIdx.x, gridDim.x); b < bricks; b += gridDim.x) {
        const uint2 cr = g.cells[(uint64_t)b * 64 + lane];
        unsigned long long occ = __ballot(cr.y > cr.x);
        while (occ) {
            const int c = __builtin_ctzll(occ);
            occ &= occ - 1ull;
            const uint32_t cs = (uint32_t)__shfl((int)cr.x, c), ce = (uint32_t)__shfl((int)cr.y, c);
            for (uint32_t t0 = cs; t0 < ce; t0 += W) {
                const int nt = (int)min(ce - t0, (uint32_t)W);
                const bool act = lane < nt;
                const int64_t i = (int64_t)t0 + (act ? lane : 0);
                const float4 p4 = pos[i];
                const Vec3 q = v3(p4.x, p4.y, p4.z);
                // the radius from the occupancy of the query's own cell (k_knn_requery<KA, true>)
                const int cx = min(max(cell_coord(q.x, g.ox, g.inv_h), 0), g.dx - 1);
                const int cy = min(max(cell_coord(q.y, g.oy, g.inv_h), 0), g.dy - 1);
                const int cz = min(max(cell_coord(q.z, g.oz, g.inv_h), 0), g.dz - 1);
                uint32_t s = 0, e = 0;
                const int n = cell_range(g, cx, cy, cz, s, e) ? (int)(e - s) : 1;
                const float rs = r_scale * g.h * cbrtf(16.f / (float)n);
                const float rr = rs * 1.0001f + 1e-30f;
                const float big = 3.0e38f;
                const float qlo[3] = {wave_min_f(act ? q.x : big), wave_min_f(act ? q.y : big), wave_min_f(act ? q.z : big)};
                const float qhi[3] = {wave_max_f(act ? q.x : -big), wave_max_f(act ? q.y : -big),
                                      wave_max_f(act ? q.z : -big)};
                const float rrmax = wave_max_f(act ? rr : 0.f);
                const float capmax = wave_max_f(act ? rs * rs : 0.f);
                // the union of the queries' boxes (cell_box of each query lies inside it: cell_coord is monotone)
                int lo[3], hi[3];
                {
                    const float o[3] = {g.ox, g.oy, g.oz};
                    const int dm[3] = {g.dx, g.dy, g.dz};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = min(max(cell_coord(qlo[a] - rrmax, o[a], g.inv_h), 0), dm[a] - 1);
                        hi[a] = min(max(cell_coord(qhi[a] + rrmax, o[a], g.inv_h), 0), dm[a] - 1);
                    }
                }
                const int64_t nbox = (int64_t)(hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1);
                int C = -1;
                if (nbox <= PCD_TILE_CELLS) C = tile_stage(g, lo, hi, qlo, qhi, capmax * 1.00001f + 1e-30f, s_cand,
                                                          &s_cells, lg);
                for (int j = 0; j < nt; ++j) {
                    const int64_t ij = (int64_t)t0 + j;
                    const Vec3 qj = v3(__shfl(q.x, j), __shfl(q.y, j), __shfl(q.z, j));
                    const float rsj = __shfl(rs, j);
                    bool clean = C >= 0;
                    int cnt = 0;
                    unsigned long long cap = ((unsigned long long)__float_as_uint(rsj * rsj) << 32) | 0xFFFFFFFFull;
                    if (clean) {
                        for (int c0 = 0; c0 < C; c0 += W * kRqRows) {
                            // room for a whole round of appends (one cut site)
                            if (cnt > RqSurv<W>::n - W * kRqRows && !rq_cut<KA, W>(s_buf, cnt, cap, lg)) {
                                clean = false;
                                break;
                            }
                            float4 cd[kRqRows];
#pragma unroll
                            for (int u = 0; u < kRqRows; ++u) {
                                const int cc = c0 + u * W + lane;
                                cd[u] = cc < C ? s_cand[cc] : make_float4(big, big, big, 0.f);
                            }
#pragma unroll
                            for (int u = 0; u < kRqRows; ++u) {
                                const int cc = c0 + u * W + lane;
                                const unsigned long long key2 =
                                    ((unsigned long long)__float_as_uint(dist2(qj, cd[u])) << 32) | __float_as_uint(cd[u].w);
                                const bool pass = cc < C && key2 < cap;
                                const unsigned long long m = __ballot(pass);
                                if (pass) s_buf[cnt + __popcll(m & ((1ull << lane) - 1ull))] = key2;
                                cnt += __popcll(m);
                            }
                        }
                    }
                    if (clean && cnt > kstore) {
                        rq_finish<KA, W>(ij, qj, rsj, N, kstore, anc, alist, idx, spill, spill_cnt, s_buf, cnt, cap,
                                         true, false, lg);
                    } else {
                        // alone: its own box (an oversized one spills in there), the radius widened when too few
                        wave_sync();
                        (void)rq_query<KA, W>(g, GridSrc{&g}, ij, qj, C >= 0 && clean ? rsj * 1.6f : rsj, N, kstore,
                                              anc, alist, idx, spill, spill_cnt, s_buf, &s_cells, lg);
                    }
                    wave_sync();
                }
                wave_sync();
            }
        }
    }
}

}  // namespace pcd
