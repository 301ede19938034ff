// Exact k-nearest-neighbour search over the frozen snapshot (replaces scipy KDTree.query on the snapshot
// taken in Selector.__init__, Pointcloud/Modules/Selector.py:141,243).
//
// Index: Morton-sorted snapshot points + a bricked cell index (GridView, cell_range).  A query scans
// its cell and the 26 around it (centre, faces, edges, corners), pruning any cell whose box is farther than
// the current k-th distance, then expands Chebyshev shells until the k-th distance is provably below the
// distance to every unscanned cell.  The top-k lives in registers as a sorted list of 64-bit keys
// (d² bits << 32 | index): fp32 (q-c)² distances (no |q|²+|c|²-2q·c cancellation), ties broken by index.
#pragma once
#include "pcd_device.h"
#include "pcd_host.h"

namespace pcd {

__host__ __device__ inline unsigned long long spread21(unsigned int v) {
    unsigned long long x = v & 0x1fffffu;
    x = (x | (x << 32)) & 0x1f00000000ffffull;
    x = (x | (x << 16)) & 0x1f0000ff0000ffull;
    x = (x | (x << 8)) & 0x100f00f00f00f00full;
    x = (x | (x << 4)) & 0x10c30c30c30c30c3ull;
    x = (x | (x << 2)) & 0x1249249249249249ull;
    return x;
}
__host__ __device__ inline unsigned long long morton3(unsigned int x, unsigned int y, unsigned int z) {
    return spread21(x) | (spread21(y) << 1) | (spread21(z) << 2);
}
__host__ __device__ inline unsigned long long hash_slot(unsigned long long key, int hbits) {
    return (key * 0x9E3779B97F4A7C15ull) >> (64 - hbits);
}

// Cells live in bricks of 4x4x4: the brick is found in a small hash of occupied bricks (L2-resident), the cell's
// row range in the brick's dense 64-entry block (contiguous in memory, and nearby bricks are nearby in Morton order),
// so the probes of neighbouring queries share cache lines instead of each touching a random hash slot.
PCD_DEV bool cell_range(const GridView& g, int cx, int cy, int cz, uint32_t& s, uint32_t& e) {
    if ((unsigned)cx >= (unsigned)g.dx || (unsigned)cy >= (unsigned)g.dy || (unsigned)cz >= (unsigned)g.dz)
        return false;
    const unsigned long long key = morton3(cx, cy, cz), bkey = key >> 6;
    unsigned long long slot = hash_slot(bkey, g.hbits);
    for (;;) {
        const uint4 sl = *reinterpret_cast<const uint4*>(g.table + slot);
        const unsigned long long k2 = (unsigned long long)sl.x | ((unsigned long long)sl.y << 32);
        if (k2 == bkey) {
            const uint2 c = g.cells[(uint64_t)sl.z * 64 + (key & 63)];
            s = c.x; e = c.y;
            return c.y > c.x;
        }
        if (k2 == kEmptyKey) return false;
        slot = (slot + 1) & g.mask;
    }
}

PCD_DEV int cell_coord(float p, float o, float inv_h) {
    float f = (p - o) * inv_h;
    f = fminf(fmaxf(f, -1.0e9f), 1.0e9f);  // NaN -> -1e9 (fmaxf drops NaN)
    return (int)floorf(f);
}

static constexpr unsigned long long kInfKey = (0x7F800000ull << 32) | 0xFFFFFFFFull;

// Sorted register list of the K best candidate keys.  `cap` is an optional acceptance bound known to be >= the
// true k-th key (a seed: the k-th distance to any k distinct snapshot points); it prunes cells and rejects
// candidates before the list has filled.
#ifdef PCD_KNN_STATS  // diagnostic build only (stats.hip): per-query work counters
#define PCD_KSTAT(tk, i, v) ((tk).stat[i] += (v))
#else
#define PCD_KSTAT(tk, i, v) ((void)0)
#endif

template <int K>
struct TopK {
    unsigned long long key[K];
    unsigned long long cap;
#ifdef PCD_KNN_STATS
    unsigned stat[6];  // cells considered, cells probed, cells found, candidates, inserts, rings
#endif
    PCD_DEV void init(unsigned long long c = kInfKey) {
#pragma unroll
        for (int i = 0; i < K; ++i) key[i] = kInfKey;
        cap = c;
#ifdef PCD_KNN_STATS
        for (int i = 0; i < 6; ++i) stat[i] = 0;
#endif
    }
    PCD_DEV unsigned long long limit() const { return key[K - 1] < cap ? key[K - 1] : cap; }
    PCD_DEV float kth() const { return __uint_as_float((unsigned)(limit() >> 32)); }
    PCD_DEV void insert(unsigned long long c) {
#pragma unroll
        for (int j = K - 1; j > 0; --j) {
            const unsigned long long prev = key[j - 1];
            const unsigned long long cur = key[j];
            key[j] = (c < prev) ? prev : ((c < cur) ? c : cur);
        }
        key[0] = (c < key[0]) ? c : key[0];
    }
    PCD_DEV int idx(int j) const { return (int)(uint32_t)(key[j] & 0xFFFFFFFFull); }
    PCD_DEV float d2(int j) const { return __uint_as_float((unsigned)(key[j] >> 32)); }
};

PCD_DEV float dist2(Vec3 q, float4 p) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    return __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
}

// Candidate key: d² bits in the high word; the low word is the snapshot point's ORIGINAL index (ORIG, kept in
// pts[r].w at build; ties then break by caller index) or its rank r in the Morton-sorted snapshot (!ORIG: the
// fused loop works in sorted order, where rank == working index).
template <bool ORIG>
PCD_DEV unsigned long long cand_key(Vec3 q, float4 p, uint32_t r) {
    return ((unsigned long long)__float_as_uint(dist2(q, p)) << 32) | (ORIG ? __float_as_uint(p.w) : r);
}

template <int K, bool ORIG>
PCD_DEV void scan_range(const float4* __restrict__ pts, uint32_t s, uint32_t e, Vec3 q, TopK<K>& tk) {
    uint32_t r = s;
    for (; r + 1 < e; r += 2) {  // two loads in flight per lane
        const float4 p0 = pts[r], p1 = pts[r + 1];
        const unsigned long long c0 = cand_key<ORIG>(q, p0, r);
        const unsigned long long c1 = cand_key<ORIG>(q, p1, r + 1);
        if (c0 < tk.limit()) { tk.insert(c0); PCD_KSTAT(tk, 4, 1); }
        if (c1 < tk.limit()) { tk.insert(c1); PCD_KSTAT(tk, 4, 1); }
    }
    if (r < e) {
        const unsigned long long c0 = cand_key<ORIG>(q, pts[r], r);
        if (c0 < tk.limit()) { tk.insert(c0); PCD_KSTAT(tk, 4, 1); }
    }
    PCD_KSTAT(tk, 3, e - s);
}

PCD_DEV float axis_gap(float q, float lo, float hi) { return fmaxf(fmaxf(lo - q, q - hi), 0.f); }

// Scan one cell unless its box is provably farther than the current k-th candidate.
template <int K, bool ORIG>
PCD_DEV void visit_cell(const GridView& g, Vec3 q, int cx, int cy, int cz, TopK<K>& tk) {
    const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
    const float gx = axis_gap(q.x, lx, lx + g.h), gy = axis_gap(q.y, ly, ly + g.h), gz = axis_gap(q.z, lz, lz + g.h);
    const float box = gx * gx + gy * gy + gz * gz;
    PCD_KSTAT(tk, 0, 1);
    if (box > tk.kth() * 1.00001f + 1e-30f) return;
    uint32_t s, e;
    PCD_KSTAT(tk, 1, 1);
    if (cell_range(g, cx, cy, cz, s, e)) { PCD_KSTAT(tk, 2, 1); scan_range<K, ORIG>(g.pts, s, e, q, tk); }
}

// 3x3x3 neighbourhood: centre, 6 faces, 12 edges, 8 corners (closest cells first -> the k-th distance
// tightens early and the far cells are pruned).
__constant__ static const signed char kRing1[27][3] = {
    {0, 0, 0},
    {-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1},
    {-1, -1, 0}, {1, -1, 0}, {-1, 1, 0}, {1, 1, 0}, {-1, 0, -1}, {1, 0, -1}, {-1, 0, 1}, {1, 0, 1},
    {0, -1, -1}, {0, 1, -1}, {0, -1, 1}, {0, 1, 1},
    {-1, -1, -1}, {1, -1, -1}, {-1, 1, -1}, {1, 1, -1}, {-1, -1, 1}, {1, -1, 1}, {-1, 1, 1}, {1, 1, 1}};

// After scanning the Chebyshev block of radius R around (cx,cy,cz): is the top-k final?
PCD_DEV bool search_done(const GridView& g, Vec3 q, int cx, int cy, int cz, int R, float kth) {
    bool exhausted = true;
    float bound = 3.0e38f;
    const int c[3] = {cx, cy, cz};
    const int dm[3] = {g.dx, g.dy, g.dz};
    const float o[3] = {g.ox, g.oy, g.oz};
    const float qa[3] = {q.x, q.y, q.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (c[a] - R > 0) {
            exhausted = false;
            bound = fminf(bound, fmaxf(qa[a] - (o[a] + (c[a] - R) * g.h), 0.f));
        }
        if (c[a] + R < dm[a] - 1) {
            exhausted = false;
            bound = fminf(bound, fmaxf((o[a] + (c[a] + R + 1) * g.h) - qa[a], 0.f));
        }
    }
    return exhausted || kth <= bound * bound * 0.99998f;
}

// Is the top-k final once every cell of the box [lo, hi] (cell coordinates) is scanned?  (The box's faces that are
// not at the grid's edge bound the distance to every unscanned cell.)
PCD_DEV bool box_done(const GridView& g, Vec3 q, const int lo[3], const int hi[3], float kth) {
    bool exhausted = true;
    float bound = 3.0e38f;
    const int dm[3] = {g.dx, g.dy, g.dz};
    const float o[3] = {g.ox, g.oy, g.oz};
    const float qa[3] = {q.x, q.y, q.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (lo[a] > 0) {
            exhausted = false;
            bound = fminf(bound, fmaxf(qa[a] - (o[a] + lo[a] * g.h), 0.f));
        }
        if (hi[a] < dm[a] - 1) {
            exhausted = false;
            bound = fminf(bound, fmaxf((o[a] + (hi[a] + 1) * g.h) - qa[a], 0.f));
        }
    }
    return exhausted || kth <= bound * bound * 0.99998f;
}

// Brick shells (4x4x4 cells) around the query's brick, after the cells within Chebyshev radius RC of (cx, cy, cz)
// have been scanned: one hash probe per brick instead of one per cell, so a query many cells away from the cloud
// (noisy points off a finely gridded surface) pays ~64x fewer probes.  Cells inside the scanned block are skipped.
static constexpr int kCellShells = 3;
template <int K, bool ORIG>
PCD_DEV void brick_shells(const GridView& g, Vec3 q, int cx, int cy, int cz, TopK<K>& tk, unsigned long long cap) {
    const int RC = kCellShells;
    const int bx = cx >> 2, by = cy >> 2, bz = cz >> 2;
    const int nbx = (g.dx + 3) >> 2, nby = (g.dy + 3) >> 2, nbz = (g.dz + 3) >> 2;
#pragma unroll 1
    for (int Rb = 0;; ++Rb) {
        const int64_t side = 2 * (int64_t)Rb + 1;
        if (Rb > 8 && side * side * side > (int64_t)g.n / 4) {   // a far outlier: one exhaustive scan is cheaper
            tk.init(cap);
            scan_range<K, ORIG>(g.pts, 0, (uint32_t)g.n, q, tk);
            return;
        }
#pragma unroll 1
        for (int dz = -Rb; dz <= Rb; ++dz) {
#pragma unroll 1
            for (int dy = -Rb; dy <= Rb; ++dy) {
                const bool rim = (dz == -Rb || dz == Rb || dy == -Rb || dy == Rb);
                const int step = rim ? 1 : 2 * Rb;
#pragma unroll 1
                for (int dx = -Rb; dx <= Rb; dx += (step > 0 ? step : 1)) {
                    const int qx = bx + dx, qy = by + dy, qz = bz + dz;
                    if ((unsigned)qx >= (unsigned)nbx || (unsigned)qy >= (unsigned)nby || (unsigned)qz >= (unsigned)nbz)
                        continue;
                    const float lx = g.ox + 4 * qx * g.h, ly = g.oy + 4 * qy * g.h, lz = g.oz + 4 * qz * g.h;
                    const float gx = axis_gap(q.x, lx, lx + 4 * g.h), gy = axis_gap(q.y, ly, ly + 4 * g.h),
                                gz = axis_gap(q.z, lz, lz + 4 * g.h);
                    if (gx * gx + gy * gy + gz * gz > tk.kth() * 1.00001f + 1e-30f) continue;
                    const unsigned long long bkey = morton3(qx, qy, qz);
                    unsigned long long slot = hash_slot(bkey, g.hbits);
                    uint32_t brick = ~0u;
                    for (;;) {
                        const uint4 sl = *reinterpret_cast<const uint4*>(g.table + slot);
                        const unsigned long long k2 = (unsigned long long)sl.x | ((unsigned long long)sl.y << 32);
                        if (k2 == bkey) { brick = sl.z; break; }
                        if (k2 == kEmptyKey) break;
                        slot = (slot + 1) & g.mask;
                    }
                    if (brick == ~0u) continue;
#pragma unroll 1
                    for (int loc = 0; loc < 64; ++loc) {
                        // local cell (x, y, z) of Morton slot loc: bits 0/3 -> x, 1/4 -> y, 2/5 -> z
                        const int ccx = 4 * qx + ((loc & 1) | ((loc >> 2) & 2));
                        const int ccy = 4 * qy + (((loc >> 1) & 1) | ((loc >> 3) & 2));
                        const int ccz = 4 * qz + (((loc >> 2) & 1) | ((loc >> 4) & 2));
                        if (abs(ccx - cx) <= RC && abs(ccy - cy) <= RC && abs(ccz - cz) <= RC) continue;   // scanned
                        const float ex = g.ox + ccx * g.h, ey = g.oy + ccy * g.h, ez = g.oz + ccz * g.h;
                        const float hx = axis_gap(q.x, ex, ex + g.h), hy = axis_gap(q.y, ey, ey + g.h),
                                    hz = axis_gap(q.z, ez, ez + g.h);
                        if (hx * hx + hy * hy + hz * hz > tk.kth() * 1.00001f + 1e-30f) continue;
                        const uint2 c = g.cells[(uint64_t)brick * 64 + loc];
                        if (c.y > c.x) scan_range<K, ORIG>(g.pts, c.x, c.y, q, tk);
                    }
                }
            }
        }
        // scanned: the bricks within Rb (and the cell block within RC, inside them from Rb >= 1 on)
        const int lo[3] = {4 * (bx - Rb), 4 * (by - Rb), 4 * (bz - Rb)};
        const int hi[3] = {4 * (bx + Rb) + 3, 4 * (by + Rb) + 3, 4 * (bz + Rb) + 3};
        if (Rb >= 1 && box_done(g, q, lo, hi, tk.kth())) return;
    }
}

// Exact top-K of the snapshot for query q (entries beyond the seed's rank are only valid when cap == inf).
template <int K, bool ORIG>
PCD_DEV void knn_search(const GridView& g, Vec3 q, TopK<K>& tk, unsigned long long cap = kInfKey) {
    tk.init(cap);
    int cx = min(max(cell_coord(q.x, g.ox, g.inv_h), 0), g.dx - 1);
    int cy = min(max(cell_coord(q.y, g.oy, g.inv_h), 0), g.dy - 1);
    int cz = min(max(cell_coord(q.z, g.oz, g.inv_h), 0), g.dz - 1);
#pragma unroll 1
    for (int t = 0; t < 27; ++t)
        visit_cell<K, ORIG>(g, q, cx + kRing1[t][0], cy + kRing1[t][1], cz + kRing1[t][2], tk);
    int R = 1;
#pragma unroll 1
    while (!search_done(g, q, cx, cy, cz, R, tk.kth())) {
        ++R;
        PCD_KSTAT(tk, 5, 1);
        if (R > kCellShells) {        // still open after the cell shells: continue brick by brick
            brick_shells<K, ORIG>(g, q, cx, cy, cz, tk, cap);
            return;
        }
#pragma unroll 1
        for (int dz = -R; dz <= R; ++dz) {
#pragma unroll 1
            for (int dy = -R; dy <= R; ++dy) {
                const bool rim = (dz == -R || dz == R || dy == -R || dy == R);
                const int step = rim ? 1 : 2 * R;
#pragma unroll 1
                for (int dx = -R; dx <= R; dx += step) visit_cell<K, ORIG>(g, q, cx + dx, cy + dy, cz + dz, tk);
            }
        }
    }
}

// ------------------------------------------------------------------ batched search (K >= 16)
// The per-candidate sorted insert above costs ~6K VALU, and in SIMT it runs whenever ANY lane of the wave accepts,
// i.e. on nearly every candidate.  The batched search flattens each lane's candidate stream across cell boundaries
// so that batch slot b is a compile-time register for every lane: B candidate rows are resolved (cell walk + hash
// probes), their B point loads issued together, the keys filtered against the k-th key, and a batch with any
// survivor is merged into the sorted list with a fixed network: bitonic sort of the batch, elementwise min against
// the list's tail (-> the K smallest of the union), then two bitonic merges.  ~100 compare-exchanges per batch
// of B = 8, instead of up to B inserts of K compare-selects each.
PCD_DEV void cswap(unsigned long long& a, unsigned long long& b) {
    const bool sw = b < a;
    const unsigned long long lo = sw ? b : a;
    b = sw ? a : b;
    a = lo;
}

// Bitonic merge of v[OFF .. OFF+N) (a bitonic sequence) into ascending (or descending) order, in place.
template <int N, int OFF, int TOT, bool DESC = false>
PCD_DEV void bitonic_merge(unsigned long long (&v)[TOT]) {
#pragma unroll
    for (int d = N / 2; d > 0; d >>= 1) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if ((i & d) == 0) {
                if (DESC) cswap(v[OFF + i + d], v[OFF + i]);
                else cswap(v[OFF + i], v[OFF + i + d]);
            }
        }
    }
}

// 32-bit keys without payload: a compare-exchange is one v_min_u32 + one v_max_u32.
PCD_DEV void cswap(uint32_t& a, uint32_t& b) {
    const uint32_t lo = min(a, b);
    b = max(a, b);
    a = lo;
}

// Ascending sort of v[0..N) by Batcher's odd-even merge network (N a power of two): 543 compare-exchanges at N = 64
// against the bitonic network's 672, every one of them between compile-time slots; as with any sorting network the
// compiler drops the exchanges whose outputs are never read (the anchor test reads the first kstore + 1).
template <int N, typename T>
PCD_DEV void oddeven_sort(T (&v)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1) {
#pragma unroll
        for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k) {
#pragma unroll
                for (int i = 0; i < k; ++i) {
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) cswap(v[i + j], v[i + j + k]);
                }
            }
        }
    }
}

// Ascending bitonic sort of v[0..N).
template <int N, typename T>
PCD_DEV void bitonic_sort(T (&v)[N]) {
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int j = i ^ stride;
                if (j > i) {
                    if ((i & size) == 0) cswap(v[i], v[j]);
                    else cswap(v[j], v[i]);
                }
            }
        }
    }
}

// key := the K smallest of key ∪ c, sorted (c: B keys, any order).  Elementwise min of the list's ascending tail
// against the descending batch keeps exactly the K smallest of the union and leaves a bitonic tail; sorting that
// tail DEscending makes the whole list bitonic (ascending head, descending tail), and one bitonic merge sorts it --
// all in place, no copy of the list.
template <int K, int B>
PCD_DEV void topk_merge(TopK<K>& tk, unsigned long long (&c)[B]) {
    static_assert(B <= K && (B & (B - 1)) == 0 && (K & (K - 1)) == 0, "power-of-two sizes");
    bitonic_sort<B>(c);
#pragma unroll
    for (int i = 0; i < B; ++i) {
        const unsigned long long x = c[B - 1 - i];
        tk.key[K - B + i] = x < tk.key[K - B + i] ? x : tk.key[K - B + i];
    }
    if constexpr (K > B) {
        bitonic_merge<B, K - B, K, true>(tk.key);
        bitonic_merge<K, 0, K>(tk.key);
    } else {
        bitonic_merge<B, 0, K>(tk.key);
    }
}

// ------------------------------------------------------------------ capped search (seeded iterations)
// With an acceptance cap known to be >= the true k-th key and close to it (the previous iteration's list re-keyed
// at the current position: median k, p99 ~1.4k keys below it on the denoise workload), a candidate below the cap
// is only APPENDED to the lane's LDS row buffer (one ds_write; no SIMT-wide sorted insert).  The register list is
// built once, at the end, by draining the buffer in chunks of 8 through topk_merge.  If a lane's buffer fills
// (rare), the lane reduces it to its K best rows and tightens the cap to their k-th key + 1, so the list is never
// live during the scan.  Exact for any cap >= the true k-th key.  Keys carry the snapshot rank (!ORIG).
// buf = this lane's column of the block's [M][kCapStride] u32 row buffer.
static constexpr int kCapStride = 256;

template <int K, int M, int S = kCapStride>
PCD_DEV void cap_drain(const GridView& g, Vec3 q, TopK<K>& tk, const uint32_t* buf, int cnt) {
    // unrolled over the (bounded) chunk count: the list stays in place, no loop-carried copy of it
#pragma unroll
    for (int base = 0; base < M; base += 8) {
        if (__any(base < cnt)) {
            unsigned long long c[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const bool ok = base + b < cnt;
                const uint32_t r = ok ? buf[(base + b) * S] : 0u;
                const float4 p = g.pts[r];
                c[b] = ok ? cand_key<false>(q, p, r) : kInfKey;
            }
            topk_merge<K, 8>(tk, c);
            PCD_KSTAT(tk, 4, 1);
        }
    }
}

template <int K, int M, int S = kCapStride>   // S: row stride of the block's LDS buffer (= threads per block)
struct CapState {
    unsigned long long lim;  // acceptance cap: every key < lim is buffered
    int cnt;                 // rows in the buffer
    uint32_t* buf;
#ifdef PCD_KNN_STATS
    unsigned* stat;
#endif
    PCD_DEV float kth() const { return __uint_as_float((unsigned)(lim >> 32)); }
};

template <int K, int M, int S>
PCD_DEV void cap_overflow(const GridView& g, Vec3 q, CapState<K, M, S>& st) {
    static_assert(M >= K + 8, "the buffer must hold the K best rows plus room to grow");
    TopK<K> t;
    t.init(st.lim);
    cap_drain<K, M, S>(g, q, t, st.buf, st.cnt);
    int n = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (t.key[j] != kInfKey) { st.buf[n * S] = (uint32_t)(t.key[j] & 0xFFFFFFFFull); ++n; }
    }
    st.cnt = n;
    if (n == K) st.lim = t.key[K - 1] + 1ull;
}

template <int K, int M, int S>
PCD_DEV void cap_scan(const GridView& g, Vec3 q, CapState<K, M, S>& st, uint32_t s, uint32_t e) {
    // groups of 4 rows: 4 loads in flight per lane; the buffer keeps 4 rows of slack for the group's appends
#pragma unroll 1
    for (uint32_t r = s; r < e; r += 4) {
        if (st.cnt > M - 4) cap_overflow<K, M, S>(g, q, st);
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = g.pts[min(r + u, e - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const unsigned long long c = cand_key<false>(q, p[u], r + u);
            if (r + u < e && c < st.lim) {
                st.buf[st.cnt * S] = r + u;
                ++st.cnt;
            }
        }
    }
}

template <int K, int M, int S>
PCD_DEV void cap_visit(const GridView& g, Vec3 q, int cx, int cy, int cz, CapState<K, M, S>& st) {
    const float lx = g.ox + cx * g.h, ly = g.oy + cy * g.h, lz = g.oz + cz * g.h;
    const float gx = axis_gap(q.x, lx, lx + g.h), gy = axis_gap(q.y, ly, ly + g.h), gz = axis_gap(q.z, lz, lz + g.h);
    if (gx * gx + gy * gy + gz * gz > st.kth() * 1.00001f + 1e-30f) return;
    uint32_t s, e;
    if (cell_range(g, cx, cy, cz, s, e)) cap_scan<K, M, S>(g, q, st, s, e);
}

template <int K, int M, int S = kCapStride>
PCD_DEV void knn_search_capped(const GridView& g, Vec3 q, TopK<K>& tk, unsigned long long cap, uint32_t* buf) {
    CapState<K, M, S> st{cap, 0, buf};
    const int cx = min(max(cell_coord(q.x, g.ox, g.inv_h), 0), g.dx - 1);
    const int cy = min(max(cell_coord(q.y, g.oy, g.inv_h), 0), g.dy - 1);
    const int cz = min(max(cell_coord(q.z, g.oz, g.inv_h), 0), g.dz - 1);
#pragma unroll 1
    for (int t = 0; t < 27; ++t) cap_visit<K, M, S>(g, q, cx + kRing1[t][0], cy + kRing1[t][1], cz + kRing1[t][2], st);
    int R = 1;
#pragma unroll 1
    while (!search_done(g, q, cx, cy, cz, R, st.kth())) {
        ++R;
        if (R > 24) {  // pathological outlier: exhaustive scan from an empty buffer
            st.cnt = 0;
            st.lim = cap;
            cap_scan<K, M, S>(g, q, st, 0, (uint32_t)g.n);
            break;
        }
#pragma unroll 1
        for (int dz = -R; dz <= R; ++dz) {
#pragma unroll 1
            for (int dy = -R; dy <= R; ++dy) {
                const bool rim = (dz == -R || dz == R || dy == -R || dy == R);
                const int step = rim ? 1 : 2 * R;
#pragma unroll 1
                for (int dx = -R; dx <= R; dx += step) cap_visit<K, M, S>(g, q, cx + dx, cy + dy, cz + dz, st);
            }
        }
    }
    tk.init(st.lim);
    cap_drain<K, M, S>(g, q, tk, buf, st.cnt);
#ifdef PCD_KNN_STATS
    tk.stat[3] += st.cnt;  // rows left in the buffer at the end
#endif
}

}  // namespace pcd
