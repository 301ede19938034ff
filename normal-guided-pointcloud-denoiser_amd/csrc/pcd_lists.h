// Per-point index lists of the fused loop in HBM (the kNN lists `idx` and the anchor sets `alist`, denoise.hip).
//
// Layout: columns in blocks of 8, each block row-major -- entry (row i, column t) at
//     base + ((t >> 3) * N + i) * 8 + (t & 7)
// so one row's 8-column block is ONE aligned 32-B sector, and a block of 64 consecutive rows is 2 KiB contiguous.
//   * a wave that re-anchors ONE row (pcd_qknn.h, pcd_wknn.h) stores whole sectors: 4 for a 32-entry list, 8 for a
//     64-entry anchor set.  The column-major layout of round 2 took 96 partial 4-B stores per re-anchored row, and
//     gfx950 retires those at ~22-28 G/s chip-wide (tools/calib_traffic.hip: one 4-B store per 128-B line costs a
//     32-B write and 45 ps of the chip): the re-anchoring kernels were bound by their list stores;
//   * a lane-per-row reader / writer (NVT, anchor test, phases) moves 16 B per instruction per lane, each instruction
//     covering 16 lines (32-B rows of a 2-KiB block), every byte of which the next instruction of the same block
//     uses -- coalesced, and the update list (columns 0..7, read by 5 passes per iteration) is block 0 alone.
// Offsets: the per-lane part i * 32 B stays below 4 GiB for N < 2^27 (checked at pcd_denoiser_create); the block
// base is uniform (SGPRs).
#pragma once
#include "pcd_device.h"

namespace pcd {

typedef int v4i __attribute__((ext_vector_type(4)));

// The two int4 of row i's block g.
PCD_DEV const v4i* lblock(const int32_t* base, int64_t N, int64_t i, int g) {
    const char* b = reinterpret_cast<const char*>(base + (int64_t)g * N * 8);
    return reinterpret_cast<const v4i*>(b + (uint32_t)((uint32_t)i * 32u));
}
PCD_DEV v4i* lblock(int32_t* base, int64_t N, int64_t i, int g) {
    char* b = reinterpret_cast<char*>(base + (int64_t)g * N * 8);
    return reinterpret_cast<v4i*>(b + (uint32_t)((uint32_t)i * 32u));
}
// Element (i, t).
PCD_DEV int64_t lpos(int64_t N, int64_t i, int t) { return ((int64_t)(t >> 3) * N + i) * 8 + (t & 7); }

// The first ceil(cnt / 8) blocks of row i into l[0 .. K) (K a multiple of 8); entries of blocks past cnt are left
// untouched.  NT: streamed past L2 (a list read once per pass).
template <int K, bool NT = false>
PCD_DEV void load_list(const int32_t* base, int64_t N, int64_t i, int cnt, int (&l)[K]) {
    static_assert(K % 8 == 0, "lists are whole 8-column blocks");
#pragma unroll
    for (int g = 0; g < K / 8; ++g) {
        if (8 * g < cnt) {
            const v4i* p = lblock(base, N, i, g);
            const v4i a = NT ? __builtin_nontemporal_load(p) : p[0];
            const v4i b = NT ? __builtin_nontemporal_load(p + 1) : p[1];
            l[8 * g + 0] = a.x; l[8 * g + 1] = a.y; l[8 * g + 2] = a.z; l[8 * g + 3] = a.w;
            l[8 * g + 4] = b.x; l[8 * g + 5] = b.y; l[8 * g + 6] = b.z; l[8 * g + 7] = b.w;
        }
    }
}
// A register list read at compile-time slots: entries past cnt repeat entry cnt - 1 (for_neighbours).  Held BY VALUE:
// a pointer to a local array keeps it in scratch memory.
template <int M>
struct RegNbC {
    int l[M];
    static constexpr bool kClamped = true;
    PCD_DEV int64_t operator()(int t) const { return l[t]; }
};
// Row i's first M columns (cnt of them valid, 1 <= cnt <= M) into l; entries past cnt repeat entry 0 (a valid row:
// for_neighbours gathers them and drops the result).  Selects against a constant slot only: a chain (l[t - 1]) is
// turned by the compiler into an indexed scratch access.
template <int M, bool NT = false>
PCD_DEV void load_list_clamped(const int32_t* base, int64_t N, int64_t i, int cnt, int (&l)[M]) {
    load_list<M, NT>(base, N, i, cnt, l);
#pragma unroll
    for (int t = 1; t < M; ++t) l[t] = t < cnt ? l[t] : l[0];
}

// load_list_clamped with 8-B loads (the windowed flat phase: 16-B loads there trip an LLVM gfx950 backend error,
// "Operand has incorrect register class", next to its LDS/global window pointer select).
template <int M>
PCD_DEV void load_list_clamped8(const int32_t* base, int64_t N, int64_t i, int cnt, int (&l)[M]) {
    typedef int v2i __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < M / 2; ++q) {
        if (8 * (q >> 2) < cnt) {                     // whole blocks (every block of a stored row is valid memory)
            const v2i x = *(reinterpret_cast<const v2i*>(lblock(base, N, i, q >> 2)) + (q & 3));
            l[2 * q] = x.x;
            l[2 * q + 1] = x.y;
        }
    }
#pragma unroll
    for (int t = 1; t < M; ++t) l[t] = t < cnt ? l[t] : l[0];
}

// Store l[0 .. ceil(cnt / 8) * 8) as row i's first blocks (entries past cnt inside the last block are whatever l holds:
// readers never use columns >= the stored count).
template <int K, bool NT = false>
PCD_DEV void store_list(int32_t* base, int64_t N, int64_t i, int cnt, const int (&l)[K]) {
    static_assert(K % 8 == 0, "lists are whole 8-column blocks");
#pragma unroll
    for (int g = 0; g < K / 8; ++g) {
        if (8 * g < cnt) {
            v4i* p = lblock(base, N, i, g);
            const v4i a = {l[8 * g + 0], l[8 * g + 1], l[8 * g + 2], l[8 * g + 3]};
            const v4i b = {l[8 * g + 4], l[8 * g + 5], l[8 * g + 6], l[8 * g + 7]};
            // (16-B halves of a sector from two instructions: measured equal to plain stores and to lane pairs that
            // write whole sectors per instruction -- L2 merges the halves)
            if (NT) { __builtin_nontemporal_store(a, p); __builtin_nontemporal_store(b, p + 1); }
            else { p[0] = a; p[1] = b; }
        }
    }
}

}  // namespace pcd
