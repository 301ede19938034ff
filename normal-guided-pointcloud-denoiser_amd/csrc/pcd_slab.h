// Spatial slabs on the device: the halo transport and one C call per slab iteration.
// The second half of denoise.hip -- included once at its end, because pcd_slab_iterate drives the same static stage
// functions as pcd_denoiser_iterate.
//
// Transport (pcd_comm): RCCL over xGMI (ncclSend / ncclRecv to the slab neighbours inside one ncclGroupStart/End,
// ncclAllReduce for the flat phase's global centre and delta, Denoiser.py:106-107), or host callbacks for callers
// without RCCL (the gloo tests: the same iteration code, with each exchange staged through pinned host memory).
//
// One slab iteration (the body of Processor.denoise, Processor.py:123-139, over the rank's own rows):
//   main stream                                        exchange stream
//   K1: anchor test, re-anchoring search  ...........  (previous iteration's position exchange in flight)
//       wait for it -> NVT1 (+ band flags)
//                                                      pack f_n of the send rows -> send / recv -> unpack
//   NVT2 of the rows that read no halo row  ........   (in flight)
//   wait -> NVT2 of the others
//   flat: sum -> all-reduce(sum) -> centre -> max distance -> all-reduce(max) -> apply
//                                                      positions after the phase -> send / recv -> unpack
//   edge: apply to the no-halo rows  ................  (in flight)
//   wait -> apply to the others
//                                                      positions -> ...
//   corner: the same; n := f_n
//                                                      positions (waited for by the next NVT1 or any other call)
// A row "reads no halo row" when its k-ball lies strictly inside the owned slab (Band, marked by NVT1 from its own
// k-th distance): every snapshot point there is owned.  The passes split each stage's rows, never its arithmetic, so
// the result is bit-identical to the staged path and to one GPU (tests/test_gpu_slab.py).

#include <rccl/rccl.h>

struct pcd_comm {
    int rank = 0, world = 1;
    ncclComm_t nccl = nullptr;    // RCCL (null: host transport)
    pcd_host_transport host{};
};

namespace pcd {

__global__ void k_xpack(XField f, const int32_t* __restrict__ rows, int64_t n, float4* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    out[t] = (f.b && ((f.moved >> (f.cls[r] & 31u)) & 1u)) ? f.b[r] : f.a[r];
}
__global__ void k_xunpack(XField f, const int32_t* __restrict__ rows, int64_t n, const float4* __restrict__ in) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    const float4 v = in[t];
    f.da[r] = v;
    if (f.db) f.db[r] = v;
}
// The RCCL path moves 12-byte rows (x, y, z: every exchanged field's w is unused -- positions and unit normals), a
// quarter less over xGMI than float4 rows; the receiver keeps its own w.
__global__ void k_xpack3(XField f, const int32_t* __restrict__ rows, int64_t n, float* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    const float4 v = (f.b && ((f.moved >> (f.cls[r] & 31u)) & 1u)) ? f.b[r] : f.a[r];
    out[3 * t] = v.x; out[3 * t + 1] = v.y; out[3 * t + 2] = v.z;
}
__global__ void k_xunpack3(XField f, const int32_t* __restrict__ rows, int64_t n, const float* __restrict__ in) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    const float x = in[3 * t], y = in[3 * t + 1], z = in[3 * t + 2];
    f.da[r] = make_float4(x, y, z, f.da[r].w);
    if (f.db) f.db[r] = make_float4(x, y, z, f.db[r].w);
}

// ---- read-set exchange: after the kNN, each rank marks the halo rows its own lists read; the peers send only those
// (masks over the routes travel as bits, each route's mask padded to whole 4-word rows)
__global__ void k_rpos(const int32_t* __restrict__ rrows, int64_t nr, int32_t* __restrict__ rpos) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < nr) rpos[rrows[t]] = (int32_t)t;
}
// the Band test of every own row (its k-ball leaves the owned slab: flag 1, it may read a halo row) from its stored
// list, and the marks of the halo rows those rows' lists hold
template <int K>
__global__ void k_readset_mark(GridView g, const float4* __restrict__ pos, const int32_t* __restrict__ idx, int64_t N,
                               RowMap rm, int kstore, Cover own, uint8_t* __restrict__ bflag,
                               const int32_t* __restrict__ rpos, uint8_t* __restrict__ rmark) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= rm.nq) return;
    const int64_t i = rm(t);
    int l[K];
    load_list<K>(idx, N, i, kstore, l);
    const float4 p4 = pos[i];
    const Vec3 vi = v3(p4.x, p4.y, p4.z);
    float dk = 0.f;
#pragma unroll
    for (int u = 0; u < K; ++u)
        if (u == kstore - 1 && (uint32_t)l[u] < (uint32_t)N) dk = dist2(vi, g.pts[l[u]]);
    const bool out = !own.holds(vi, dk);
    bflag[t] = out ? 1 : 0;
    if (!out) return;
#pragma unroll
    for (int u = 0; u < K; ++u) {
        if (u < kstore && (uint32_t)l[u] < (uint32_t)N) {
            const int32_t r = rpos[l[u]];
            if (r >= 0) rmark[r] = 1;
        }
    }
}
// segments of a route (per peer): rows [off[q], off[q+1]), mask words [woff[q], woff[q+1])
struct SegLayout {
    int n;
    const int64_t* off;
    const int64_t* woff;
    PCD_DEV int seg(int64_t w) const { int q = 0; while (q + 1 < n && w >= woff[q + 1]) ++q; return q; }
};
__global__ void k_mask_words(const uint8_t* __restrict__ mark, SegLayout L, int64_t W, uint32_t* __restrict__ words,
                             uint32_t* __restrict__ popc) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w >= W) return;
    const int q = L.seg(w);
    const int64_t base = L.off[q] + 32 * (w - L.woff[q]);
    const int64_t cnt = L.off[q + 1] - base;
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b)
        if (b < cnt && mark[base + b]) bits |= 1u << b;
    words[w] = bits;
    popc[w] = (uint32_t)__popc(bits);
}
__global__ void k_word_popc(const uint32_t* __restrict__ words, int64_t W, uint32_t* __restrict__ popc) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w < W) popc[w] = (uint32_t)__popc(words[w]);
}
// exclusive scan of W counts (one block; W is a route's row count / 32), out[W] = the total
__global__ __launch_bounds__(1024) void k_scan_excl(const uint32_t* __restrict__ in, int64_t W, uint32_t* __restrict__ out) {
    __shared__ uint32_t s[1024];
    const int64_t per = (W + 1023) / 1024;
    const int64_t a = threadIdx.x * per, b = a + per < W ? a + per : W;
    uint32_t sum = 0;
    for (int64_t i = a; i < b; ++i) sum += in[i];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t v = (int)threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - sum;
    for (int64_t i = a; i < b; ++i) { out[i] = run; run += in[i]; }
    if (threadIdx.x == 1023) out[W] = s[1023];
}
__global__ void k_compact_words(const uint32_t* __restrict__ words, const uint32_t* __restrict__ scan, SegLayout L,
                                int64_t W, const int32_t* __restrict__ rows, int32_t* __restrict__ sel) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w >= W) return;
    uint32_t bits = words[w];
    if (!bits) return;
    const int q = L.seg(w);
    const int64_t base = L.off[q] + 32 * (w - L.woff[q]);
    uint32_t o = scan[w];
    while (bits) {
        const int b = __ffs(bits) - 1;
        bits &= bits - 1;
        sel[o++] = rows[base + b];
    }
}
__global__ void k_seg_offsets(const uint32_t* __restrict__ scan, const int64_t* __restrict__ woff, int n,
                              int64_t* __restrict__ out) {
    const int q = (int)threadIdx.x;
    if (q <= n) out[q] = (int64_t)scan[woff[q]];
}
// the refresh at K1: position (both buffers) and normal of each selected row, 6 floats (RCCL) or 2 float4 (host)
__global__ void k_rpack6(const float4* __restrict__ pos, const float4* __restrict__ nrm, const int32_t* __restrict__ rows,
                         int64_t n, int stride, float* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    const float4 a = pos[r], b = nrm[r];
    float* o = out + (int64_t)stride * t;
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = b.x; o[4] = b.y; o[5] = b.z;
}
__global__ void k_runpack6(float4* __restrict__ pa, float4* __restrict__ pb, float4* __restrict__ nrm,
                           const int32_t* __restrict__ rows, int64_t n, int stride, const float* __restrict__ in) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t r = rows[t];
    const float* v = in + (int64_t)stride * t;
    pa[r] = make_float4(v[0], v[1], v[2], pa[r].w);
    if (pb) pb[r] = make_float4(v[0], v[1], v[2], pb[r].w);
    nrm[r] = make_float4(v[3], v[4], v[5], nrm[r].w);
}

}  // namespace pcd

static int rccl_fail(ncclResult_t r, const char* what) {
    return fail(PCD_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}
#define PCD_NCCL(call)                                                   \
    do {                                                                 \
        const ncclResult_t r_ = (call);                                  \
        if (r_ != ncclSuccess) return rccl_fail(r_, #call);              \
    } while (0)

// the main stream waits for an exchange in flight (any call that reads or writes the state does this first)
static int settle(pcd_denoiser* dn, hipStream_t st) {
    if (dn->xpending) {
        PCD_HIP(hipStreamWaitEvent(st, dn->xev_out, 0));
        dn->xpending = false;
    }
    return PCD_OK;
}

static int ensure_xstream(pcd_denoiser* dn) {
    if (!dn->xst) {
        PCD_HIP(hipStreamCreateWithFlags(&dn->xst, hipStreamNonBlocking));
        PCD_HIP(hipEventCreateWithFlags(&dn->xev_in, hipEventDisableTiming));
        PCD_HIP(hipEventCreateWithFlags(&dn->xev_out, hipEventDisableTiming));
    }
    return PCD_OK;
}

// Start exchanging field f with every peer, ordered after the work already on st.  RCCL: the whole exchange is
// enqueued on the exchange stream.  Host transport: the pack and the device -> host copy; xchg_end runs the callback.
// the routes an exchange uses: every halo row, or this iteration's read set (use_sel)
struct XRoutes {
    const int32_t* s;
    const int32_t* r;
    const std::vector<int64_t>& so;
    const std::vector<int64_t>& ro;
};
static XRoutes xroutes(const pcd_denoiser* dn) {
    return dn->use_sel ? XRoutes{dn->sel_srows, dn->sel_rrows, dn->sel_soff, dn->sel_roff}
                       : XRoutes{dn->srows, dn->rrows, dn->soff, dn->roff};
}

static int xchg_begin(pcd_denoiser* dn, pcd_comm* c, hipStream_t st, const XField& f) {
    if (dn->npeers == 0) return PCD_OK;
    const int rc = ensure_xstream(dn);
    if (rc != PCD_OK) return rc;
    hipStream_t xs = dn->xst;
    const XRoutes R = xroutes(dn);
    const int64_t ns = R.so[dn->npeers], nr = R.ro[dn->npeers];
    PCD_HIP(hipEventRecord(dn->xev_in, st));
    PCD_HIP(hipStreamWaitEvent(xs, dn->xev_in, 0));
    dn->xfield = f;
    if (c->nccl) {
        float* sb = reinterpret_cast<float*>(dn->sbuf);
        float* rb = reinterpret_cast<float*>(dn->rbuf);
        if (ns > 0) hipLaunchKernelGGL(k_xpack3, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, f, R.s, ns, sb);
        PCD_LAUNCH_CHECK();
        PCD_NCCL(ncclGroupStart());
        for (int q = 0; q < dn->npeers; ++q) {
            const int64_t s0 = R.so[q], s1 = R.so[q + 1], r0 = R.ro[q], r1 = R.ro[q + 1];
            if (s1 > s0) PCD_NCCL(ncclSend(sb + 3 * s0, (size_t)(s1 - s0) * 3, ncclFloat, dn->peers[q], c->nccl, xs));
            if (r1 > r0) PCD_NCCL(ncclRecv(rb + 3 * r0, (size_t)(r1 - r0) * 3, ncclFloat, dn->peers[q], c->nccl, xs));
        }
        PCD_NCCL(ncclGroupEnd());
        if (nr > 0) hipLaunchKernelGGL(k_xunpack3, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, f, R.r, nr, rb);
        PCD_LAUNCH_CHECK();
        PCD_HIP(hipEventRecord(dn->xev_out, xs));
        dn->xpending = true;
    } else {
        if (ns > 0) hipLaunchKernelGGL(k_xpack, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, f, R.s, ns, dn->sbuf);
        PCD_LAUNCH_CHECK();
        if (ns > 0) PCD_HIP(hipMemcpyAsync(dn->hs, dn->sbuf, ns * sizeof(float4), hipMemcpyDeviceToHost, xs));
        dn->xbegun = true;
    }
    return PCD_OK;
}

// Host transport: wait for the packed rows, hand them to the callback, unpack what it received.
static int xchg_end(pcd_denoiser* dn, pcd_comm* c) {
    if (!dn->xbegun) return PCD_OK;
    dn->xbegun = false;
    hipStream_t xs = dn->xst;
    const XRoutes R = xroutes(dn);
    const int64_t nr = R.ro[dn->npeers];
    PCD_HIP(hipStreamSynchronize(xs));
    if (c->host.exchange(c->host.user, dn->npeers, dn->peers.data(), reinterpret_cast<const float*>(dn->hs),
                         R.so.data(), reinterpret_cast<float*>(dn->hr), R.ro.data()) != 0)
        return fail(PCD_ERR_RCCL, "pcd_slab: host transport exchange callback failed");
    if (nr > 0) {
        PCD_HIP(hipMemcpyAsync(dn->rbuf, dn->hr, nr * sizeof(float4), hipMemcpyHostToDevice, xs));
        hipLaunchKernelGGL(k_xunpack, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, dn->xfield, R.r, nr, dn->rbuf);
        PCD_LAUNCH_CHECK();
    }
    PCD_HIP(hipEventRecord(dn->xev_out, xs));
    dn->xpending = true;
    return PCD_OK;
}

static int xchg_wait(pcd_denoiser* dn, pcd_comm* c, hipStream_t st) {
    int rc = xchg_end(dn, c);
    if (rc != PCD_OK) return rc;
    return settle(dn, st);
}

static ncclDataType_t nccl_dtype(int dt) {
    return dt == PCD_DT_F64 ? ncclFloat64 : dt == PCD_DT_I32 ? ncclInt32 : ncclFloat32;
}
static size_t dt_bytes(int dt) { return dt == PCD_DT_F64 ? 8 : 4; }

static int allreduce(pcd_comm* c, void* buf, int count, int dt, int op, hipStream_t st) {
    if (count == 0 || (c->world == 1 && !c->nccl)) return PCD_OK;
    if (c->nccl) {
        PCD_NCCL(ncclAllReduce(buf, buf, (size_t)count, nccl_dtype(dt), op == PCD_OP_MAX ? ncclMax : ncclSum,
                               c->nccl, st));
        return PCD_OK;
    }
    std::vector<unsigned char> h((size_t)count * dt_bytes(dt));
    PCD_HIP(hipMemcpyAsync(h.data(), buf, h.size(), hipMemcpyDeviceToHost, st));
    PCD_HIP(hipStreamSynchronize(st));
    if (c->host.allreduce(c->host.user, h.data(), count, dt, op) != 0)
        return fail(PCD_ERR_RCCL, "pcd_slab: host transport all-reduce callback failed");
    PCD_HIP(hipMemcpyAsync(buf, h.data(), h.size(), hipMemcpyHostToDevice, st));
    PCD_HIP(hipStreamSynchronize(st));
    return PCD_OK;
}

static void free_routes(pcd_denoiser* dn) {
    (void)hipFree(dn->srows); (void)hipFree(dn->rrows); (void)hipFree(dn->sbuf); (void)hipFree(dn->rbuf);
    (void)hipHostFree(dn->hs); (void)hipHostFree(dn->hr); (void)hipFree(dn->bflag);
    (void)hipFree(dn->rpos); (void)hipFree(dn->rmark); (void)hipFree(dn->rwords); (void)hipFree(dn->swords);
    (void)hipFree(dn->wpopc); (void)hipFree(dn->wscan); (void)hipFree(dn->sel_srows); (void)hipFree(dn->sel_rrows);
    (void)hipFree(dn->xoff_d); (void)hipFree(dn->seloff_d); (void)hipHostFree(dn->seloff_h);
    dn->srows = dn->rrows = nullptr;
    dn->sbuf = dn->rbuf = dn->hs = dn->hr = nullptr;
    dn->bflag = nullptr;
    dn->rpos = dn->sel_srows = dn->sel_rrows = nullptr;
    dn->rmark = nullptr;
    dn->rwords = dn->swords = dn->wpopc = dn->wscan = nullptr;
    dn->xoff_d = dn->seloff_d = dn->seloff_h = nullptr;
    dn->use_sel = false;
    dn->npeers = 0;
    dn->peers.clear();
    dn->soff.assign(1, 0);
    dn->roff.assign(1, 0);
    dn->rwoff.assign(1, 0);
    dn->swoff.assign(1, 0);
    dn->sel_soff.assign(1, 0);
    dn->sel_roff.assign(1, 0);
}

static void destroy_slab_state(pcd_denoiser* dn) {
    if (dn->xst) (void)hipStreamSynchronize(dn->xst);
    free_routes(dn);
    if (dn->xst) (void)hipStreamDestroy(dn->xst);
    if (dn->xev_in) (void)hipEventDestroy(dn->xev_in);
    if (dn->xev_out) (void)hipEventDestroy(dn->xev_out);
    if (dn->rs_ev) (void)hipEventDestroy(dn->rs_ev);
}

// Read-set exchange, part A (main stream, after a lists-only K1): the band flags, the marks of the halo rows the
// flagged rows' lists hold, and this rank's receive selection (rs_ev after it; its per-peer offsets -> pinned host).
static int readset_mark(pcd_denoiser* dn, const pcd_denoise_params* p, hipStream_t st) {
    const RowMap rm = dn->rowmap();
    const int np = dn->npeers;
    const int64_t nr = dn->roff[np], RW = dn->rwoff[np];
    const int kstore = std::max(p->k, p->k_update);
    if (nr > 0) PCD_HIP(hipMemsetAsync(dn->rmark, 0, nr, st));
    if (rm.nq > 0) {
        const dim3 blk(256), grd((unsigned)cdiv(rm.nq, 256));
        const GridView gv = dn->g->view;
        const float4* P = dn->pos[dn->cur];
        switch (list_cap(p)) {
            case 8: hipLaunchKernelGGL(k_readset_mark<8>, grd, blk, 0, st, gv, P, dn->idx, dn->n, rm, kstore, dn->own,
                                       dn->bflag, dn->rpos, dn->rmark); break;
            case 16: hipLaunchKernelGGL(k_readset_mark<16>, grd, blk, 0, st, gv, P, dn->idx, dn->n, rm, kstore, dn->own,
                                        dn->bflag, dn->rpos, dn->rmark); break;
            case 32: hipLaunchKernelGGL(k_readset_mark<32>, grd, blk, 0, st, gv, P, dn->idx, dn->n, rm, kstore, dn->own,
                                        dn->bflag, dn->rpos, dn->rmark); break;
            default: return fail(PCD_ERR_ARG, "readset_mark: unsupported k");
        }
        PCD_LAUNCH_CHECK();
    }
    const SegLayout L{np, dn->xoff_d, dn->xoff_d + 2 * (np + 1)};
    if (RW > 0) hipLaunchKernelGGL(k_mask_words, dim3((unsigned)cdiv(RW, 256)), dim3(256), 0, st, dn->rmark, L, RW, dn->rwords, dn->wpopc);
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, st, dn->wpopc, RW, dn->wscan);
    if (RW > 0) hipLaunchKernelGGL(k_compact_words, dim3((unsigned)cdiv(RW, 256)), dim3(256), 0, st, dn->rwords, dn->wscan, L, RW, dn->rrows, dn->sel_rrows);
    hipLaunchKernelGGL(k_seg_offsets, dim3(1), dim3(64), 0, st, dn->wscan, L.woff, np, dn->seloff_d);
    PCD_LAUNCH_CHECK();
    PCD_HIP(hipMemcpyAsync(dn->seloff_h, dn->seloff_d, (np + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PCD_HIP(hipEventRecord(dn->rs_ev, st));
    return PCD_OK;
}

// Part B (host waits for part A; the main stream runs NVT1 of the rows that read no halo row meanwhile): the masks
// to / from the peers, this rank's send selection, then the refresh of the selected rows' position + normal in
// flight on the exchange stream (xev_out).  The iteration's later exchanges use the selection (use_sel).
static int readset_exchange(pcd_denoiser* dn, pcd_comm* c) {
    const int np = dn->npeers;
    hipStream_t xs = dn->xst;
    PCD_HIP(hipEventSynchronize(dn->rs_ev));
    dn->sel_roff.assign(dn->seloff_h, dn->seloff_h + np + 1);
    const int64_t RW = dn->rwoff[np], SW = dn->swoff[np];
    if (c->nccl) {
        PCD_HIP(hipStreamWaitEvent(xs, dn->rs_ev, 0));
        PCD_NCCL(ncclGroupStart());
        for (int q = 0; q < np; ++q) {
            const int64_t w0 = dn->rwoff[q], w1 = dn->rwoff[q + 1], v0 = dn->swoff[q], v1 = dn->swoff[q + 1];
            if (w1 > w0) PCD_NCCL(ncclSend(dn->rwords + w0, (size_t)(w1 - w0), ncclUint32, dn->peers[q], c->nccl, xs));
            if (v1 > v0) PCD_NCCL(ncclRecv(dn->swords + v0, (size_t)(v1 - v0), ncclUint32, dn->peers[q], c->nccl, xs));
        }
        PCD_NCCL(ncclGroupEnd());
    } else {
        // host transport: the words as float4 rows (every segment is whole 4-word rows)
        if (RW > 0) PCD_HIP(hipMemcpyAsync(dn->hs, dn->rwords, RW * sizeof(uint32_t), hipMemcpyDeviceToHost, xs));
        PCD_HIP(hipStreamSynchronize(xs));
        std::vector<int64_t> so(np + 1), ro(np + 1);
        for (int q = 0; q <= np; ++q) { so[q] = dn->rwoff[q] / 4; ro[q] = dn->swoff[q] / 4; }
        if (c->host.exchange(c->host.user, np, dn->peers.data(), reinterpret_cast<const float*>(dn->hs), so.data(),
                             reinterpret_cast<float*>(dn->hr), ro.data()) != 0)
            return fail(PCD_ERR_RCCL, "pcd_slab: host transport exchange callback failed (read-set masks)");
        if (SW > 0) PCD_HIP(hipMemcpyAsync(dn->swords, dn->hr, SW * sizeof(uint32_t), hipMemcpyHostToDevice, xs));
    }
    const SegLayout L{np, dn->xoff_d + (np + 1), dn->xoff_d + 3 * (np + 1)};
    if (SW > 0) hipLaunchKernelGGL(k_word_popc, dim3((unsigned)cdiv(SW, 256)), dim3(256), 0, xs, dn->swords, SW, dn->wpopc);
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, xs, dn->wpopc, SW, dn->wscan);
    if (SW > 0) hipLaunchKernelGGL(k_compact_words, dim3((unsigned)cdiv(SW, 256)), dim3(256), 0, xs, dn->swords, dn->wscan, L, SW, dn->srows, dn->sel_srows);
    hipLaunchKernelGGL(k_seg_offsets, dim3(1), dim3(64), 0, xs, dn->wscan, L.woff, np, dn->seloff_d + (np + 1));
    PCD_LAUNCH_CHECK();
    PCD_HIP(hipMemcpyAsync(dn->seloff_h + (np + 1), dn->seloff_d + (np + 1), (np + 1) * sizeof(int64_t),
                           hipMemcpyDeviceToHost, xs));
    PCD_HIP(hipStreamSynchronize(xs));
    dn->sel_soff.assign(dn->seloff_h + np + 1, dn->seloff_h + 2 * (np + 1));
    dn->use_sel = true;
    const int64_t ns = dn->sel_soff[np], nr = dn->sel_roff[np];
    dn->rs_iters += 1;
    dn->rs_send_rows += ns;
    dn->rs_recv_rows += nr;
    // the refresh: position (both buffers: the copy-free phases read either) and normal of each selected row
    float4* pa = dn->pos[dn->cur];
    float4* pb = dn->pos[dn->cur ^ 1];
    float* sb = reinterpret_cast<float*>(dn->sbuf);
    float* rb = reinterpret_cast<float*>(dn->rbuf);
    if (c->nccl) {
        if (ns > 0) hipLaunchKernelGGL(k_rpack6, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, pa, dn->nrm, dn->sel_srows, ns, 6, sb);
        PCD_LAUNCH_CHECK();
        PCD_NCCL(ncclGroupStart());
        for (int q = 0; q < np; ++q) {
            const int64_t s0 = dn->sel_soff[q], s1 = dn->sel_soff[q + 1], r0 = dn->sel_roff[q], r1 = dn->sel_roff[q + 1];
            if (s1 > s0) PCD_NCCL(ncclSend(sb + 6 * s0, (size_t)(s1 - s0) * 6, ncclFloat, dn->peers[q], c->nccl, xs));
            if (r1 > r0) PCD_NCCL(ncclRecv(rb + 6 * r0, (size_t)(r1 - r0) * 6, ncclFloat, dn->peers[q], c->nccl, xs));
        }
        PCD_NCCL(ncclGroupEnd());
        if (nr > 0) hipLaunchKernelGGL(k_runpack6, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, pa, pb, dn->nrm, dn->sel_rrows, nr, 6, rb);
        PCD_LAUNCH_CHECK();
    } else {
        if (ns > 0) hipLaunchKernelGGL(k_rpack6, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, pa, dn->nrm, dn->sel_srows, ns, 8, sb);
        PCD_LAUNCH_CHECK();
        if (ns > 0) PCD_HIP(hipMemcpyAsync(dn->hs, sb, ns * 2 * sizeof(float4), hipMemcpyDeviceToHost, xs));
        PCD_HIP(hipStreamSynchronize(xs));
        std::vector<int64_t> so(np + 1), ro(np + 1);
        for (int q = 0; q <= np; ++q) { so[q] = 2 * dn->sel_soff[q]; ro[q] = 2 * dn->sel_roff[q]; }
        if (c->host.exchange(c->host.user, np, dn->peers.data(), reinterpret_cast<const float*>(dn->hs), so.data(),
                             reinterpret_cast<float*>(dn->hr), ro.data()) != 0)
            return fail(PCD_ERR_RCCL, "pcd_slab: host transport exchange callback failed (read-set refresh)");
        if (nr > 0) {
            PCD_HIP(hipMemcpyAsync(rb, dn->hr, nr * 2 * sizeof(float4), hipMemcpyHostToDevice, xs));
            hipLaunchKernelGGL(k_runpack6, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, pa, pb, dn->nrm, dn->sel_rrows, nr, 8, rb);
            PCD_LAUNCH_CHECK();
        }
    }
    PCD_HIP(hipEventRecord(dn->xev_out, xs));
    dn->xpending = true;
    return PCD_OK;
}

extern "C" {

int pcd_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int pcd_comm_id(void* id_out) {
    PCD_CHECK_ARG(id_out != nullptr, "null argument");
    ncclUniqueId id;
    PCD_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof id);
    return PCD_OK;
}

int pcd_comm_create(const void* id, int world, int rank, pcd_comm** out) {
    PCD_CHECK_ARG(out != nullptr, "out is null");
    *out = nullptr;
    PCD_CHECK_ARG(id != nullptr, "id is null");
    PCD_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "bad world / rank");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    pcd_comm* c = new pcd_comm();
    c->rank = rank;
    c->world = world;
    const ncclResult_t r = ncclCommInitRank(&c->nccl, world, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return rccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
    return PCD_OK;
}

int pcd_comm_create_host(const pcd_host_transport* t, int world, int rank, pcd_comm** out) {
    PCD_CHECK_ARG(out != nullptr, "out is null");
    *out = nullptr;
    PCD_CHECK_ARG(t && t->exchange && t->allreduce, "host transport needs exchange and allreduce callbacks");
    PCD_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "bad world / rank");
    pcd_comm* c = new pcd_comm();
    c->rank = rank;
    c->world = world;
    c->host = *t;
    *out = c;
    return PCD_OK;
}

int pcd_comm_destroy(pcd_comm* c) {
    if (!c) return PCD_OK;
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    delete c;
    return PCD_OK;
}

int pcd_comm_info(const pcd_comm* c, int* world, int* rank, int* transport) {
    PCD_CHECK_ARG(c != nullptr, "null comm");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    if (transport) *transport = c->nccl ? PCD_COMM_RCCL : PCD_COMM_HOST;
    return PCD_OK;
}

int pcd_comm_sendrecv(pcd_comm* c, int send_peer, const void* send, int64_t send_bytes, int recv_peer, void* recv,
                      int64_t recv_bytes, void* stream) {
    PCD_CHECK_ARG(c != nullptr, "null comm");
    PCD_CHECK_ARG(send_peer >= -1 && send_peer < c->world && recv_peer >= -1 && recv_peer < c->world, "bad peer");
    PCD_CHECK_ARG(send_bytes >= 0 && recv_bytes >= 0 && send_bytes % 4 == 0 && recv_bytes % 4 == 0,
                  "byte counts must be non-negative multiples of 4");
    const bool tx = send_peer >= 0 && send_bytes > 0, rx = recv_peer >= 0 && recv_bytes > 0;
    PCD_CHECK_ARG((!tx || send) && (!rx || recv), "null buffer");
    if (!tx && !rx) return PCD_OK;
    hipStream_t st = as_stream(stream);
    if (c->nccl) {
        PCD_NCCL(ncclGroupStart());
        if (tx) PCD_NCCL(ncclSend(send, (size_t)send_bytes, ncclChar, send_peer, c->nccl, st));
        if (rx) PCD_NCCL(ncclRecv(recv, (size_t)recv_bytes, ncclChar, recv_peer, c->nccl, st));
        PCD_NCCL(ncclGroupEnd());
        return PCD_OK;
    }
    // host transport: one exchange callback over at most two peers, the payloads as whole float4 rows
    const int64_t srows = tx ? (send_bytes + 15) / 16 : 0, rrows = rx ? (recv_bytes + 15) / 16 : 0;
    std::vector<float4> hs((size_t)std::max<int64_t>(srows, 1)), hr((size_t)std::max<int64_t>(rrows, 1));
    if (tx) PCD_HIP(hipMemcpyAsync(hs.data(), send, (size_t)send_bytes, hipMemcpyDeviceToHost, st));
    PCD_HIP(hipStreamSynchronize(st));
    std::vector<int> peers;
    std::vector<int64_t> so(1, 0), ro(1, 0);
    if (tx) { peers.push_back(send_peer); so.push_back(srows); ro.push_back(send_peer == recv_peer && rx ? rrows : 0); }
    if (rx && !(tx && send_peer == recv_peer)) { peers.push_back(recv_peer); so.push_back(so.back()); ro.push_back(rrows); }
    if (c->host.exchange(c->host.user, (int)peers.size(), peers.data(), reinterpret_cast<const float*>(hs.data()),
                         so.data(), reinterpret_cast<float*>(hr.data()), ro.data()) != 0)
        return fail(PCD_ERR_RCCL, "pcd_comm_sendrecv: host transport exchange callback failed");
    if (rx) {
        PCD_HIP(hipMemcpyAsync(recv, hr.data(), (size_t)recv_bytes, hipMemcpyHostToDevice, st));
        PCD_HIP(hipStreamSynchronize(st));
    }
    return PCD_OK;
}

int pcd_allreduce_scalars(pcd_comm* c, void* buf, int count, int dtype, int op, void* stream) {
    PCD_CHECK_ARG(c != nullptr, "null comm");
    PCD_CHECK_ARG(count >= 0 && (count == 0 || buf), "null buffer");
    PCD_CHECK_ARG(dtype >= PCD_DT_F32 && dtype <= PCD_DT_I32 && (op == PCD_OP_SUM || op == PCD_OP_MAX), "bad dtype / op");
    return allreduce(c, buf, count, dtype, op, as_stream(stream));
}

int pcd_denoiser_set_routes(pcd_denoiser* dn, int npeers, const int* peers, const int64_t* n_send,
                            const int32_t* send_rows, const int64_t* n_recv, const int32_t* recv_rows,
                            const float* own_lo3, const float* own_hi3, void* stream) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    PCD_CHECK_ARG(npeers >= 0 && (npeers == 0 || (peers && n_send && n_recv)), "bad peer list");
    hipStream_t st = as_stream(stream);
    int rc = settle(dn, st);
    if (rc != PCD_OK) return rc;
    if (dn->xst) PCD_HIP(hipStreamSynchronize(dn->xst));
    free_routes(dn);
    std::vector<int64_t> so(1, 0), ro(1, 0);
    for (int q = 0; q < npeers; ++q) {
        PCD_CHECK_ARG(n_send[q] >= 0 && n_recv[q] >= 0, "negative row count");
        so.push_back(so.back() + n_send[q]);
        ro.push_back(ro.back() + n_recv[q]);
    }
    PCD_CHECK_ARG(so.back() == 0 || send_rows, "send_rows is null");
    PCD_CHECK_ARG(ro.back() == 0 || recv_rows, "recv_rows is null");
    const int64_t ns = so.back(), nr = ro.back();
    if (npeers > 0) {
        // read-set masks: per peer ceil(rows / 32) words, padded to whole 4-word rows (the host transport's unit)
        std::vector<int64_t> sw(1, 0), rw(1, 0);
        for (int q = 0; q < npeers; ++q) {
            sw.push_back(sw.back() + 4 * cdiv(cdiv(n_send[q], 32), 4));
            rw.push_back(rw.back() + 4 * cdiv(cdiv(n_recv[q], 32), 4));
        }
        const int64_t SW = sw.back(), RW = rw.back(), MW = std::max<int64_t>(std::max(SW, RW), 1);
        // staging: 2 float4 a row (the read-set refresh moves position + normal), and the mask words
        const int64_t sst = std::max<int64_t>(2 * ns, SW / 4) + 1, rst = std::max<int64_t>(2 * nr, RW / 4) + 1;
        if (hipMalloc(&dn->srows, std::max<int64_t>(ns, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->rrows, std::max<int64_t>(nr, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->sbuf, sst * sizeof(float4)) != hipSuccess ||
            hipMalloc(&dn->rbuf, rst * sizeof(float4)) != hipSuccess ||
            hipHostMalloc(&dn->hs, sst * sizeof(float4), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&dn->hr, rst * sizeof(float4), hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&dn->rpos, std::max<int64_t>(dn->n, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->rmark, std::max<int64_t>(nr, 1)) != hipSuccess ||
            hipMalloc(&dn->rwords, std::max<int64_t>(RW, 1) * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&dn->swords, std::max<int64_t>(SW, 1) * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&dn->wpopc, MW * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&dn->wscan, (MW + 1) * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&dn->sel_srows, std::max<int64_t>(ns, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->sel_rrows, std::max<int64_t>(nr, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->xoff_d, 4 * (npeers + 1) * sizeof(int64_t)) != hipSuccess ||
            hipMalloc(&dn->seloff_d, 2 * (npeers + 1) * sizeof(int64_t)) != hipSuccess ||
            hipHostMalloc(&dn->seloff_h, 2 * (npeers + 1) * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) {
            free_routes(dn);
            return fail(PCD_ERR_OOM, "pcd_denoiser_set_routes: buffers");
        }
        if (ns > 0) PCD_HIP(hipMemcpyAsync(dn->srows, send_rows, ns * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        if (nr > 0) PCD_HIP(hipMemcpyAsync(dn->rrows, recv_rows, nr * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        PCD_HIP(hipMemsetAsync(dn->rpos, 0xFF, std::max<int64_t>(dn->n, 1) * sizeof(int32_t), st));
        if (nr > 0) hipLaunchKernelGGL(k_rpos, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, st, dn->rrows, nr, dn->rpos);
        PCD_LAUNCH_CHECK();
        std::vector<int64_t> xo;
        for (const auto* v : {&ro, &so, &rw, &sw}) xo.insert(xo.end(), v->begin(), v->end());
        PCD_HIP(hipMemcpyAsync(dn->xoff_d, xo.data(), xo.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
        dn->peers.assign(peers, peers + npeers);
        dn->soff = so;
        dn->roff = ro;
        dn->swoff = sw;
        dn->rwoff = rw;
        dn->npeers = npeers;
        if (!dn->rs_ev) PCD_HIP(hipEventCreateWithFlags(&dn->rs_ev, hipEventDisableTiming));
        const char* e = std::getenv("PCD_SLAB_READSET");
        dn->readset = !(e && e[0] == '0');
        dn->rs_iters = dn->rs_send_rows = dn->rs_recv_rows = 0;
    }
    if (own_lo3 && own_hi3) {
        for (int a = 0; a < 3; ++a) {
            PCD_CHECK_ARG(!(own_lo3[a] > own_hi3[a]), "owned slab has lo > hi");
            dn->own.lo[a] = own_lo3[a];
            dn->own.hi[a] = own_hi3[a];
        }
        if (hipMalloc(&dn->bflag, dn->n) != hipSuccess) return fail(PCD_ERR_OOM, "pcd_denoiser_set_routes: band flags");
        PCD_HIP(hipMemsetAsync(dn->bflag, 1, dn->n, st));
    }
    PCD_HIP(hipStreamSynchronize(st));     // (the caller may free its row arrays once this returns)
    return ensure_xstream(dn);
}

int pcd_halo_exchange(pcd_denoiser* dn, pcd_comm* c, int field, void* stream) {
    PCD_CHECK_ARG(dn && c, "null argument");
    float4* f = field_ptr(dn, field);
    PCD_CHECK_ARG(f != nullptr, "bad field");
    hipStream_t st = as_stream(stream);
    int rc = settle(dn, st);
    if (rc != PCD_OK) return rc;
    dn->use_sel = false;                   // every halo row
    if (field == PCD_FIELD_POS || field == PCD_FIELD_NRM) dn->part_ph = dn->scan_ph = -1;
    if ((rc = xchg_begin(dn, c, st, XField{f, nullptr, nullptr, 0u, f, nullptr})) != PCD_OK) return rc;
    if ((rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
    if (field == PCD_FIELD_NRM) dn->unit_nrm = false;
    return PCD_OK;
}

int pcd_denoiser_set_readset(pcd_denoiser* dn, int on) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    dn->readset = on != 0;
    if (!dn->readset) dn->use_sel = false;
    return PCD_OK;
}

int pcd_denoiser_readset_stats(const pcd_denoiser* dn, int64_t* iterations, int64_t* send_rows, int64_t* recv_rows) {
    PCD_CHECK_ARG(dn != nullptr, "null denoiser");
    if (iterations) *iterations = dn->rs_iters;
    if (send_rows) *send_rows = dn->rs_send_rows;
    if (recv_rows) *recv_rows = dn->rs_recv_rows;
    return PCD_OK;
}

int pcd_slab_iterate(pcd_denoiser* dn, pcd_comm* c, const pcd_denoise_params* p, int iterations, void* stream) {
    int rc = check_params(dn, p);
    if (rc != PCD_OK) return rc;
    PCD_CHECK_ARG(c != nullptr, "null comm");
    PCD_CHECK_ARG(iterations >= 0, "iterations must be >= 0");
    hipStream_t st = as_stream(stream);
    const bool xchg = dn->npeers > 0;
    const bool overlap = xchg && dn->bflag != nullptr;
    // read-set exchange: the anchored K1 (its lists before its NVT1) with the owned slab's band flags.  Decided
    // from settings every rank shares (its protocol's messages pair across the ranks)
    const bool rs = overlap && dn->readset && dn->seeding && dn->anchoring && list_cap(p) <= 32 &&
                    knn_cap(dn->kcap) <= 32;
    if (rs && !k1_anchored(dn, p))
        return fail(PCD_ERR_ARG, "pcd_slab_iterate: the read-set exchange needs >= 2k local rows on every rank "
                                 "(PCD_SLAB_READSET=0 exchanges every halo row)");
    const RowSel all{nullptr, 0}, core{dn->bflag, 0}, edge_rows{dn->bflag, 1};
    const Band band = overlap ? Band{dn->own, dn->bflag} : kNoBand;
    // the fused loop's copy-free Gauss-Seidel phases (pcd_denoiser_iterate's condition): halo rows receive their
    // positions in both buffers, so a neighbour read through SplitRows sees the current position either way
    const bool split = !p->jacobi && p->nphases == 3 &&
                       ((1u << p->phase_class[0]) | (1u << p->phase_class[1]) | (1u << p->phase_class[2])) == 7u &&
                       !phase_is_global(p, 1) && !phase_is_global(p, 2);
    for (int it = 0; it < iterations; ++it) {
        hipEvent_t* ev = nullptr;
        if (dn->timing && dn->ev_used < kTimingSets) ev = &dn->ev[(size_t)dn->ev_used++ * kTimingEvents];
        if (ev) PCD_HIP(hipEventRecord(ev[0], st));
        // K1; its neighbour gathers (NVT1) wait for the previous iteration's position exchange
        if ((rc = xchg_end(dn, c)) != PCD_OK) return rc;
        if (rs) {
            // lists -> flags + marks -> NVT1 of the no-halo rows || masks, send selection, refresh -> NVT1 of the rest
            if ((rc = settle(dn, st)) != PCD_OK) return rc;
            dn->use_sel = false;
            if ((rc = stage_k1(dn, p, st, ev, kNoBand, nullptr, true)) != PCD_OK) return rc;
            if ((rc = readset_mark(dn, p, st)) != PCD_OK) return rc;
            if ((rc = stage_nvt1(dn, p, st, core)) != PCD_OK) return rc;
            if ((rc = readset_exchange(dn, c)) != PCD_OK) return rc;
            if ((rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
            if ((rc = stage_nvt1(dn, p, st, edge_rows)) != PCD_OK) return rc;
        } else {
            hipEvent_t before = dn->xpending ? dn->xev_out : nullptr;
            if (dn->rowmap().nq == 0 && before) PCD_HIP(hipStreamWaitEvent(st, before, 0));
            if ((rc = stage_k1(dn, p, st, ev, band, before)) != PCD_OK) return rc;
            dn->xpending = false;
        }
        if (ev) PCD_HIP(hipEventRecord(ev[4], st));
        // f_n of the send rows -> the peers; NVT2 of the rows that read no halo row meanwhile
        if (xchg && (rc = xchg_begin(dn, c, st, XField{dn->fn, nullptr, nullptr, 0u, dn->fn, nullptr})) != PCD_OK) return rc;
        if (overlap && (rc = stage_k2(dn, p, st, core)) != PCD_OK) return rc;
        if (xchg && (rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
        if ((rc = stage_k2(dn, p, st, overlap ? edge_rows : all)) != PCD_OK) return rc;
        if (ev) PCD_HIP(hipEventRecord(ev[5], st));
        uint32_t moved = 0;
        for (int ph = 0; ph < p->nphases; ++ph) {
            const bool inflight = dn->xbegun || dn->xpending;
            if (phase_is_global(p, ph)) {
                // the global centre / delta read every flat row's neighbours, halo rows included
                if (inflight && (rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
                double* red4 = dn->red + 4 * ph;
                float* delta = dn->gscal + 4 * ph + 3;
                if ((rc = stage_sum(dn, p, ph, red4, st)) != PCD_OK) return rc;
                if ((rc = allreduce(c, red4, 4, PCD_DT_F64, PCD_OP_SUM, st)) != PCD_OK) return rc;
                if ((rc = stage_centre(dn, ph, red4, st)) != PCD_OK) return rc;
                if ((rc = stage_maxdist(dn, p, ph, nullptr, st)) != PCD_OK) return rc;
                if ((rc = allreduce(c, delta, 1, PCD_DT_F32, PCD_OP_MAX, st)) != PCD_OK) return rc;
                if ((rc = stage_apply(dn, p, ph, nullptr, st, split, split ? moved : 0u)) != PCD_OK) return rc;
            } else if (inflight && overlap) {
                if ((rc = stage_apply(dn, p, ph, nullptr, st, split, split ? moved : 0u, core, false)) != PCD_OK) return rc;
                if ((rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
                if ((rc = stage_apply(dn, p, ph, nullptr, st, split, split ? moved : 0u, edge_rows, true)) != PCD_OK) return rc;
            } else {
                if (inflight && (rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
                if ((rc = stage_apply(dn, p, ph, nullptr, st, split, split ? moved : 0u)) != PCD_OK) return rc;
            }
            moved |= 1u << p->phase_class[ph];
            if (ev) PCD_HIP(hipEventRecord(ev[6 + ph], st));
            // Gauss-Seidel: the next phase (or the next iteration) reads these positions (read-set: the next
            // iteration's rows arrive with its refresh)
            if (xchg && !p->jacobi && !(rs && ph == p->nphases - 1)) {
                XField f = split ? XField{dn->pos[dn->cur], dn->pos[dn->cur ^ 1], dn->cls, moved, dn->pos[dn->cur],
                                          dn->pos[dn->cur ^ 1]}
                                 : XField{dn->pos[dn->cur], nullptr, nullptr, 0u, dn->pos[dn->cur], nullptr};
                if (split && ph == p->nphases - 1)   // (cur flipped after the last phase: every own row is in pos[cur])
                    f = XField{dn->pos[dn->cur], nullptr, nullptr, 0u, dn->pos[dn->cur], dn->pos[dn->cur ^ 1]};
                if ((rc = xchg_begin(dn, c, st, f)) != PCD_OK) return rc;
            }
        }
        if (ev)
            for (int ph = p->nphases; ph < 3; ++ph) PCD_HIP(hipEventRecord(ev[6 + ph], st));
        stage_finish(dn, p);
        if (xchg && p->jacobi && !rs &&
            (rc = xchg_begin(dn, c, st, XField{dn->pos[dn->cur], nullptr, nullptr, 0u, dn->pos[dn->cur], nullptr})) != PCD_OK)
            return rc;
        if (ev) PCD_HIP(hipEventRecord(ev[9], st));
        if (ev) PCD_HIP(hipEventRecord(ev[10], st));
    }
    // the last position exchange stays in flight (RCCL) for the next call to wait on; the host transport finishes it
    // now, so every rank's blocking callbacks stay paired within the call
    return xchg_end(dn, c);
}

}  // extern "C"
