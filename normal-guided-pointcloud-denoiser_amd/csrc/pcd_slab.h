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
static int xchg_begin(pcd_denoiser* dn, pcd_comm* c, hipStream_t st, const XField& f) {
    if (dn->npeers == 0) return PCD_OK;
    const int rc = ensure_xstream(dn);
    if (rc != PCD_OK) return rc;
    hipStream_t xs = dn->xst;
    const int64_t ns = dn->soff[dn->npeers], nr = dn->roff[dn->npeers];
    PCD_HIP(hipEventRecord(dn->xev_in, st));
    PCD_HIP(hipStreamWaitEvent(xs, dn->xev_in, 0));
    dn->xfield = f;
    if (c->nccl) {
        float* sb = reinterpret_cast<float*>(dn->sbuf);
        float* rb = reinterpret_cast<float*>(dn->rbuf);
        if (ns > 0) hipLaunchKernelGGL(k_xpack3, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, f, dn->srows, ns, sb);
        PCD_LAUNCH_CHECK();
        PCD_NCCL(ncclGroupStart());
        for (int q = 0; q < dn->npeers; ++q) {
            const int64_t s0 = dn->soff[q], s1 = dn->soff[q + 1], r0 = dn->roff[q], r1 = dn->roff[q + 1];
            if (s1 > s0) PCD_NCCL(ncclSend(sb + 3 * s0, (size_t)(s1 - s0) * 3, ncclFloat, dn->peers[q], c->nccl, xs));
            if (r1 > r0) PCD_NCCL(ncclRecv(rb + 3 * r0, (size_t)(r1 - r0) * 3, ncclFloat, dn->peers[q], c->nccl, xs));
        }
        PCD_NCCL(ncclGroupEnd());
        if (nr > 0) hipLaunchKernelGGL(k_xunpack3, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, f, dn->rrows, nr, rb);
        PCD_LAUNCH_CHECK();
        PCD_HIP(hipEventRecord(dn->xev_out, xs));
        dn->xpending = true;
    } else {
        if (ns > 0) hipLaunchKernelGGL(k_xpack, dim3((unsigned)cdiv(ns, 256)), dim3(256), 0, xs, f, dn->srows, ns, dn->sbuf);
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
    const int64_t nr = dn->roff[dn->npeers];
    PCD_HIP(hipStreamSynchronize(xs));
    if (c->host.exchange(c->host.user, dn->npeers, dn->peers.data(), reinterpret_cast<const float*>(dn->hs),
                         dn->soff.data(), reinterpret_cast<float*>(dn->hr), dn->roff.data()) != 0)
        return fail(PCD_ERR_RCCL, "pcd_slab: host transport exchange callback failed");
    if (nr > 0) {
        PCD_HIP(hipMemcpyAsync(dn->rbuf, dn->hr, nr * sizeof(float4), hipMemcpyHostToDevice, xs));
        hipLaunchKernelGGL(k_xunpack, dim3((unsigned)cdiv(nr, 256)), dim3(256), 0, xs, dn->xfield, dn->rrows, nr, dn->rbuf);
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
    dn->srows = dn->rrows = nullptr;
    dn->sbuf = dn->rbuf = dn->hs = dn->hr = nullptr;
    dn->bflag = nullptr;
    dn->npeers = 0;
    dn->peers.clear();
    dn->soff.assign(1, 0);
    dn->roff.assign(1, 0);
}

static void destroy_slab_state(pcd_denoiser* dn) {
    if (dn->xst) (void)hipStreamSynchronize(dn->xst);
    free_routes(dn);
    if (dn->xst) (void)hipStreamDestroy(dn->xst);
    if (dn->xev_in) (void)hipEventDestroy(dn->xev_in);
    if (dn->xev_out) (void)hipEventDestroy(dn->xev_out);
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
        if (hipMalloc(&dn->srows, std::max<int64_t>(ns, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->rrows, std::max<int64_t>(nr, 1) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&dn->sbuf, std::max<int64_t>(ns, 1) * sizeof(float4)) != hipSuccess ||
            hipMalloc(&dn->rbuf, std::max<int64_t>(nr, 1) * sizeof(float4)) != hipSuccess ||
            hipHostMalloc(&dn->hs, std::max<int64_t>(ns, 1) * sizeof(float4), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&dn->hr, std::max<int64_t>(nr, 1) * sizeof(float4), hipHostMallocDefault) != hipSuccess) {
            free_routes(dn);
            return fail(PCD_ERR_OOM, "pcd_denoiser_set_routes: buffers");
        }
        if (ns > 0) PCD_HIP(hipMemcpyAsync(dn->srows, send_rows, ns * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        if (nr > 0) PCD_HIP(hipMemcpyAsync(dn->rrows, recv_rows, nr * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        dn->peers.assign(peers, peers + npeers);
        dn->soff = so;
        dn->roff = ro;
        dn->npeers = npeers;
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
    if (field == PCD_FIELD_POS || field == PCD_FIELD_NRM) dn->part_ph = dn->scan_ph = -1;
    if ((rc = xchg_begin(dn, c, st, XField{f, nullptr, nullptr, 0u, f, nullptr})) != PCD_OK) return rc;
    if ((rc = xchg_wait(dn, c, st)) != PCD_OK) return rc;
    if (field == PCD_FIELD_NRM) dn->unit_nrm = false;
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
        hipEvent_t before = dn->xpending ? dn->xev_out : nullptr;
        if (dn->rowmap().nq == 0 && before) PCD_HIP(hipStreamWaitEvent(st, before, 0));
        if ((rc = stage_k1(dn, p, st, ev, band, before)) != PCD_OK) return rc;
        dn->xpending = false;
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
            // Gauss-Seidel: the next phase (or the next iteration) reads these positions
            if (xchg && !p->jacobi) {
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
        if (xchg && p->jacobi &&
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
