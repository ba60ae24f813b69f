// RCCL communicator behind the C ABI (pd_comm_*): the device collectives of
// the sharded train.  They replace Spark's data movement in the reference:
//   all_to_all_v  partitionBy(max_partitions) shuffle of the halo records
//                 (R:dbscan/dbscan.py:114-118)
//   all_gather_v  collect() of the local cluster ids to the driver and the
//                 broadcast of the merged map (R:dbscan/dbscan.py:153-161)
//   all_reduce    the KD partitioner's aggregate() of counts / moments /
//                 bbox over the RDD slices (R:dbscan/partition.py:60-63,86-89,
//                 135-137)
// One rank per device.  xGMI is point-to-point (MI355X: 7 links per GPU), so
// the variable-size exchanges are grouped ncclSend/ncclRecv straight to each
// peer rather than ring collectives over padded buffers.
#include <cstdlib>
#include <cstring>
#include <vector>
#include <rccl/rccl.h>

#include "internal.hpp"

namespace pd {

struct Comm {
    ncclComm_t nc = nullptr;
    int device = 0;
    int n_ranks = 1;
    int rank = 0;
};

namespace {

void check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess)
        throw Error(-4, std::string(what) + ": " + ncclGetErrorString(r));
}

ncclDataType_t elem_type(int elem) {
    switch (elem) {
        case 0: return ncclUint8;
        case 1: return ncclInt32;
        case 2: return ncclUint32;
        case 3: return ncclInt64;
        case 4: return ncclUint64;
        case 5: return ncclFloat32;
        case 6: return ncclFloat64;
    }
    throw Error(-1, "unknown element type " + std::to_string(elem));
}

size_t elem_bytes(int elem) {
    static const size_t b[] = {1, 4, 4, 8, 8, 4, 8};
    if (elem < 0 || elem > 6) throw Error(-1, "unknown element type " + std::to_string(elem));
    return b[elem];
}

ncclRedOp_t red_op(int op) {
    switch (op) {
        case 0: return ncclSum;
        case 1: return ncclMax;
        case 2: return ncclMin;
    }
    throw Error(-1, "unknown reduction " + std::to_string(op));
}

}  // namespace

// PD_COMM_SELF_CHECK=0 turns off the W > 1 check at communicator creation.
bool self_check_enabled() {
    const char* e = std::getenv("PD_COMM_SELF_CHECK");
    return !(e && e[0] == '0');
}

void comm_unique_id(uint8_t* id) {
    static_assert(sizeof(ncclUniqueId) == 128, "PD_COMM_ID_BYTES");
    ncclUniqueId u;
    check(ncclGetUniqueId(&u), "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
}

Comm* comm_init(int device, int n_ranks, int rank, const uint8_t* id) {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) throw Error(-1, "bad rank / n_ranks");
    PD_HIP(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    Comm* c = new Comm;
    c->device = device;
    c->n_ranks = n_ranks;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->nc, n_ranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        check(r, "ncclCommInitRank");
    }
    if (n_ranks > 1 && self_check_enabled()) {
        try {
            comm_self_check(&c, 1);
        } catch (...) {
            comm_destroy(c);
            throw;
        }
    }
    return c;
}

void comm_init_all(int n, const int32_t* devices, Comm** out) {
    if (n < 1) throw Error(-1, "need at least one device");
    std::vector<ncclComm_t> nc(n);
    std::vector<int> dev(devices, devices + n);
    check(ncclCommInitAll(nc.data(), n, dev.data()), "ncclCommInitAll");
    for (int i = 0; i < n; ++i) {
        out[i] = new Comm;
        out[i]->nc = nc[i];
        out[i]->device = dev[i];
        out[i]->n_ranks = n;
        out[i]->rank = i;
    }
    if (n > 1 && self_check_enabled()) {
        try {
            comm_self_check(out, n);
        } catch (...) {
            for (int i = 0; i < n; ++i) {
                comm_destroy(out[i]);
                out[i] = nullptr;
            }
            throw;
        }
    }
}

void comm_destroy(Comm* c) {
    if (!c) return;
    if (c->nc) (void)ncclCommDestroy(c->nc);
    delete c;
}

int comm_device(const Comm* c) { return c->device; }

// Rank count and this rank as RCCL itself reports them (not the values the
// communicator was created with): the bench line's rccl_ranks.
void comm_size(const Comm* c, int* n_ranks, int* rank) {
    if (!c->nc) throw Error(-4, "communicator was aborted");
    int n = 0, r = -1;
    check(ncclCommCount(c->nc, &n), "ncclCommCount");
    check(ncclCommUserRank(c->nc, &r), "ncclCommUserRank");
    *n_ranks = n;
    *rank = r;
}

void comm_all_reduce(Comm* c, const void* send, void* recv, int64_t count, int elem, int op,
                     hipStream_t s) {
    if (count <= 0) return;
    check(ncclAllReduce(send, recv, (size_t)count, elem_type(elem), red_op(op), c->nc, s),
          "ncclAllReduce");
}

// recv = concat over ranks r of counts[r] elements (this rank's `send` has
// counts[rank] of them): every rank sends its block to each peer directly.
void comm_all_gather_v(Comm* c, const void* send, void* recv, const int64_t* counts, int elem,
                       hipStream_t s) {
    const ncclDataType_t t = elem_type(elem);
    const size_t eb = elem_bytes(elem);
    const int W = c->n_ranks, me = c->rank;
    std::vector<size_t> off(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        if (counts[r] < 0) throw Error(-1, "negative count");
        off[r + 1] = off[r] + (size_t)counts[r];
    }
    char* out = (char*)recv;
    if (counts[me])
        PD_HIP(hipMemcpyAsync(out + off[me] * eb, send, (size_t)counts[me] * eb,
                              hipMemcpyDeviceToDevice, s));
    if (W == 1) return;
    check(ncclGroupStart(), "ncclGroupStart");
    for (int k = 1; k < W; ++k) {
        const int to = (me + k) % W, from = (me - k + W) % W;
        if (counts[me]) check(ncclSend(send, (size_t)counts[me], t, to, c->nc, s), "ncclSend");
        if (counts[from])
            check(ncclRecv(out + off[from] * eb, (size_t)counts[from], t, from, c->nc, s),
                  "ncclRecv");
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
}

// send = blocks grouped by destination rank (send_counts), recv = blocks
// grouped by source rank (recv_counts), element counts.
void comm_all_to_all_v(Comm* c, const void* send, const int64_t* send_counts, void* recv,
                       const int64_t* recv_counts, int elem, hipStream_t s) {
    const ncclDataType_t t = elem_type(elem);
    const size_t eb = elem_bytes(elem);
    const int W = c->n_ranks, me = c->rank;
    std::vector<size_t> so(W + 1, 0), ro(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        if (send_counts[r] < 0 || recv_counts[r] < 0) throw Error(-1, "negative count");
        so[r + 1] = so[r] + (size_t)send_counts[r];
        ro[r + 1] = ro[r] + (size_t)recv_counts[r];
    }
    if (send_counts[me] != recv_counts[me]) throw Error(-1, "self block sizes differ");
    const char* in = (const char*)send;
    char* out = (char*)recv;
    if (send_counts[me])
        PD_HIP(hipMemcpyAsync(out + ro[me] * eb, in + so[me] * eb, (size_t)send_counts[me] * eb,
                              hipMemcpyDeviceToDevice, s));
    if (W == 1) return;
    check(ncclGroupStart(), "ncclGroupStart");
    for (int k = 1; k < W; ++k) {
        const int to = (me + k) % W, from = (me - k + W) % W;
        if (send_counts[to])
            check(ncclSend(in + so[to] * eb, (size_t)send_counts[to], t, to, c->nc, s),
                  "ncclSend");
        if (recv_counts[from])
            check(ncclRecv(out + ro[from] * eb, (size_t)recv_counts[from], t, from, c->nc, s),
                  "ncclRecv");
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
}

// Several fields (coords, ids, flags, ...) of one exchange in ONE group:
// block r of field f is rec_bytes[f] * counts[r] bytes at offset
// rec_bytes[f] * off[r]; skip_self: the self blocks were written in place
// (pd_pack2 packs them straight into the receive buffers).
void comm_exchange(Comm* c, int nf, const void* const* send, void* const* recv,
                   const int64_t* rec_bytes, const int64_t* send_counts, const int64_t* send_off,
                   const int64_t* recv_counts, const int64_t* recv_off, bool skip_self,
                   hipStream_t s) {
    const int W = c->n_ranks, me = c->rank;
    for (int r = 0; r < W; ++r)
        if (send_counts[r] < 0 || recv_counts[r] < 0 || send_off[r] < 0 || recv_off[r] < 0)
            throw Error(-1, "negative count or offset");
    if (send_counts[me] != recv_counts[me]) throw Error(-1, "self block sizes differ");
    for (int f = 0; f < nf; ++f)
        if (rec_bytes[f] <= 0) throw Error(-1, "field record size must be > 0");
    if (!skip_self && send_counts[me])
        for (int f = 0; f < nf; ++f)
            PD_HIP(hipMemcpyAsync((char*)recv[f] + rec_bytes[f] * recv_off[me],
                                  (const char*)send[f] + rec_bytes[f] * send_off[me],
                                  (size_t)(rec_bytes[f] * send_counts[me]),
                                  hipMemcpyDeviceToDevice, s));
    if (W == 1) return;
    check(ncclGroupStart(), "ncclGroupStart");
    for (int k = 1; k < W; ++k) {
        const int to = (me + k) % W, from = (me - k + W) % W;
        for (int f = 0; f < nf; ++f) {
            if (send_counts[to])
                check(ncclSend((const char*)send[f] + rec_bytes[f] * send_off[to],
                               (size_t)(rec_bytes[f] * send_counts[to]), ncclUint8, to, c->nc, s),
                      "ncclSend");
            if (recv_counts[from])
                check(ncclRecv((char*)recv[f] + rec_bytes[f] * recv_off[from],
                               (size_t)(rec_bytes[f] * recv_counts[from]), ncclUint8, from, c->nc,
                               s),
                      "ncclRecv");
        }
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
}

// Unblock every rank waiting on this communicator (a failed rank of a
// one-process group); the communicator is unusable afterwards.
void comm_abort(Comm* c) {
    if (c && c->nc) {
        (void)ncclCommAbort(c->nc);
        c->nc = nullptr;
    }
}

namespace {
// Self-check pattern: rank r sends (r + 2 q) % 3 + (r == q) u32 values to
// rank q in the all-to-all (zero-sized blocks included), value (r << 20) |
// (q << 10) | k; in the all-gather rank r contributes r % 3 + 1 values
// (r << 20) | k.  recv_expected_* restate it on the receiving rank.
__host__ __device__ inline int64_t a2a_count(int r, int q) { return (r + 2 * q) % 3 + (r == q ? 1 : 0); }
__host__ __device__ inline int64_t ag_count(int r) { return r % 3 + 1; }

__global__ void self_check_fill(uint32_t* a2a, uint32_t* ag, int W, int me) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t o = 0;
    for (int q = 0; q < W; ++q)
        for (int64_t k = 0; k < a2a_count(me, q); ++k) a2a[o++] = ((uint32_t)me << 20) | ((uint32_t)q << 10) | (uint32_t)k;
    for (int64_t k = 0; k < ag_count(me); ++k) ag[k] = ((uint32_t)me << 20) | (uint32_t)k;
}

__global__ void self_check_verify(const uint32_t* a2a, const uint32_t* ag, int W, int me,
                                  uint32_t* bad) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t b = 0;
    int64_t o = 0;
    for (int p = 0; p < W; ++p)
        for (int64_t k = 0; k < a2a_count(p, me); ++k)
            b |= a2a[o++] != (((uint32_t)p << 20) | ((uint32_t)me << 10) | (uint32_t)k) ? 1u : 0u;
    o = 0;
    for (int p = 0; p < W; ++p)
        for (int64_t k = 0; k < ag_count(p); ++k)
            b |= ag[o++] != (((uint32_t)p << 20) | (uint32_t)k) ? 2u : 0u;
    *bad = b;
}
}  // namespace

void comm_self_check(Comm* const* comms, int n) {
    if (n < 1) return;
    const int W = comms[0]->n_ranks;
    if (W > 1000) throw Error(-1, "self check: too many ranks");
    struct Bufs {
        hipStream_t s = nullptr;
        uint32_t *sa = nullptr, *ra = nullptr, *sg = nullptr, *rg = nullptr, *bad = nullptr;
        std::vector<int64_t> sc, so, rc, ro, gc;
    };
    std::vector<Bufs> b(n);
    auto release = [&]() {
        for (int i = 0; i < n; ++i) {
            (void)hipSetDevice(comms[i]->device);
            if (b[i].s) (void)hipStreamSynchronize(b[i].s);
            for (uint32_t* p : {b[i].sa, b[i].ra, b[i].sg, b[i].rg, b[i].bad})
                if (p) (void)hipFree(p);
            if (b[i].s) (void)hipStreamDestroy(b[i].s);
        }
    };
    try {
        for (int i = 0; i < n; ++i) {
            Comm* c = comms[i];
            const int me = c->rank;
            Bufs& x = b[i];
            x.sc.resize(W);
            x.so.resize(W);
            x.rc.resize(W);
            x.ro.resize(W);
            x.gc.resize(W);
            int64_t st = 0, rt = 0, gt = 0;
            for (int q = 0; q < W; ++q) {
                x.sc[q] = a2a_count(me, q);
                x.so[q] = st;
                st += x.sc[q];
                x.rc[q] = a2a_count(q, me);
                x.ro[q] = rt;
                rt += x.rc[q];
                x.gc[q] = ag_count(q);
                gt += x.gc[q];
            }
            PD_HIP(hipSetDevice(c->device));
            PD_HIP(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking));
            PD_HIP(hipMalloc(&x.sa, sizeof(uint32_t) * (st + 1)));
            PD_HIP(hipMalloc(&x.ra, sizeof(uint32_t) * (rt + 1)));
            PD_HIP(hipMalloc(&x.sg, sizeof(uint32_t) * (ag_count(me) + 1)));
            PD_HIP(hipMalloc(&x.rg, sizeof(uint32_t) * (gt + 1)));
            PD_HIP(hipMalloc(&x.bad, sizeof(uint32_t)));
            PD_HIP(hipMemsetAsync(x.ra, 0xFF, sizeof(uint32_t) * (rt + 1), x.s));
            PD_HIP(hipMemsetAsync(x.rg, 0xFF, sizeof(uint32_t) * (gt + 1), x.s));
            hipLaunchKernelGGL(self_check_fill, dim3(1), dim3(64), 0, x.s, x.sa, x.sg, W, me);
            PD_HIP(hipGetLastError());
        }
        // one group over every rank this process drives (init_all), so the
        // point-to-point pairs of all ranks launch together
        check(ncclGroupStart(), "ncclGroupStart");
        for (int i = 0; i < n; ++i) {
            PD_HIP(hipSetDevice(comms[i]->device));
            comm_all_to_all_v(comms[i], b[i].sa, b[i].sc.data(), b[i].ra, b[i].rc.data(), 2, b[i].s);
        }
        check(ncclGroupEnd(), "ncclGroupEnd");
        check(ncclGroupStart(), "ncclGroupStart");
        for (int i = 0; i < n; ++i) {
            PD_HIP(hipSetDevice(comms[i]->device));
            comm_all_gather_v(comms[i], b[i].sg, b[i].rg, b[i].gc.data(), 2, b[i].s);
        }
        check(ncclGroupEnd(), "ncclGroupEnd");
        for (int i = 0; i < n; ++i) {
            PD_HIP(hipSetDevice(comms[i]->device));
            hipLaunchKernelGGL(self_check_verify, dim3(1), dim3(64), 0, b[i].s, b[i].ra, b[i].rg, W,
                               comms[i]->rank, b[i].bad);
            PD_HIP(hipGetLastError());
        }
        // every rank learns every rank's verdict (max of the flags), so a
        // check that fails on some ranks fails on all of them: none returns a
        // communicator its peers have destroyed
        std::vector<uint32_t> local(n, 0), any(n, 0);
        for (int i = 0; i < n; ++i) {
            PD_HIP(hipSetDevice(comms[i]->device));
            PD_HIP(hipMemcpyAsync(&local[i], b[i].bad, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  b[i].s));
        }
        if (W > 1) {
            check(ncclGroupStart(), "ncclGroupStart");
            for (int i = 0; i < n; ++i) {
                PD_HIP(hipSetDevice(comms[i]->device));
                check(ncclAllReduce(b[i].bad, b[i].bad, 1, ncclUint32, ncclMax, comms[i]->nc,
                                    b[i].s),
                      "ncclAllReduce");
            }
            check(ncclGroupEnd(), "ncclGroupEnd");
        }
        for (int i = 0; i < n; ++i) {
            PD_HIP(hipSetDevice(comms[i]->device));
            PD_HIP(hipMemcpyAsync(&any[i], b[i].bad, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  b[i].s));
            PD_HIP(hipStreamSynchronize(b[i].s));
        }
        for (int i = 0; i < n; ++i) {
            const uint32_t hb = local[i] ? local[i] : any[i];
            if (hb)
                throw Error(-4, std::string("RCCL self check failed ") +
                                    (local[i] ? "on rank " + std::to_string(comms[i]->rank)
                                              : "on another rank (seen from rank " +
                                                    std::to_string(comms[i]->rank) + ")") +
                                    " of " + std::to_string(W) + ((hb & 1) ? ": all_to_all_v" : "") +
                                    ((hb & 2) ? ": all_gather_v" : "") +
                                    " delivered wrong data (PD_COMM_SELF_CHECK=0 skips this check)");
        }
    } catch (...) {
        release();
        throw;
    }
    release();
}

void comm_broadcast(Comm* c, void* buf, int64_t count, int elem, int root, hipStream_t s) {
    if (count <= 0) return;
    if (root < 0 || root >= c->n_ranks) throw Error(-1, "bad root");
    check(ncclBroadcast(buf, buf, (size_t)count, elem_type(elem), root, c->nc, s), "ncclBroadcast");
}

}  // namespace pd
