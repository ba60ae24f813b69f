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
#include <cstring>
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
}

void comm_destroy(Comm* c) {
    if (!c) return;
    if (c->nc) (void)ncclCommDestroy(c->nc);
    delete c;
}

int comm_device(const Comm* c) { return c->device; }

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

void comm_broadcast(Comm* c, void* buf, int64_t count, int elem, int root, hipStream_t s) {
    if (count <= 0) return;
    if (root < 0 || root >= c->n_ranks) throw Error(-1, "bad root");
    check(ncclBroadcast(buf, buf, (size_t)count, elem_type(elem), root, c->nc, s), "ncclBroadcast");
}

}  // namespace pd
