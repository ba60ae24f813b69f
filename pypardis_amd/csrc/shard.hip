// Sharded (multi-device) train: routing of points to the devices that own
// their neighbourhoods, the global key merge, and global label ranks.
//
// The reference has no device split: its equivalent is Spark's
// partitionBy(max_partitions) shuffle of the halo records
// (R:dbscan/dbscan.py:114-118) and the driver-side ClusterAggregator merge
// (R:dbscan/dbscan.py:153-165, R:dbscan/aggregator.py:9-73).  Here each
// device holds a slice of the input; a point travels once to every device
// whose neighbourhoods' expanded boxes contain it (pd_route / pd_pack), each
// device clusters its neighbourhoods (pd_train_begin), exports the component
// keys of its cross-device core points, and the union of all exports
// (pd_merge_exports, identical on every device) maps local keys to global
// ones (pd_train_end).  Labels are ranks of the global keys
// (pd_select_roots, pd_sort_u32, pd_rank_labels) - the same numbering
// single-device pd_train gives.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "compact.hpp"
#include "internal.hpp"

namespace pd {
namespace {

constexpr int kMaxRanks = 64;   // one bit per device in the route mask

inline unsigned blocks(uint64_t n) { return n ? (unsigned)((n + kBlock - 1) / kBlock) : 1u; }

template <typename F>
void dispatch(int dtype, int d, F&& f) {
    auto by_d = [&](auto tp) {
        switch (d) {
            case 1: f(tp, std::integral_constant<int, 1>{}); break;
            case 2: f(tp, std::integral_constant<int, 2>{}); break;
            case 3: f(tp, std::integral_constant<int, 3>{}); break;
            case 4: f(tp, std::integral_constant<int, 4>{}); break;
            default: throw Error(-5, "dimension " + std::to_string(d) + " > 4 not supported yet");
        }
    };
    if (dtype == 0)
        by_d((float*)nullptr);
    else if (dtype == 1)
        by_d((double*)nullptr);
    else
        throw Error(-1, "dtype must be 0 (float32) or 1 (float64)");
}

// Route mask: bit r set when some neighbourhood assigned to device r has an
// expanded box containing the point (inclusive bounds, the test pd_train's
// halo uses).  One LDS counter per device, one global atomic per block.
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void route_kernel(const T* __restrict__ X, uint64_t n,
                                                       const double* __restrict__ ebox, int P,
                                                       const int32_t* __restrict__ part_rank,
                                                       int n_ranks,
                                                       uint64_t* __restrict__ mask,
                                                       unsigned long long* __restrict__ counts) {
    __shared__ unsigned int sc[kMaxRanks];
    for (int k = threadIdx.x; k < n_ranks; k += kBlock) sc[k] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        double v[D];
#pragma unroll
        for (int j = 0; j < D; ++j) v[j] = (double)X[i * D + j];
        uint64_t m = 0;
        for (int L = 0; L < P; ++L) {
            const double* b = ebox + (size_t)L * 2 * D;
            bool in = true;
#pragma unroll
            for (int j = 0; j < D; ++j) in &= (b[j] <= v[j]) & (b[D + j] >= v[j]);
            if (in) m |= 1ull << part_rank[L];
        }
        mask[i] = m;
        while (m) {
            const int r = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            atomicAdd(&sc[r], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n_ranks; k += kBlock)
        if (sc[k]) atomicAdd(counts + k, (unsigned long long)sc[k]);
}

struct HasBit {
    const uint64_t* mask;
    int bit;
    __device__ bool operator()(uint32_t i) const { return (mask[i] >> bit) & 1ull; }
};

template <typename T, int D>
__global__ __launch_bounds__(kBlock) void pack_kernel(
    const T* __restrict__ X, const uint32_t* __restrict__ list, uint32_t m,
    const uint64_t* __restrict__ mask, const int32_t* __restrict__ kdlab,
    const int32_t* __restrict__ part_rank, const int32_t* __restrict__ local_index, int P,
    int dest, uint32_t gid_base, T* __restrict__ coords, uint32_t* __restrict__ gid,
    int32_t* __restrict__ owner, uint8_t* __restrict__ xr) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    const uint32_t i = list[k];
#pragma unroll
    for (int j = 0; j < D; ++j) coords[(size_t)k * D + j] = X[(size_t)i * D + j];
    gid[k] = gid_base + i;
    const int32_t L = kdlab[i];
    owner[k] = (L >= 0 && L < P && part_rank[L] == dest) ? local_index[L] : -1;
    xr[k] = __popcll(mask[i]) > 1 ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void iota_kernel(uint32_t* __restrict__ p, uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) p[i] = i;
}

// Union-find over the compacted export ids (index into the ascending id
// list), smaller root wins, so a component's root is its smallest id = its
// smallest core point.
__device__ __forceinline__ uint32_t find_root(uint32_t* par, uint32_t x) {
    uint32_t p = __hip_atomic_load(par + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(par + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return x;
}

__device__ __forceinline__ uint32_t lower_bound(const uint32_t* a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void unite_kernel(const uint32_t* __restrict__ ga,
                                                       const uint32_t* __restrict__ gb, int64_t m,
                                                       const uint32_t* __restrict__ ids,
                                                       uint32_t u, uint32_t* __restrict__ par) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    // both ids are in the list (it is the set of all of them)
    uint32_t a = find_root(par, lower_bound(ids, u, ga[i]));
    uint32_t b = find_root(par, lower_bound(ids, u, gb[i]));
    while (a != b) {
        if (a > b) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t expected = b;
        if (__hip_atomic_compare_exchange_strong(par + b, &expected, a, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        b = find_root(par, expected);
        a = find_root(par, a);
    }
}

// keys_out[j] = id of the root of ids[j]'s component (after every union).
__global__ __launch_bounds__(kBlock) void map_keys_kernel(const uint32_t* __restrict__ par,
                                                          const uint32_t* __restrict__ ids,
                                                          uint32_t u,
                                                          uint32_t* __restrict__ keys_out) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= u) return;
    uint32_t x = par[j];
    while (true) {
        const uint32_t p = par[x];
        if (p == x) break;
        x = p;
    }
    keys_out[j] = ids[x];
}

// Owned core point whose key is its own global id.  One per cluster over all
// devices: a cluster's key is the global id of its smallest core point, and
// pd_train_end writes keys for owned records only (a point is owned by exactly
// one device: the one holding its KD partition; halo copies keep kNone), so
// the smallest core point passes this test on exactly one device.
struct IsRoot {
    const uint32_t* keys;
    const uint32_t* gid;
    __device__ bool operator()(uint32_t i) const {
        const uint32_t k = keys[i];
        return k != kNone && k == (gid ? gid[i] : i);
    }
};

__global__ __launch_bounds__(kBlock) void map_gid_kernel(uint32_t* __restrict__ p, uint32_t m,
                                                         const uint32_t* __restrict__ gid) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < m) p[i] = gid[p[i]];
}

__global__ __launch_bounds__(kBlock) void rank_kernel(const uint32_t* __restrict__ keys, uint64_t n,
                                                      const uint32_t* __restrict__ roots,
                                                      uint32_t nr, int32_t* __restrict__ labels,
                                                      uint32_t* __restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    if (k == kNone) {
        labels[i] = -1;
        return;
    }
    const uint32_t lo = lower_bound(roots, nr, k);
    if (lo < nr && roots[lo] == k) {
        labels[i] = (int32_t)lo;
    } else {   // a key with no root: the exports / roots were not gathered from every device
        labels[i] = -2;
        atomicOr(bad, 1u);
    }
}

// Owned records of a sharded train packed for the return to the devices that
// hold the points: (global id, (label + 1) | core << 31), in the input order
// (ascending global id); per destination device r (ids in
// [gid_off[r], gid_off[r + 1])) a count.  Ids must ascend (pd_pack order), so
// each destination's block is contiguous; `bad` flags a descent.
__global__ __launch_bounds__(kBlock) void owned_pack_kernel(
    const uint32_t* __restrict__ list, uint32_t m, const uint32_t* __restrict__ gid,
    const int32_t* __restrict__ labels, const uint8_t* __restrict__ core,
    const int64_t* __restrict__ gid_off, int n_ranks, uint32_t* __restrict__ out,
    unsigned long long* __restrict__ counts, uint32_t* __restrict__ bad) {
    __shared__ unsigned int sc[kMaxRanks];
    for (int k = threadIdx.x; k < n_ranks; k += kBlock) sc[k] = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k < m) {
        const uint32_t i = list[k];
        const uint32_t g = gid[i];
        if (k && gid[list[k - 1]] >= g) atomicOr(bad, 1u);
        int r = 0;
        while (r + 1 < n_ranks && (int64_t)g >= gid_off[r + 1]) ++r;
        if ((int64_t)g < gid_off[0] || (int64_t)g >= gid_off[n_ranks]) atomicOr(bad, 2u);
        atomicAdd(&sc[r], 1u);
        out[2 * (size_t)k] = g;
        out[2 * (size_t)k + 1] = (uint32_t)(labels[i] + 1) | (core && core[i] ? 0x80000000u : 0u);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n_ranks; q += kBlock)
        if (sc[q]) atomicAdd(counts + q, (unsigned long long)sc[q]);
}

struct IsOwned {
    const int32_t* owner;
    __device__ bool operator()(uint32_t i) const { return owner[i] >= 0; }
};

constexpr int32_t kUnset = (int32_t)0x80000000;

__global__ __launch_bounds__(kBlock) void fill_i32_kernel(int32_t* __restrict__ p, uint64_t n,
                                                          int32_t v) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ __launch_bounds__(kBlock) void scatter_results_kernel(
    const uint32_t* __restrict__ pairs, uint64_t m, uint32_t gid_base, uint64_t n,
    int32_t* __restrict__ labels, uint8_t* __restrict__ core, uint32_t* __restrict__ bad) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    const uint32_t g = pairs[2 * k], v = pairs[2 * k + 1];
    if (g < gid_base || (uint64_t)(g - gid_base) >= n) {
        atomicOr(bad, 1u);
        return;
    }
    labels[g - gid_base] = (int32_t)(v & 0x7FFFFFFFu) - 1;
    if (core) core[g - gid_base] = (uint8_t)(v >> 31);
}

__global__ __launch_bounds__(kBlock) void unset_check_kernel(const int32_t* __restrict__ labels,
                                                             uint64_t n, uint32_t* __restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && labels[i] == kUnset) atomicOr(bad, 2u);
}

// ---- one-pass exchange (pd_route2 / pd_pack2): tiles of 4 * kBlock points;
// lane l of wave w takes points base + 256 w + 64 q + l (q = 0..3), so a
// tile's points are visited in ascending index order (w, q, l) and every
// destination receives its points in ascending local index.
constexpr int kRTile = 4 * kBlock;

template <typename T, int D>
__device__ __forceinline__ uint64_t route_mask(const T* __restrict__ X, uint64_t i,
                                               const double* __restrict__ eb, int P,
                                               const int32_t* __restrict__ part_rank) {
    double v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (double)X[i * D + j];
    uint64_t m = 0;
    for (int L = 0; L < P; ++L) {
        const double* b = eb + (size_t)L * 2 * D;
        bool in = true;
#pragma unroll
        for (int j = 0; j < D; ++j) in &= (b[j] <= v[j]) & (b[D + j] >= v[j]);
        if (in) m |= 1ull << part_rank[L];
    }
    return m;
}

// Pass 1: destination mask per point, per-tile counts (dest-major:
// cnt[r * tiles + tile]) and per-destination totals of the points that
// destination owns (its KD partition holds them).
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void route_tile_kernel(
    const T* __restrict__ X, uint64_t n, const double* __restrict__ ebox, int P,
    const int32_t* __restrict__ part_rank, const int32_t* __restrict__ kdlab, int n_ranks,
    unsigned tiles, uint64_t* __restrict__ mask, uint32_t* __restrict__ cnt,
    unsigned long long* __restrict__ own) {
    __shared__ unsigned int sc[kMaxRanks], so[kMaxRanks];
    for (int k = threadIdx.x; k < n_ranks; k += kBlock) sc[k] = so[k] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kRTile + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + 64 * q;
        if (i >= n) continue;
        uint64_t m = route_mask<T, D>(X, i, ebox, P, part_rank);
        mask[i] = m;
        const int32_t L = kdlab[i];
        if (L >= 0 && L < P) atomicAdd(&so[part_rank[L]], 1u);
        while (m) {
            const int r = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            atomicAdd(&sc[r], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n_ranks; k += kBlock) {
        cnt[(size_t)k * tiles + blockIdx.x] = sc[k];
        if (so[k]) atomicAdd(own + k, (unsigned long long)so[k]);
    }
}

// Per destination: its block's start in the dest-major scan (off[r * tiles])
// and total, for the host.
__global__ void route_totals_kernel(const uint64_t* __restrict__ off, unsigned tiles, int n_ranks,
                                    unsigned long long* __restrict__ out) {
    const int r = threadIdx.x;
    if (r < n_ranks)
        out[r] = (unsigned long long)(off[(size_t)(r + 1) * tiles] - off[(size_t)r * tiles]);
}

struct PackOut {
    void* const* coords;
    uint32_t* const* gid;
    int32_t* const* owner;
    uint8_t* const* xr;
};

// Pass 2: every point written to each of its destinations at (its position
// among the tile's points for that destination) + the tile's offset.
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void pack_tile_kernel(
    const T* __restrict__ X, uint64_t n, const uint64_t* __restrict__ mask,
    const uint64_t* __restrict__ off, unsigned tiles, const int32_t* __restrict__ kdlab,
    const int32_t* __restrict__ part_rank, const int32_t* __restrict__ local_index, int P,
    int n_ranks, uint32_t gid_base, PackOut out) {
    __shared__ unsigned int wc[kBlock / 64][kMaxRanks];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kRTile + w * 256 + lane;
    uint64_t m[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) m[q] = base + 64 * q < n ? mask[base + 64 * q] : 0ull;
    unsigned long long any = m[0] | m[1] | m[2] | m[3];
    for (int o = 32; o > 0; o >>= 1) any |= (unsigned long long)__shfl_xor((long long)any, o, 64);
    for (int r = 0; r < n_ranks; ++r) {
        uint32_t t = 0;
        if ((any >> r) & 1ull) {
#pragma unroll
            for (int q = 0; q < 4; ++q) t += (uint32_t)__popcll(__ballot((m[q] >> r) & 1ull));
        }
        if (lane == 0) wc[w][r] = t;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int r = 0; r < n_ranks; ++r) {
        if (!((any >> r) & 1ull)) continue;   // wave-uniform
        uint64_t pos = off[(size_t)r * tiles + blockIdx.x] - off[(size_t)r * tiles];
        for (int u = 0; u < w; ++u) pos += wc[u][r];
        T* co = (T*)out.coords[r];
        uint32_t* gi = out.gid[r];
        int32_t* ow = out.owner[r];
        uint8_t* xr = out.xr[r];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool in = (m[q] >> r) & 1ull;
            const unsigned long long b = __ballot(in);
            if (in) {
                const uint64_t i = base + 64 * q;
                const uint64_t k = pos + (uint64_t)__popcll(b & lt);
#pragma unroll
                for (int j = 0; j < D; ++j) co[k * D + j] = X[i * D + j];
                gi[k] = gid_base + (uint32_t)i;
                const int32_t L = kdlab[i];
                ow[k] = (L >= 0 && L < P && part_rank[L] == r) ? local_index[L] : -1;
                xr[k] = __popcll(m[q]) > 1 ? 1 : 0;
            }
            pos += (uint64_t)__popcll(b);
        }
    }
}

// ---- results: labels of the owned records back to the ranks that hold the
// points.  A record's source rank is its block of the exchange (records
// arrive grouped by source), so the owned records of the self block are
// written straight into this rank's outputs and the others are compacted in
// order, block by block = destination by destination.
// A cluster key's label is its rank among the sorted roots of every device.
// RootIndex cuts the binary search over all roots (~15 dependent L2 reads per
// record at C4's 3.7e4 clusters) to two table reads and a search over the
// few roots sharing the key's top bits: idx[t] = first root >= t << sh, for
// t <= kRootIdx (keys < 2^32, sh chosen so key >> sh < kRootIdx).
constexpr uint32_t kRootIdx = 1u << 16;

struct RootIndex {
    const uint32_t* roots;
    const uint32_t* idx;
    uint32_t nr;
    uint32_t sh;
};

__global__ __launch_bounds__(kBlock) void root_index_kernel(const uint32_t* __restrict__ roots,
                                                            uint32_t nr, uint32_t sh,
                                                            uint32_t* __restrict__ idx) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t > kRootIdx) return;
    const uint64_t v = (uint64_t)t << sh;
    idx[t] = v > 0xFFFFFFFFull ? nr : lower_bound(roots, nr, (uint32_t)v);
}

__device__ __forceinline__ int32_t root_rank(const RootIndex& R, uint32_t k) {
    if (k == kNone) return -1;
    const uint32_t t = k >> R.sh;
    if (t >= kRootIdx) return -2;   // beyond every key: no such root
    uint32_t lo = R.idx[t];
    const uint32_t hi = R.idx[t + 1];
    uint32_t n = hi - lo;   // roots in [t << sh, (t + 1) << sh)
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (R.roots[lo + h] < k) {
            lo += h + 1;
            n -= h + 1;
        } else {
            n = h;
        }
    }
    return (lo < hi && R.roots[lo] == k) ? (int32_t)lo : -2;
}

// kResPer records per thread (coalesced rounds of kBlock), their root
// lookups interleaved: four independent two-table-read chains per lane in
// flight instead of one (the lookups are L2 latency, not bandwidth)
constexpr int kResPer = 4;
__global__ __launch_bounds__(kBlock) void results_self_kernel(
    const uint32_t* __restrict__ keys, const uint8_t* __restrict__ core,
    const int32_t* __restrict__ owner, const uint32_t* __restrict__ gid, uint64_t lo, uint64_t hi,
    RootIndex RI, uint32_t gid_base, uint64_t n_local,
    int32_t* __restrict__ labels, uint8_t* __restrict__ core_out, uint32_t* __restrict__ bad) {
    const uint64_t i0 = lo + (uint64_t)blockIdx.x * kBlock * kResPer + threadIdx.x;
    uint32_t k[kResPer];
    bool ok[kResPer];
#pragma unroll
    for (int q = 0; q < kResPer; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        ok[q] = i < hi && owner[i] >= 0;
        k[q] = ok[q] ? keys[i] : kNone;
    }
    int32_t lab[kResPer];
#pragma unroll
    for (int q = 0; q < kResPer; ++q) lab[q] = root_rank(RI, k[q]);
#pragma unroll
    for (int q = 0; q < kResPer; ++q) {
        if (!ok[q]) continue;
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        const uint32_t g = gid ? gid[i] : (uint32_t)i;
        if (lab[q] == -2) atomicOr(bad, 4u);
        if (g < gid_base || (uint64_t)(g - gid_base) >= n_local) {
            atomicOr(bad, 1u);
            continue;
        }
        labels[g - gid_base] = lab[q];
        if (core_out) core_out[g - gid_base] = core ? core[i] : 0;
    }
}

struct IsRemoteOwned {
    const int32_t* owner;
    uint64_t lo, hi;
    __device__ bool operator()(uint32_t i) const { return owner[i] >= 0 && (i < lo || i >= hi); }
};

__global__ __launch_bounds__(kBlock) void results_pack_kernel(
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ count, int64_t expect,
    const uint32_t* __restrict__ keys, const uint8_t* __restrict__ core,
    const uint32_t* __restrict__ gid, RootIndex RI,
    uint32_t* __restrict__ pairs, uint32_t* __restrict__ bad) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t m = *count;
    if (k == 0 && (int64_t)m != expect) atomicOr(bad, 8u);
    if ((int64_t)k >= expect) return;
    if (k >= m) {   // short: the slots the peers expect carry an invalid id, so the
        pairs[2 * (size_t)k] = kNone;   // receivers fail in results_scatter too
        pairs[2 * (size_t)k + 1] = 0u;
        return;
    }
    const uint32_t i = list[k];
    const int32_t lab = root_rank(RI, keys[i]);
    if (lab == -2) atomicOr(bad, 4u);
    pairs[2 * (size_t)k] = gid ? gid[i] : i;
    pairs[2 * (size_t)k + 1] = (uint32_t)(lab + 1) | (core && core[i] ? 0x80000000u : 0u);
}

__global__ __launch_bounds__(kBlock) void results_scatter_kernel(
    const uint32_t* __restrict__ pairs, uint64_t m, uint32_t gid_base, uint64_t n,
    int32_t* __restrict__ labels, uint8_t* __restrict__ core, uint32_t* __restrict__ bad) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    const uint32_t g = pairs[2 * k], v = pairs[2 * k + 1];
    if (g < gid_base || (uint64_t)(g - gid_base) >= n) {
        atomicOr(bad, 1u);
        return;
    }
    labels[g - gid_base] = (int32_t)(v & 0x7FFFFFFFu) - 1;
    if (core) core[g - gid_base] = (uint8_t)(v >> 31);
}

}  // namespace

void route(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P, const double* ebox_host,
           const int32_t* part_rank_host, int n_ranks, uint64_t* mask, int64_t* counts_host,
           hipStream_t s) {
    if (n_ranks < 1 || n_ranks > kMaxRanks) throw Error(-1, "n_ranks must be in [1, 64]");
    if (P < 1) throw Error(-1, "need at least one neighbourhood");
    for (int L = 0; L < P; ++L)
        if (part_rank_host[L] < 0 || part_rank_host[L] >= n_ranks)
            throw Error(-1, "part_rank out of range");
    const size_t tb = sizeof(double) * P * 2 * d + sizeof(int32_t) * P;
    char* h = (char*)pinned(ctx, tb + 64);
    std::memcpy(h, ebox_host, sizeof(double) * P * 2 * d);
    std::memcpy(h + sizeof(double) * P * 2 * d, part_rank_host, sizeof(int32_t) * P);
    char* dt = ctx.arena.get<char>("route_tab", tb + 64);
    PD_HIP(hipMemcpyAsync(dt, h, tb, hipMemcpyHostToDevice, s));
    unsigned long long* dc = ctx.arena.get<unsigned long long>("route_cnt", kMaxRanks);
    PD_HIP(hipMemsetAsync(dc, 0, sizeof(unsigned long long) * kMaxRanks, s));
    if (n) {
        dispatch(dtype, d, [&](auto tp, auto Dc) {
            using T = std::remove_pointer_t<decltype(tp)>;
            constexpr int D = decltype(Dc)::value;
            hipLaunchKernelGGL((route_kernel<T, D>), dim3(grid_for(n, 8192)), dim3(kBlock), 0, s,
                               (const T*)X, (uint64_t)n, (const double*)dt, P,
                               (const int32_t*)(dt + sizeof(double) * P * 2 * d), n_ranks, mask,
                               dc);
        });
        PD_HIP(hipGetLastError());
    }
    unsigned long long* hc = (unsigned long long*)pinned(ctx, sizeof(unsigned long long) * kMaxRanks);
    PD_HIP(hipMemcpyAsync(hc, dc, sizeof(unsigned long long) * n_ranks, hipMemcpyDeviceToHost, s));
    sync(s);
    for (int r = 0; r < n_ranks; ++r) counts_host[r] = (int64_t)hc[r];
}

int64_t pack(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const uint64_t* mask, int dest,
             const int32_t* kdlab, int P, const int32_t* part_rank_host,
             const int32_t* local_index_host, uint32_t gid_base, void* coords_out,
             uint32_t* gid_out, int32_t* owner_out, uint8_t* xr_out, int64_t cap, hipStream_t s) {
    if (dest < 0 || dest >= kMaxRanks) throw Error(-1, "dest out of range");
    if (n > (int64_t)kIdMask) throw Error(-5, "n must be < 2^30 points per device");
    if ((uint64_t)gid_base + (uint64_t)n > 0xFFFFFFFEull)
        throw Error(-5, "global ids must stay below 2^32 - 1");
    const size_t tb = sizeof(int32_t) * 2 * P;
    int32_t* h = (int32_t*)pinned(ctx, tb + 64);
    std::memcpy(h, part_rank_host, sizeof(int32_t) * P);
    std::memcpy(h + P, local_index_host, sizeof(int32_t) * P);
    int32_t* dt = ctx.arena.get<int32_t>("pack_tab", 2 * P + 16);
    PD_HIP(hipMemcpyAsync(dt, h, tb, hipMemcpyHostToDevice, s));
    uint32_t* list = ctx.arena.get<uint32_t>("pack_list", n + 1);
    uint32_t* dcount = ctx.arena.get<uint32_t>("pack_count", 4);
    const uint32_t m =
        (uint32_t)compact_ordered(ctx, "pack_cmp", (uint64_t)n, HasBit{mask, dest}, list, dcount, s);
    if ((int64_t)m > cap) throw Error(-1, "pack: output buffers too small");
    if (m) {
        dispatch(dtype, d, [&](auto tp, auto Dc) {
            using T = std::remove_pointer_t<decltype(tp)>;
            constexpr int D = decltype(Dc)::value;
            hipLaunchKernelGGL((pack_kernel<T, D>), dim3(blocks(m)), dim3(kBlock), 0, s,
                               (const T*)X, list, m, mask, kdlab, dt, dt + P, P, dest, gid_base,
                               (T*)coords_out, gid_out, owner_out, xr_out);
        });
        PD_HIP(hipGetLastError());
    }
    return (int64_t)m;
}

void train_exports(Ctx& ctx, uint32_t* gid_out, uint32_t* key_out, int64_t cap, hipStream_t s) {
    const PhaseState& st = ctx.st;
    if (!st.valid) throw Error(-1, "pd_train_exports without a matching pd_train_begin");
    if ((int64_t)st.n_exports > cap) throw Error(-1, "exports buffers too small");
    if (!st.n_exports) return;
    PD_HIP(hipMemcpyAsync(gid_out, st.exp_gid, sizeof(uint32_t) * st.n_exports,
                          hipMemcpyDeviceToDevice, s));
    PD_HIP(hipMemcpyAsync(key_out, st.exp_key, sizeof(uint32_t) * st.n_exports,
                          hipMemcpyDeviceToDevice, s));
}

// O(exports): the union of the pairs runs over the distinct ids they name
// (sorted, unique), not over the whole id space.
int64_t merge_exports(Ctx& ctx, const uint32_t* gid, const uint32_t* key, int64_t m,
                      uint32_t* ids_out, uint32_t* keys_out, hipStream_t s) {
    if (m <= 0) return 0;
    if (m > (int64_t)0x7FFFFFFF) throw Error(-5, "too many exports");
    const size_t m2 = 2 * (size_t)m;
    uint32_t* buf = ctx.arena.get<uint32_t>("mx_buf", m2);
    uint32_t* alt = ctx.arena.get<uint32_t>("mx_alt", m2);
    PD_HIP(hipMemcpyAsync(buf, gid, sizeof(uint32_t) * m, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipMemcpyAsync(buf + m, key, sizeof(uint32_t) * m, hipMemcpyDeviceToDevice, s));
    rocprim::double_buffer<uint32_t> kb(buf, alt);
    size_t tb = 0;
    PD_HIP(rocprim::radix_sort_keys(nullptr, tb, kb, m2, 0u, 32u, s));
    void* tmp = ctx.arena.get<char>("mx_tmp", tb);
    PD_HIP(rocprim::radix_sort_keys(tmp, tb, kb, m2, 0u, 32u, s));
    uint32_t* du = ctx.arena.get<uint32_t>("mx_count", 4);
    tb = 0;
    PD_HIP(rocprim::unique(nullptr, tb, kb.current(), ids_out, du, m2, rocprim::equal_to<uint32_t>(), s));
    tmp = ctx.arena.get<char>("mx_tmp2", tb);
    PD_HIP(rocprim::unique(tmp, tb, kb.current(), ids_out, du, m2, rocprim::equal_to<uint32_t>(), s));
    uint32_t* hu = (uint32_t*)pinned(ctx, sizeof(uint32_t));
    PD_HIP(hipMemcpyAsync(hu, du, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    const uint32_t u = *hu;
    uint32_t* par = ctx.arena.get<uint32_t>("mx_par", u);
    hipLaunchKernelGGL(iota_kernel, dim3(blocks(u)), dim3(kBlock), 0, s, par, u);
    hipLaunchKernelGGL(unite_kernel, dim3(blocks((uint64_t)m)), dim3(kBlock), 0, s, gid, key, m,
                       ids_out, u, par);
    hipLaunchKernelGGL(map_keys_kernel, dim3(blocks(u)), dim3(kBlock), 0, s, par, ids_out, u,
                       keys_out);
    PD_HIP(hipGetLastError());
    return (int64_t)u;
}

int64_t select_roots(Ctx& ctx, const uint32_t* keys, const uint32_t* gid, int64_t n, uint32_t* out,
                     hipStream_t s) {
    if (n > (int64_t)kIdMask) throw Error(-5, "n must be < 2^30 points per device");
    uint32_t* dcount = ctx.arena.get<uint32_t>("roots_count", 4);
    const uint32_t m =
        (uint32_t)compact_ordered(ctx, "roots_cmp", (uint64_t)n, IsRoot{keys, gid}, out, dcount, s);
    if (m && gid) {
        hipLaunchKernelGGL(map_gid_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, out, m, gid);
        PD_HIP(hipGetLastError());
    }
    return (int64_t)m;
}

void sort_u32(Ctx& ctx, uint32_t* data, int64_t n, hipStream_t s) {
    if (n <= 1) return;
    uint32_t* alt = ctx.arena.get<uint32_t>("sortu_alt", (size_t)n);
    rocprim::double_buffer<uint32_t> kb(data, alt);
    size_t tb = 0;
    PD_HIP(rocprim::radix_sort_keys(nullptr, tb, kb, (size_t)n, 0u, 32u, s));
    void* tmp = ctx.arena.get<char>("sortu_tmp", tb);
    PD_HIP(rocprim::radix_sort_keys(tmp, tb, kb, (size_t)n, 0u, 32u, s));
    if (kb.current() != data)
        PD_HIP(hipMemcpyAsync(data, kb.current(), sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipGetLastError());
}

void rank_labels(Ctx& ctx, const uint32_t* keys, int64_t n, const uint32_t* roots, int64_t nr,
                 int32_t* labels, hipStream_t s) {
    if (nr > (int64_t)0x7FFFFFFF) throw Error(-5, "too many clusters");
    if (!n) return;
    uint32_t* dbad = ctx.arena.get<uint32_t>("rank_bad", 4);
    PD_HIP(hipMemsetAsync(dbad, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(rank_kernel, dim3(blocks((uint64_t)n)), dim3(kBlock), 0, s, keys,
                       (uint64_t)n, roots, (uint32_t)nr, labels, dbad);
    PD_HIP(hipGetLastError());
    uint32_t* hb = (uint32_t*)pinned(ctx, sizeof(uint32_t));
    PD_HIP(hipMemcpyAsync(hb, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    if (*hb) throw Error(-1, "rank_labels: a cluster key has no root among the roots given "
                             "(roots must be gathered from every device)");
}

int64_t owned_results(Ctx& ctx, int64_t n, const int32_t* owner, const uint32_t* gid,
                      const int32_t* labels, const uint8_t* core, int n_ranks,
                      const int64_t* gid_off_host, uint32_t* out, int64_t cap,
                      int64_t* counts_host, hipStream_t s) {
    if (n_ranks < 1 || n_ranks > kMaxRanks) throw Error(-1, "n_ranks must be in [1, 64]");
    if (n > (int64_t)kIdMask) throw Error(-5, "n must be < 2^30 points per device");
    for (int r = 0; r < n_ranks; ++r)
        if (gid_off_host[r + 1] < gid_off_host[r]) throw Error(-1, "gid offsets must ascend");
    int64_t* doff = ctx.arena.get<int64_t>("own_off", kMaxRanks + 1);
    int64_t* hoff = (int64_t*)pinned(ctx, sizeof(int64_t) * (kMaxRanks + 1));
    std::memcpy(hoff, gid_off_host, sizeof(int64_t) * (n_ranks + 1));
    PD_HIP(hipMemcpyAsync(doff, hoff, sizeof(int64_t) * (n_ranks + 1), hipMemcpyHostToDevice, s));
    uint32_t* list = ctx.arena.get<uint32_t>("own_list", n + 1);
    uint32_t* dcount = ctx.arena.get<uint32_t>("own_count", 4);
    PD_HIP(hipMemsetAsync(dcount, 0, sizeof(uint32_t), s));
    if (n) {
        rocprim::counting_iterator<uint32_t> it(0u);
        size_t tb = 0;
        IsOwned pred{owner};
        PD_HIP(rocprim::select(nullptr, tb, it, list, dcount, (size_t)n, pred, s));
        void* tmp = ctx.arena.get<char>("own_tmp", tb);
        PD_HIP(rocprim::select(tmp, tb, it, list, dcount, (size_t)n, pred, s));
    }
    // one pinned block: m, bad, counts (the offsets were copied already)
    PD_HIP(hipStreamSynchronize(s));
    uint32_t* hm = (uint32_t*)pinned(ctx, 16 + sizeof(unsigned long long) * kMaxRanks);
    PD_HIP(hipMemcpyAsync(hm, dcount, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    const uint32_t m = hm[0];
    if ((int64_t)m > cap) throw Error(-1, "owned_results: output buffer too small");
    unsigned long long* dc = ctx.arena.get<unsigned long long>("own_cnt", kMaxRanks);
    uint32_t* dbad = ctx.arena.get<uint32_t>("own_bad", 4);
    PD_HIP(hipMemsetAsync(dc, 0, sizeof(unsigned long long) * kMaxRanks, s));
    PD_HIP(hipMemsetAsync(dbad, 0, sizeof(uint32_t), s));
    if (m)
        hipLaunchKernelGGL(owned_pack_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, list, m, gid,
                           labels, core, doff, n_ranks, out, dc, dbad);
    PD_HIP(hipGetLastError());
    unsigned long long* hc = (unsigned long long*)((char*)hm + 16);
    PD_HIP(hipMemcpyAsync(hm + 1, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PD_HIP(hipMemcpyAsync(hc, dc, sizeof(unsigned long long) * n_ranks, hipMemcpyDeviceToHost, s));
    sync(s);
    if (hm[1] & 1) throw Error(-1, "owned_results: global ids do not ascend");
    if (hm[1] & 2) throw Error(-1, "owned_results: global id outside the offsets");
    for (int r = 0; r < n_ranks; ++r) counts_host[r] = (int64_t)hc[r];
    return (int64_t)m;
}

void scatter_results(Ctx& ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base, int64_t n,
                     int32_t* labels, uint8_t* core, hipStream_t s) {
    if (m != n) throw Error(-1, "scatter_results: " + std::to_string(m) + " results for " +
                                    std::to_string(n) + " points");
    if (!n) return;
    uint32_t* dbad = ctx.arena.get<uint32_t>("scat_bad", 4);
    PD_HIP(hipMemsetAsync(dbad, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(fill_i32_kernel, dim3(blocks((uint64_t)n)), dim3(kBlock), 0, s, labels,
                       (uint64_t)n, kUnset);
    hipLaunchKernelGGL(scatter_results_kernel, dim3(blocks((uint64_t)m)), dim3(kBlock), 0, s,
                       pairs, (uint64_t)m, gid_base, (uint64_t)n, labels, core, dbad);
    hipLaunchKernelGGL(unset_check_kernel, dim3(blocks((uint64_t)n)), dim3(kBlock), 0, s, labels,
                       (uint64_t)n, dbad);
    PD_HIP(hipGetLastError());
    uint32_t* hb = (uint32_t*)pinned(ctx, sizeof(uint32_t));
    PD_HIP(hipMemcpyAsync(hb, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    if (*hb & 1) throw Error(-1, "scatter_results: global id outside this device's points");
    if (*hb & 2) throw Error(-1, "scatter_results: a point received no result (each point must "
                                 "be owned by exactly one device)");
}

// ---------------------------------------------------------------- one-pass exchange
void route2(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P, const double* ebox_host,
            const int32_t* part_rank_host, const int32_t* kdlab, int n_ranks, int64_t* counts_host,
            hipStream_t s) {
    RouteState& rt = ctx.rt;
    rt = RouteState{};
    if (n_ranks < 1 || n_ranks > kMaxRanks) throw Error(-1, "n_ranks must be in [1, 64]");
    if (P < 1) throw Error(-1, "need at least one neighbourhood");
    if (n > (int64_t)kIdMask) throw Error(-5, "n must be < 2^30 points per device");
    for (int L = 0; L < P; ++L)
        if (part_rank_host[L] < 0 || part_rank_host[L] >= n_ranks)
            throw Error(-1, "part_rank out of range");
    const size_t tb = sizeof(double) * P * 2 * d + sizeof(int32_t) * P;
    char* h = (char*)pinned(ctx, tb + 64);
    std::memcpy(h, ebox_host, sizeof(double) * P * 2 * d);
    std::memcpy(h + sizeof(double) * P * 2 * d, part_rank_host, sizeof(int32_t) * P);
    char* dt = ctx.arena.get<char>("route_tab", tb + 64);
    PD_HIP(hipMemcpyAsync(dt, h, tb, hipMemcpyHostToDevice, s));
    const unsigned tiles = (unsigned)std::max<int64_t>(1, (n + kRTile - 1) / kRTile);
    const size_t nt = (size_t)tiles * n_ranks;
    uint64_t* mask = ctx.arena.get<uint64_t>("route_mask", (size_t)n + 1);
    uint32_t* cnt = ctx.arena.get<uint32_t>("route_tcnt", nt + 1);
    uint64_t* off = ctx.arena.get<uint64_t>("route_toff", nt + 1);
    unsigned long long* dres = ctx.arena.get<unsigned long long>("route_res", 2 * kMaxRanks);
    PD_HIP(hipMemsetAsync(dres, 0, sizeof(unsigned long long) * 2 * kMaxRanks, s));
    PD_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (nt + 1), s));
    if (n) {
        dispatch(dtype, d, [&](auto tp, auto Dc) {
            using T = std::remove_pointer_t<decltype(tp)>;
            constexpr int D = decltype(Dc)::value;
            hipLaunchKernelGGL((route_tile_kernel<T, D>), dim3(tiles), dim3(kBlock), 0, s,
                               (const T*)X, (uint64_t)n, (const double*)dt, P,
                               (const int32_t*)(dt + sizeof(double) * P * 2 * d), kdlab, n_ranks,
                               tiles, mask, cnt, dres + kMaxRanks);
        });
        PD_HIP(hipGetLastError());
    }
    size_t sb = 0;
    PD_HIP(rocprim::exclusive_scan(nullptr, sb, cnt, off, (uint64_t)0, nt + 1,
                                   rocprim::plus<uint64_t>(), s));
    void* tmp = ctx.arena.get<char>("route_scan_tmp", sb);
    PD_HIP(rocprim::exclusive_scan(tmp, sb, cnt, off, (uint64_t)0, nt + 1,
                                   rocprim::plus<uint64_t>(), s));
    hipLaunchKernelGGL(route_totals_kernel, dim3(1), dim3(kMaxRanks), 0, s, off, tiles, n_ranks,
                       dres);
    PD_HIP(hipGetLastError());
    unsigned long long* hc =
        (unsigned long long*)pinned(ctx, sizeof(unsigned long long) * 2 * kMaxRanks);
    PD_HIP(hipMemcpyAsync(hc, dres, sizeof(unsigned long long) * 2 * kMaxRanks,
                          hipMemcpyDeviceToHost, s));
    sync(s);
    for (int r = 0; r < n_ranks; ++r) {
        counts_host[2 * r] = (int64_t)hc[r];
        counts_host[2 * r + 1] = (int64_t)hc[kMaxRanks + r];
    }
    rt.valid = true;
    rt.n = n;
    rt.n_ranks = n_ranks;
    rt.tiles = tiles;
    rt.mask = mask;
    rt.off = off;
}

void pack2(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* kdlab, int P,
           const int32_t* part_rank_host, const int32_t* local_index_host, uint32_t gid_base,
           int n_ranks, void* const* coords, uint32_t* const* gid, int32_t* const* owner,
           uint8_t* const* xr, hipStream_t s) {
    RouteState& rt = ctx.rt;
    if (!rt.valid || rt.n != n || rt.n_ranks != n_ranks)
        throw Error(-1, "pd_pack2 without a matching pd_route2 on this context");
    if ((uint64_t)gid_base + (uint64_t)n > 0xFFFFFFFEull)
        throw Error(-5, "global ids must stay below 2^32 - 1");
    // tables: part_rank | local_index | 4 x n_ranks output pointers
    const size_t ib = sizeof(int32_t) * 2 * P, pb = sizeof(void*) * 4 * n_ranks;
    const size_t ibp = (ib + 15) & ~size_t(15);
    char* h = (char*)pinned(ctx, ibp + pb + 64);
    std::memcpy(h, part_rank_host, sizeof(int32_t) * P);
    std::memcpy(h + sizeof(int32_t) * P, local_index_host, sizeof(int32_t) * P);
    void** hp = (void**)(h + ibp);
    for (int r = 0; r < n_ranks; ++r) {
        hp[r] = coords[r];
        hp[n_ranks + r] = gid[r];
        hp[2 * n_ranks + r] = owner[r];
        hp[3 * n_ranks + r] = xr[r];
    }
    char* dt = ctx.arena.get<char>("pack2_tab", ibp + pb + 64);
    PD_HIP(hipMemcpyAsync(dt, h, ibp + pb, hipMemcpyHostToDevice, s));
    void** dp = (void**)(dt + ibp);
    const PackOut po{(void* const*)dp, (uint32_t* const*)(dp + n_ranks),
                     (int32_t* const*)(dp + 2 * n_ranks), (uint8_t* const*)(dp + 3 * n_ranks)};
    if (n) {
        dispatch(dtype, d, [&](auto tp, auto Dc) {
            using T = std::remove_pointer_t<decltype(tp)>;
            constexpr int D = decltype(Dc)::value;
            hipLaunchKernelGGL((pack_tile_kernel<T, D>), dim3(rt.tiles), dim3(kBlock), 0, s,
                               (const T*)X, (uint64_t)n, rt.mask, rt.off, rt.tiles, kdlab,
                               (const int32_t*)dt, (const int32_t*)dt + P, P, n_ranks, gid_base,
                               po);
        });
        PD_HIP(hipGetLastError());
    }
    sync(s);   // the pinned tables are reused by later calls
    rt.valid = false;
}

void results(Ctx& ctx, int64_t nr, const uint32_t* keys, const uint8_t* core, const int32_t* owner,
             const uint32_t* gid, const uint32_t* roots, int64_t n_roots, int64_t n_total,
             uint32_t gid_base, int64_t n_local, int n_ranks, int me, const int64_t* src_off,
             int64_t expect_remote, int32_t* labels, uint8_t* core_out, uint32_t* pairs,
             hipStream_t s) {
    if (n_ranks < 1 || n_ranks > kMaxRanks || me < 0 || me >= n_ranks)
        throw Error(-1, "bad rank / n_ranks");
    if (nr > (int64_t)kIdMask || n_local > (int64_t)kIdMask)
        throw Error(-5, "n must be < 2^30 points per device");
    if (n_roots > (int64_t)0x7FFFFFFF || n_roots > n_total) throw Error(-5, "too many clusters");
    for (int r = 0; r < n_ranks; ++r)
        if (src_off[r + 1] < src_off[r]) throw Error(-1, "source offsets must ascend");
    if (src_off[0] != 0 || src_off[n_ranks] != nr) throw Error(-1, "source offsets must span the records");
    uint32_t* dbad = ctx.arena.get<uint32_t>("res_bad", 4);
    PD_HIP(hipMemsetAsync(dbad, 0, sizeof(uint32_t), s));
    if (n_local) {
        hipLaunchKernelGGL(fill_i32_kernel, dim3(blocks((uint64_t)n_local)), dim3(kBlock), 0, s,
                           labels, (uint64_t)n_local, kUnset);
        if (core_out) PD_HIP(hipMemsetAsync(core_out, 0, (size_t)n_local, s));
    }
    const uint64_t lo = (uint64_t)src_off[me], hi = (uint64_t)src_off[me + 1];
    // the roots' index table (keys are global point ids < n_total)
    uint32_t sh = 0;
    while (sh < 32 && ((uint64_t)n_total >> sh) >= (uint64_t)kRootIdx) ++sh;
    uint32_t* ridx = ctx.arena.get<uint32_t>("root_idx", kRootIdx + 1);
    hipLaunchKernelGGL(root_index_kernel, dim3(blocks((uint64_t)kRootIdx + 1)), dim3(kBlock), 0, s,
                       roots, (uint32_t)n_roots, sh, ridx);
    const RootIndex RI{roots, ridx, (uint32_t)n_roots, sh};
    if (hi > lo)
        hipLaunchKernelGGL(results_self_kernel,
                           dim3((unsigned)((hi - lo + (uint64_t)kBlock * kResPer - 1) /
                                           ((uint64_t)kBlock * kResPer))),
                           dim3(kBlock), 0, s, keys,
                           core, owner, gid, lo, hi, RI, gid_base,
                           (uint64_t)n_local, labels, core_out, dbad);
    if (expect_remote > 0) {
        uint32_t* list = ctx.arena.get<uint32_t>("res_list", (size_t)nr + 1);
        uint32_t* dcount = ctx.arena.get<uint32_t>("res_count", 4);
        compact_ordered(ctx, "res_cmp", (uint64_t)nr, IsRemoteOwned{owner, lo, hi}, list, dcount, s,
                        false);
        hipLaunchKernelGGL(results_pack_kernel, dim3(blocks((uint64_t)expect_remote)), dim3(kBlock),
                           0, s, list, dcount, expect_remote, keys, core, gid, RI, pairs, dbad);
    }
    PD_HIP(hipGetLastError());
}

void results_scatter(Ctx& ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base, int64_t n,
                     int32_t* labels, uint8_t* core, hipStream_t s) {
    uint32_t* dbad = ctx.arena.get<uint32_t>("res_bad", 4);
    if (m)
        hipLaunchKernelGGL(results_scatter_kernel, dim3(blocks((uint64_t)m)), dim3(kBlock), 0, s,
                           pairs, (uint64_t)m, gid_base, (uint64_t)n, labels, core, dbad);
    if (n)
        hipLaunchKernelGGL(unset_check_kernel, dim3(blocks((uint64_t)n)), dim3(kBlock), 0, s, labels,
                           (uint64_t)n, dbad);
    PD_HIP(hipGetLastError());
    uint32_t* hb = (uint32_t*)pinned(ctx, sizeof(uint32_t));
    PD_HIP(hipMemcpyAsync(hb, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    const uint32_t b = *hb;
    if (b & 1) throw Error(-1, "results: a global id outside this device's points (or a sender's "
                               "owned records differed from the exchanged counts)");
    if (b & 2) throw Error(-1, "results: a point received no result (each point must be owned by "
                               "exactly one device)");
    if (b & 4) throw Error(-1, "results: a cluster key has no root among the roots given (roots "
                               "must be gathered from every device)");
    if (b & 8) throw Error(-1, "results: the owned records to return differ from the exchanged "
                               "counts");
}

}  // namespace pd
