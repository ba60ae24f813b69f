// The per-neighbourhood DBSCAN engine, batched over every KD neighbourhood
// held by this device, plus the cross-neighbourhood label merge.
//
// Replaces, in one device-resident pipeline:
//   DBSCAN._create_neighborhoods   (halo records)        R:dbscan/dbscan.py:136-151
//   partitionBy(P) shuffle         (sort by key)         R:dbscan/dbscan.py:116-118
//   dbscan_partition -> sklearn    (count/core/union)    R:dbscan/dbscan.py:12-34
//   _remap_cluster_ids + ClusterAggregator (merge)       R:dbscan/dbscan.py:153-165,
//                                                        R:dbscan/aggregator.py:9-73
//
// Data layout in HBM (R = halo records = sum of neighbourhood sizes):
//   keys  K[R]   neighbourhood base + row-major eps-cell index (axis 0 fastest)
//   vals  u32[R] point id | owner bit (record is the point's own KD partition)
//   Xs    T[R*d] coordinates gathered into key order (AoS, input precision)
//   dir   u64[W] occupancy bit per cell + u32[W] prefix ranks (W = G/64):
//         rank_lt(k) = number of occupied cells with key < k, O(1)
//   cstart u32[ncells+1] first record of each occupied cell
//   core  u8[R], parent u32[R] (union-find, root = min record in component)
//
// Exactness: the neighbour predicate is sklearn's kd_tree leaf test
// (SK:neighbors/_binary_tree.pxi.tp:1951-1955, SK:metrics/_dist_metrics.pxd.tp:
// 39-49): fp64, per-axis difference, squared and summed in axis order with
// every product and sum rounded separately (__dmul_rn/__dadd_rn: no FMA), then
// `<= eps*eps`.  Inputs (fp32 or fp64) are widened exactly.  For fp32 inputs
// a pair is first screened in fp32 (Pred, PD_OPT_FP32_SCREEN, default on):
// distances outside a 2^-18 relative band around the threshold are decided
// there, the rest by the exact fp64 predicate — the answer is identical
// either way (the band bounds the fp32 rounding error), only cheaper.
//
// Labels: components of the core graph get the id of their smallest core
// point (global index); a border point takes the smallest id among its core
// neighbours; ids are ranked.  That is precisely sklearn's dbscan_inner order
// (SK:cluster/_dbscan_inner.pyx:19-41), so fit_predict labels come out equal,
// not merely equal up to permutation.
#include <cstring>
#include <rocprim/rocprim.hpp>
#ifndef PD_SORT_ROCPRIM
#define PD_SORT_ROCPRIM 0
#endif

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstring>
#include <vector>

#include "compact.hpp"
#include "internal.hpp"
#include "rsort.hpp"
#include "scan.hpp"
#include "stream.hpp"
#include "uf.hpp"

namespace pd {
namespace {

// Device-side bounds checks (debug builds: -DPD_CHECK_BOUNDS=1, e.g.
// tools/build_variant.sh): every checked access that would leave its buffer
// is skipped and the first one recorded (site << 48 | index); the host reads
// the record after the kernel (check_bounds) and throws.  Off (the default),
// PD_OK is `true` and costs nothing.
#ifndef PD_CHECK_BOUNDS
#define PD_CHECK_BOUNDS 0
#endif
#if PD_CHECK_BOUNDS
__device__ unsigned long long g_oob[2];   // [0] violations, [1] the first
__device__ __forceinline__ bool pd_ok(bool c, unsigned site, uint64_t idx) {
    if (!c && atomicAdd(&g_oob[0], 1ull) == 0ull)
        g_oob[1] = ((unsigned long long)site << 48) | (idx & 0xFFFFFFFFFFFFull);
    return c;
}
#define PD_OK(cond, site, idx) pd_ok((cond), (site), (uint64_t)(idx))
#else
#define PD_OK(cond, site, idx) true
#endif

// ------------------------------------------------------------------ helpers
// (union-find primitives: uf.hpp)

// L1-cacheable variant for the hot link loop: workgroup-scope relaxed loads
// compile to plain global_loads; stale values are older ancestors, which the
// algorithm tolerates (every retry starts from the CAS's returned value, and
// indices only decrease, so it terminates).  Halving stores stay write-through.
__device__ __forceinline__ uint32_t ld_l1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint32_t uf_find_l1(uint32_t* par, uint32_t x) {
    uint32_t p = ld_l1(par + x);
    while (p != x) {
        uint32_t g = ld_l1(par + p);
        if (g == p) return p;
        st_rlx(par + x, g);
        x = g;
        p = ld_l1(par + x);
    }
    return x;
}

// Link two roots (a = caller's current root); returns the caller's new root.
__device__ __forceinline__ uint32_t uf_link_roots(uint32_t* par, uint32_t a, uint32_t b) {
    while (a != b) {
        if (a > b) {
            uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t expected = b;
        if (__hip_atomic_compare_exchange_strong(par + b, &expected, a, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return a;
        b = uf_find_l1(par, expected);
        a = uf_find_l1(par, a);
    }
    return a;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

// atomicMin(base[key], val) for the lanes with `valid`, one atomic per
// distinct key per wave: consecutive records mostly share a component, and a
// big cluster's root otherwise takes ~1e5 serialised atomics.  Every lane of
// the wave must call this (no early return before it).
#ifndef PD_GMIN_CACHED
#define PD_GMIN_CACHED 0
#endif
// The skip test's read of the current minimum: any stale value is >= the
// current one, so an L1-cached read is as exact as an L2 one (it may only
// cost an atomic the fresher read would have skipped).
__device__ __forceinline__ uint32_t gmin_peek(const uint32_t* p) {
    if constexpr (PD_GMIN_CACHED) return *p;
    else return ld_rlx(p);
}

__device__ __forceinline__ void wave_atomic_min(uint32_t* base, bool valid, uint32_t key,
                                                uint32_t val) {
    const int lane = threadIdx.x & 63;
    unsigned long long active = __ballot(valid);
    while (active) {
        const int leader = __ffsll(active) - 1;
        const uint32_t lk = (uint32_t)__shfl((int)key, leader, 64);
        const bool mine = valid && ((active >> lane) & 1ull) && key == lk;
        const uint32_t m = wave_min_u32(mine ? val : kNone);
        // keys only decrease: a stale read is >= the current minimum, so
        // skipping when it is already <= m is exact; a hot root (a city of
        // 1e8 records) then takes reads, not a queue of atomics
        if (lane == leader && m < gmin_peek(base + lk)) atomicMin(base + lk, m);
        active &= ~__ballot(mine);
    }
}

// Append val to list where pred holds, one atomic per wave: a wave's entries
// land contiguously (in lane order), so lists keep the spatial locality of
// the records that produced them.  Every lane of the wave must call this.
__device__ __forceinline__ void wave_append(uint32_t* __restrict__ list, uint32_t* __restrict__ count,
                                            bool pred, uint32_t val) {
    const unsigned long long b = __ballot(pred);
    if (!b) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(b) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (pred) list[base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = val;
}

template <typename T, int D>
__device__ __forceinline__ void load_d(const T* __restrict__ X, uint64_t i, double (&v)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (double)X[i * D + j];
}

// Sorted-record layout: 3-D records are padded to 4 components so one
// 16-byte (fp32) load fetches a candidate; other D are packed.
template <int D>
struct Stride {
    static constexpr int v = (D == 3) ? 4 : D;
};

template <typename T, int D>
__device__ __forceinline__ void load_rec(const T* __restrict__ Xs, uint32_t j, double (&v)[D]) {
    constexpr int S = Stride<D>::v;
    if constexpr (std::is_same<T, float>::value && S == 4) {
        const float4 f = *reinterpret_cast<const float4*>(Xs + (uint64_t)j * 4);
        v[0] = f.x;
        v[1] = f.y;
        v[2] = f.z;
        if constexpr (D == 4) v[3] = f.w;
    } else if constexpr (std::is_same<T, float>::value && S == 2) {
        const float2 f = *reinterpret_cast<const float2*>(Xs + (uint64_t)j * 2);
        v[0] = f.x;
        v[1] = f.y;
    } else if constexpr (std::is_same<T, double>::value && S >= 2) {
        const double2* p = reinterpret_cast<const double2*>(Xs + (uint64_t)j * S);
        const double2 u = p[0];
        v[0] = u.x;
        v[1] = u.y;
        if constexpr (S == 4) {
            const double2 w = p[1];
            v[2] = w.x;
            if constexpr (D == 4) v[3] = w.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) v[k] = (double)Xs[(uint64_t)j * S + k];
    }
}

// sklearn kd_tree leaf predicate, exact: fp64, axis order, every product and
// sum rounded separately (no FMA), `<= eps*eps` (cityblock: `<= eps`).
template <int D, int M>
__device__ __forceinline__ bool within(const double (&a)[D], const double (&b)[D], double eps,
                                       double eps2) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const double t = __dadd_rn(a[j], -b[j]);
        if constexpr (M == 0)
            acc = __dadd_rn(acc, __dmul_rn(t, t));
        else
            acc = __dadd_rn(acc, fabs(t));
    }
    return M == 0 ? (acc <= eps2) : (acc <= eps);
}

// Raw candidate load (input precision).
template <typename T, int D>
__device__ __forceinline__ void load_raw(const T* __restrict__ Xs, uint32_t j, T (&v)[D]) {
    constexpr int S = Stride<D>::v;
    if constexpr (std::is_same<T, float>::value && S == 4) {
        const float4 f = *reinterpret_cast<const float4*>(Xs + (uint64_t)j * 4);
        v[0] = f.x;
        v[1] = f.y;
        v[2] = f.z;
        if constexpr (D == 4) v[3] = f.w;
    } else if constexpr (std::is_same<T, float>::value && S == 2) {
        const float2 f = *reinterpret_cast<const float2*>(Xs + (uint64_t)j * 2);
        v[0] = f.x;
        v[1] = f.y;
    } else if constexpr (std::is_same<T, double>::value && S >= 2) {
        const double2* p = reinterpret_cast<const double2*>(Xs + (uint64_t)j * S);
        const double2 u = p[0];
        v[0] = u.x;
        v[1] = u.y;
        if constexpr (S == 4) {
            const double2 w = p[1];
            v[2] = w.x;
            if constexpr (D == 4) v[3] = w.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) v[k] = Xs[(uint64_t)j * S + k];
    }
}

// The neighbour predicate as the sweeps use it.  fp32 inputs are screened
// in fp32 first: with every coordinate an fp32 value, the fp32 distance has
// relative error <= (D+2)*2^-24 < 2^-18, so a result below eps^2*(1-2^-18)
// (rounded down to fp32) or above eps^2*(1+2^-18) (rounded up) already
// decides the exact fp64 test; only pairs inside that band (ties) run it.
// fp64 inputs always take the exact path.
template <typename T, int D, int M>
struct Pred {
    double a[D];
    T ar[D];
    double eps, eps2;
    float lo, hi;
    __device__ __forceinline__ bool operator()(const T (&b)[D]) const {
        if constexpr (std::is_same<T, float>::value) {
            float d = 0.0f;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float t = ar[j] - b[j];
                if constexpr (M == 0)
                    d = __builtin_fmaf(t, t, d);
                else
                    d += fabsf(t);
            }
            if (d <= lo) return true;
            if (!(d <= hi)) return false;
        }
        double bb[D];
#pragma unroll
        for (int j = 0; j < D; ++j) bb[j] = (double)b[j];
        return within<D, M>(a, bb, eps, eps2);
    }
    // Branch-free screen: in = decided inside, maybe = needs exact(); fp64
    // inputs are always "maybe".
    __device__ __forceinline__ void screen(const T (&b)[D], bool& in, bool& maybe) const {
        if constexpr (std::is_same<T, float>::value) {
            float d = 0.0f;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float t = ar[j] - b[j];
                if constexpr (M == 0)
                    d = __builtin_fmaf(t, t, d);
                else
                    d += fabsf(t);
            }
            in = d <= lo;
            maybe = !in & (d <= hi);
        } else {
            in = false;
            maybe = true;
        }
    }
    __device__ __forceinline__ bool exact(const T (&b)[D]) const {
        double bb[D];
#pragma unroll
        for (int j = 0; j < D; ++j) bb[j] = (double)b[j];
        return within<D, M>(a, bb, eps, eps2);
    }
};

template <typename T, int D, int M>
__device__ __forceinline__ Pred<T, D, M> make_pred(const T* __restrict__ Xs, uint32_t r,
                                                   const double (&a)[D], double eps, double eps2,
                                                   float lo, float hi) {
    Pred<T, D, M> p;
#pragma unroll
    for (int j = 0; j < D; ++j) p.a[j] = a[j];
    load_raw<T, D>(Xs, r, p.ar);
    p.eps = eps;
    p.eps2 = eps2;
    p.lo = lo;
    p.hi = hi;
    return p;
}

template <int D>
__device__ __forceinline__ void cell_of(const double (&v)[D], const PartGrid& g, int64_t (&c)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        int64_t q = (int64_t)floor((v[j] - g.lo[j]) * g.inv[j]);
        q = q < 0 ? 0 : q;
        q = q >= g.nc[j] ? g.nc[j] - 1 : q;
        c[j] = q;
    }
}

template <int D>
__device__ __forceinline__ uint64_t lin_of(const int64_t (&c)[D], const PartGrid& g) {
    uint64_t k = 0;
#pragma unroll
    for (int j = D - 1; j >= 0; --j) k = k * (uint64_t)g.nc[j] + (uint64_t)c[j];
    return k;
}

// Box test in the input precision: for fp32 coordinates v, (double)v >= elo
// iff v >= flo (flo = the smallest float >= elo), likewise for ehi / fhi.
template <typename T, int D>
__device__ __forceinline__ bool in_box_t(const T (&v)[D], const PartGrid& g) {
    bool in = true;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if constexpr (std::is_same<T, float>::value)
            in &= (g.flo[j] <= v[j]) & (g.fhi[j] >= v[j]);
        else
            in &= (g.elo[j] <= v[j]) & (g.ehi[j] >= v[j]);
    }
    return in;
}


// Partition of a record: part_start is sorted.
__device__ __forceinline__ int part_of(const uint32_t* __restrict__ ps, int P, uint32_t r) {
    int lo = 0, hi = P - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (ps[mid] <= r)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t rec_index() {
    return xcd_block(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
}

// Shared view of the cell structure for the neighbour sweeps.
struct Cells {
    const PartGrid* parts;
    const uint32_t* part_start;
    int P;
    const uint4* dir;
    const uint32_t* cstart;
    const uint4* pages;   // paged directory (null: flat, dir[k >> 6]); see dir_word
};

template <int D>
struct NRows {
    static constexpr int v = (D == 1) ? 1 : (D == 2 ? 3 : (D == 3 ? 9 : 27));
};

// Occupied cells with key < k, from the key's directory word.
__device__ __forceinline__ uint32_t dir_rank(const uint4& w, uint64_t k) {
    const uint64_t bits = ((uint64_t)w.y << 32) | (uint64_t)w.x;
    const uint32_t sh = (uint32_t)(k & 63);
    const uint64_t m = sh ? (bits & ((~0ull) >> (64 - sh))) : 0ull;
    return w.z + (uint32_t)__popcll(m);
}

// Paged directory (PD_OPT_DIR_PAGED; automatic when the grid has more
// directory words than points).  Keys are grouped in pages of 64 words (4096
// cells); pages[p] = {occupancy mask of the page's 64 words (x, y), number of
// occupied words before the page (z)}, and only the occupied words are
// stored, in key order, followed by a terminal word {0, 0, ncells}.  The word
// of key k is one page load and one word load; an empty word reads as the
// next occupied word with its bits cleared — the same prefix rank — so
// dir_rank and every sweep are unchanged.  Memory: 16 B per page + 16 B per
// occupied word, instead of 16 B per word of the bounding box.
__device__ __forceinline__ uint64_t page_slot(const uint4& pg, uint64_t wid, bool& occ) {
    const uint64_t m = ((uint64_t)pg.y << 32) | (uint64_t)pg.x;
    const uint32_t b = (uint32_t)(wid & 63);
    occ = (m >> b) & 1ull;
    const uint64_t below = b ? (m & ((~0ull) >> (64 - b))) : 0ull;
    return (uint64_t)pg.z + (uint64_t)__popcll(below);
}

// Directory word of key k (either layout).
__device__ __forceinline__ uint4 dir_word(const Cells& C, uint64_t k) {
    if (!C.pages) return C.dir[k >> 6];
    bool occ;
    const uint64_t s = page_slot(C.pages[k >> 12], k >> 6, occ);
    uint4 w = C.dir[s];
    if (!occ) {
        w.x = 0u;
        w.y = 0u;
    }
    return w;
}

// Word slot of an occupied cell key (flat: k >> 6).
__device__ __forceinline__ uint64_t word_slot(const uint4* __restrict__ pages, uint64_t k) {
    if (!pages) return k >> 6;
    bool occ;
    return page_slot(pages[k >> 12], k >> 6, occ);
}

// Word root (wroot: per directory word slot) of key k's word; kNone for an
// empty word.
__device__ __forceinline__ uint32_t word_root_at(const Cells& C, const uint32_t* __restrict__ wroot,
                                                 uint64_t k) {
    if (!C.pages) return wroot[k >> 6];
    bool occ;
    const uint64_t s = page_slot(C.pages[k >> 12], k >> 6, occ);
    return occ ? wroot[s] : kNone;
}

// Partition of a record.  Waves almost always sit inside one partition: try
// the first lane's partition on the scalar path, fall back per lane.
__device__ __forceinline__ int part_of_wave(const uint32_t* __restrict__ ps, int P, uint32_t r) {
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(r);
    const int L0 = part_of(ps, P, r0);
    const uint32_t lo = ps[L0], hi = ps[L0 + 1];
    if (__all(r >= lo && r < hi)) return L0;
    return part_of(ps, P, r);
}

// ------------------------------------------------------------------ kernels
// The KD partition's split tree (pd_train_tree): a point's owner label is
// found by replaying the BFS splits on its coordinates — level l, the label's
// slot: v[axis] >= boundary moves it to the new label (the kd_pass split,
// R:dbscan/partition.py:66-68) — so pd_train needs no owner array and the
// partitioner no final split pass.
struct KdTree {
    int nl = 0;                  // levels (0: no tree)
    int ntab[16], toff[16], eoff[16];
    int nslot = 0, ne = 0;       // table sizes
    const int32_t* slot;         // per level: label -> slot (-1: not split)
    const int32_t* ax_new;       // per split: axis, new label
    const double* bound;         // per split: boundary
};
// tables up to this size are staged in LDS by halo_write_kernel (P <= 64)
constexpr int kTreeSlots = 256, kTreeSplits = 128;

template <typename T, int D>
__device__ __forceinline__ int tree_owner(const KdTree& t, const int32_t* slot,
                                          const int32_t* ax_new, const double* bound,
                                          const T (&v)[D]) {
    int lab = 0;
    for (int l = 0; l < t.nl; ++l) {
        if (lab >= t.ntab[l]) continue;
        if (!PD_OK(t.toff[l] + lab < t.nslot, 1, t.toff[l] + lab)) continue;
        const int sl = slot[t.toff[l] + lab];
        if (sl < 0) continue;
        const int e = t.eoff[l] + sl;
        if (!PD_OK(e < t.ne, 2, e)) continue;
        const int ax = ax_new[2 * e];
        if (!PD_OK(ax >= 0 && ax < D, 3, ax)) continue;
        T x = v[0];
#pragma unroll
        for (int j = 1; j < D; ++j) x = ax == j ? v[j] : x;
        if ((double)x >= bound[e]) lab = ax_new[2 * e + 1];
    }
    return lab;
}

// tree_owner, and whether the point lies within `marg` (2 eps, grown) of a
// split plane on its path, or of a non-finite one.  A point farther than
// 2 eps from every plane on its path lies in its owner's expanded box only:
// any other KD box is separated from it by one of those planes (the first
// split where the two paths part), so its 2 eps expansion cannot reach it.
template <typename T, int D>
__device__ __forceinline__ int tree_owner_near(const KdTree& t, const int32_t* slot,
                                               const int32_t* ax_new, const double* bound,
                                               double marg, const T (&v)[D], bool& near) {
    int lab = 0;
    near = false;
    for (int l = 0; l < t.nl; ++l) {
        if (lab >= t.ntab[l]) continue;
        if (!PD_OK(t.toff[l] + lab < t.nslot, 1, t.toff[l] + lab)) continue;
        const int sl = slot[t.toff[l] + lab];
        if (sl < 0) continue;
        const int e = t.eoff[l] + sl;
        if (!PD_OK(e < t.ne, 2, e)) continue;
        const int ax = ax_new[2 * e];
        if (!PD_OK(ax >= 0 && ax < D, 3, ax)) continue;
        T x = v[0];
#pragma unroll
        for (int j = 1; j < D; ++j) x = ax == j ? v[j] : x;
        const double xd = (double)x, b = bound[e];
        // (2^-20 |b|: far beyond the fp64 expand's and the fp32 bounds' rounding)
        near |= !(fabs(xd - b) > marg + 9.5367431640625e-07 * fabs(b));
        if (xd >= b) lab = ax_new[2 * e + 1];
    }
    return lab;
}

// Halo records (R:dbscan/dbscan.py:136-151) in two ordered passes over the
// points: halo_tile_kernel counts each tile's records (a tile = one block's
// 4·256 points), the host scans the tile counts (rocPRIM), and
// halo_write_kernel recomputes the memberships and writes the (cell key,
// point id | owner bit | duplicate bit) records at tile offset + wave
// offset.  No per-point count array, no inter-block waiting (the dispatch
// order is undefined: cdna_hip_programming.md Guideline 16).
// Lane l of wave w takes points base + 256 w + 64 q + l (q = 0..3): every
// load and every record store of one step q is contiguous across the wave.
// The membership of each point is a bit mask over the neighbourhoods (P <=
// 64; MASK = false recomputes instead), built branch-free in the input
// precision with one wave-uniform grid load per neighbourhood.
// The near-plane points of a tile, listed in LDS: (thread << 2 | step), and
// each one's full-test record count and neighbourhood mask.
struct NearLds {
    uint32_t n;
    uint32_t list[4 * kBlock];
    uint32_t cnt[4 * kBlock];
    unsigned long long mask[4 * kBlock];
};

template <typename T, int D, bool MASK>
__device__ __forceinline__ void halo_points(const T* __restrict__ X, uint64_t n,
                                            const PartGrid* __restrict__ parts, int P,
                                            uint64_t tile,
                                            uint64_t (&idx)[4], T (&v)[4][D],
                                            unsigned long long (&m)[4], uint32_t (&cnt)[4]) {
    const uint64_t base = tile * (4 * kBlock) + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        idx[q] = base + 64 * q;
        m[q] = 0;
        cnt[q] = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) v[q][j] = idx[q] < n ? X[idx[q] * D + j] : T(NAN);
    }
    for (int L = 0; L < P; ++L) {
        const PartGrid& g = parts[L];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool in = in_box_t<T, D>(v[q], g);
            cnt[q] += in ? 1u : 0u;
            if constexpr (MASK) m[q] |= (unsigned long long)in << L;
        }
    }
}

// halo_points with the split tree in LDS (P <= 64, pd_train_tree): each
// point's owner by the tree replay; a point far from every split plane on its
// path is in its owner's expanded box alone (tree_owner_near) — one record, no
// box tests; the few near a plane (the halo duplicates and their
// neighbours, ~1-2 % at the BASELINE configs) are listed block-wide and take
// the full test, one list entry per lane.  Same counts and masks as
// halo_points.  own[q]: the owner (-1 past n).  The caller zeroes nl.n and
// synchronises before the call.
template <typename T, int D>
__device__ __forceinline__ void halo_points_tree(const T* __restrict__ X, uint64_t n,
                                                 const PartGrid* __restrict__ parts, int P,
                                                 uint64_t tile, const KdTree& tree,
                                                 const int32_t* t_slot, const int32_t* t_axn,
                                                 const double* t_bd, double marg, NearLds& nl,
                                                 uint64_t (&idx)[4], T (&v)[4][D],
                                                 unsigned long long (&m)[4], uint32_t (&cnt)[4],
                                                 int (&own)[4]) {
    const uint64_t base = tile * (4 * kBlock) + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
    int slotq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        idx[q] = base + 64 * q;
        const bool ok = idx[q] < n;
#pragma unroll
        for (int j = 0; j < D; ++j) v[q][j] = ok ? X[idx[q] * D + j] : T(NAN);
        bool near = false;
        own[q] = ok ? tree_owner_near<T, D>(tree, t_slot, t_axn, t_bd, marg, v[q], near) : -1;
        cnt[q] = ok ? 1u : 0u;
        m[q] = ok ? 1ull << (own[q] & 63) : 0ull;
        slotq[q] = -1;
        if (ok && near) {
            slotq[q] = (int)atomicAdd(&nl.n, 1u);
            nl.list[slotq[q]] = (threadIdx.x << 2) | (uint32_t)q;
        }
    }
    __syncthreads();
    const uint32_t nn = nl.n;
    const uint64_t tb = tile * (4 * kBlock);
    for (uint32_t k = threadIdx.x; k < nn; k += kBlock) {
        const uint32_t e = nl.list[k], th = e >> 2, q = e & 3;
        const uint64_t i = tb + (th >> 6) * 256 + (th & 63) + 64 * q;
        T u[D];
#pragma unroll
        for (int j = 0; j < D; ++j) u[j] = X[i * D + j];
        uint32_t c = 0;
        unsigned long long mm = 0;
        for (int Lb = 0; Lb < P; ++Lb) {
            const bool in = in_box_t<T, D>(u, parts[Lb]);
            c += in ? 1u : 0u;
            mm |= (unsigned long long)in << Lb;
        }
        nl.cnt[k] = c;
        nl.mask[k] = mm;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (slotq[q] >= 0) {
            cnt[q] = nl.cnt[slotq[q]];
            m[q] = nl.mask[slotq[q]];
        }
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v) {
    __shared__ uint32_t ws[kBlock / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int u = 0; u < kBlock / 64; ++u) t += ws[u];
    return t;
}

// A tile kernel's count (tile_offsets scans tiles + 1 entries): block 0 also
// zeroes the trailing entry, so no fill runs before the scan.
__device__ __forceinline__ void tile_count_out(uint32_t* tile_cnt, uint32_t c) {
    tile_cnt[blockIdx.x] = c;
    if (blockIdx.x == 0) tile_cnt[gridDim.x] = 0;
}

constexpr int kCtrs = 16;   // train counters: [0..7] lists, [8..9] big / mid cells, [10] pairs

// TREE (the split tree in LDS, P <= 64): the near-plane fast path
// (halo_points_tree); marg = 2 eps, slightly grown.
template <typename T, int D, bool TREE>
__global__ __launch_bounds__(kBlock) void halo_tile_kernel(const T* __restrict__ X, uint64_t n,
                                                           const PartGrid* __restrict__ parts,
                                                           int P, KdTree tree, double marg,
                                                           uint32_t* __restrict__ tile_cnt,
                                                           uint32_t* __restrict__ ctrs,
                                                           uint32_t* __restrict__ sort_hist) {
    // the train's small counters (dup / root / core / border lists, big and
    // mid cells, cell pairs) and the record sort's digit histograms: zeroed
    // here, the first kernel of the train, instead of by fills
    if (blockIdx.x == 0) {
        if (threadIdx.x < kCtrs) ctrs[threadIdx.x] = 0;
        if (sort_hist)
            for (int i = threadIdx.x; i < 8 * rsort::kRadix; i += kBlock) sort_hist[i] = 0;
    }
    uint64_t idx[4];
    T v[4][D];
    unsigned long long m[4];
    uint32_t cnt[4];
    if constexpr (TREE) {
        __shared__ int32_t t_slot[kTreeSlots], t_axn[2 * kTreeSplits];
        __shared__ double t_bd[kTreeSplits];
        __shared__ NearLds nl;
        for (int k = threadIdx.x; k < tree.nslot; k += kBlock) t_slot[k] = tree.slot[k];
        for (int k = threadIdx.x; k < 2 * tree.ne; k += kBlock) t_axn[k] = tree.ax_new[k];
        for (int k = threadIdx.x; k < tree.ne; k += kBlock) t_bd[k] = tree.bound[k];
        if (threadIdx.x == 0) nl.n = 0;
        __syncthreads();
        int own[4];
        halo_points_tree<T, D>(X, n, parts, P, blockIdx.x, tree, t_slot, t_axn, t_bd, marg, nl, idx,
                               v, m, cnt, own);
    } else {
        halo_points<T, D, false>(X, n, parts, P, blockIdx.x, idx, v, m, cnt);
    }
    const uint32_t t = block_sum_u32(cnt[0] + cnt[1] + cnt[2] + cnt[3]);
    if (threadIdx.x == 0) tile_count_out(tile_cnt, t);
}

template <typename T, int D, typename K>
__device__ __forceinline__ void halo_record(const T (&tv)[D], const PartGrid& g, K& key) {
    double v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (double)tv[j];
    int64_t c[D];
    cell_of<D>(v, g, c);
    key = (K)(g.base + lin_of<D>(c, g));
}

// The grid fields a record key needs, per neighbourhood, staged in LDS: the
// lanes of a wave key their points in different neighbourhoods, and per-lane
// global loads of the grids cost more than the arithmetic.
// The linear cell index is accumulated in double: every term is an integer
// and the grid has fewer than 2^53 cells (checked on the host), so each fma
// is exact and equals the int64 form, with one conversion per key instead of
// one per axis (the halo write is VALU-issue bound).
template <int D>
struct KeyGrid {
    double lo[D], inv[D];
    double nc[D], top[D];   // cells per axis, and the last cell index
    uint64_t base;
};

template <typename T, int D, typename K>
__device__ __forceinline__ K key_of(const T (&tv)[D], const KeyGrid<D>& g) {
    double k = 0.0;
#pragma unroll
    for (int j = D - 1; j >= 0; --j) {
        double q = floor(((double)tv[j] - g.lo[j]) * g.inv[j]);
        q = fmin(fmax(q, 0.0), g.top[j]);
        k = fma(k, g.nc[j], q);
    }
    return (K)(g.base + (uint64_t)k);
}

// Records of a tile in (wave, step, lane, neighbourhood) order:
// deterministic.  Each point's first record (its lowest neighbourhood) is
// computed for all lanes at once and stored after the loop, so one step's
// stores are contiguous; the extra records of the few halo duplicates follow.
// (92 VGPRs, 5 waves/SIMD: capping it at 6 or 8 waves measured slower — C2
// halo 1.29 / 1.81 vs 1.22 ms, the cap spills the per-point state)
// Every record store is bounded by `cap` (the buffers' length): the
// single-pass form writes before it knows the total, and a tile past the
// capacity must not store (the host then reruns the two-pass form).
template <int D>
struct HaloLds {
    uint32_t ws[kBlock / 64];
    KeyGrid<D> kg[64];
    int32_t t_slot[kTreeSlots], t_axn[2 * kTreeSplits];
    double t_bd[kTreeSplits];
};

// the per-wave exclusive record offsets of the four steps; the wave's total
template <int Q>
__device__ __forceinline__ uint32_t wave_offsets(const uint32_t (&cnt)[Q], uint32_t (&ex)[Q]) {
    const int lane = threadIdx.x & 63;
    uint32_t wtot = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        uint32_t x = cnt[q];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= o) x += y;
        }
        ex[q] = wtot + x - cnt[q];
        wtot += (uint32_t)__shfl((int)x, 63, 64);
    }
    return wtot;
}

// stage the split tree and the key grids in LDS (MASK: P <= 64); returns
// whether the tree is read from LDS.  The caller synchronises after.
template <typename T, int D, bool MASK>
__device__ __forceinline__ bool halo_stage(HaloLds<D>& L, const PartGrid* __restrict__ parts,
                                           int P, const KdTree& tree) {
    const bool tree_lds = MASK && tree.nl && tree.nslot <= kTreeSlots && tree.ne <= kTreeSplits;
    if (tree_lds) {
        for (int k = threadIdx.x; k < tree.nslot; k += kBlock) L.t_slot[k] = tree.slot[k];
        for (int k = threadIdx.x; k < 2 * tree.ne; k += kBlock) L.t_axn[k] = tree.ax_new[k];
        for (int k = threadIdx.x; k < tree.ne; k += kBlock) L.t_bd[k] = tree.bound[k];
    }
    if constexpr (MASK) {
        for (int q = threadIdx.x; q < P; q += kBlock) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                L.kg[q].lo[j] = parts[q].lo[j];
                L.kg[q].inv[j] = parts[q].inv[j];
                L.kg[q].nc[j] = (double)parts[q].nc[j];
                L.kg[q].top[j] = (double)(parts[q].nc[j] - 1);
            }
            L.kg[q].base = parts[q].base;
        }
    }
    return tree_lds;
}

// write the records of one tile's points from record offset wbase (this
// wave's first record); stores at or past cap are dropped
// PRE: the owners are already known (own_in, halo_points_tree)
template <typename T, int D, typename K, bool MASK, bool PRE = false>
__device__ __forceinline__ void halo_emit(const HaloLds<D>& L, const PartGrid* __restrict__ parts,
                                          int P, const int32_t* __restrict__ owner,
                                          const KdTree& tree, bool tree_lds, uint64_t n,
                                          const uint64_t (&idx)[4], const T (&v)[4][D],
                                          const unsigned long long (&m)[4],
                                          const uint32_t (&cnt)[4], const uint32_t (&ex)[4],
                                          uint64_t wbase, uint64_t cap, K* __restrict__ keys,
                                          uint32_t* __restrict__ vals, const int (&own_in)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!cnt[q]) continue;
        if (!PD_OK(idx[q] < n, 4, idx[q])) continue;
        // P == 1: neighbourhood 0
        const int own = PRE      ? own_in[q]
                        : owner  ? owner[idx[q]]
                        : !tree.nl ? 0
                        : tree_lds ? tree_owner<T, D>(tree, L.t_slot, L.t_axn, L.t_bd, v[q])
                                   : tree_owner<T, D>(tree, tree.slot, tree.ax_new, tree.bound, v[q]);
        (void)PD_OK(own >= 0 && own < P, 5, (uint32_t)own);
        const uint32_t tag = (uint32_t)idx[q] | (cnt[q] >= 2 ? kDupBit : 0u);
        uint64_t o = wbase + ex[q];
        if constexpr (MASK) {
            unsigned long long mm = m[q];
            do {
                const int Lb = __ffsll(mm) - 1;
                mm &= mm - 1;
                const K key = key_of<T, D, K>(v[q], L.kg[Lb]);
                if (o < cap) {
                    keys[o] = key;
                    vals[o] = tag | (own == Lb ? kOwnerBit : 0u);
                }
                ++o;
            } while (mm);
        } else {
            for (int Lb = 0; Lb < P; ++Lb) {
                const PartGrid& g = parts[Lb];
                if (!in_box_t<T, D>(v[q], g)) continue;
                K key;
                halo_record<T, D, K>(v[q], g, key);
                if (o < cap) {
                    keys[o] = key;
                    vals[o] = tag | (own == Lb ? kOwnerBit : 0u);
                }
                ++o;
            }
        }
        (void)PD_OK(o - (wbase + ex[q]) == cnt[q], 6, o);
    }
}

template <typename T, int D, typename K, bool MASK, bool TREE = false>
__global__ __launch_bounds__(kBlock) void halo_write_kernel(
    const T* __restrict__ X, uint64_t n, const PartGrid* __restrict__ parts, int P,
    const int32_t* __restrict__ owner, KdTree tree, double marg,
    const uint64_t* __restrict__ tile_off, uint64_t cap, K* __restrict__ keys,
    uint32_t* __restrict__ vals) {
    static_assert(!TREE || MASK, "the near-plane path builds masks");
    uint64_t idx[4];
    T v[4][D];
    unsigned long long m[4];
    uint32_t cnt[4], ex[4];
    int own[4] = {0, 0, 0, 0};
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ HaloLds<D> L;
    __shared__ std::conditional_t<TREE, NearLds, char> nl;
    bool tree_lds;
    if constexpr (TREE) {
        tree_lds = halo_stage<T, D, MASK>(L, parts, P, tree);   // (true by the host's choice)
        if (threadIdx.x == 0) nl.n = 0;
        __syncthreads();
        halo_points_tree<T, D>(X, n, parts, P, blockIdx.x, tree, L.t_slot, L.t_axn, L.t_bd, marg,
                               nl, idx, v, m, cnt, own);
    } else {
        halo_points<T, D, MASK>(X, n, parts, P, blockIdx.x, idx, v, m, cnt);
        tree_lds = halo_stage<T, D, MASK>(L, parts, P, tree);
    }
    const uint32_t wtot = wave_offsets<4>(cnt, ex);
    if (lane == 0) L.ws[w] = wtot;
    __syncthreads();
    uint64_t wbase = tile_off[blockIdx.x];
#pragma unroll
    for (int u = 0; u < kBlock / 64; ++u) wbase += u < w ? L.ws[u] : 0u;
    halo_emit<T, D, K, MASK, TREE>(L, parts, P, owner, tree, tree_lds, n, idx, v, m, cnt, ex, wbase,
                                   cap, keys, vals, own);
}

// Single-pass halo (PD_OPT_HALO_PASSES = 1): each tile counts its records,
// learns the records of the tiles before it by decoupled look-back, and
// writes them — one read of the points instead of two, no scan, at the price
// of buffers sized before the total is known (cap; the host reruns the
// two-pass form when the total passes it).  Tiles take their index from a
// ticket (atomicAdd - tick0), so the tiles a tile waits for were dispatched
// before it: forward progress without assuming a dispatch order.  Look-back
// words: tag << 32 | records (tag 2 epoch + 1: the tile's own count, 2 epoch
// + 2: inclusive of every tile before; older epochs' tags read as
// unpublished); counts saturate at 2^32 - 1, far past any capacity.  The
// last tile writes the total (64-bit) for the host.  Tile 0 zeroes the
// train's counters and the sort histograms (the tile kernel's job in the
// two-pass form).
template <typename T, int D, typename K, bool MASK>
__global__ __launch_bounds__(kBlock) void halo1_kernel(
    const T* __restrict__ X, uint64_t n, const PartGrid* __restrict__ parts, int P,
    const int32_t* __restrict__ owner, KdTree tree, uint64_t cap, K* __restrict__ keys,
    uint32_t* __restrict__ vals, uint64_t* __restrict__ look, uint32_t epoch,
    unsigned long long* __restrict__ ticket, unsigned long long tick0, uint32_t ntiles,
    unsigned long long* __restrict__ total, uint32_t* __restrict__ ctrs,
    uint32_t* __restrict__ sort_hist) {
    __shared__ HaloLds<D> L;
    __shared__ uint32_t s_tile;
    __shared__ unsigned long long s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tick0);
    const bool tree_lds = halo_stage<T, D, MASK>(L, parts, P, tree);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (!PD_OK(tile < ntiles, 7, tile)) return;   // (a ticket past the grid: never)
    if (tile == 0) {
        if (threadIdx.x < kCtrs) ctrs[threadIdx.x] = 0;
        if (sort_hist)
            for (int i = threadIdx.x; i < 8 * rsort::kRadix; i += kBlock) sort_hist[i] = 0;
    }
    uint64_t idx[4];
    T v[4][D];
    unsigned long long m[4];
    uint32_t cnt[4], ex[4];
    halo_points<T, D, MASK>(X, n, parts, P, tile, idx, v, m, cnt);
    const uint32_t wtot = wave_offsets<4>(cnt, ex);
    if (lane == 0) L.ws[w] = wtot;
    __syncthreads();
    if (w == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int u = 0; u < kBlock / 64; ++u) t += L.ws[u];
        const uint32_t agg = 2u * epoch + 1u, inc = 2u * epoch + 2u;
        if (lane == 0) rsort::st_lb(look + tile, ((uint64_t)(tile == 0 ? inc : agg) << 32) | t);
        uint64_t excl = 0;
        // look back 64 tiles at a time: lane l reads tile (front - l); the
        // nearest inclusive word ends the walk, every word up to it must be
        // published (else spin)
        for (int64_t front = (int64_t)tile - 1; front >= 0;) {
            const int64_t tt = front - lane;
            const uint64_t wv = tt >= 0 ? rsort::ld_lb(look + tt) : ((uint64_t)inc << 32);
            const uint32_t tag = (uint32_t)(wv >> 32);
            const unsigned long long pub = __ballot(tag == agg || tag == inc);
            const unsigned long long incl = __ballot(tag == inc);
            const int stop = incl ? __ffsll((long long)incl) - 1 : 63;
            const unsigned long long need = stop == 63 ? ~0ull : ((2ull << stop) - 1ull);
            if ((pub & need) != need) continue;   // a tile up to `stop` not published yet
            uint64_t x = lane <= stop ? (uint32_t)wv : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += (uint64_t)__shfl_xor((long long)x, o, 64);
            excl += x;
            if (incl) break;
            front -= 64;
        }
        if (lane == 0) {
            const uint64_t it = excl + t;
            if (tile > 0) rsort::st_lb(look + tile, ((uint64_t)inc << 32) | (it < 0xFFFFFFFFull ? it : 0xFFFFFFFFull));
            if (tile == ntiles - 1) *total = it;
            s_base = excl;
        }
    }
    __syncthreads();
    uint64_t wbase = s_base;
#pragma unroll
    for (int u = 0; u < kBlock / 64; ++u) wbase += u < w ? L.ws[u] : 0u;
    const int own0[4] = {0, 0, 0, 0};
    halo_emit<T, D, K, MASK>(L, parts, P, owner, tree, tree_lds, n, idx, v, m, cnt, ex, wbase, cap,
                             keys, vals, own0);
}

// Coordinates into key order (padded rows); also lists the records of halo
// points that live in several neighbourhoods (the merge only touches those)
// and starts those points' merge representative (rep) at kNone.
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void gather_kernel(const T* __restrict__ X, uint64_t R,
                                                        const uint32_t* __restrict__ vals,
                                                        T* __restrict__ Xs,
                                                        uint32_t* __restrict__ dup_list,
                                                        uint32_t* __restrict__ dup_count,
                                                        uint32_t* __restrict__ rep) {
    const uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t v = r < R ? vals[r] : 0u;
    if (r < R) {
        const uint64_t i = v & kIdMask;
        constexpr int S = Stride<D>::v;
#pragma unroll
        for (int j = 0; j < S; ++j) Xs[r * S + j] = j < D ? X[i * D + j] : T(0);
        if (rep && (v & kDupBit)) rep[i] = kNone;
    }
    wave_append(dup_list, dup_count, r < R && (v & kDupBit), (uint32_t)r);
}

template <typename K>
__global__ void part_start_kernel(const K* __restrict__ keys, uint64_t R,
                                  const PartGrid* __restrict__ parts, int P,
                                  uint32_t* __restrict__ ps) {
    const int L = blockIdx.x * blockDim.x + threadIdx.x;
    if (L > P) return;
    if (L == P) {
        ps[P] = (uint32_t)R;
        return;
    }
    const uint64_t b = parts[L].base;
    uint64_t lo = 0, hi = R;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if ((uint64_t)keys[mid] < b)
            lo = mid + 1;
        else
            hi = mid;
    }
    ps[L] = (uint32_t)lo;
}

// Cell starts, two ordered passes over the sorted keys (four records per
// lane): a record whose key differs from its predecessor's starts a cell;
// cell_tile_kernel counts each tile's starts, the host scans the counts, and
// cell_write_kernel numbers the cells (tile offset + block scan), so
// cstart[cell] = record.
template <typename K>
__device__ __forceinline__ uint32_t cell_starts4(const K* __restrict__ keys, uint64_t R,
                                                 uint64_t r0, uint32_t (&st)[4],
                                                 uint64_t (&kv)[4]) {
    uint32_t c = 0;
    uint64_t prev = r0 > 0 && r0 < R ? (uint64_t)keys[r0 - 1] : ~0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t r = r0 + q;
        st[q] = 0;
        kv[q] = 0;
        if (r < R) {
            const uint64_t k = (uint64_t)keys[r];
            st[q] = (r == 0 || k != prev) ? 1u : 0u;
            kv[q] = k;
            prev = k;
        }
        c += st[q];
    }
    return c;
}

template <typename K>
__global__ __launch_bounds__(kBlock) void cell_tile_kernel(const K* __restrict__ keys, uint64_t R,
                                                           uint32_t* __restrict__ tile_cnt) {
    uint32_t st[4];
    uint64_t kv[4];
    const uint64_t r0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    const uint32_t t = block_sum_u32(cell_starts4<K>(keys, R, r0, st, kv));
    if (threadIdx.x == 0) tile_count_out(tile_cnt, t);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void cell_write_kernel(const K* __restrict__ keys, uint64_t R,
                                                            const uint64_t* __restrict__ tile_off,
                                                            uint32_t* __restrict__ cstart,
                                                            K* __restrict__ ckeys,
                                                            uint32_t* __restrict__ ncells) {
    uint32_t st[4];
    uint64_t kv[4];
    const uint64_t r0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    uint32_t btot;
    const uint32_t c = cell_starts4<K>(keys, R, r0, st, kv);
    uint32_t cid = (uint32_t)tile_off[blockIdx.x] + block_excl_scan(c, btot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (st[q]) {
            cstart[cid] = (uint32_t)(r0 + q);
            ckeys[cid] = (K)kv[q];   // the cell's key, dense: the directory passes read it in order
        }
        cid += st[q];
        if (r0 + q == R - 1) {
            cstart[cid] = (uint32_t)R;
            *ncells = cid;
        }
    }
}

// Wave shuffles of a directory word / page id: 32-bit when the ids fit (one
// ds_bpermute per step instead of two; W32 below — C2's 32-bit keys always,
// C4's 37-bit ones too), else 64-bit.
template <typename WT>
__device__ __forceinline__ WT shfl_up_w(WT x, int o) {
    if constexpr (sizeof(WT) == 4) return (WT)__shfl_up((int)x, o, 64);
    else return (WT)__shfl_up((long long)x, o, 64);
}
template <typename WT>
__device__ __forceinline__ WT shfl_down_w(WT x, int o) {
    if constexpr (sizeof(WT) == 4) return (WT)__shfl_down((int)x, o, 64);
    else return (WT)__shfl_down((long long)x, o, 64);
}
template <typename WT>
__device__ __forceinline__ WT shfl_w(WT x, int l) {
    if constexpr (sizeof(WT) == 4) return (WT)__shfl((int)x, l, 64);
    else return (WT)__shfl((long long)x, l, 64);
}

// Directory occupancy bits, one lane per cell: the cells are sorted, so the
// lanes of one directory word are contiguous and a segmented OR-scan across
// the wave (Hillis-Steele; equal words at distance o imply equal words in
// between) leaves each word's bits in its last lane, which adds them with
// one atomicOr (a word can continue into the neighbouring waves).
// SH = 6: the paged directory's page masks (one bit per occupied word of
// the page; the units are then words, k >> 6).
template <typename K, int SH, bool W32>
__global__ __launch_bounds__(kBlock) void dir_bits_kernel(const K* __restrict__ ckeys,
                                                          const uint32_t* __restrict__ ncells,
                                                          uint4* __restrict__ dir) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t nc = *ncells;
    // the grid covers the records (the cell count stays on the device): the
    // waves past the last cell (C4: 2/3 of them) leave before the scan
    if (c - (uint32_t)(threadIdx.x & 63) >= nc) return;
    const bool in = c < nc;
    using WT = std::conditional_t<W32, uint32_t, uint64_t>;
    const uint64_t k = in ? ((uint64_t)ckeys[c] >> SH) : ~0ull;
    const WT word = (WT)(k >> 6);   // W32: ids < 2^31, the sentinel 0xFFFFFFFF
    unsigned long long v = in ? (1ull << (k & 63)) : 0ull;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const WT wo = shfl_up_w(word, o);
        const unsigned long long vo = (unsigned long long)__shfl_up((long long)v, o, 64);
        if (lane >= o && wo == word) v |= vo;
    }
    const WT wn = shfl_down_w(word, 1);
    const bool last = lane == 63 || wn != word;
    if (in && last) atomicOr(reinterpret_cast<unsigned long long*>(dir + (uint64_t)word), v);
}

// Paged directory, the occupied words (pages already hold their masks and
// word prefixes): each word is written whole, by the lane of its first cell —
// bits = a segmented suffix OR of the word's cells across the wave (a word
// whose cells run past the wave's last lane continues with a serial walk of
// at most 63 cells), z = that cell's index (the occupied cells before the
// word).  The last cell also writes the terminal word {0, 0, ncells}.
template <typename K, bool W32>
__global__ __launch_bounds__(kBlock) void word_write_kernel(const K* __restrict__ ckeys,
                                                            const uint32_t* __restrict__ ncells,
                                                            const uint4* __restrict__ pages,
                                                            uint4* __restrict__ words) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t nc = *ncells;
    if (c - (uint32_t)(threadIdx.x & 63) >= nc) return;   // a wave past the last cell
    const bool in = c < nc;
    using WT = std::conditional_t<W32, uint32_t, uint64_t>;
    const uint64_t k = in ? (uint64_t)ckeys[c] : ~0ull;
    const WT word = (WT)(k >> 6);   // W32: ids < 2^31, the sentinel 0xFFFFFFFF
    unsigned long long v = in ? (1ull << (k & 63)) : 0ull;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const WT wo = shfl_down_w(word, o);
        const unsigned long long vo = (unsigned long long)__shfl_down((long long)v, o, 64);
        if (lane + o < 64 && wo == word) v |= vo;
    }
    const WT wp = shfl_up_w(word, 1);
    const WT w63 = shfl_w(word, 63);
    // Only the wave's last word can continue into the next wave (a word has
    // <= 64 cells, so it ends there): the whole wave reads the next 64 cells
    // and ORs their bits (a serial walk of up to 63 cells by the word's first
    // lane held its wave on C4's dense rows: word_write 6.8 ms).
    const uint32_t cb = c - (uint32_t)lane;   // the wave's first cell (uniform)
    unsigned long long vx = 0;
    if (cb + 64 < nc && (WT)((uint64_t)ckeys[cb + 64] >> 6) == w63) {   // uniform
        const uint32_t c2 = cb + 64 + (uint32_t)lane;
        const uint64_t k2 = c2 < nc ? (uint64_t)ckeys[c2] : ~0ull;
        vx = c2 < nc && (WT)(k2 >> 6) == w63 ? 1ull << (k2 & 63) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vx |= (unsigned long long)__shfl_xor((long long)vx, o, 64);
    }
    if (!in) return;
    bool first = c == 0;
    if (!first) first = lane ? wp != word : (WT)((uint64_t)ckeys[c - 1] >> 6) != word;
    bool occ;
    const uint64_t slot = page_slot(pages[(uint64_t)word >> 6], (uint64_t)word, occ);
    if (first) {
        if (w63 == word) v |= vx;   // the word continues past this wave
        words[slot] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), c, 0u);
    }
    if (c == nc - 1) words[slot + 1] = make_uint4(0u, 0u, nc, 0u);
}

// Directory ranks dir[w].z = occupied cells in words < w: per-tile popcount
// sums, a host-side scan of the tile sums, then the block-scan write (four
// words per lane).
__device__ __forceinline__ uint32_t dir_popc4(const uint4* __restrict__ dir, uint64_t W,
                                              uint64_t w0, uint32_t (&pc)[4]) {
    uint32_t t = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        pc[q] = 0;
        if (w0 + q < W) {
            const uint4 d = dir[w0 + q];
            pc[q] = (uint32_t)__popc(d.x) + (uint32_t)__popc(d.y);
        }
        t += pc[q];
    }
    return t;
}

__global__ __launch_bounds__(kBlock) void dir_tile_kernel(const uint4* __restrict__ dir, uint64_t W,
                                                          uint32_t* __restrict__ tile_cnt) {
    uint32_t pc[4];
    const uint32_t t =
        block_sum_u32(dir_popc4(dir, W, ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4, pc));
    if (threadIdx.x == 0) tile_count_out(tile_cnt, t);
}

__global__ __launch_bounds__(kBlock) void dir_write_kernel(uint4* __restrict__ dir, uint64_t W,
                                                           const uint64_t* __restrict__ tile_off) {
    uint32_t pc[4], btot;
    const uint64_t w0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    uint32_t z = (uint32_t)tile_off[blockIdx.x] + block_excl_scan(dir_popc4(dir, W, w0, pc), btot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (w0 + q < W) dir[w0 + q].z = z;
        z += pc[q];
    }
}

// Initial forest.  parent doubles as the core flag: kNone marks a non-core
// record, so an edge test costs one load.
// The count pass keeps the two smallest neighbours it saw (mn2[r]): the
// parent is the smaller of them that is core and below r — two candidates
// leave about half the trees of one (tools/init_forest_study.py).
constexpr int kSubTiles = 4;   // init_kernel / roots_kernel: record tiles per block
#ifndef PD_ROOTS_SUB
#define PD_ROOTS_SUB 4
#endif
constexpr int kRootSub = PD_ROOTS_SUB;   // roots_kernel: record tiles per block
constexpr int kRootLists = 64, kRootCntStride = 32;   // root lists, one 128-B counter line each
// Also starts the per-record component keys (gmin) and the directory-word
// roots (wroot, W words) at kNone — the fills they needed before.
__global__ __launch_bounds__(kBlock) void init_kernel(uint32_t R, const uint8_t* __restrict__ core,
                                                      const uint32_t* __restrict__ mn,
                                                      int use_mn, uint32_t* __restrict__ par,
                                                      uint32_t* __restrict__ gmin,
                                                      uint32_t* __restrict__ wroot, uint64_t W,
                                                      uint32_t* __restrict__ kbits, uint64_t NW) {
    // kSubTiles record tiles of kBlock per block (fewer workgroups for the
    // light per-record passes over 1e9 records)
#pragma unroll
    for (int q = 0; q < kSubTiles; ++q) {
        const uint64_t r64 = ((uint64_t)blockIdx.x * kSubTiles + q) * kBlock + threadIdx.x;
        if (r64 < W) wroot[r64] = kNone;
        if (r64 < NW) kbits[r64] = 0u;   // the component-key bitmap (rank_roots)
        if (r64 >= R) continue;
        const uint32_t r = (uint32_t)r64;
        gmin[r] = kNone;
        uint32_t p = kNone;
        if (core[r] & 1) {
            p = r;
            if (use_mn) {
                const uint2 m = reinterpret_cast<const uint2*>(mn)[r];
                if (m.x < r && (core[m.x] & 1))
                    p = m.x;
                else if (m.y < r && (core[m.y] & 1))
                    p = m.y;
            }
        }
        par[r] = p;
    }
}

struct LinkStats {
    uint32_t cand = 0, hit = 0, core = 0, same = 0, find_same = 0, unions = 0;
};

// A point's copies in several neighbourhoods (the dup list): link every core
// copy to one representative (the smallest record), gluing the
// neighbourhoods' clusters.
__global__ __launch_bounds__(kBlock) void rep_kernel(const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ count,
                                                     const uint32_t* __restrict__ vals,
                                                     const uint32_t* __restrict__ par,
                                                     uint32_t* __restrict__ rep) {
    const uint32_t nl = *count;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nl; i += gridDim.x * kBlock) {
        const uint32_t r = list[i];
        if (par[r] != kNone) atomicMin(rep + (vals[r] & kIdMask), r);
    }
}

__global__ __launch_bounds__(kBlock) void merge_kernel(const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ count,
                                                       const uint32_t* __restrict__ vals,
                                                       const uint32_t* __restrict__ rep,
                                                       uint32_t* __restrict__ par) {
    // The copies of a cluster's boundary points all join the same two trees:
    // thousands of lanes racing one CAS on the same root (C2: 0.56 ms for
    // 2.2M listed records).  Each lane finds its pair of roots first and
    // skips the union when the lane before holds the same pair (the list is
    // in record order, so a wave's neighbours mostly do).
    const uint32_t nl = *count;
    const int lane = threadIdx.x & 63;
    for (uint32_t b0 = blockIdx.x * kBlock; b0 < nl; b0 += gridDim.x * kBlock) {   // uniform
        const uint32_t i = b0 + threadIdx.x;
        uint32_t ra = kNone, rb = kNone;
        if (i < nl) {
            const uint32_t r = list[i];
            if (ld_rlx(par + r) != kNone) {   // core (par is the core flag)
                const uint32_t q = rep[vals[r] & kIdMask];
                if (q != r) {
                    ra = uf_find(par, r);
                    rb = uf_find(par, q);
                    if (ra > rb) {
                        const uint32_t t = ra;
                        ra = rb;
                        rb = t;
                    }
                    if (ra == rb) ra = rb = kNone;
                }
            }
        }
        const uint32_t pa = (uint32_t)__shfl_up((int)ra, 1, 64);
        const uint32_t pb = (uint32_t)__shfl_up((int)rb, 1, 64);
        const bool same = lane > 0 && pa == ra && pb == rb;
        if (ra != kNone && !same) uf_unite(par, ra, rb);
    }
}

// Roots: every core record's parent becomes its root (flatten) and each root
// gets the smallest (global) point id of its component (wave-aggregated
// atomicMin); with stats, the count of core records.
__global__ __launch_bounds__(kBlock) void roots_kernel(uint32_t R, const uint32_t* __restrict__ vals,
                                                       const uint32_t* __restrict__ gid,
                                                       uint32_t* __restrict__ par,
                                                       uint32_t* __restrict__ gmin,
                                                       uint32_t* __restrict__ rlist,
                                                       uint32_t* __restrict__ rcnt, uint32_t seg,
                                                       uint32_t* __restrict__ counts, int stats) {
    // kRootSub record tiles of kBlock per block; a lane's kRootSub records
    // are read together (parents, first parent step, point ids) and their
    // minima folded per root in the lane before the wave-aggregated atomics:
    // one aggregation per distinct root of the lane (usually one), not one
    // per record
    uint32_t ncore = 0;
    uint32_t rr[kRootSub], x0[kRootSub], root[kRootSub], pt[kRootSub];
    bool core[kRootSub];
#pragma unroll
    for (int q = 0; q < kRootSub; ++q) {
        rr[q] = (blockIdx.x * kRootSub + q) * kBlock + threadIdx.x;
        x0[q] = rr[q] < R ? par[rr[q]] : kNone;
        core[q] = x0[q] != kNone;
    }
#pragma unroll
    for (int q = 0; q < kRootSub; ++q) {
        root[q] = core[q] ? par[x0[q]] : 0u;   // the first step, all four in flight
        pt[q] = core[q] ? (vals[rr[q]] & kIdMask) : kNone;
    }
    // longer chains (a tree the verify / pair / merge unions hung under
    // another after the cell roots flattened it): the lane's kRootSub walks
    // advance together, one round of loads in flight per step, instead of
    // one walk after another
    bool more[kRootSub];
#pragma unroll
    for (int q = 0; q < kRootSub; ++q) more[q] = core[q] && root[q] != x0[q];
    while (true) {
        bool any = false;
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) any |= more[q];
        if (!__any(any)) break;
        uint32_t p[kRootSub];
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) p[q] = more[q] ? par[root[q]] : root[q];
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) {
            if (p[q] == root[q]) more[q] = false;
            root[q] = p[q];
        }
    }
#pragma unroll
    for (int q = 0; q < kRootSub; ++q) {
        if (!core[q]) continue;
        if (root[q] != x0[q]) par[rr[q]] = root[q];
        if (gid) pt[q] = gid[pt[q]];
        ncore += 1u;
    }
    bool left[kRootSub];
#pragma unroll
    for (int q = 0; q < kRootSub; ++q) left[q] = core[q];
    while (true) {
        // the lane's first remaining root and the smallest point id under it
        bool have = false;
        uint32_t key = 0, m = kNone;
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) {
            if (left[q] && !have) {
                have = true;
                key = root[q];
            }
        }
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) {
            if (left[q] && root[q] == key) {
                m = pt[q] < m ? pt[q] : m;
                left[q] = false;
            }
        }
        if (!__any(have)) break;
        wave_atomic_min(gmin, have, key, m);
    }
    // the roots, listed (single device) into kRootLists lists, one
    // reservation per block: one list counter taking an append per wave
    // with a root (96K on C2) serialised at its L2 channel — 0.8 of the
    // kernel's 1.06 ms; block b appends to list b % kRootLists, whose blocks
    // hold at most seg records
    if (rlist) {
        __shared__ uint32_t s_rbase;
        uint32_t nr = 0;
#pragma unroll
        for (int q = 0; q < kRootSub; ++q) nr += core[q] && root[q] == rr[q] ? 1u : 0u;
        uint32_t tot;
        uint32_t off = block_excl_scan(nr, tot);
        const uint32_t k = blockIdx.x % kRootLists;
        if (threadIdx.x == 0 && tot) s_rbase = atomicAdd(rcnt + k * kRootCntStride, tot);
        __syncthreads();
        if (tot) {
            uint32_t* out = rlist + (size_t)k * seg + s_rbase;
#pragma unroll
            for (int q = 0; q < kRootSub; ++q)
                if (core[q] && root[q] == rr[q]) out[off++] = rr[q];
        }
    }
    if (stats) {   // core records (sweep statistics): one atomic per block
        const uint32_t c = block_sum_u32(ncore);
        if (threadIdx.x == 0 && c) atomicAdd(counts + 1, c);
    }
}

// Single device: each component's key becomes its label — the rank of its
// smallest core point id among all components (sklearn's numbering).  The
// keys are distinct point ids < n, so the rank is a bitmap population count:
// mark each component's key in an n-bit map, scan the words' popcounts, and
// a root's label is its word's prefix plus the bits below it in the word —
// no sort, and the component count stays on the device (no host sync).
// The lists' slots: list k holds rcnt[k * kRootCntStride] roots from slot
// k * seg; block b of a grid of kRootLists * m blocks walks list b % kRootLists.
__global__ __launch_bounds__(kBlock) void root_mark_kernel(const uint32_t* __restrict__ rlist,
                                                           const uint32_t* __restrict__ rcnt,
                                                           uint32_t seg,
                                                           const uint32_t* __restrict__ gmin,
                                                           uint32_t* __restrict__ kbits) {
    const uint32_t k = blockIdx.x % kRootLists, m = gridDim.x / kRootLists;
    const uint32_t c = rcnt[k * kRootCntStride];
    const uint32_t* l = rlist + (size_t)k * seg;
    for (uint32_t i = (blockIdx.x / kRootLists) * kBlock + threadIdx.x; i < c; i += m * kBlock) {
        const uint32_t g = gmin[l[i]];
        atomicOr(kbits + (g >> 5), 1u << (g & 31));
    }
}

// ... and the component count (the map's population: one bit per component
// key) into *count, read with the train's last copy back.
__global__ __launch_bounds__(kBlock) void root_rank_kernel(const uint32_t* __restrict__ rlist,
                                                           const uint32_t* __restrict__ rcnt,
                                                           uint32_t seg,
                                                           const uint32_t* __restrict__ kbits,
                                                           const uint32_t* __restrict__ kpre,
                                                           uint64_t NW, uint32_t* __restrict__ gmin,
                                                           uint32_t* __restrict__ count) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
        *count = kpre[NW - 1] + (uint32_t)__popc(kbits[NW - 1]);
    const uint32_t k = blockIdx.x % kRootLists, m = gridDim.x / kRootLists;
    const uint32_t c = rcnt[k * kRootCntStride];
    const uint32_t* l = rlist + (size_t)k * seg;
    for (uint32_t i = (blockIdx.x / kRootLists) * kBlock + threadIdx.x; i < c; i += m * kBlock) {
        const uint32_t r = l[i], g = gmin[r];
        gmin[r] = kpre[g >> 5] + (uint32_t)__popc(kbits[g >> 5] & ((1u << (g & 31)) - 1u));
    }
}

struct PopcOp {
    __device__ uint32_t operator()(uint32_t w) const { return (uint32_t)__popc(w); }
};

// Sharded train, phase A exports: (global id, local component key) of every
// core record whose point was also routed to another device.
struct IsExport {
    const uint8_t* core;
    const uint32_t* vals;
    const uint8_t* xr;
    __device__ bool operator()(uint32_t r) const {
        return (core[r] & 1) && xr[vals[r] & kIdMask];
    }
};

__global__ __launch_bounds__(kBlock) void export_kernel(uint32_t NL,
                                                        const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ par,
                                                        const uint32_t* __restrict__ gmin,
                                                        const uint32_t* __restrict__ gid,
                                                        uint32_t* __restrict__ out_gid,
                                                        uint32_t* __restrict__ out_key) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= NL) return;
    const uint32_t r = list[i];
    const uint32_t pt = vals[r] & kIdMask;
    out_gid[i] = gid ? gid[pt] : pt;
    out_key[i] = gmin[par[r]];
}

// Phase B: replace each local component's key by its global key (ids in no
// export keep their own: the component never left this device).  Every key
// a record of this device can take is such a root's; with the core flag in
// the keys (core_mask, PD_OPT_SHARD_CORE_BIT) a key with that bit already set
// would be read back as a core flag, so it raises *err instead.
__global__ __launch_bounds__(kBlock) void remap_kernel(uint32_t R, const uint8_t* __restrict__ core,
                                                       const uint32_t* __restrict__ par,
                                                       const uint32_t* __restrict__ map_ids,
                                                       const uint32_t* __restrict__ map_keys,
                                                       uint32_t n_map, uint32_t core_mask,
                                                       uint32_t* __restrict__ gmin,
                                                       uint32_t* __restrict__ err) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= R || !(core[r] & 1) || par[r] != r) return;
    uint32_t k = gmin[r];
    uint32_t lo = 0, hi = n_map;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (map_ids[mid] < k)
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo < n_map && map_ids[lo] == k) {
        k = map_keys[lo];
        gmin[r] = k;
    }
    if (k & core_mask) atomicOr(err, 1u);
}

// Owner records: publish core flag / count, and the cluster key of core
// points (their component's smallest core point).  core_mask (single device,
// ids < 2^30: bit 30; sharded phase B with global ids < 2^31: bit 31): the
// core flag rides in the key instead of a byte scattered to core_out — the
// label pass (split_core_kernel) writes the core mask coalesced.
constexpr uint32_t kKeyCoreBit = 0x40000000u;
constexpr int kOwnPer = 4;                    // owner_kernel / border_list_kernel records per thread
constexpr uint32_t kOwnTile = kBlock * kOwnPer;

__global__ __launch_bounds__(kBlock) void owner_kernel(uint32_t R, const uint32_t* __restrict__ vals,
                                                       const uint8_t* __restrict__ core,
                                                       const uint32_t* __restrict__ par,
                                                       const uint32_t* __restrict__ gmin,
                                                       const uint32_t* __restrict__ cnt_rec,
                                                       const uint2* __restrict__ mn,
                                                       uint32_t core_mask,
                                                       uint32_t* __restrict__ key_out,
                                                       uint8_t* __restrict__ core_out,
                                                       uint32_t* __restrict__ cnt_out,
                                                       uint32_t* __restrict__ tile_cnt,
                                                       uint2* __restrict__ recs) {
    // kOwnPer consecutive records per thread (a tile of kOwnTile records per
    // block: a quarter of the workgroups of one record per thread, which
    // dominated these light passes over C4's 1e9 records)
    // (the thread's four values / flags in one 16-B / 4-B load each, and the
    // pairs staged in LDS and written out as whole 16-B runs: stored one
    // record per lane at a 32-B stride, the pairs' partial sectors reached
    // HBM separately — 3.1 GB written per C2 launch for 0.8 GB of pairs)
    __shared__ uint2 s_rec[kOwnTile];
    const uint32_t r0 = (blockIdx.x * kBlock + threadIdx.x) * kOwnPer;
    uint32_t vq[kOwnPer];
    uint8_t cq[kOwnPer];
    if (r0 + kOwnPer <= R && !((uintptr_t)vals & 15)) {
        const uint4 v4 = *reinterpret_cast<const uint4*>(vals + r0);
        const uint32_t c4 = *reinterpret_cast<const uint32_t*>(core + r0);
        vq[0] = v4.x, vq[1] = v4.y, vq[2] = v4.z, vq[3] = v4.w;
#pragma unroll
        for (int q = 0; q < kOwnPer; ++q) cq[q] = (uint8_t)(c4 >> (8 * q));
    } else {
#pragma unroll
        for (int q = 0; q < kOwnPer; ++q) {
            vq[q] = r0 + q < R ? vals[r0 + q] : 0u;
            cq[q] = r0 + q < R ? core[r0 + q] : 0;
        }
    }
    uint32_t nb = 0;
#pragma unroll
    for (int q = 0; q < kOwnPer; ++q) {
        const uint32_t r = r0 + q;
        const uint32_t v = vq[q];
        const bool own = r < R && (v & kOwnerBit);
        const uint8_t fl = own ? cq[q] : 0;
        // the record's key: core -> its component's; a border record with a
        // single neighbour (bit 2) -> that neighbour's if it is core (the
        // border sweep's smallest core key, over one candidate); else none
        uint32_t key = kNone;
        if (fl & 1) {
            key = gmin[par[r]] | core_mask;
        } else if ((fl & 7) == 6 && mn) {
            const uint2 m = mn[r];
            const uint32_t j = m.x == r ? m.y : m.x;
            const uint32_t pj = par[j];
            key = pj != kNone ? gmin[pj] : kNone;
        }
        if (recs)   // bucketed labels: the pair in record order
            s_rec[threadIdx.x * kOwnPer + q] = make_uint2(own ? v & kIdMask : kNone, key);
        if (own) {
            const uint32_t pt = v & kIdMask;
            if (core_out && !core_mask) core_out[pt] = fl & 1;
            if (cnt_out) cnt_out[pt] = cnt_rec[r];
            // (noise and unattached border points keep key_out's kNone fill:
            // writing kNone here instead measured 1.67 -> 2.11 ms on C2, the
            // extra scattered sectors cost more than the 55 us fill)
            if (key != kNone && key_out) key_out[pt] = key;
        }
        // the rest of the border candidates go to the sweep
        nb += own && (fl & 3) == 2 && !((fl & 4) && mn) ? 1u : 0u;
    }
    if (recs) {
        __syncthreads();
        const uint32_t base = blockIdx.x * kOwnTile;
        for (uint32_t i = threadIdx.x; i < kOwnTile / 2; i += kBlock) {
            const uint32_t r = base + 2 * i;
            if (r + 1 < R)
                *reinterpret_cast<uint4*>(recs + r) =
                    make_uint4(s_rec[2 * i].x, s_rec[2 * i].y, s_rec[2 * i + 1].x, s_rec[2 * i + 1].y);
            else if (r < R)
                recs[r] = s_rec[2 * i];
        }
    }
    // border candidates (owner record, not core, has a neighbour) per tile;
    // border_list_kernel lists them in order after a scan of the counts
    const uint32_t c = block_sum_u32(nb);
    if (threadIdx.x == 0) tile_count_out(tile_cnt, c);
}

__global__ __launch_bounds__(kBlock) void border_list_kernel(uint32_t R,
                                                             const uint32_t* __restrict__ vals,
                                                             const uint8_t* __restrict__ core,
                                                             const uint64_t* __restrict__ tile_off,
                                                             uint32_t* __restrict__ blist) {
    // the owner_kernel tiling: kOwnPer consecutive records per thread, so the
    // list stays in ascending record order
    bool cand[kOwnPer];
    uint32_t nc = 0;
    const uint32_t r0 = (blockIdx.x * kBlock + threadIdx.x) * kOwnPer;
    uint32_t c4 = 0;   // the four flags in one load; vals read only for candidates
    if (r0 + kOwnPer <= R)
        c4 = *reinterpret_cast<const uint32_t*>(core + r0);
    else
        for (int q = 0; q < kOwnPer; ++q) c4 |= r0 + q < R ? (uint32_t)core[r0 + q] << (8 * q) : 0u;
#pragma unroll
    for (int q = 0; q < kOwnPer; ++q) {
        const uint32_t r = r0 + q;
        const uint32_t fl = (c4 >> (8 * q)) & 0xFFu;
        // (owner_kernel's rule: single-neighbour records are attached there)
        cand[q] = r < R && (fl & 3) == 2 && !(fl & 4) && (vals[r] & kOwnerBit);
        nc += cand[q] ? 1u : 0u;
    }
    uint32_t btot;
    uint32_t off = block_excl_scan(nc, btot);
    if (btot == 0) return;
    const uint64_t base = tile_off[blockIdx.x];
#pragma unroll
    for (int q = 0; q < kOwnPer; ++q)
        if (cand[q]) blist[base + off++] = r0 + q;
}

// ------------------------------------------------------------------ lane sweeps
// One lane per record, restructured for latency: the neighbourhood index is
// made wave-uniform (almost always one per wave), so the grid parameters sit
// in scalar registers; rows are taken three at a time and the three ranges
// are swept as ONE virtual list, four candidates per round trip with no
// per-row remainder loops.  Fewer live registers, more waves in flight.
__device__ __forceinline__ double uniform_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xFFFFFFFFll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xFFFFFFFFll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return ((int64_t)hi << 32) | (unsigned int)lo;
}

// Runs body(L, uniform): when the whole wave lies in one neighbourhood (all
// but at most P - 1 waves of a sweep) with L wave-uniform, so the grid
// parameters sit in scalar registers; otherwise with each lane's own L.
template <typename F>
__device__ __forceinline__ void with_part(const uint32_t* __restrict__ ps, int P, uint32_t r,
                                          F&& body) {
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(r);
    const int L0 = part_of(ps, P, r0);
    const uint32_t lo = ps[L0], hi = ps[L0 + 1];
    if (__all(r >= lo && r < hi))
        body(__builtin_amdgcn_readfirstlane(L0), std::true_type{});
    else
        body(part_of(ps, P, r), std::false_type{});
}

// A long centre list (dense cells, PD_OPT_COUNT_ROTATE): the sweep starts at
// record r & ~(kRotAlign - 1) when that lies in the query's centre row, and
// wraps.  The records of a dense row then do not all stream the same first
// lines (one hot L2 channel per row start), the early exit comes sooner (the
// block's records are in the query's own cell), and the smallest neighbour
// found is still near a shared record, so the initial forest stays shallow.
constexpr uint32_t kRotAlign = 256;

// ------------------------------------------------------------------ cheap-row count
// count4_kernel: the neighbour count sweep.  Rows are taken three at a time
// (centre batch first, centre row first) and the three record ranges swept
// as ONE virtual list, four candidates per round trip, with a rotated start
// in long centre rows.  A row's candidate range costs about a third of the
// instructions of the fp64 chord (sqrt, two floors, 64-bit key arithmetic
// from the cell coordinates: ~130 instructions a row, nine rows, which was
// most of the earlier sweep's 3.29e9 VALU instructions per C2 launch).  (At
// the guide's issue rate — a wave64 VALU instruction takes 2 cycles on a
// SIMD-32, so 2 wave-instructions per CU per cycle — count4's 2.66e9 are
// 0.44 of the issue budget: the sweep is bound by the latency of its
// dependent record -> directory word -> cell start -> candidate chain;
// DESIGN.md §4.)  Here, per record once: the fp64 cell index exactly as the
// record keys were built, the in-cell fractions, the squared distances to the
// neighbour rows; per row: the chord in fp32 from those (distances shrunk by
// 2^-16 relative + 2^-20 of a cell, the chord grown by 2^-16 relative + 2^-16
// of an axis-0 cell: a superset of the fp64 chord, so no neighbour is ever
// cut), the row's key as integer offsets from the query cell's key, rows
// outside the grid at an infinite distance.
//   (A persistent-lane variant — a lane that finishes takes the next record
//   of its wave's chunk — was measured and rejected: C2 count 7.0 -> 14.6 ms,
//   8.5e9 VALU instructions: rows hold ~5-10 candidates, so the advance step
//   ran on almost every sweep step)
template <int D>
struct RowGeo {
    uint64_t kc;             // key of the query cell
    int32_t lim_lo, lim_hi;  // axis-0 offsets that stay inside the grid
    float f0;                // in-cell fraction along axis 0
    float tl[D], th[D];      // (j >= 1) distance to the lower / upper row (squared for
                             // euclidean; +inf: no such row)
};

// Row q's axis offsets (-1, 0, +1) for axes 1.., centre row first: digit t of
// q in base 3 (axis 1 fastest) -> offset 0, -1, +1 for t = 0, 1, 2.
template <int D>
__device__ __forceinline__ int row_off(int q, int j) {
    int t = q;
    for (int k = 1; k < j; ++k) t /= 3;
    t %= 3;
    return t == 0 ? 0 : (t == 1 ? -1 : 1);
}

template <typename T, int D, int M, bool U>
struct Count3Grid {
    // neighbourhood grid fields (U: wave-uniform, scalar registers)
    double lo[D], inv[D];
    double cs[D];
    int64_t nc[D];
    uint64_t base;
    uint64_t S[D];           // key strides
    float wsc, wsl;          // chord -> axis-0 cells: w * wsc + wsl
    __device__ __forceinline__ void load(const PartGrid* gp) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            lo[j] = U ? uniform_f64(gp->lo[j]) : gp->lo[j];
            inv[j] = U ? uniform_f64(gp->inv[j]) : gp->inv[j];
            cs[j] = U ? uniform_f64(gp->cs[j]) : gp->cs[j];
            nc[j] = U ? uniform_i64(gp->nc[j]) : gp->nc[j];
        }
        base = U ? (uint64_t)uniform_i64((int64_t)gp->base) : gp->base;
        uint64_t s = 1;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            S[j] = s;
            s *= (uint64_t)nc[j];
        }
        wsc = (float)(inv[0] * (1.0 + 1.0 / 65536.0));
        wsl = 1.0f / 65536.0f;
    }
};

template <typename T, int D, int M, bool U>
__device__ __forceinline__ RowGeo<D> row_geo(const Count3Grid<T, D, M, U>& g, const double (&a)[D]) {
    RowGeo<D> R;
    uint64_t lin = 0;
#pragma unroll
    for (int j = D - 1; j >= 0; --j) {
        const double u = (a[j] - g.lo[j]) * g.inv[j];
        // the cell index exactly as the record keys were built (key_of)
        int64_t c = (int64_t)floor(u);
        c = c < 0 ? 0 : c;
        c = c >= g.nc[j] ? g.nc[j] - 1 : c;
        lin = lin * (uint64_t)g.nc[j] + (uint64_t)c;
        double fr = u - (double)c;
        fr = fr < 0.0 ? 0.0 : (fr > 1.0 ? 1.0 : fr);
        const float f = (float)fr;
        if (j == 0) {
            R.f0 = f;
            R.lim_lo = -(int32_t)(c < 64 ? c : 64);
            const int64_t up = g.nc[0] - 1 - c;
            R.lim_hi = (int32_t)(up < 64 ? up : 64);
        } else {
            const float csf = (float)g.cs[j];
            const float shrink = 1.0f - 1.0f / 65536.0f, abs_s = csf * (1.0f / 1048576.0f);
            float dl = fmaxf(f * csf * shrink - abs_s, 0.0f);
            float dh = fmaxf((1.0f - f) * csf * shrink - abs_s, 0.0f);
            if constexpr (M == 0) {
                dl *= dl;
                dh *= dh;
            }
            R.tl[j] = c > 0 ? dl : INFINITY;
            R.th[j] = c < g.nc[j] - 1 ? dh : INFINITY;
        }
    }
    R.kc = g.base + lin;
    return R;
}

// Candidate record range [s, e) of row q (e <= s: empty).
template <typename T, int D, int M, bool U>
__device__ __forceinline__ void row_range3(const Cells& C, const Count3Grid<T, D, M, U>& g,
                                           const RowGeo<D>& R, float e2, int q, uint32_t& s,
                                           uint32_t& e) {
    float d2 = 0.0f;
    int64_t koff = 0;
#pragma unroll
    for (int j = 1; j < D; ++j) {
        const int o = row_off<D>(q, j);
        d2 += o < 0 ? R.tl[j] : (o > 0 ? R.th[j] : 0.0f);
        koff += o < 0 ? -(int64_t)g.S[j] : (o > 0 ? (int64_t)g.S[j] : 0);
    }
    const bool ok = d2 <= e2;
    float w;
    if constexpr (M == 0)
        // the raw v_sqrt_f32 (<= 1 ulp; the chord is widened by 2^-16 relative
        // below) instead of the correctly rounded sequence (~20 instructions a
        // row).  It may flush a denormal input to 0; the floor at sqrt(FLT_MIN)
        // keeps w >= the true root then (a superset of the chord either way)
        w = fmaxf(__builtin_amdgcn_sqrtf(fmaxf(e2 - d2, 0.0f)), 1.0842022e-19f);
    else
        w = fmaxf(e2 - d2, 0.0f);
    const float wc = w * g.wsc + g.wsl;
    int32_t dx0 = (int32_t)floorf(R.f0 - wc), dx1 = (int32_t)floorf(R.f0 + wc);
    dx0 = dx0 > R.lim_lo ? dx0 : R.lim_lo;
    dx1 = dx1 < R.lim_hi ? dx1 : R.lim_hi;
    const uint64_t rb = R.kc + (uint64_t)koff;
    const uint64_t k0 = ok ? rb + (uint64_t)(int64_t)dx0 : R.kc;
    const uint64_t k1 = ok ? rb + (uint64_t)(int64_t)(dx1 + 1) : R.kc;
    const uint4 w0 = dir_word(C, k0), w1 = dir_word(C, k1);
    const uint32_t i0 = dir_rank(w0, k0), i1 = dir_rank(w1, k1);
    s = C.cstart[i0];
    e = C.cstart[i1];
    e = e > s ? e : s;
}

#ifndef PD_COUNT_WPE
#define PD_COUNT_WPE 8
#endif
#ifndef PD_BORDER_WPE
#define PD_BORDER_WPE 8
#endif
constexpr int kCountWpe = PD_COUNT_WPE, kBorderWpe = PD_BORDER_WPE;   // (A/B builds override)
// WPE: the minimum waves per SIMD the register allocation must allow (1: no
// constraint, the instrumented sweep; 8: at most 64 VGPRs, the default — the
// candidate gathers want the occupancy: C2 count 4.87 -> 4.58 ms).
// REPLAY (measurement only, PD_OPT_COUNT_REPLAY): R launched lanes sweep
// record r % rmod — replicas of a small record set whose chain of loads
// (record, directory words, cell starts, candidates) stays in L2, at full
// occupancy and steady state: the sweep's latency ceiling
// (tools/count_ceiling.py).  Replicas write the same values.
template <typename T, int D, int M, bool ST, int WPE = 1, bool REPLAY = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void count4_kernel(
    const T* __restrict__ Xs, uint32_t R, Cells C, double eps, double eps2, float lo, float hi,
    uint32_t ms, int full, uint32_t rot_min, uint8_t* __restrict__ core,
    uint32_t* __restrict__ mn_out, uint32_t* __restrict__ cnt_out,
    unsigned long long* __restrict__ stats, uint32_t rmod) {
    constexpr int NR = NRows<D>::v;
    constexpr int B = NR < 3 ? NR : 3, NB = NR / B;
    uint32_t r = rec_index();
    if (r >= R) return;
    if constexpr (REPLAY) r = r % rmod;
    (void)rmod;
    double a[D];
    load_rec<T, D>(Xs, r, a);
    const Pred<T, D, M> pr = make_pred<T, D, M>(Xs, r, a, eps, eps2, lo, hi);
    const uint32_t stop = full ? 0xFFFFFFFFu : ms;
    float e2 = M == 0 ? (float)eps2 : (float)eps;
    e2 = e2 * (1.0f + 1.0f / 65536.0f);
    uint32_t cnt = 0, mn = kNone, mn2 = kNone, n_cand = 0;
    with_part(C.part_start, C.P, r, [&](int L, auto U) {
        Count3Grid<T, D, M, decltype(U)::value> g;
        g.load(C.parts + L);
        const RowGeo<D> geo = row_geo<T, D, M, decltype(U)::value>(g, a);
        for (int bt = 0; bt < NB; ++bt) {   // batch 0: the centre batch, centre row first
            uint32_t s0, e0, s1 = 0, e1 = 0, s2 = 0, e2r = 0;
            row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B, s0, e0);
            if constexpr (B > 1) row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B + 1, s1, e1);
            if constexpr (B > 2) row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B + 2, s2, e2r);
            const uint32_t l0 = e0 - s0, l01 = l0 + (e1 - s1), tot = l01 + (e2r - s2);
            // virtual position w -> record (three rows, no dynamic indexing)
            auto jpos = [&](uint32_t w) -> uint32_t {
                uint32_t j = s0 + w;
                if constexpr (B > 1) j = w >= l0 ? s1 + (w - l0) : j;
                if constexpr (B > 2) j = w >= l01 ? s2 + (w - l01) : j;
                return j;
            };
            // a long centre batch: start at record r & ~(kRotAlign - 1) when it
            // lies in the centre row, and wrap
            uint32_t v0 = 0;
            if (bt == 0 && tot > rot_min) {
                const uint32_t vr = (r & ~(kRotAlign - 1u)) - s0;
                v0 = vr < l0 ? vr : 0u;
            }
            auto sweep = [&](auto ROT) -> bool {
                for (uint32_t v = 0; v < tot; v += 4) {
                    uint32_t j[4];
                    T b[4][D];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        uint32_t w = v + u;
                        if constexpr (decltype(ROT)::value) {
                            w += v0;
                            w = w >= tot ? w - tot : w;
                        }
                        j[u] = jpos(w);
                        load_raw<T, D>(Xs, v + u < tot ? j[u] : r, b[u]);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool h = (v + u < tot) && pr(b[u]);
                        cnt += h ? 1u : 0u;
                        const uint32_t x = h ? j[u] : kNone;
                        mn2 = min(mn2, max(mn, x));   // the two smallest hits
                        mn = min(mn, x);
                    }
                    if constexpr (ST) n_cand += (tot - v < 4u ? tot - v : 4u);
                    if (cnt >= stop) return true;
                }
                return false;
            };
            const bool stopped = __any(v0 != 0) ? sweep(std::true_type{}) : sweep(std::false_type{});
            if (stopped) return;
        }
    });
    // bit 2: exactly one neighbour besides the record itself (no early exit
    // below min_samples, so the sweep saw it, and it is the other of the two
    // smallest hits): owner_kernel attaches such a border record directly
    core[r] = (cnt >= ms ? 1 : 0) | (cnt >= 2 ? 2 : 0) | (cnt == 2 ? 4 : 0);
    reinterpret_cast<uint2*>(mn_out)[r] = make_uint2(mn, mn2);
    if (cnt_out) cnt_out[r] = full ? cnt : (cnt < ms ? cnt : ms);
    if constexpr (ST) atomicAdd(stats + 0, (unsigned long long)n_cand);
}

// ------------------------------------------------------------------ link
// The union-find over core-core edges (sklearn's dbscan_inner components,
// SK:cluster/_dbscan_inner.pyx:19-41): (1) an initial forest from the count
// sweep's two smallest neighbours (init_kernel); (2) a union over record
// windows (window_uf_kernel: each core record against the W records after it
// in key order, its own cell and row first); (3) per cell the common root of
// its core records (kMixed: several roots) and per directory word the common
// root of its cells; (4) per cell its forward neighbour cells (higher key,
// within the eps stencil): a pair of cells whose roots agree is already
// connected and skipped (a directory-word summary lets whole neighbour rows
// go unread), only the rest test their core records against each other.
// Every core-core edge lies in one cell or two neighbouring cells, so every
// edge is either proven connected or tested; (1) and (2) are heuristics that
// make (4) cheap, never a source of labels.
constexpr uint32_t kMixed = 0xFFFFFFFEu;

// Root of x without path writes (L1 reads: a stale parent is still an
// ancestor, so the walk ends at a root of some moment).
__device__ __forceinline__ uint32_t root_l1(const uint32_t* par, uint32_t x) {
    uint32_t p = ld_l1(par + x);
    while (p != x) {
        x = p;
        p = ld_l1(par + x);
    }
    return x;
}

__device__ __forceinline__ uint32_t lds_find(const uint32_t* lp, uint32_t x) {
    uint32_t p = lp[x];
    while (p != x) {
        x = p;
        p = lp[x];
    }
    return x;
}

// Union in an LDS forest (smaller index wins; CAS on the larger root).
__device__ __forceinline__ void lds_union(uint32_t* lp, uint32_t a, uint32_t b) {
    while (true) {
        a = lds_find(lp, a);
        b = lds_find(lp, b);
        if (a == b) return;
        if (a > b) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(lp + b, b, a) == b) return;
    }
}

// The window union (link step 2), with the flatten fused into the staging
// and the edges reduced in LDS first.  A wave stages its 64 records
// and the W after them with each one's current root (own records get it
// written back: the flatten), each core lane tests the W records after it
// and unions the core ones within eps of another tree in an LDS forest over
// the window's slots; then each slot whose tree differs from its LDS
// component's representative unites the two trees in the global forest —
// one global union per pair of trees the window joins (the wave's edges
// between the same two trees cost one), instead of a find per edge.
template <typename T, int D, int M, int W, bool ST>
__global__ __launch_bounds__(kBlock) void window_uf_kernel(const T* __restrict__ Xs, uint32_t R,
                                                           double eps, double eps2, float lo,
                                                           float hi, uint32_t* __restrict__ par,
                                                           unsigned long long* __restrict__ stats) {
    constexpr int E = 64 + W;
    static_assert(E <= 128, "two slots per lane");
    __shared__ T sx[kBlock / 64][E][D];
    __shared__ uint32_t sp[kBlock / 64][E];
    __shared__ uint32_t lp[kBlock / 64][E];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t b = xcd_block(blockIdx.x, gridDim.x) * kBlock + w * 64;
    for (int e = lane; e < E; e += 64) {
        const uint32_t j = b + e;
        T v[D];
        uint32_t p = kNone;
        if (j < R) {
            load_raw<T, D>(Xs, j, v);
            p = ld_l1(par + j);
            if (p != kNone && p != j) {
                const uint32_t root = root_l1(par, p);
                if (e < 64 && root != p) st_rlx(par + j, root);   // the flatten
                p = root;
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) v[k] = T(0);
        }
#pragma unroll
        for (int k = 0; k < D; ++k) sx[w][e][k] = v[k];
        sp[w][e] = p;
        lp[w][e] = (uint32_t)e;
    }
    __syncthreads();
    const uint32_t r = b + lane;
    const uint32_t p0 = r < R ? sp[w][lane] : kNone;
    LinkStats st;
    if (p0 != kNone) {
        Pred<T, D, M> pr;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            pr.ar[k] = sx[w][lane][k];
            pr.a[k] = (double)pr.ar[k];
        }
        pr.eps = eps;
        pr.eps2 = eps2;
        pr.lo = lo;
        pr.hi = hi;
#pragma unroll 4
        for (int k = 1; k <= W; ++k) {
            const uint32_t pj = sp[w][lane + k];
            if (pj == kNone || pj == p0 || r + k >= R) continue;   // non-core / same tree
            T bj[D];
#pragma unroll
            for (int q = 0; q < D; ++q) bj[q] = sx[w][lane + k][q];
            if constexpr (ST) ++st.cand;
            if (pr(bj)) {
                if constexpr (ST) ++st.hit;
                lds_union(lp[w], (uint32_t)lane, (uint32_t)(lane + k));
            }
        }
    }
    __syncthreads();
    for (int e = lane; e < E; e += 64) {
        const uint32_t pe = sp[w][e];
        if (pe == kNone) continue;
        const uint32_t lr = lds_find(lp[w], (uint32_t)e);
        const uint32_t pl = sp[w][lr];
        if (pl == pe) continue;
        // the slot before carries the same pair of trees: its lane unites them
        if (e > 0 && sp[w][e - 1] == pe && lds_find(lp[w], (uint32_t)(e - 1)) == lr) continue;
        if constexpr (ST) ++st.unions;
        uf_link_roots(par, uf_find_l1(par, pl), uf_find_l1(par, pe));
    }
    if constexpr (ST) {   // one atomic per block and counter
        const uint32_t c = block_sum_u32(st.cand), h = block_sum_u32(st.hit),
                       u = block_sum_u32(st.unions);
        if (threadIdx.x == 0) {
            atomicAdd(stats + 1, (unsigned long long)c);
            atomicAdd(stats + 2, (unsigned long long)h);
            atomicAdd(stats + 6, (unsigned long long)u);
        }
    }
}

// Per cell, the common root of its core records (kNone: no core record,
// kMixed: several roots); also flattens: each core record gets its root
// written back, so no separate flatten pass runs before (no unions run
// concurrently, so a chain read by another cell stays valid).
__device__ __forceinline__ uint32_t root_merge(uint32_t a, uint32_t b) {
    return a == kNone ? b : (b == kNone ? a : (a == b ? a : kMixed));
}

__device__ __forceinline__ uint32_t core_root(uint32_t* __restrict__ par, uint32_t r) {
    const uint32_t p0 = par[r];
    if (p0 == kNone) return kNone;   // not core
    uint32_t p = p0;
    while (true) {
        const uint32_t q = par[p];
        if (q == p) break;
        p = q;
    }
    if (p != p0) par[r] = p;
    return p;
}

// wroot[w] = root_merge(wroot[w], v) atomically (monotone: kNone -> a root
// -> kMixed).
__device__ __forceinline__ void word_merge(uint32_t* wroot, uint64_t w, uint32_t v) {
    if (v == kNone) return;
    uint32_t cur = ld_rlx(wroot + w);
    while (true) {
        const uint32_t want = root_merge(cur, v);
        if (want == cur) return;
        const uint32_t prev = atomicCAS(wroot + w, cur, want);
        if (prev == cur) return;
        cur = prev;
    }
}

// Cell roots with the word roots fused in: the cells of a wave are
// consecutive in key order, so lanes of one directory word (key >> 6) merge
// their cell roots by a segmented shuffle scan and the segment's last lane
// merges the result into the word atomically (a word can span two waves).
// wroot must start at kNone.
// Tiers: a thread walks a cell of <= kMidCell records, a wave one of
// <= kWordBig (mid_cell_word_root_kernel), a block a larger one
// (big_cell_word_root_kernel).  A thread walking up to 256 records held its
// whole wave on C4's dense cells: 55 ms of the 1B-point link.
constexpr uint32_t kMidCell = 16, kWordBig = 1024;

template <typename K, bool W32>
__global__ __launch_bounds__(kBlock) void cell_word_root_kernel(
    const uint32_t* __restrict__ cstart, const uint32_t* __restrict__ ncells,
    const K* __restrict__ ckeys, uint32_t* __restrict__ par, uint32_t* __restrict__ croot,
    uint32_t* __restrict__ wroot, uint32_t* __restrict__ mid, uint32_t* __restrict__ nmid,
    uint32_t* __restrict__ big, uint32_t* __restrict__ nbig, const uint4* __restrict__ pages) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t nc = *ncells;
    if (c - (uint32_t)lane >= nc) return;   // a wave past the last cell (grid over records)
    using WT = std::conditional_t<W32, uint32_t, uint64_t>;   // W32: slots < 2^32 - 1
    uint32_t v = kNone;
    WT word = (WT)~0ull;
    uint32_t sz = 0, s = 0;
    if (c < nc) {
        s = cstart[c];
        sz = cstart[c + 1] - s;
        word = (WT)word_slot(pages, (uint64_t)ckeys[c]);
    }
    // the larger cells' roots join their words in the mid / big kernels
    wave_append(mid, nmid, sz > kMidCell && sz <= kWordBig, c);
    wave_append(big, nbig, sz > kWordBig, c);
    if (c < nc && sz <= kMidCell) {
        // four records at a time: their parents, then the parents' parents,
        // all in flight together (core_root walked one record's chain after
        // another: C4's 3.4e8 cells took 8.4 ms)
        for (uint32_t b = s; b < s + sz; b += 4) {
            uint32_t p0[4], p1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) p0[q] = b + q < s + sz ? par[b + q] : kNone;
#pragma unroll
            for (int q = 0; q < 4; ++q) p1[q] = p0[q] != kNone ? par[p0[q]] : kNone;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (p0[q] == kNone) continue;   // not core
                uint32_t x = p0[q];
                if (p1[q] != x) {               // p0 is not a root: walk on
                    x = p1[q];
                    while (true) {
                        const uint32_t y = par[x];
                        if (y == x) break;
                        x = y;
                    }
                    par[b + q] = x;             // the flatten (core_root's write)
                }
                v = root_merge(v, x);
            }
        }
        croot[c] = v;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t nv = (uint32_t)__shfl_up((int)v, o, 64);
        const WT nw = shfl_up_w(word, o);
        if (lane >= o && nw == word) v = root_merge(v, nv);
    }
    const WT next = shfl_down_w(word, 1);
    if (c < nc && (lane == 63 || next != word)) word_merge(wroot, (uint64_t)word, v);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void mid_cell_word_root_kernel(
    const uint32_t* __restrict__ cstart, const K* __restrict__ ckeys,
    const uint32_t* __restrict__ mid, const uint32_t* __restrict__ nmid,
    uint32_t* __restrict__ par, uint32_t* __restrict__ croot, uint32_t* __restrict__ wroot,
    const uint4* __restrict__ pages) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nm = *nmid;
    const uint32_t nw = gridDim.x * (kBlock / 64);
    for (uint32_t i = (blockIdx.x * kBlock + threadIdx.x) >> 6; i < nm; i += nw) {
        const uint32_t c = mid[i];
        const uint32_t s = cstart[c], e = cstart[c + 1];
        uint32_t v = kNone;
        for (uint32_t r = s + lane; r < e; r += 64) v = root_merge(v, core_root(par, r));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = root_merge(v, (uint32_t)__shfl_xor((int)v, o, 64));
        if (lane == 0) {
            croot[c] = v;
            word_merge(wroot, word_slot(pages, (uint64_t)ckeys[c]), v);
        }
    }
}

template <typename K>
__global__ __launch_bounds__(kBlock) void big_cell_word_root_kernel(
    const uint32_t* __restrict__ cstart, const K* __restrict__ ckeys,
    const uint32_t* __restrict__ big, const uint32_t* __restrict__ nbig,
    uint32_t* __restrict__ par, uint32_t* __restrict__ croot, uint32_t* __restrict__ wroot,
    const uint4* __restrict__ pages) {
    __shared__ uint32_t part[kBlock / 64];
    const uint32_t nb = *nbig;
    for (uint32_t i = blockIdx.x; i < nb; i += gridDim.x) {
        const uint32_t c = big[i];
        const uint32_t e = cstart[c + 1];
        uint32_t v = kNone;
        for (uint32_t r = cstart[c] + threadIdx.x; r < e; r += kBlock) v = root_merge(v, core_root(par, r));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = root_merge(v, (uint32_t)__shfl_xor((int)v, o, 64));
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t w = kNone;
#pragma unroll
            for (int k = 0; k < kBlock / 64; ++k) w = root_merge(w, part[k]);
            croot[c] = w;
            word_merge(wroot, word_slot(pages, (uint64_t)ckeys[c]), w);
        }
        __syncthreads();
    }
}

// Test the core records of [s0, e0) against those of [s1, e1) (b > a when the
// ranges are the same cell) and unite the pairs within eps; pairs already
// under one root (live) skip the distance test.
template <typename T, int D, int M>
__device__ __noinline__ void pair_block(const T* __restrict__ Xs, uint32_t s0, uint32_t e0,
                                        uint32_t s1, uint32_t e1, bool same, bool uniform,
                                        double eps, double eps2, float lo, float hi,
                                        uint32_t* par) {
    // uniform: two different cells, each under one root (the cell_root
    // snapshot; later unions only merge trees), so the first pair found
    // connected settles the whole block — a dense cell pair costs a few
    // tests, not occupancy^2.  ra may go stale under concurrent unions: a
    // match still proves a and b share a tree (trees only merge).
    for (uint32_t a = s0; a < e0; ++a) {
        if (ld_rlx(par + a) == kNone) continue;
        double av[D];
        load_rec<T, D>(Xs, a, av);
        const Pred<T, D, M> pr = make_pred<T, D, M>(Xs, a, av, eps, eps2, lo, hi);
        uint32_t ra = uf_find(par, a);
        for (uint32_t b = same ? a + 1 : s1; b < e1; ++b) {
            if (ld_rlx(par + b) == kNone) continue;
            if (uf_find(par, b) == ra) {
                if (uniform) return;
                continue;
            }
            T bv[D];
            load_raw<T, D>(Xs, b, bv);
            if (pr(bv)) {
                uf_unite(par, a, b);
                if (uniform) return;
                ra = uf_find(par, a);
            }
        }
    }
}

// The forward rows of cell c (its own row from the cell on, and the rows
// after it: key order is lexicographic from the last axis; row q's offsets
// o_j = digit j-1 of q in base 3, minus 1): their key ranges [k0, k1).
template <int D, typename K>
struct ForwardRows {
    static constexpr int NF = (NRows<D>::v + 1) / 2;
    uint64_t k0[NF], k1[NF];
    bool ok[NF];
};

template <int D, typename K>
__device__ __forceinline__ void forward_rows(const K* __restrict__ keys, const Cells& C, uint32_t s0,
                                             int xsub, ForwardRows<D, K>& fr) {
    constexpr int NR = NRows<D>::v;
    constexpr int NF = ForwardRows<D, K>::NF;
    // the cell's grid coordinates (wave-uniform neighbourhood in the common case)
    const int L = part_of_wave(C.part_start, C.P, s0);
    const PartGrid* gp = C.parts + L;
    int64_t nc[D], cc[D];
#pragma unroll
    for (int j = 0; j < D; ++j) nc[j] = gp->nc[j];
    const uint64_t base = gp->base;
    uint64_t lin = (uint64_t)keys[s0] - base;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        uint64_t qt;
        if (lin < (1ull << 52) && nc[j] < (1ll << 31)) {
            // exact via fp64 (both operands exact), one-step correction
            qt = (uint64_t)floor((double)lin / (double)nc[j]);
            int64_t rem = (int64_t)(lin - qt * (uint64_t)nc[j]);
            if (rem < 0) {
                --qt;
                rem += nc[j];
            } else if (rem >= nc[j]) {
                ++qt;
                rem -= nc[j];
            }
            cc[j] = rem;
        } else {
            qt = lin / (uint64_t)nc[j];
            cc[j] = (int64_t)(lin - qt * (uint64_t)nc[j]);
        }
        lin = qt;
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const int q = NR / 2 + f;   // rows NR/2 .. NR-1 are the own row and those after
        int t = q, o[D];
        o[0] = 0;
        bool okq = true;
#pragma unroll
        for (int j = 1; j < D; ++j) {
            o[j] = (t % 3) - 1;
            t /= 3;
            okq &= (cc[j] + o[j] >= 0) & (cc[j] + o[j] < nc[j]);
        }
        const int64_t x0 = f == 0 ? cc[0] : (cc[0] - xsub < 0 ? 0 : cc[0] - xsub);
        const int64_t x1 = cc[0] + xsub >= nc[0] ? nc[0] - 1 : cc[0] + xsub;
        uint64_t kk = 0;
#pragma unroll
        for (int j = D - 1; j >= 0; --j)
            kk = kk * (uint64_t)nc[j] + (uint64_t)(j == 0 ? x0 : cc[j] + o[j]);
        fr.k0[f] = okq ? kk + base : 0;
        fr.k1[f] = okq ? kk + base + (uint64_t)(x1 - x0) + 1 : 1;
        fr.ok[f] = okq;
    }
}

// Cell verify, first pass: which cells need record-level work at all.  A
// cell with one root R (not mixed) whose forward rows' directory words hold
// no root but R is settled; the others are flagged (flag byte per cell, and
// per-tile counts for the ordered work list).
template <int D, typename K>
__global__ __launch_bounds__(kBlock) void verify_screen_kernel(
    const K* __restrict__ keys, const uint32_t* __restrict__ ncells,
    const uint32_t* __restrict__ croot, const uint32_t* __restrict__ wroot, Cells C, int xsub,
    uint8_t* __restrict__ flags, uint32_t* __restrict__ tile_cnt) {
    constexpr int NF = ForwardRows<D, K>::NF;
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t nc = *ncells;
    if (blockIdx.x * kBlock >= nc) {   // a tile past the last cell (grid over records)
        if (threadIdx.x == 0) tile_count_out(tile_cnt, 0);
        return;
    }
    const uint32_t rc = c < nc ? croot[c] : kNone;
    bool work = rc == kMixed;
    if (rc != kNone && rc != kMixed) {
        ForwardRows<D, K> fr;
        forward_rows<D, K>(keys, C, C.cstart[c], xsub, fr);
        uint32_t wa[NF], wb[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            wa[f] = word_root_at(C, wroot, fr.k0[f]);
            wb[f] = word_root_at(C, wroot, fr.k1[f] - 1);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f)
            work |= fr.ok[f] && !((wa[f] == kNone || wa[f] == rc) && (wb[f] == kNone || wb[f] == rc));
    }
    if (c < nc) flags[c] = work ? 1 : 0;
    const uint32_t t = block_sum_u32(work ? 1u : 0u);
    if (threadIdx.x == 0) tile_count_out(tile_cnt, t);
}

// Ordered list of the indices i < n with flags[i] set (tile offsets from a
// scan of the per-tile counts).
__global__ __launch_bounds__(kBlock) void flag_list_kernel(const uint8_t* __restrict__ flags,
                                                           const uint32_t* __restrict__ n_dev,
                                                           const uint64_t* __restrict__ tile_off,
                                                           uint32_t* __restrict__ list) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t nd = *n_dev;
    if (blockIdx.x * kBlock >= nd) return;   // a tile past the last cell: no entries
    const bool f = i < nd && flags[i];
    uint32_t btot;
    const uint32_t off = block_excl_scan(f ? 1u : 0u, btot);
    if (f) list[tile_off[blockIdx.x] + off] = i;
}

// Cell verify, second pass, over the flagged cells only: per forward row
// whose words hold another root, the neighbouring cells whose root differs
// are deferred as cell pairs.
template <typename T, int D, int M, typename K>
__global__ __launch_bounds__(kBlock) void cell_verify_kernel(
    const T* __restrict__ Xs, const K* __restrict__ keys, const uint32_t* __restrict__ clist,
    uint32_t nlist, const uint32_t* __restrict__ croot, const uint32_t* __restrict__ wroot,
    Cells C, int xsub, double eps, double eps2, float lo, float hi, uint32_t* __restrict__ par,
    uint2* __restrict__ plist, uint32_t pcap, uint32_t* __restrict__ pcount,
    unsigned long long* __restrict__ stats, const uint32_t* __restrict__ ncells) {
    constexpr int NF = ForwardRows<D, K>::NF;
    constexpr uint32_t kBuf = 1024;
    // clist == nullptr (PD_OPT_VERIFY_FUSED): every cell, i.e. the screen
    // fused in (the grid covers the records; blocks past the last cell leave)
    if (!clist) {
        nlist = *ncells;
        if (blockIdx.x * kBlock >= nlist) return;
    }
    // cell pairs whose roots differ go to a list, resolved by pair_kernel, so
    // the rare record-level work does not stall this kernel's waves: staged
    // per block in LDS, one global reservation per block (overflow of the
    // block buffer or of the list: resolved in place)
    __shared__ uint2 lbuf[kBuf];
    __shared__ uint32_t lcnt, lbase;
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t c = i < nlist ? (clist ? clist[i] : i) : 0u;
    const uint32_t rc = i < nlist ? croot[c] : kNone;
    uint32_t pairs = 0;
    if (rc != kNone) {
    const uint32_t s0 = C.cstart[c], e0 = C.cstart[c + 1];
    auto defer = [&](uint32_t c2) {
        ++pairs;
        const uint32_t slot = atomicAdd(&lcnt, 1u);
        if (slot < kBuf) {
            lbuf[slot] = make_uint2(c, c2);
        } else {
            const bool same = c2 == c;
            const bool uni = !same && rc != kMixed && croot[c2] != kMixed;
            pair_block<T, D, M>(Xs, s0, e0, same ? s0 : C.cstart[c2], same ? e0 : C.cstart[c2 + 1],
                                same, uni, eps, eps2, lo, hi, par);
        }
    };
    if (rc == kMixed) defer(c);
    ForwardRows<D, K> fr;
    forward_rows<D, K>(keys, C, s0, xsub, fr);
    uint32_t wa[NF], wb[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        wa[f] = word_root_at(C, wroot, fr.k0[f]);
        wb[f] = word_root_at(C, wroot, fr.k1[f] - 1);
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        if (!fr.ok[f]) continue;
        // the row's words hold no root but ours: nothing to test
        if (rc != kMixed && (wa[f] == kNone || wa[f] == rc) && (wb[f] == kNone || wb[f] == rc))
            continue;
        const uint32_t i0 = dir_rank(dir_word(C, fr.k0[f]), fr.k0[f]);
        const uint32_t i1 = dir_rank(dir_word(C, fr.k1[f]), fr.k1[f]);
        for (uint32_t c2 = i0 > c + 1 ? i0 : c + 1; c2 < i1; ++c2) {
            const uint32_t r2 = croot[c2];
            if (r2 == kNone || (r2 == rc && rc != kMixed)) continue;
            defer(c2);
        }
    }
    }   // rc != kNone
    __syncthreads();
    const uint32_t nb = lcnt < kBuf ? lcnt : kBuf;
    if (threadIdx.x == 0) lbase = nb ? atomicAdd(pcount, nb) : 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nb; k += kBlock) {
        const uint2 pr = lbuf[k];
        if (lbase + k < pcap) {
            plist[lbase + k] = pr;
        } else {
            const bool same = pr.x == pr.y;
            const bool uni = !same && croot[pr.x] != kMixed && croot[pr.y] != kMixed;
            pair_block<T, D, M>(Xs, C.cstart[pr.x], C.cstart[pr.x + 1], C.cstart[pr.y],
                                C.cstart[pr.y + 1], same, uni, eps, eps2, lo, hi, par);
        }
    }
    if (stats && pairs) atomicAdd(stats + 7, (unsigned long long)pairs);
}

// The deferred cell pairs: a live root comparison of two uniform cells may
// settle a pair (earlier unions merged their trees); otherwise their core
// records are tested against each other.
template <typename T, int D, int M>
__global__ __launch_bounds__(kBlock) void pair_kernel(const T* __restrict__ Xs,
                                                      const uint2* __restrict__ plist,
                                                      const uint32_t* __restrict__ pcount,
                                                      uint32_t pcap,
                                                      const uint32_t* __restrict__ cstart,
                                                      const uint32_t* __restrict__ croot, double eps,
                                                      double eps2, float lo, float hi,
                                                      uint32_t* __restrict__ par) {
    const uint32_t np0 = *pcount;
    const uint32_t np = np0 < pcap ? np0 : pcap;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < np; i += gridDim.x * kBlock) {
        const uint2 pr = plist[i];
        const uint32_t ra = croot[pr.x], rb = croot[pr.y];
        if (pr.x != pr.y && ra != kMixed && rb != kMixed && uf_find(par, ra) == uf_find(par, rb))
            continue;
        const bool same = pr.x == pr.y;
        const bool uni = !same && ra != kMixed && rb != kMixed;
        pair_block<T, D, M>(Xs, cstart[pr.x], cstart[pr.x + 1], cstart[pr.y], cstart[pr.y + 1],
                            same, uni, eps, eps2, lo, hi, par);
    }
}

// border4_kernel: the smallest cluster key among the core neighbours of a
// border candidate (sklearn's first-discovered-cluster rule, every row), with
// count4's cheap rows.
template <typename T, int D, int M, int WPE = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void border4_kernel(
    const T* __restrict__ Xs, uint32_t NL, const uint32_t* __restrict__ list, Cells C, double eps,
    double eps2, float lo, float hi, const uint32_t* __restrict__ vals,
    const uint32_t* __restrict__ par, const uint32_t* __restrict__ gmin,
    uint32_t* __restrict__ key_out, uint32_t* __restrict__ rec_out) {
    constexpr int NR = NRows<D>::v;
    constexpr int B = NR < 3 ? NR : 3, NB = NR / B;
    const uint32_t i = rec_index();
    if (i >= NL) return;
    const uint32_t r = list[i];   // owner, non-core records with a neighbour, ascending
    double a[D];
    load_rec<T, D>(Xs, r, a);
    const Pred<T, D, M> pr = make_pred<T, D, M>(Xs, r, a, eps, eps2, lo, hi);
    float e2 = M == 0 ? (float)eps2 : (float)eps;
    e2 = e2 * (1.0f + 1.0f / 65536.0f);
    uint32_t best = kNone;
    with_part(C.part_start, C.P, r, [&](int L, auto U) {
        Count3Grid<T, D, M, decltype(U)::value> g;
        g.load(C.parts + L);
        const RowGeo<D> geo = row_geo<T, D, M, decltype(U)::value>(g, a);
        for (int bt = 0; bt < NB; ++bt) {
            uint32_t s0, e0, s1 = 0, e1 = 0, s2 = 0, e2r = 0;
            row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B, s0, e0);
            if constexpr (B > 1) row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B + 1, s1, e1);
            if constexpr (B > 2) row_range3<T, D, M, decltype(U)::value>(C, g, geo, e2, bt * B + 2, s2, e2r);
            const uint32_t l0 = e0 - s0, l01 = l0 + (e1 - s1), tot = l01 + (e2r - s2);
            const uint32_t o1 = s1 - l0, o2 = s2 - l01;
            for (uint32_t v = 0; v < tot; v += 4) {
                uint32_t j[4], pj[4];
                T b[4][D];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t w = v + u;
                    uint32_t o = s0;
                    if constexpr (B > 1) o = w >= l0 ? o1 : o;
                    if constexpr (B > 2) o = w >= l01 ? o2 : o;
                    j[u] = w < tot ? w + o : r;
                    load_raw<T, D>(Xs, j[u], b[u]);
                    pj[u] = par[j[u]];
                }
                bool h[4], mb[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    pr.screen(b[u], h[u], mb[u]);
                    const bool ok = (v + u < tot) & (pj[u] != kNone);
                    h[u] &= ok;
                    mb[u] &= ok;
                }
                if (__any(mb[0] | mb[1] | mb[2] | mb[3])) {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (mb[u]) h[u] = pr.exact(b[u]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (h[u]) {
                        const uint32_t k = gmin[pj[u]];
                        best = k < best ? k : best;
                    }
            }
        }
    });
    // rec_out: by record, into the pairs of the bucketed label pass
    if (rec_out)
        rec_out[2 * (size_t)r] = best;   // the key half of the record's (point, key) pair
    else
        key_out[vals[r] & kIdMask] = best;
}

// ---- labels into input order in two coalesced passes (single device).  The
// owner records sit in key order, their points in input order: a permutation
// whose direct scatter (owner_kernel: one 4-B write per record, anywhere in
// n) moved 28 GB for C4's 1e9 records.  Here label_bucket_kernel partitions
// the (point, key) pairs of a tile by the point's high bits (buckets of
// 2^kLabBits points): the tile is counting-sorted by bucket in LDS and each
// bucket's run is written out by consecutive threads (whole lines, one
// global reservation per tile and bucket, ~15 pairs per run); then
// label_scatter_kernel writes each bucket's keys into its 4 MB of key_out
// from blocks of one XCD, so the random writes combine in that XCD's L2.
// (Round 3, first form: 2^17-point buckets and pairs written straight from
// an LDS atomic slot — partial lines; C4 label_bucket 12.2 ms.)
constexpr int kLabBlock = 1024;                 // threads per label_bucket tile
constexpr int kLabPer = 15;                     // pairs per thread
constexpr int kLabTile = kLabBlock * kLabPer;   // 15360 pairs (120 KiB staged)
constexpr int kLabMaxBk = 2048;                 // buckets (2 per thread in the scan)
// Block-local form: buckets of 2^15 points, one workgroup per bucket places
// its keys in an LDS image of the bucket's labels (128 KiB) and writes labels
// and core flags coalesced.
constexpr int kLabBitsL = 15;
constexpr int kLabPerL = 12;                    // label_split tile: 12288 pairs (96 KiB staged)

// (point, key) pairs in record order: pairs[r] = (owner record ? its point :
// kNone, core: the cluster key | kKeyCoreBit; else kNone — the border sweep
// fills in its key afterwards).  Written by owner_kernel in bucketed mode.
template <int PER, int MAXBK>
__global__ __launch_bounds__(kLabBlock) void label_bucket_kernel(uint32_t R,
                                                                 const uint2* __restrict__ recs,
                                                                 int kLabBits, int nbk,
                                                                 uint32_t* __restrict__ bcnt,
                                                                 uint2* __restrict__ pairs) {
    constexpr int TILE = kLabBlock * PER, BPT = MAXBK / kLabBlock;
    __shared__ uint2 stage[TILE];
    __shared__ uint32_t cnt[MAXBK], off[MAXBK], gbase[MAXBK];
    const int tid = threadIdx.x;
    for (int k = tid; k < MAXBK; k += kLabBlock) cnt[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    uint2 q[PER];
    uint32_t lr[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kLabBlock + tid;
        q[i] = make_uint2(kNone, kNone);
        if (r < R) {   // streamed once: non-temporal
            const unsigned long long w =
                __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(recs + r));
            q[i] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
        }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const bool ok = q[i].x != kNone && q[i].y != kNone;
        lr[i] = ok ? atomicAdd(&cnt[q[i].x >> kLabBits], 1u) : 0u;
        if (!ok) q[i].x = kNone;
    }
    __syncthreads();
    uint32_t total, c[BPT], sum = 0;   // BPT consecutive buckets per thread
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        const int k = BPT * tid + u;
        c[u] = k < nbk ? cnt[k] : 0u;
        sum += c[u];
    }
    uint32_t ex = block_excl_scan<kLabBlock>(sum, total);
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        const int k = BPT * tid + u;
        if (k < nbk) {
            off[k] = ex;
            gbase[k] = c[u] ? atomicAdd(bcnt + k, c[u]) : 0u;
        }
        ex += c[u];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if (q[i].x != kNone) stage[off[q[i].x >> kLabBits] + lr[i]] = q[i];
    __syncthreads();
    for (uint32_t p = tid; p < total; p += kLabBlock) {
        const uint2 v = stage[p];
        const uint32_t b = v.x >> kLabBits;
        pairs[((uint64_t)b << kLabBits) + gbase[b] + (p - off[b])] = v;
    }
}

__global__ __launch_bounds__(kBlock) void label_scatter_kernel(const uint2* __restrict__ pairs,
                                                               const uint32_t* __restrict__ bcnt,
                                                               int kLabBits, int nbk, unsigned bpb,
                                                               uint32_t* __restrict__ key_out) {
    const unsigned lb = xcd_block(blockIdx.x, gridDim.x);   // a bucket's blocks share an XCD
    const unsigned b = lb / bpb, part = lb % bpb;
    if ((int)b >= nbk) return;
    const uint32_t c = bcnt[b];
    const uint2* p = pairs + ((uint64_t)b << kLabBits);
    for (uint32_t k = part * kBlock + threadIdx.x; k < c; k += bpb * kBlock) {
        // streamed: non-temporal, the L2 is kept for key_out
        const unsigned long long w =
            __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(p + k));
        key_out[(uint32_t)w] = (uint32_t)(w >> 32);
    }
}

// The coarse buckets of 2^kLabBits points (label_bucket_kernel) are split
// into their 2^(kLabBits - kLabBitsL) sub-buckets of 2^kLabBitsL points, a
// tile of one coarse bucket per workgroup (counting sort by sub-bucket in LDS,
// runs of ~700 pairs written whole), for label_local_kernel.  (Bucketing
// straight into 2^15-point buckets — 3052 for C2, runs of ~3 pairs per tile —
// measured slower: label_bucket 0.78 vs 0.31 + 0.24 split ms, C2 border
// 3.80 vs 3.65 ms.)
constexpr int kLabMaxSub = 64;   // kLabBits <= kLabBitsL + 6 (n < 2^32 needs <= 21)
__global__ __launch_bounds__(kLabBlock) void label_split_kernel(const uint2* __restrict__ pairs,
                                                                const uint32_t* __restrict__ bcnt,
                                                                int kLabBits, uint32_t tpb,
                                                                uint32_t* __restrict__ bcnt2,
                                                                uint2* __restrict__ pairs2) {
    constexpr int PER = kLabPerL, TILE = kLabBlock * PER;
    __shared__ uint2 stage[TILE];
    __shared__ uint32_t cnt[kLabMaxSub], off[kLabMaxSub], gbase[kLabMaxSub], s_total;
    const uint32_t b = blockIdx.x / tpb, t = blockIdx.x % tpb;
    const uint32_t c = bcnt[b];
    const uint64_t t0 = (uint64_t)t * TILE;
    if (t0 >= c) return;   // whole workgroup
    const int tid = threadIdx.x;
    const int sb = kLabBits - kLabBitsL;
    const uint32_t nsub = 1u << sb, smask = nsub - 1;
    if (tid < kLabMaxSub) cnt[tid] = 0;
    __syncthreads();
    const uint2* src = pairs + ((uint64_t)b << kLabBits);
    uint2 q[PER];
    uint32_t lr[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint64_t k = t0 + (uint64_t)i * kLabBlock + tid;
        q[i] = make_uint2(kNone, kNone);
        if (k < c) {   // streamed once: non-temporal
            const unsigned long long w =
                __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(src + k));
            q[i] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
        }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i)
        lr[i] = q[i].x != kNone ? atomicAdd(&cnt[(q[i].x >> kLabBitsL) & smask], 1u) : 0u;
    __syncthreads();
    if (tid < 64) {   // wave 0: scan of the <= 64 sub-bucket counts
        const uint32_t v = (uint32_t)tid < nsub ? cnt[tid] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (tid >= o) x += y;
        }
        off[tid] = x - v;
        gbase[tid] = v ? atomicAdd(bcnt2 + ((uint64_t)b << sb) + tid, v) : 0u;
        if (tid == 63) s_total = x;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if (q[i].x != kNone) stage[off[(q[i].x >> kLabBitsL) & smask] + lr[i]] = q[i];
    __syncthreads();
    const uint32_t total = s_total;
    for (uint32_t p = tid; p < total; p += kLabBlock) {
        const uint2 v = stage[p];
        const uint32_t g = v.x >> kLabBitsL, u = g & smask;
        pairs2[((uint64_t)g << kLabBitsL) + gbase[u] + (p - off[u])] = v;
    }
}

// Block-local label pass: one workgroup per bucket of 2^kLabBitsL points.
// The bucket's (point, key) pairs (in bucket order, from label_bucket_kernel)
// are placed into an LDS image of its labels (kNone = noise), then the
// labels (core bit stripped) and the core mask are written coalesced — no
// key_out fill, no scattered HBM writes, no separate final_label_kernel.
__global__ __launch_bounds__(kLabBlock) void label_local_kernel(const uint2* __restrict__ pairs,
                                                                const uint32_t* __restrict__ bcnt,
                                                                uint64_t n,
                                                                int32_t* __restrict__ labels,
                                                                uint8_t* __restrict__ core_out) {
    constexpr uint32_t NB = 1u << kLabBitsL, MASK = NB - 1;
    __shared__ uint32_t img[NB];
    const uint32_t b = blockIdx.x;
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < NB; i += kLabBlock) img[i] = kNone;
    __syncthreads();
    const uint32_t c = bcnt[b];
    const unsigned long long* p =
        reinterpret_cast<const unsigned long long*>(pairs + ((uint64_t)b << kLabBitsL));
    constexpr int U = 4;   // loads in flight per thread
    for (uint32_t k0 = 0; k0 < c; k0 += U * kLabBlock) {
        unsigned long long w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * kLabBlock + tid;
            w[u] = k < c ? __builtin_nontemporal_load(p + k) : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u * kLabBlock + tid < c) img[(uint32_t)w[u] & MASK] = (uint32_t)(w[u] >> 32);
    }
    __syncthreads();
    const uint64_t base = (uint64_t)b << kLabBitsL;
    const uint32_t m = (uint32_t)std::min<uint64_t>(NB, n - base);
    for (uint32_t i = tid; i < m; i += kLabBlock) {
        const uint32_t k = img[i];
        labels[base + i] = k == kNone ? -1 : (int32_t)(k & ~kKeyCoreBit);
        if (core_out) core_out[base + i] = (k != kNone && (k & kKeyCoreBit)) ? 1 : 0;
    }
}

// Single device: key_out holds each point's label (rank; kNone = noise) with
// the core flag in bit 30 — split it into labels and the core mask.
__global__ __launch_bounds__(kBlock) void final_label_kernel(const uint32_t* __restrict__ key,
                                                             uint64_t n, int32_t* __restrict__ labels,
                                                             uint8_t* __restrict__ core_out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = key[i];
    labels[i] = k == kNone ? -1 : (int32_t)(k & ~kKeyCoreBit);
    if (core_out) core_out[i] = (k != kNone && (k & kKeyCoreBit)) ? 1 : 0;
}

// Sharded phase B: the core flag out of bit `mask` of each key into a byte,
// both coalesced (kNone stays: a noise point).
__global__ __launch_bounds__(kBlock) void split_core_kernel(uint32_t* __restrict__ key, uint64_t n,
                                                            uint32_t mask,
                                                            uint8_t* __restrict__ core) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = key[i];
    const bool c = k != kNone && (k & mask);
    if (core) core[i] = c ? 1 : 0;
    if (c) key[i] = k & ~mask;
}

// Keys may carry kKeyCoreBit (owner_kernel core_bit mode): strip it.
__device__ __forceinline__ uint32_t key_id(uint32_t k, int core_bit) {
    return (core_bit && k != kNone) ? (k & ~kKeyCoreBit) : k;
}

__global__ __launch_bounds__(kBlock) void root_flag_kernel(const uint32_t* __restrict__ key,
                                                           uint64_t n, int core_bit,
                                                           uint32_t* __restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) flag[i] = key_id(key[i], core_bit) == (uint32_t)i ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void label_kernel(const uint32_t* __restrict__ key,
                                                       const uint32_t* __restrict__ rnk,
                                                       const uint32_t* __restrict__ flag,
                                                       uint64_t n, int core_bit,
                                                       int32_t* __restrict__ labels,
                                                       uint8_t* __restrict__ core_out,
                                                       int64_t* __restrict__ ncl) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = key[i];
    const uint32_t id = key_id(k, core_bit);
    labels[i] = k == kNone ? -1 : (int32_t)rnk[id];
    if (core_bit && core_out) core_out[i] = (k != kNone && (k & kKeyCoreBit)) ? 1 : 0;
    if (i == n - 1) *ncl = (int64_t)rnk[i] + flag[i];
}

// ------------------------------------------------------------------ driver
struct EvTimer {
    Ctx& ctx;
    hipStream_t s;
    int k = 0;
    explicit EvTimer(Ctx& c, hipStream_t st) : ctx(c), s(st) {}
    void mark() {
        if (!ctx.timing) return;
        if (!ctx.ev[k]) PD_HIP(hipEventCreate(&ctx.ev[k]));
        PD_HIP(hipEventRecord(ctx.ev[k], s));
        ++k;
    }
    float span(int a, int b) {
        if (!ctx.timing || b >= k) return 0;
        float ms = 0;
        PD_HIP(hipEventElapsedTime(&ms, ctx.ev[a], ctx.ev[b]));
        return ms;
    }
};

inline unsigned blocks(uint64_t n) { return n ? (unsigned)((n + kBlock - 1) / kBlock) : 1u; }
// blocks of `sub` record tiles (init_kernel: kSubTiles, roots_kernel: kRootSub)
inline unsigned sub_blocks(uint64_t n, int sub = kSubTiles) {
    return n ? (unsigned)((n + (uint64_t)kBlock * sub - 1) / ((uint64_t)kBlock * sub)) : 1u;
}

// Exclusive scan of `tiles` per-tile counts into u64 offsets (off[tiles] =
// total); with `read_total` the total is copied back (syncs) and returned.
uint64_t tile_offsets(Ctx& ctx, uint32_t* cnt, unsigned tiles, uint64_t* off, hipStream_t s,
                      bool read_total) {
    // (cnt[tiles] = 0: written by the tile kernel's block 0, tile_count_out)
    size_t tb = 0;
    PD_HIP(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint64_t)0, (size_t)tiles + 1,
                                   rocprim::plus<uint64_t>(), s));
    void* tmp = ctx.arena.get<char>("tile_scan_tmp", tb);
    PD_HIP(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint64_t)0, (size_t)tiles + 1,
                                   rocprim::plus<uint64_t>(), s));
    if (!read_total) return 0;
    uint64_t* h = (uint64_t*)pinned(ctx, sizeof(uint64_t));
    PD_HIP(hipMemcpyAsync(h, off + tiles, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    sync(s);
    return *h;
}
inline int xsub_of(const Ctx& ctx) { return ctx.xsub < 1 ? 1 : ctx.xsub; }

// Launch helpers for the two neighbour sweeps.  The count sweep runs at 8
// waves per SIMD (64 VGPRs); its instrumented form (PD_OPT_SWEEP_STATS)
// without the register cap.
template <typename T, int D, int M, bool ST>
void launch_count(hipStream_t s, const T* Xs, uint32_t R, const Cells& C, double eps, double eps2,
                  float lo, float hi, uint32_t ms, int full, uint32_t rot_min, uint8_t* core,
                  uint32_t* mn, uint32_t* cnt, unsigned long long* st) {
    if constexpr (ST)
        hipLaunchKernelGGL((count4_kernel<T, D, M, true, 1>), dim3(blocks(R)), dim3(kBlock), 0, s,
                           Xs, R, C, eps, eps2, lo, hi, ms, full, rot_min, core, mn, cnt, st, 0u);
    else
        hipLaunchKernelGGL((count4_kernel<T, D, M, false, kCountWpe>), dim3(blocks(R)), dim3(kBlock), 0, s,
                           Xs, R, C, eps, eps2, lo, hi, ms, full, rot_min, core, mn, cnt, st, 0u);
}

// PD_OPT_COUNT_REPLAY (measurement): the shipped count sweep over `reps`
// replicas of the R records (lane i sweeps record i % R), timed with its own
// events into PD_T_COUNT_KERNEL.
template <typename T, int D, int M>
float replay_count(hipStream_t s, const T* Xs, uint32_t R, uint32_t reps, const Cells& C,
                   double eps, double eps2, float lo, float hi, uint32_t ms, int full,
                   uint32_t rot_min, uint8_t* core, uint32_t* mn, uint32_t* cnt) {
    const uint64_t RL = (uint64_t)R * reps;
    if (RL >= 0xFFFFFFFFull) throw Error(-1, "count replay: more than 2^32 - 1 lanes");
    hipEvent_t e0, e1;
    PD_HIP(hipEventCreate(&e0));
    PD_HIP(hipEventCreate(&e1));
    PD_HIP(hipEventRecord(e0, s));
    hipLaunchKernelGGL((count4_kernel<T, D, M, false, kCountWpe, true>), dim3(blocks(RL)), dim3(kBlock), 0,
                       s, Xs, (uint32_t)RL, C, eps, eps2, lo, hi, ms, full, rot_min, core, mn, cnt,
                       (unsigned long long*)nullptr, R);
    PD_HIP(hipEventRecord(e1, s));
    PD_HIP(hipEventSynchronize(e1));
    float msec = 0;
    PD_HIP(hipEventElapsedTime(&msec, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return msec;
}

template <typename T, int D, int M>
void launch_border(hipStream_t s, const T* Xs, uint32_t NL, const uint32_t* list, const Cells& C,
                   double eps, double eps2, float lo, float hi, const uint32_t* vals,
                   const uint32_t* par, const uint32_t* gmin, uint32_t* key_out,
                   uint32_t* rec_out = nullptr) {
    hipLaunchKernelGGL((border4_kernel<T, D, M, kBorderWpe>), dim3(blocks(NL)), dim3(kBlock), 0, s, Xs, NL,
                       list, C, eps, eps2, lo, hi, vals, par, gmin, key_out, rec_out);
}

// The record sort: the library's onesweep (rsort.hpp), stable, bits [0,
// key_bits).  Its look-back words and ticket live in the arena and are
// zeroed only when (re)allocated.  hist_zeroed (required): true only where
// the caller knows "rsort_hist" was zeroed on the stream since its last use
// (the train's halo tile pass does it; the scan then overwrites the
// histograms with offsets, so a second sort must pass false).
// (PD_SORT_ROCPRIM=1 builds rocPRIM's radix_sort_pairs instead, for A/B runs.)
template <typename K>
void sort_records(Ctx& ctx, K*& keys, uint32_t*& vals, K* keys2, uint32_t* vals2, uint64_t R,
                  int key_bits, hipStream_t s, bool hist_zeroed) {
#if PD_SORT_ROCPRIM
    rocprim::double_buffer<K> kb(keys, keys2);
    rocprim::double_buffer<uint32_t> vb(vals, vals2);
    size_t tb = 0;
    PD_HIP(rocprim::radix_sort_pairs(nullptr, tb, kb, vb, (size_t)R, 0u, (unsigned)key_bits, s));
    void* tmp = ctx.arena.get<char>("sort_tmp", tb);
    PD_HIP(rocprim::radix_sort_pairs(tmp, tb, kb, vb, (size_t)R, 0u, (unsigned)key_bits, s));
    keys = kb.current();
    vals = vb.current();
#else
    const uint64_t tiles = rsort::tiles_for(R, (int)sizeof(K));
    const uint64_t want = std::max<uint64_t>(tiles, ctx.rs_look_tiles);
    uint64_t* look = ctx.arena.get<uint64_t>("rsort_look", want * rsort::kRadix);
    if (look != ctx.rs_look || want > ctx.rs_look_tiles) {   // new words: zero them once
        PD_HIP(hipMemsetAsync(look, 0, sizeof(uint64_t) * rsort::kRadix * want, s));
        ctx.rs_look = look;
        ctx.rs_look_tiles = want;
        ctx.rs_epoch = 0;
    }
    rsort::State st;
    st.look = look;
    st.look_tiles = ctx.rs_look_tiles;
    st.hist = ctx.arena.get<uint32_t>("rsort_hist", 8 * rsort::kRadix);
    st.ticket = ctx.arena.get<unsigned long long>("rsort_ticket", 1);   // (restarted per sort)
    st.epoch = ctx.rs_epoch;
    K* ko;
    uint32_t* vo;
    // (st.hist zeroed by the halo pass in the train)
    rsort::sort_pairs<K>(st, keys, vals, keys2, vals2, R, key_bits, s, &ko, &vo, hist_zeroed);
    ctx.rs_epoch = st.epoch;
    keys = ko;
    vals = vo;
#endif
}

// Ordered compaction of record ids satisfying `pred` (keeps the spatial
// order, so a wave's records stay neighbours).  Returns the count (syncs).
template <typename Pred>
uint32_t select_records(Ctx& ctx, const char* name, uint32_t R, Pred pred, uint32_t** out,
                        hipStream_t s) {
    uint32_t* list = ctx.arena.get<uint32_t>(name, R);
    *out = list;
    return (uint32_t)compact_ordered(ctx, "sel_cmp", (uint64_t)R, pred, list, nullptr, s);
}

// PD_CHECK_BOUNDS builds: after a checked kernel, read the violation record
// and throw with the site and the first index (nothing in normal builds).
void check_bounds(hipStream_t s, const char* kernel) {
#if PD_CHECK_BOUNDS
    unsigned long long h[2] = {0, 0};
    PD_HIP(hipStreamSynchronize(s));
    PD_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_oob), sizeof(h), 0, hipMemcpyDeviceToHost));
    if (h[0]) {
        const unsigned long long z[2] = {0, 0};
        PD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_oob), z, sizeof(z), 0, hipMemcpyHostToDevice));
        throw Error(-1, std::string("bounds check failed in ") + kernel + ": " +
                            std::to_string(h[0]) + " violation(s), first at site " +
                            std::to_string(h[1] >> 48) + " index " +
                            std::to_string(h[1] & 0xFFFFFFFFFFFFull));
    }
#else
    (void)s;
    (void)kernel;
#endif
}

// Phase A: halo records, sort, cell directory, core counts, union-find,
// component keys (marks 0..8).  Leaves its device state in ctx.st.
template <typename T, int D, typename K, int M>
void run_a(Ctx& ctx, TrainArgs& a, const std::vector<PartGrid>& hparts, uint64_t Gtot,
           int key_bits, EvTimer& tm) {
    hipStream_t s = a.stream;
    const uint64_t n = (uint64_t)a.n;
    const int P = a.P;
    // key_of accumulates cell indices in double (exact below 2^53 cells)
    if (Gtot >= (1ull << 53)) throw Error(-5, "eps grid of 2^53 cells or more");
    tm.mark();   // 0

    PartGrid* parts = ctx.arena.get<PartGrid>("parts", P);
    const T* X = (const T*)a.X;

    // the split tree (pd_train_tree): per level a label -> slot table, per
    // split (axis, new label) and the boundary — host tables first, then ONE
    // pinned block carries the grids and the tree (no sync between uploads)
    KdTree tree;
    std::vector<int32_t> t_int;
    std::vector<double> t_bd;
    if (!a.owner && a.tree_levels > 0) {
        const int nl = a.tree_levels;
        if (nl > 16) throw Error(-5, "KD split tree deeper than 16 levels");
        std::vector<int> ntab(nl, 1), toff(nl, 0), eoff(nl, 0);
        int nslot = 0, ne = 0;
        for (int l = 0; l < nl; ++l) {
            for (int k = 0; k < a.tree_sizes[l]; ++k)
                ntab[l] = std::max(ntab[l], a.tree_cur[ne + k] + 1);
            toff[l] = nslot;
            eoff[l] = ne;
            nslot += ntab[l];
            ne += a.tree_sizes[l];
        }
        t_int.assign((size_t)nslot + 2 * ne, -1);
        t_bd.assign(ne, 0.0);
        for (int l = 0; l < nl; ++l)
            for (int k = 0; k < a.tree_sizes[l]; ++k) {
                const int e = eoff[l] + k, L = a.tree_cur[e];
                if (L < 0 || L >= P || a.tree_new[e] < 0 || a.tree_new[e] >= P ||
                    a.tree_axis[e] < 0 || a.tree_axis[e] >= D || t_int[toff[l] + L] != -1)
                    throw Error(-1, "bad KD split tree");
                t_int[toff[l] + L] = k;
                t_int[nslot + 2 * e] = a.tree_axis[e];
                t_int[nslot + 2 * e + 1] = a.tree_new[e];
                t_bd[e] = a.tree_bound[e];
            }
        tree.nl = nl;
        for (int l = 0; l < nl; ++l) {
            tree.ntab[l] = ntab[l];
            tree.toff[l] = toff[l];
            tree.eoff[l] = eoff[l];
        }
        tree.nslot = nslot;
        tree.ne = ne;
    }
    {
        const size_t pb = (sizeof(PartGrid) * P + 15) & ~size_t(15);
        const size_t ib = (sizeof(int32_t) * t_int.size() + 7) & ~size_t(7);
        const size_t tb = ib + sizeof(double) * t_bd.size();
        char* h = (char*)pinned(ctx, pb + tb);
        std::memcpy(h, hparts.data(), sizeof(PartGrid) * P);
        PD_HIP(hipMemcpyAsync(parts, h, sizeof(PartGrid) * P, hipMemcpyHostToDevice, s));
        if (tree.nl) {
            std::memcpy(h + pb, t_int.data(), sizeof(int32_t) * t_int.size());
            std::memcpy(h + pb + ib, t_bd.data(), sizeof(double) * t_bd.size());
            char* dt = ctx.arena.get<char>("kd_tree", tb);
            PD_HIP(hipMemcpyAsync(dt, h + pb, tb, hipMemcpyHostToDevice, s));
            tree.slot = (const int32_t*)dt;
            tree.ax_new = (const int32_t*)dt + tree.nslot;
            tree.bound = (const double*)(dt + ib);
        }
        // (the block is next written by a D2H copy ordered after these on s,
        // and read by the host only after a sync)
    }

    // ---- halo records (R:dbscan/dbscan.py:136-151)
    const unsigned htiles = (unsigned)std::max<uint64_t>(1, (n + 4 * kBlock - 1) / (4 * kBlock));
    uint32_t* ctrs = ctx.arena.get<uint32_t>("train_ctrs", kCtrs);
    uint32_t* sort_hist = PD_SORT_ROCPRIM ? nullptr : ctx.arena.get<uint32_t>("rsort_hist", 8 * rsort::kRadix);
    uint64_t R64 = ~0ull;
    K *keys = nullptr, *keys2 = nullptr;
    uint32_t *vals = nullptr, *vals2 = nullptr;
    ctx.t.halo_fallback = 0;
    if (ctx.halo_passes == 1) {
        // single pass into buffers of a guessed capacity: n/8 + 4096 records
        // of halo copies (the BASELINE configs duplicate 0.004-1 % at full
        // size), or 5 % over the last train's records per point when that was
        // more (small sets / many partitions duplicate more); a total past it
        // reruns the two-pass form below
        const double grow = std::max(1.125, 1.05 * ctx.h1_ratio);
        const uint64_t cap = std::min<uint64_t>(
            ctx.halo_cap > 0 ? (uint64_t)ctx.halo_cap : (uint64_t)(grow * (double)n) + 4096,
            0xFFFFFFFDull);
        keys = ctx.arena.get<K>("keys", cap);
        vals = ctx.arena.get<uint32_t>("vals", cap);
        uint64_t* look = ctx.arena.get<uint64_t>("halo_look", htiles);
        auto* tick = ctx.arena.get<unsigned long long>("halo_ticket", 2);   // [0] ticket, [1] total
        if (look != ctx.h1_look || htiles > ctx.h1_look_tiles || tick != ctx.h1_tick ||
            ctx.h1_epoch >= 0x7FFFFFF0u) {   // new words: zero them once
            PD_HIP(hipMemsetAsync(look, 0, sizeof(uint64_t) * htiles, s));
            PD_HIP(hipMemsetAsync(tick, 0, sizeof(unsigned long long) * 2, s));
            ctx.h1_look = look;
            ctx.h1_look_tiles = htiles;
            ctx.h1_tick = tick;
            ctx.h1_epoch = 0;
            ctx.h1_tick0 = 0;
        }
        const uint32_t ep = ctx.h1_epoch++;
        const unsigned long long t0 = ctx.h1_tick0;
        ctx.h1_tick0 += htiles;
        if (P <= 64)
            hipLaunchKernelGGL((halo1_kernel<T, D, K, true>), dim3(htiles), dim3(kBlock), 0, s, X, n,
                               parts, P, a.owner, tree, cap, keys, vals, look, ep, tick, t0,
                               htiles, tick + 1, ctrs, sort_hist);
        else
            hipLaunchKernelGGL((halo1_kernel<T, D, K, false>), dim3(htiles), dim3(kBlock), 0, s, X,
                               n, parts, P, a.owner, tree, cap, keys, vals, look, ep, tick, t0,
                               htiles, tick + 1, ctrs, sort_hist);
        PD_HIP(hipGetLastError());
        check_bounds(s, "halo1_kernel");
        uint64_t* h = (uint64_t*)pinned(ctx, sizeof(uint64_t));
        PD_HIP(hipMemcpyAsync(h, tick + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        sync(s);
        if (*h <= cap) R64 = *h;
        ctx.t.halo_fallback = R64 == ~0ull ? 1 : 0;
    }
    if (R64 == ~0ull) {
        // two passes: tile counts, scan, write
        uint32_t* tcnt = ctx.arena.get<uint32_t>("tile_cnt", (size_t)htiles + 1);
        uint64_t* toff = ctx.arena.get<uint64_t>("tile_off", (size_t)htiles + 1);
        // the near-plane fast path needs the split tree in LDS (P <= 64)
        const bool tree_fast = ctx.halo_tree && P <= 64 && !a.owner && tree.nl &&
                               tree.nslot <= kTreeSlots && tree.ne <= kTreeSplits;
        const double marg = 2.0 * a.eps * (1.0 + 9.5367431640625e-07);
        if (tree_fast)
            hipLaunchKernelGGL((halo_tile_kernel<T, D, true>), dim3(htiles), dim3(kBlock), 0, s, X, n,
                               parts, P, tree, marg, tcnt, ctrs, sort_hist);
        else
            hipLaunchKernelGGL((halo_tile_kernel<T, D, false>), dim3(htiles), dim3(kBlock), 0, s, X,
                               n, parts, P, tree, marg, tcnt, ctrs, sort_hist);
        R64 = tile_offsets(ctx, tcnt, htiles, toff, s, true);
        if (R64 >= 0xFFFFFFFEull) throw Error(-5, "more than 2^32-2 halo records on one device");
        keys = ctx.arena.get<K>("keys", R64);
        vals = ctx.arena.get<uint32_t>("vals", R64);
        if (tree_fast)
            hipLaunchKernelGGL((halo_write_kernel<T, D, K, true, true>), dim3(htiles), dim3(kBlock), 0,
                               s, X, n, parts, P, a.owner, tree, marg, toff, R64, keys, vals);
        else if (P <= 64)
            hipLaunchKernelGGL((halo_write_kernel<T, D, K, true>), dim3(htiles), dim3(kBlock), 0, s,
                               X, n, parts, P, a.owner, tree, marg, toff, R64, keys, vals);
        else
            hipLaunchKernelGGL((halo_write_kernel<T, D, K, false>), dim3(htiles), dim3(kBlock), 0,
                               s, X, n, parts, P, a.owner, tree, marg, toff, R64, keys, vals);
        PD_HIP(hipGetLastError());
        check_bounds(s, "halo_write_kernel");
    }
    const uint32_t R = (uint32_t)R64;
    ctx.t.records = R;
    ctx.h1_ratio = n ? (double)R / (double)n : 1.0;
    keys2 = ctx.arena.get<K>("keys2", R);
    vals2 = ctx.arena.get<uint32_t>("vals2", R);
    tm.mark();   // 1

    // ---- shuffle by neighbourhood == sort by (neighbourhood, cell) key:
    // the library's onesweep (rsort.hpp: stable, one kernel per 8-bit digit,
    // C2 2.6 vs rocPRIM's 3.0 ms) over (key, id) pairs, then a gather of the
    // coordinates into key order.  (Round 5 measured an MSD bucket sort that
    // carries the coordinate rows instead — slower: C2 8.76 vs 5.91 ms, C4
    // 84 vs 64 ms; DESIGN.md §6, tools/msd_probe.hip.  Also measured: C4's
    // 37-bit keys in four passes of 10-bit digits, 1024-thread blocks —
    // sort 46.1 vs 40.6 ms, profiles/r05_v3_ab_sort_10bit.txt.)
    T* Xs = ctx.arena.get<T>("Xs", (size_t)R * Stride<D>::v);
    uint32_t* dup_list = ctx.arena.get<uint32_t>("dup_list", R);
    uint32_t* lcount = ctrs;   // dup, roots, core, border (zeroed by the halo pass)
    // the merge's representative per point, initialised for the points of the
    // duplicated records only (by the gather, which lists them), not a fill over n
    uint32_t* rep = P > 1 ? ctx.arena.get<uint32_t>("rep", n) : nullptr;
    sort_records<K>(ctx, keys, vals, keys2, vals2, (uint64_t)R, key_bits, s,
                    /*hist_zeroed=*/!PD_SORT_ROCPRIM);   // by the halo pass above
    tm.mark();   // 2
    hipLaunchKernelGGL((gather_kernel<T, D>), dim3(blocks(R)), dim3(kBlock), 0, s, X, (uint64_t)R,
                       vals, Xs, dup_list, lcount, rep);
    tm.mark();   // 3

    // ---- cell directory
#ifndef PD_NC_SYNC
#define PD_NC_SYNC 1   // (A/B builds: 0 = directory bits over the records, no sync)
#endif
    uint32_t* part_start = ctx.arena.get<uint32_t>("part_start", P + 1);
    hipLaunchKernelGGL((part_start_kernel<K>), dim3((P + 1 + 63) / 64), dim3(64), 0, s, keys,
                       (uint64_t)R, parts, P, part_start);
    uint32_t* cstart = ctx.arena.get<uint32_t>("cstart", (size_t)R + 1);
    K* ckeys = ctx.arena.get<K>("cell_keys", (size_t)R + 1);   // key of each occupied cell
    uint32_t* dncells = ctx.arena.get<uint32_t>("ncells", 4);
    if (R) {
        const unsigned ctiles = (unsigned)((R + 4 * kBlock - 1) / (4 * kBlock));
        uint32_t* ccnt = ctx.arena.get<uint32_t>("tile_cnt", (size_t)ctiles + 1);
        uint64_t* coff = ctx.arena.get<uint64_t>("tile_off", (size_t)ctiles + 1);
        hipLaunchKernelGGL((cell_tile_kernel<K>), dim3(ctiles), dim3(kBlock), 0, s, keys,
                           (uint64_t)R, ccnt);
        tile_offsets(ctx, ccnt, ctiles, coff, s, false);
        hipLaunchKernelGGL((cell_write_kernel<K>), dim3(ctiles), dim3(kBlock), 0, s, keys,
                           (uint64_t)R, coff, cstart, ckeys, dncells);
    } else {
        PD_HIP(hipMemsetAsync(cstart, 0, sizeof(uint32_t), s));
        PD_HIP(hipMemsetAsync(dncells, 0, sizeof(uint32_t), s));
    }
    // the cell count on the host (one sync): the directory passes then launch
    // over the cells, not the records (C2: 57 % of the waves, C4: 66 %)
    uint64_t cgrid0 = R;
#if PD_NC_SYNC
    if (R) {
        uint32_t* hnc = (uint32_t*)((char*)pinned(ctx, 16) + 8);
        PD_HIP(hipMemcpyAsync(hnc, dncells, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        sync(s);
        cgrid0 = std::max<uint64_t>(1, std::min<uint64_t>(*hnc, R));
    }
#endif
    // per-tile popcount prefix over a uint4 array's (x, y) bits into .z
    auto prefix_words = [&](uint4* d, uint64_t nw, bool read_total) -> uint64_t {
        const unsigned wtiles = (unsigned)std::max<uint64_t>(1, (nw + 4 * kBlock - 1) / (4 * kBlock));
        uint32_t* wcnt = ctx.arena.get<uint32_t>("tile_cnt", (size_t)wtiles + 1);
        uint64_t* woff = ctx.arena.get<uint64_t>("tile_off", (size_t)wtiles + 1);
        hipLaunchKernelGGL(dir_tile_kernel, dim3(wtiles), dim3(kBlock), 0, s, d, nw, wcnt);
        const uint64_t tot = tile_offsets(ctx, wcnt, wtiles, woff, s, read_total);
        hipLaunchKernelGGL(dir_write_kernel, dim3(wtiles), dim3(kBlock), 0, s, d, nw, woff);
        return tot;
    };
    uint64_t W;            // directory words (flat: the whole grid; paged: occupied + terminal)
    uint4* dir;
    uint4* pages = nullptr;
    if (!a.dir_paged) {
        W = (Gtot >> 6) + 2;
        dir = ctx.arena.get<uint4>("dir", W);
        PD_HIP(hipMemsetAsync(dir, 0, sizeof(uint4) * W, s));
        if (R) {
            if (sizeof(K) == 4 || key_bits <= 37)   // word ids < 2^31
                hipLaunchKernelGGL((dir_bits_kernel<K, 0, true>), dim3(blocks(cgrid0)), dim3(kBlock), 0, s,
                                   ckeys, dncells, dir);
            else
                hipLaunchKernelGGL((dir_bits_kernel<K, 0, false>), dim3(blocks(cgrid0)), dim3(kBlock), 0,
                                   s, ckeys, dncells, dir);
        }
        prefix_words(dir, W, false);
    } else {
        // pages: word masks, then the occupied words before each page (the
        // total sizes the word array: one sync); then the words themselves
        const uint64_t NP = (Gtot >> 12) + 2;
        pages = ctx.arena.get<uint4>("dir_pages", NP);
        PD_HIP(hipMemsetAsync(pages, 0, sizeof(uint4) * NP, s));
        if (R) {
            if (sizeof(K) == 4 || key_bits <= 43)   // page ids < 2^31
                hipLaunchKernelGGL((dir_bits_kernel<K, 6, true>), dim3(blocks(cgrid0)), dim3(kBlock), 0, s,
                                   ckeys, dncells, pages);
            else
                hipLaunchKernelGGL((dir_bits_kernel<K, 6, false>), dim3(blocks(cgrid0)), dim3(kBlock), 0,
                                   s, ckeys, dncells, pages);
        }
        // (the word pass launches over the cells too; without the count sync
        // it rides on this one, beside the total in the pinned block)
        if (R && !PD_NC_SYNC)
            PD_HIP(hipMemcpyAsync((char*)pinned(ctx, 16) + 8, dncells, sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, s));
        const uint64_t nw = prefix_words(pages, NP, true);
        W = nw + 1;
        dir = ctx.arena.get<uint4>("dir", W);
        if (R)
        {
            const uint32_t nch = *(const uint32_t*)((const char*)pinned(ctx, 16) + 8);
            const uint64_t wg = std::max<uint64_t>(1, std::min<uint64_t>(nch, R));
            if (sizeof(K) == 4 || key_bits <= 37)   // word ids < 2^31
                hipLaunchKernelGGL((word_write_kernel<K, true>), dim3(blocks(wg)), dim3(kBlock), 0, s,
                                   ckeys, dncells, pages, dir);
            else
                hipLaunchKernelGGL((word_write_kernel<K, false>), dim3(blocks(wg)), dim3(kBlock), 0, s,
                                   ckeys, dncells, pages, dir);
        }
        else
            PD_HIP(hipMemsetAsync(dir, 0, sizeof(uint4), s));
    }
    ctx.t.dir_words = (int64_t)W;
    PD_HIP(hipGetLastError());
    tm.mark();   // 4

    Cells C{parts, part_start, P, dir, cstart, pages};
    const double eps = a.eps, eps2 = a.eps * a.eps;
    // fp32 screening band (see Pred): thresholds rounded outward
    float slo = -1.0f, shi = INFINITY;
    {
        const double thr = a.metric == 0 ? eps2 : eps;
        if (std::is_same<T, float>::value && thr > 1e-30 && thr < 1e30 && ctx.screen) {
            slo = std::nextafter((float)(thr * (1.0 - 1.0 / 262144.0)), 0.0f);
            shi = std::nextafter((float)(thr * (1.0 + 1.0 / 262144.0)), INFINITY);
        }
    }
    uint8_t* core = ctx.arena.get<uint8_t>("core", R);
    uint32_t* mn = ctx.arena.get<uint32_t>("minnbr", 2 * (size_t)R);   // two smallest (uint2)
    uint32_t* cnt_rec = a.counts ? ctx.arena.get<uint32_t>("cnt_rec", R) : nullptr;
    unsigned long long* sst = nullptr;
    if (ctx.sweep_stats) {
        sst = ctx.arena.get<unsigned long long>("sweep_stats", 10);
        PD_HIP(hipMemsetAsync(sst, 0, sizeof(unsigned long long) * 10, s));
    }
    // the auto window's cell count (link step 2) is copied back before the
    // count sweep and waited for after it is queued: the host learns it while
    // the sweep runs, and the window union launches with no gap
    uint32_t* h_nc = nullptr;
    hipEvent_t ev_nc = nullptr;
    if (R && ctx.centre_window < 0) {
        h_nc = (uint32_t*)pinned(ctx, sizeof(uint32_t));
        PD_HIP(hipEventCreateWithFlags(&ev_nc, hipEventDisableTiming));
        PD_HIP(hipMemcpyAsync(h_nc, dncells, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        PD_HIP(hipEventRecord(ev_nc, s));
    }
    if (R) {
        const uint32_t rot = ctx.count_rotate ? (uint32_t)ctx.count_rotate : 0xFFFFFFFFu;
        if (sst)
            launch_count<T, D, M, true>(s, Xs, R, C, eps, eps2, slo, shi, (uint32_t)a.min_samples,
                                        ctx.full_counts ? 1 : 0, rot, core, mn, cnt_rec, sst);
        else
            launch_count<T, D, M, false>(s, Xs, R, C, eps, eps2, slo, shi, (uint32_t)a.min_samples,
                                         ctx.full_counts ? 1 : 0, rot, core, mn, cnt_rec, sst);
        if (ctx.count_replay > 0 && !sst)
            ctx.t.count_kernel = replay_count<T, D, M>(
                s, Xs, R, (uint32_t)ctx.count_replay, C, eps, eps2, slo, shi,
                (uint32_t)a.min_samples, ctx.full_counts ? 1 : 0, rot, core, mn, cnt_rec);
    }
    PD_HIP(hipGetLastError());
    tm.mark();   // 5

    uint32_t* par = ctx.arena.get<uint32_t>("parent", R);
    uint32_t* gmin = ctx.arena.get<uint32_t>("gmin", R);
    if (R) {
        // (1) forest from the count pass's two smallest neighbours
        uint32_t* wroot = ctx.arena.get<uint32_t>("word_root", W);
        // (single device: the n-bit component-key map of rank_roots, zeroed here)
        // (+ the root lists' counters after it, from a 128-B boundary)
        const uint64_t NW = a.phase == 0 ? (n + 31) / 32 : 0;
        const uint64_t NWz = NW ? ((NW + 31) & ~uint64_t(31)) + kRootLists * kRootCntStride : 0;
        uint32_t* kbits = NW ? ctx.arena.get<uint32_t>("key_bits", NWz) : nullptr;
        hipLaunchKernelGGL(init_kernel, dim3(sub_blocks(std::max<uint64_t>(std::max<uint64_t>(R, W), NWz))),
                           dim3(kBlock), 0, s, R, core, mn, 1, par, gmin, wroot, (uint64_t)W, kbits, NWz);
        // (2) window union.  Auto window (PD_OPT_CENTRE_WINDOW < 0): sparse
        // cells (a few records each, C2: 2.3) gain little from the window
        // beyond the fused flatten, so a short one is cheapest (C2 link 6.59
        // -> 5.96 ms at 16 -> 4; round 5: 5.45 / 5.33 / 5.42 ms at 4 / 2 / 1,
        // and 56 ms with the flatten alone); dense cells (C4 city centres)
        // want the long one (C4 link 71.5 -> 60.6 ms at 4 -> 16)
        int cw = ctx.centre_window;
        // the per-cell kernels' grid: the cells when the host knows their
        // count (the auto window), else the records (a bound: the kernels
        // read the count on the device and leave past it)
        uint64_t cgrid = R;
        if (cw < 0) {
            PD_HIP(hipEventSynchronize(ev_nc));
            (void)hipEventDestroy(ev_nc);
            const uint32_t nc = *h_nc ? *h_nc : 1u;
            cgrid = std::min<uint64_t>(nc, R);
            // records per occupied cell: <= 2.5 -> 2 (C2: 2.32), <= 8 -> 8
            // (C4: 2.96, dense cities in sparse noise: link 37.1 / 32.2 /
            // 56.3 / 142.9 ms at 4 / 8 / 16 / 32; C1: 4.96, 0.58 / 0.60 /
            // 0.61 ms at 4 / 8 / 16), else 16
            cw = 2 * (uint64_t)R <= 5ull * nc ? 2 : ((uint64_t)R <= 8ull * nc ? 8 : 16);
        }
        auto go = [&](auto Wc) {
            constexpr int Wv = decltype(Wc)::value;
            if (sst)
                hipLaunchKernelGGL((window_uf_kernel<T, D, M, Wv, true>), dim3(blocks(R)),
                                   dim3(kBlock), 0, s, Xs, R, eps, eps2, slo, shi, par, sst);
            else
                hipLaunchKernelGGL((window_uf_kernel<T, D, M, Wv, false>), dim3(blocks(R)),
                                   dim3(kBlock), 0, s, Xs, R, eps, eps2, slo, shi, par, sst);
        };
        if (cw <= 2)
            go(std::integral_constant<int, 2>{});
        else if (cw <= 4)
            go(std::integral_constant<int, 4>{});
        else if (cw <= 8)
            go(std::integral_constant<int, 8>{});
        else if (cw <= 16)
            go(std::integral_constant<int, 16>{});
        else if (cw <= 32)
            go(std::integral_constant<int, 32>{});
        else
            go(std::integral_constant<int, 64>{});
        uint32_t* croot = ctx.arena.get<uint32_t>("cell_root", R);
        {   // (3) cell and word roots in one pass
            uint32_t* big = ctx.arena.get<uint32_t>("big_cells", R / (kWordBig + 1) + 1);
            uint32_t* mid = ctx.arena.get<uint32_t>("mid_cells", R / (kMidCell + 1) + 1);
            uint32_t* nbig = ctrs + 8;   // [0] big, [1] mid (zeroed by the halo pass)
            // (wroot starts at kNone: init_kernel)
            if ((uint64_t)W < 0xFFFFFFFFull)   // directory slots < 2^32 - 1
                hipLaunchKernelGGL((cell_word_root_kernel<K, true>), dim3(blocks(cgrid)), dim3(kBlock), 0,
                                   s, cstart, dncells, ckeys, par, croot, wroot, mid, nbig + 1, big,
                                   nbig, pages);
            else
                hipLaunchKernelGGL((cell_word_root_kernel<K, false>), dim3(blocks(cgrid)), dim3(kBlock),
                                   0, s, cstart, dncells, ckeys, par, croot, wroot, mid, nbig + 1,
                                   big, nbig, pages);
            hipLaunchKernelGGL((mid_cell_word_root_kernel<K>), dim3(2048), dim3(kBlock), 0, s,
                               cstart, ckeys, mid, nbig + 1, par, croot, wroot, pages);
            hipLaunchKernelGGL((big_cell_word_root_kernel<K>), dim3(1024), dim3(kBlock), 0, s,
                               cstart, ckeys, big, nbig, par, croot, wroot, pages);
        }
        const uint32_t pcap = (uint32_t)std::min<uint64_t>(R, 64ull << 20);
        uint2* plist = ctx.arena.get<uint2>("pair_list", pcap);
        uint32_t* pcount = ctrs + 10;   // (zeroed by the halo pass)
        // (4) verify: screen every cell, then work on the flagged ones only
        const unsigned vtiles = blocks(cgrid);
        uint8_t* vflag = ctx.arena.get<uint8_t>("verify_flags", R);
        uint32_t* vlist = ctx.arena.get<uint32_t>("verify_list", R);
        uint32_t* vcnt = ctx.arena.get<uint32_t>("tile_cnt", (size_t)vtiles + 1);
        uint64_t* voff = ctx.arena.get<uint64_t>("tile_off", (size_t)vtiles + 1);
        if (ctx.verify_fused) {
            // one pass over every cell: the screen's test inline (no flags,
            // no list, no scan, no host read of the flagged count)
            hipLaunchKernelGGL((cell_verify_kernel<T, D, M, K>), dim3(vtiles), dim3(kBlock), 0, s,
                               Xs, keys, nullptr, 0u, croot, wroot, C, xsub_of(ctx), eps, eps2,
                               slo, shi, par, plist, pcap, pcount, sst, dncells);
        } else {
            hipLaunchKernelGGL((verify_screen_kernel<D, K>), dim3(vtiles), dim3(kBlock), 0, s, keys,
                               dncells, croot, wroot, C, xsub_of(ctx), vflag, vcnt);
            const uint32_t NV = (uint32_t)tile_offsets(ctx, vcnt, vtiles, voff, s, true);
            if (NV) {
                hipLaunchKernelGGL(flag_list_kernel, dim3(vtiles), dim3(kBlock), 0, s, vflag, dncells,
                                   voff, vlist);
                hipLaunchKernelGGL((cell_verify_kernel<T, D, M, K>), dim3(blocks(NV)), dim3(kBlock), 0,
                                   s, Xs, keys, vlist, NV, croot, wroot, C, xsub_of(ctx), eps, eps2,
                                   slo, shi, par, plist, pcap, pcount, sst, nullptr);
            }
        }
        hipLaunchKernelGGL((pair_kernel<T, D, M>), dim3(std::min(blocks(pcap), 4096u)), dim3(kBlock), 0, s, Xs, plist,
                           pcount, pcap, cstart, croot, eps, eps2, slo, shi, par);
    }
    PD_HIP(hipGetLastError());
    tm.mark();   // 6
    if (P > 1 && R) {
        // the merge touches only the records of points in several neighbourhoods
        const unsigned gb = std::min(blocks(R), 2048u);
        hipLaunchKernelGGL(rep_kernel, dim3(gb), dim3(kBlock), 0, s, dup_list, lcount, vals, par,
                           rep);
        hipLaunchKernelGGL(merge_kernel, dim3(gb), dim3(kBlock), 0, s, dup_list, lcount, vals, rep,
                           par);
    }
    tm.mark();   // 7
    if (R) {
        // single device: the component keys are ranked here (labels);
        // sharded: keys stay global ids (merge first)
        // (gmin starts at kNone: init_kernel)
        const unsigned rb = sub_blocks(R, kRootSub);
        const uint32_t seg = ((rb + kRootLists - 1) / kRootLists) * (uint32_t)(kRootSub * kBlock);
        const uint64_t NW = a.phase == 0 ? (n + 31) / 32 : 0;
        uint32_t* rlist = NW ? ctx.arena.get<uint32_t>("root_list", (size_t)seg * kRootLists) : nullptr;
        uint32_t* rcnt = NW ? ctx.arena.get<uint32_t>("key_bits", 1) + ((NW + 31) & ~uint64_t(31))
                            : nullptr;   // (zeroed by init_kernel)
        hipLaunchKernelGGL(roots_kernel, dim3(rb), dim3(kBlock), 0, s, R, vals, a.gid, par, gmin, rlist,
                           rcnt, seg, lcount + 1, ctx.sweep_stats ? 1 : 0);
        if (a.phase == 0) {
            // rank the component keys on the device; the component count is
            // read with the train's last copy back (finish)
            uint32_t* kbits = ctx.arena.get<uint32_t>("key_bits", 1);
            uint32_t* kpre = ctx.arena.get<uint32_t>("key_pre", NW);
            const unsigned gb = kRootLists * 16;
            hipLaunchKernelGGL(root_mark_kernel, dim3(gb), dim3(kBlock), 0, s, rlist, rcnt, seg, gmin,
                               kbits);
            rocprim::transform_iterator<const uint32_t*, PopcOp, uint32_t> pc(kbits, PopcOp{});
            size_t tb = 0;
            PD_HIP(rocprim::exclusive_scan(nullptr, tb, pc, kpre, 0u, (size_t)NW,
                                           rocprim::plus<uint32_t>(), s));
            void* tmp = ctx.arena.get<char>("key_scan_tmp", tb);
            PD_HIP(rocprim::exclusive_scan(tmp, tb, pc, kpre, 0u, (size_t)NW,
                                           rocprim::plus<uint32_t>(), s));
            hipLaunchKernelGGL(root_rank_kernel, dim3(gb), dim3(kBlock), 0, s, rlist, rcnt, seg, kbits,
                               kpre, NW, gmin, lcount + 1);
        } else if (ctx.sweep_stats) {
            uint32_t* h = (uint32_t*)pinned(ctx, sizeof(uint32_t) * 4);
            PD_HIP(hipMemcpyAsync(h, lcount + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            sync(s);
            ctx.t.core_records = h[0];
        }
    }
    ctx.st.n_roots = 0;   // single device: set by finish
    PD_HIP(hipGetLastError());
    tm.mark();   // 8

    PhaseState& st = ctx.st;
    st.R = R;
    st.n = n;
    st.G = Gtot;
    st.P = P;
    st.d = D;
    st.dtype = std::is_same<T, float>::value ? 0 : 1;
    st.metric = M;
    st.min_samples = a.min_samples;
    st.key_bits = key_bits;
    st.eps = a.eps;
    st.slo = slo;
    st.shi = shi;
    st.Xs = Xs;
    st.parts = parts;
    st.part_start = part_start;
    st.dir = dir;
    st.pages = pages;
    st.cstart = cstart;
    st.vals = vals;
    st.core = core;
    st.par = par;
    st.gmin = gmin;
    st.cnt_rec = cnt_rec;
    st.mn = mn;
    st.n_exports = 0;
    if (a.phase == 1 && R && a.xr) {
        uint32_t* elist = nullptr;
        const uint32_t NE = select_records(ctx, "export_list", R, IsExport{core, vals, a.xr},
                                           &elist, s);
        st.exp_gid = ctx.arena.get<uint32_t>("exp_gid", NE + 1);
        st.exp_key = ctx.arena.get<uint32_t>("exp_key", NE + 1);
        if (NE)
            hipLaunchKernelGGL(export_kernel, dim3(blocks(NE)), dim3(kBlock), 0, s, NE, elist, vals,
                               par, gmin, a.gid, st.exp_gid, st.exp_key);
        PD_HIP(hipGetLastError());
        st.n_exports = NE;
    }
    a.n_exports = st.n_exports;
    st.valid = true;
}


// Phase B: (sharded: global key remap,) owner records, border attach,
// then labels (single device) or keys (sharded).
template <typename T, int D, int M>
void run_b(Ctx& ctx, TrainArgs& a, EvTimer& tm) {
    hipStream_t s = a.stream;
    PhaseState& st = ctx.st;
    const uint64_t n = st.n;
    const uint32_t R = st.R;
    const T* Xs = (const T*)st.Xs;
    const uint32_t* vals = st.vals;
    const uint8_t* core = st.core;
    const uint32_t* par = st.par;
    uint32_t* gmin = st.gmin;
    const Cells C{(const PartGrid*)st.parts, st.part_start, st.P, (const uint4*)st.dir, st.cstart,
                  (const uint4*)st.pages};
    const double eps = st.eps, eps2 = st.eps * st.eps;
    const float slo = st.slo, shi = st.shi;
    uint32_t* shard_err = nullptr;
    if (a.phase == 2) {
        tm.mark();   // 0
        const uint32_t cm = ctx.shard_core_bit ? 0x80000000u : 0u;
        if (cm) {
            shard_err = ctx.arena.get<uint32_t>("shard_err", 1);
            PD_HIP(hipMemsetAsync(shard_err, 0, sizeof(uint32_t), s));
        }
        if ((a.n_map > 0 || cm) && R)
            hipLaunchKernelGGL(remap_kernel, dim3(blocks(R)), dim3(kBlock), 0, s, R, core, par,
                               a.map_ids, a.map_keys, (uint32_t)a.n_map, cm, gmin, shard_err);
    }
    // core flags travel in the keys: single device bit 30 (ids < 2^30);
    // sharded (global ids) bit 31 when the caller vouches for ids < 2^31
    // (PD_OPT_SHARD_CORE_BIT), else a byte scattered per owner record
    const uint32_t core_mask =
        a.phase == 2 ? (ctx.shard_core_bit ? 0x80000000u : 0u) : kKeyCoreBit;
    const int core_bit = a.phase == 2 ? 0 : 1;
    if (a.core && !core_mask) PD_HIP(hipMemsetAsync(a.core, 0, n, s));
    // single device, no counts wanted: labels reach input order through the
    // bucketed pair passes instead of owner_kernel's scatter
    // (ctx.label_buckets, PD_OPT_LABEL_BUCKETS)
    // (automatic from 2^22 points since the block-local passes: C2 1e8
    // border + label 4.35 -> 3.65 ms, C1 1e7 0.33 -> 0.29 ms, round 5)
    const bool want_buckets = ctx.label_buckets > 0 || (ctx.label_buckets < 0 && n >= (1ull << 22));
    const bool bucketed = a.phase != 2 && core_bit && !a.counts && want_buckets && n > 0;
    // block-local passes (coarse buckets split into 2^15-point ones, each
    // written from an LDS image): every label and core flag is written there,
    // so there is no key_out buffer, fill or key -> label pass.
    // PD_OPT_LABEL_BUCKETS 2: the round-4 L2-bucket scatter instead
    const uint64_t nbkL = (n + (1ull << kLabBitsL) - 1) >> kLabBitsL;
    const bool local = bucketed && R && ctx.label_buckets != 2;
    uint32_t* key_out = a.phase == 2 ? a.keys_out
                        : local      ? nullptr
                                     : ctx.arena.get<uint32_t>("key_out", n);
    if (!local) PD_HIP(hipMemsetAsync(key_out, 0xFF, sizeof(uint32_t) * n, s));
    if (R) {
        uint32_t* blist = ctx.arena.get<uint32_t>("border_list", R);
        const unsigned tiles = (unsigned)(((uint64_t)R + kOwnTile - 1) / kOwnTile);
        uint32_t* tcnt = ctx.arena.get<uint32_t>("tile_cnt", (size_t)tiles + 1);
        uint64_t* toff = ctx.arena.get<uint64_t>("tile_off", (size_t)tiles + 1);
        // bucketed: owner_kernel writes the (point, key) pairs in record order
        // instead of scattering key_out; the border sweep fills in its keys
        uint2* recs = bucketed ? ctx.arena.get<uint2>("lab_recs", R) : nullptr;
        // count4 flags records with exactly one neighbour besides themselves
        // (core bit 2): owner_kernel attaches those border records from the
        // count pass's two smallest hits, the sweep takes the rest
        hipLaunchKernelGGL(owner_kernel, dim3(tiles), dim3(kBlock), 0, s, R, vals, core, par, gmin,
                           st.cnt_rec, (const uint2*)st.mn, core_mask,
                           bucketed ? nullptr : key_out, a.core, a.counts, tcnt, recs);
        const uint32_t NB = (uint32_t)tile_offsets(ctx, tcnt, tiles, toff, s, true);
        if (NB)
            hipLaunchKernelGGL(border_list_kernel, dim3(tiles), dim3(kBlock), 0, s, R, vals, core,
                               toff, blist);
        if (NB)
            launch_border<T, D, M>(s, Xs, NB, blist, C, eps, eps2, slo, shi, vals, par, gmin,
                                   key_out, recs ? (uint32_t*)recs + 1 : nullptr);
        if (local) {
            int kLabBits = 19;
            while (((n + (1ull << kLabBits) - 1) >> kLabBits) > (uint64_t)kLabMaxBk) ++kLabBits;
            const int nbk = (int)((n + (1ull << kLabBits) - 1) >> kLabBits);
            const int sb = kLabBits - kLabBitsL;
            if (nbk > kLabMaxBk || sb > 6) throw Error(-5, "label buckets: too many points");
            uint32_t* bcnt = ctx.arena.get<uint32_t>("lab_bcnt", (size_t)nbk);
            uint2* pairs = ctx.arena.get<uint2>("lab_pairs", (size_t)nbk << kLabBits);
            const size_t nsub = (size_t)nbk << sb;   // >= nbkL
            uint32_t* bcnt2 = ctx.arena.get<uint32_t>("lab_bcnt2", nsub);
            uint2* pairs2 = ctx.arena.get<uint2>("lab_pairs2", (size_t)nbkL << kLabBitsL);
            PD_HIP(hipMemsetAsync(bcnt, 0, sizeof(uint32_t) * nbk, s));
            PD_HIP(hipMemsetAsync(bcnt2, 0, sizeof(uint32_t) * nsub, s));
            const unsigned ltiles = (unsigned)(((uint64_t)R + kLabTile - 1) / kLabTile);
            hipLaunchKernelGGL((label_bucket_kernel<kLabPer, kLabMaxBk>), dim3(ltiles),
                               dim3(kLabBlock), 0, s, R, recs, kLabBits, nbk, bcnt, pairs);
            constexpr uint32_t tile = kLabBlock * kLabPerL;
            const uint32_t tpb = ((1u << kLabBits) + tile - 1) / tile;
            hipLaunchKernelGGL(label_split_kernel, dim3((unsigned)nbk * tpb), dim3(kLabBlock), 0, s,
                               pairs, bcnt, kLabBits, tpb, bcnt2, pairs2);
            hipLaunchKernelGGL(label_local_kernel, dim3((unsigned)nbkL), dim3(kLabBlock), 0, s,
                               pairs2, bcnt2, (uint64_t)n, a.labels, a.core);
        } else if (bucketed) {
            // buckets of 2^19 points: a bucket's 2 MB of key_out stays in one
            // XCD's 4 MB L2 (C4 border: 2^20 29.2, 2^19 27.9, 2^18 29.5 ms)
            int kLabBits = 19;
            while (((n + (1ull << kLabBits) - 1) >> kLabBits) > (uint64_t)kLabMaxBk) ++kLabBits;
            const int nbk = (int)((n + (1ull << kLabBits) - 1) >> kLabBits);
            if (nbk > kLabMaxBk) throw Error(-5, "label buckets: too many points");
            uint32_t* bcnt = ctx.arena.get<uint32_t>("lab_bcnt", (size_t)nbk);
            uint2* pairs = ctx.arena.get<uint2>("lab_pairs", (size_t)nbk << kLabBits);
            PD_HIP(hipMemsetAsync(bcnt, 0, sizeof(uint32_t) * nbk, s));
            const unsigned ltiles = (unsigned)(((uint64_t)R + kLabTile - 1) / kLabTile);
            hipLaunchKernelGGL((label_bucket_kernel<kLabPer, kLabMaxBk>), dim3(ltiles),
                               dim3(kLabBlock), 0, s, R, recs,
                               kLabBits, nbk, bcnt, pairs);
            const unsigned bpb = (1u << kLabBits) / (kBlock * 8);
            hipLaunchKernelGGL(label_scatter_kernel, dim3((unsigned)nbk * bpb), dim3(kBlock), 0, s,
                               pairs, bcnt, kLabBits, nbk, bpb, key_out);
        }
    }
    PD_HIP(hipGetLastError());
    tm.mark();   // 9 (phase 2: 1)
    if (a.phase == 2) {
        if (core_mask && n)
            hipLaunchKernelGGL(split_core_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, key_out, n,
                               core_mask, a.core);
        PD_HIP(hipGetLastError());
        tm.mark();
        if (shard_err) {   // PD_OPT_SHARD_CORE_BIT's guarantee, checked
            uint32_t* h = (uint32_t*)pinned(ctx, sizeof(uint32_t));
            PD_HIP(hipMemcpyAsync(h, shard_err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            sync(s);
            if (*h)
                throw Error(-1, "PD_OPT_SHARD_CORE_BIT: a cluster key (global id) is >= 2^31; "
                                "the keys cannot carry the core flag — unset the option");
        }
        return;
    }
    // single device: key_out already holds ranks (root_rank_kernel)
    if (n && !local)
        hipLaunchKernelGGL(final_label_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, key_out, n,
                           a.labels, a.core);
    PD_HIP(hipGetLastError());
    tm.mark();   // 10
}

// Host-side bookkeeping after phase A (and B): cell count, stage times.
void finish(Ctx& ctx, TrainArgs& a, EvTimer& tm) {
    hipStream_t s = a.stream;
    if (a.phase != 2) {
        // cell count, and (single device) the component count and core
        // records (roots_kernel's counters): one copy back, one sync
        uint32_t* hnc = (uint32_t*)pinned(ctx, 4 * sizeof(uint32_t));
        hnc[0] = hnc[1] = hnc[2] = 0;
        if (ctx.st.R) {
            PD_HIP(hipMemcpyAsync(hnc, ctx.arena.get<uint32_t>("ncells", 4), sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, s));
            if (a.phase == 0)
                PD_HIP(hipMemcpyAsync(hnc + 1, ctx.arena.get<uint32_t>("train_ctrs", kCtrs) + 1,
                                      2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        }
        sync(s);
        ctx.t.cells_n = hnc[0];
        if (a.phase == 0) {
            ctx.st.n_roots = hnc[1];
            a.n_clusters = hnc[1];
            if (ctx.sweep_stats) ctx.t.core_records = hnc[2];
        }
        if (ctx.sweep_stats && ctx.st.R) {
            unsigned long long* hs = (unsigned long long*)pinned(ctx, 10 * sizeof(unsigned long long));
            PD_HIP(hipMemcpyAsync(hs, ctx.arena.get<unsigned long long>("sweep_stats", 10),
                                  10 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            sync(s);
            for (int k = 0; k < 10; ++k) ctx.t.sweep[k] = (int64_t)hs[k];
        }
        ctx.t.grid_cells = (int64_t)ctx.st.G;
        ctx.t.key_bits = ctx.st.key_bits;
    } else {
        sync(s);
    }
    if (!ctx.timing) return;
    if (a.phase == 2) {
        ctx.t.border = tm.span(0, 1);
        ctx.t.label = tm.span(1, 2);
        ctx.t.total += tm.span(0, 2);
        return;
    }
    ctx.t.halo = tm.span(0, 1);
    ctx.t.sort = tm.span(1, 2);
    ctx.t.gather = tm.span(2, 3);
    ctx.t.cells = tm.span(3, 4);
    ctx.t.count = tm.span(4, 5);
    ctx.t.link = tm.span(5, 6);
    ctx.t.merge = tm.span(6, 7);
    ctx.t.roots = tm.span(7, 8);
    if (a.phase == 1) {
        ctx.t.total = tm.span(0, 8);
        return;
    }
    ctx.t.border = tm.span(8, 9);
    ctx.t.label = tm.span(9, 10);
    ctx.t.total = tm.span(0, 10);
}

template <typename T, int D, typename K, int M>
void run(Ctx& ctx, TrainArgs& a, const std::vector<PartGrid>& hparts, uint64_t Gtot,
         int key_bits) {
    EvTimer tm(ctx, a.stream);
    run_a<T, D, K, M>(ctx, a, hparts, Gtot, key_bits, tm);
    if (a.phase == 0) run_b<T, D, M>(ctx, a, tm);
    finish(ctx, a, tm);
}

template <typename T, int D>
void run_b_m(Ctx& ctx, TrainArgs& a) {
    EvTimer tm(ctx, a.stream);
    if (ctx.st.metric == 0)
        run_b<T, D, 0>(ctx, a, tm);
    else
        run_b<T, D, 1>(ctx, a, tm);
    finish(ctx, a, tm);
}

template <typename T>
void run_b_d(Ctx& ctx, TrainArgs& a) {
    switch (ctx.st.d) {
        case 1: run_b_m<T, 1>(ctx, a); break;
        case 2: run_b_m<T, 2>(ctx, a); break;
        case 3: run_b_m<T, 3>(ctx, a); break;
        case 4: run_b_m<T, 4>(ctx, a); break;
        default: throw Error(-5, "grid path supports d <= 4");
    }
}

template <typename T, int D, typename K>
void run_m(Ctx& ctx, TrainArgs& a, const std::vector<PartGrid>& p, uint64_t G, int kb) {
    if (a.metric == 0)
        run<T, D, K, 0>(ctx, a, p, G, kb);
    else
        run<T, D, K, 1>(ctx, a, p, G, kb);
}

template <typename T, typename K>
void run_d(Ctx& ctx, TrainArgs& a, const std::vector<PartGrid>& p, uint64_t G, int kb) {
    switch (a.d) {
        case 1: run_m<T, 1, K>(ctx, a, p, G, kb); break;
        case 2: run_m<T, 2, K>(ctx, a, p, G, kb); break;
        case 3: run_m<T, 3, K>(ctx, a, p, G, kb); break;
        case 4: run_m<T, 4, K>(ctx, a, p, G, kb); break;
        default: throw Error(-5, "grid path supports d <= 4");
    }
}

}  // namespace

// pd_sort_pairs: the record sort on caller arrays (in place, stable).
void sort_pairs_inplace(Ctx& ctx, void* keys, int key_bytes, uint32_t* vals, uint64_t n,
                        int key_bits, hipStream_t s) {
    if (n == 0) return;
    auto go = [&](auto* k) {
        using K = std::remove_pointer_t<decltype(k)>;
        K* kk = k;
        uint32_t* vv = vals;
        K* k2 = ctx.arena.get<K>("usort_keys2", n);
        uint32_t* v2 = ctx.arena.get<uint32_t>("usort_vals2", n);
        sort_records<K>(ctx, kk, vv, k2, v2, n, key_bits, s, false);
        if (kk != k) {
            PD_HIP(hipMemcpyAsync(k, kk, sizeof(K) * n, hipMemcpyDeviceToDevice, s));
            PD_HIP(hipMemcpyAsync(vals, vv, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s));
        }
    };
    if (key_bytes == 4)
        go((uint32_t*)keys);
    else
        go((uint64_t*)keys);
    PD_HIP(hipGetLastError());
}


// Labels from cluster keys (key[i] = smallest core point id of i's cluster,
// 0xFFFFFFFF noise): a key's rank among the cluster roots (points whose key
// is their own id) is the label — sklearn's numbering.  Async on s; the
// cluster count is read back by rank_labels_count.
void rank_labels_async(Ctx& ctx, const uint32_t* key, uint64_t n, int32_t* labels,
                       hipStream_t s, int core_bit, uint8_t* core_from_key) {
    uint32_t* rflag = ctx.arena.get<uint32_t>("rflag", n);
    uint32_t* rnk = ctx.arena.get<uint32_t>("rnk", n);
    int64_t* dncl = ctx.arena.get<int64_t>("ncl", 2);
    PD_HIP(hipMemsetAsync(dncl, 0, sizeof(int64_t), s));
    if (n) {
        hipLaunchKernelGGL(root_flag_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, key, n, core_bit,
                           rflag);
        size_t tb = 0;
        PD_HIP(rocprim::exclusive_scan(nullptr, tb, rflag, rnk, 0u, (size_t)n,
                                       rocprim::plus<uint32_t>(), s));
        void* tmp = ctx.arena.get<char>("scan_tmp", tb);
        PD_HIP(rocprim::exclusive_scan(tmp, tb, rflag, rnk, 0u, (size_t)n,
                                       rocprim::plus<uint32_t>(), s));
        hipLaunchKernelGGL(label_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, key, rnk, rflag, n,
                           core_bit, labels, core_from_key, dncl);
    }
    PD_HIP(hipGetLastError());
}

int64_t rank_labels_count(Ctx& ctx, hipStream_t s) {
    int64_t* hres = (int64_t*)pinned(ctx, sizeof(int64_t));
    PD_HIP(hipMemcpyAsync(hres, ctx.arena.get<int64_t>("ncl", 2), sizeof(int64_t),
                          hipMemcpyDeviceToHost, s));
    sync(s);
    return hres[0];
}

void train(Ctx& ctx, TrainArgs& a) {
    if (a.phase == 2) {   // resume a sharded train after the global key merge
        PhaseState& st = ctx.st;
        if (!st.valid) throw Error(-1, "pd_train_end without a matching pd_train_begin");
        if (a.n != (int64_t)st.n) throw Error(-1, "pd_train_end: n differs from pd_train_begin");
        if (!a.keys_out && a.n) throw Error(-1, "keys output is required");
        if (a.n) {
            if (st.dtype == 0)
                run_b_d<float>(ctx, a);
            else
                run_b_d<double>(ctx, a);
        }
        st.valid = false;
        return;
    }
    ctx.st.valid = false;
    if (a.n < 0 || a.d < 1) throw Error(-1, "invalid shape");
    if (!(a.eps > 0) || !std::isfinite(a.eps)) throw Error(-1, "eps must be a finite value > 0");
    if (a.min_samples < 1) throw Error(-1, "min_samples must be >= 1");
    if (a.metric != 0 && a.metric != 1) throw Error(-1, "metric must be 0 (euclidean) or 1 (cityblock)");
    if (a.P < 1) throw Error(-1, "need at least one neighbourhood");
    if (a.n > (int64_t)kIdMask) throw Error(-5, "n must be < 2^30 points per device");
    if (a.phase == 0 && !a.labels && a.n) throw Error(-1, "labels output is required");
    ctx.t = Timings{};
    if (a.d > kMaxDim) {
        // dense tiles (dense.hip): one pass over all points; the halo + merge
        // of the neighbourhoods would reproduce exactly this global answer
        std::vector<double> dbox(2 * (size_t)a.d);
        if (a.data_box) {
            std::memcpy(dbox.data(), a.data_box, sizeof(double) * 2 * a.d);
        } else if (a.n) {
            int64_t bad = 0;
            bbox(ctx, a.X, a.dtype, a.n, a.d, dbox.data(), &bad, a.stream);
            if (bad) throw Error(-1, "input contains NaN or infinity");
        }
        if (a.n == 0) {
            if (a.phase == 1) throw Error(-5, "the sharded train is built for d <= 4 only");
            a.n_clusters = 0;
            return;
        }
        a.data_box = dbox.data();
        dense_train(ctx, a);
        a.data_box = nullptr;
        return;
    }
    const int d = a.d;
    double box[2 * kMaxDim];
    if (a.data_box) {
        std::memcpy(box, a.data_box, sizeof(double) * 2 * d);
    } else if (a.n) {
        int64_t bad = 0;
        bbox(ctx, a.X, a.dtype, a.n, d, box, &bad, a.stream);
        if (bad) throw Error(-1, "input contains NaN or infinity");
    }
    if (a.n == 0) {
        a.n_clusters = 0;
        a.n_exports = 0;
        if (a.phase == 1) {
            ctx.st = PhaseState{};
            ctx.st.valid = true;
        }
        return;
    }
    // per-neighbourhood grids.  Cells are eps (eps/xsub along axis 0) wide.
    // The directory is flat (20 B per 64 cells of the bounding box:
    // occupancy word + word root) or paged (16 B per 4096 cells + the
    // occupied words; PD_OPT_DIR_PAGED, automatic for sparse grids); when its
    // extent-dependent part would pass the budget (PD_OPT_DIR_BUDGET, default
    // 32 GiB), every cell grows by a common factor k >= 1 until it fits.  Any width >=
    // eps is exact: the sweeps derive their candidate ranges from the cell
    // geometry (chords along axis 0, rows +-1 beyond it) and the cell verify
    // covers +-xsub axis-0 cells of width >= eps/xsub; wider cells only add
    // candidates (globe-sized extents at a small eps).
    const int xsub = ctx.xsub < 1 ? 1 : ctx.xsub;
    std::vector<PartGrid> parts(a.P);
    uint64_t G = 0;
    const long double budget = (long double)ctx.dir_budget;
    double grow = 1.0;
    bool paged = false;
    for (int attempt = 0;; ++attempt) {
        const double cw = a.eps * (1.0 + 1.0 / 1048576.0) * grow;
        G = 0;
        bool too_big = false;
        long double gsum = 0;
        for (int L = 0; L < a.P && !too_big; ++L) {
            PartGrid& g = parts[L];
            std::memset(&g, 0, sizeof(g));
            for (int j = 0; j < d; ++j) {
                g.cs[j] = j == 0 ? cw / (double)xsub : cw;
                g.inv[j] = j == 0 ? (double)xsub / cw : 1.0 / cw;
            }
            g.base = G;
            bool empty = false;
            long double cells = 1;
            for (int j = 0; j < d; ++j) {
                g.elo[j] = a.ebox[(size_t)L * 2 * d + j];
                g.ehi[j] = a.ebox[(size_t)L * 2 * d + d + j];
                const double lo = std::max(g.elo[j], box[j]);
                const double hi = std::min(g.ehi[j], box[d + j]);
                if (!(lo <= hi)) empty = true;
                g.lo[j] = lo;
                if (!empty) {
                    const double nc = std::floor((hi - lo) * g.inv[j]) + 1.0;
                    if (!(nc < 4.0e18)) {
                        too_big = true;
                        break;
                    }
                    g.nc[j] = (int64_t)nc;
                    cells *= (long double)g.nc[j];
                }
            }
            if (too_big) break;
            for (int j = 0; j < d; ++j) {
                float fl = (float)g.elo[j], fh = (float)g.ehi[j];
                if ((double)fl < g.elo[j]) fl = std::nextafter(fl, INFINITY);
                if ((double)fh > g.ehi[j]) fh = std::nextafter(fh, -INFINITY);
                g.flo[j] = fl;
                g.fhi[j] = fh;
            }
            if (empty) {
                for (int j = 0; j < d; ++j) {
                    g.nc[j] = 0;
                    g.elo[j] = g.flo[j] = INFINITY;   // a box no point is in
                    g.ehi[j] = g.fhi[j] = -INFINITY;
                }
                continue;
            }
            gsum += cells;
            if (gsum > 4.0e18L) {
                too_big = true;
                break;
            }
            G += (uint64_t)cells;
        }
        // the extent-dependent bytes: flat, 20 B per 64 cells of the grid;
        // paged, 16 B per 4096 cells (its occupied words, 20 B each, follow
        // the data like the records do, not the extent)
        const long double words = gsum / 64.0L;
        paged = ctx.dir_paged > 0 ||
                (ctx.dir_paged < 0 && (words > (long double)a.n || words * 20.0L > budget));
        const long double dir_bytes =
            too_big ? 1e30L : (paged ? gsum / 4096.0L * 16.0L : words * 20.0L);
        if (dir_bytes <= budget) break;
        if (attempt >= 64 || !std::isfinite(grow * 2.0))
            throw Error(-5, "eps-grid directory does not fit the budget at any cell size");
        // the directory shrinks by k^d: aim below the budget in one step
        double k = too_big ? 1024.0
                           : (double)std::pow((double)(dir_bytes / budget), 1.0 / (double)d) * 1.01;
        grow *= std::max(k, 1.25);
    }
    ctx.t.grid_grow = grow;
    ctx.t.dir_paged = paged ? 1 : 0;
    a.dir_paged = paged;
    int key_bits = 1;
    while (key_bits < 64 && ((G - (G ? 1 : 0)) >> key_bits)) ++key_bits;
    if (a.dtype == 0) {
        if (G < 0xFFFFFFFFull)
            run_d<float, uint32_t>(ctx, a, parts, G, key_bits);
        else
            run_d<float, uint64_t>(ctx, a, parts, G, key_bits);
    } else if (a.dtype == 1) {
        if (G < 0xFFFFFFFFull)
            run_d<double, uint32_t>(ctx, a, parts, G, key_bits);
        else
            run_d<double, uint64_t>(ctx, a, parts, G, key_bits);
    } else {
        throw Error(-1, "dtype must be 0 (float32) or 1 (float64)");
    }
}

}  // namespace pd
