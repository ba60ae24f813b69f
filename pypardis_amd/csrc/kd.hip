// KD partition stages: R:dbscan/partition.py:33-183 on the device.
//
//  bbox       — data.aggregate(BoundingBox(k), union)          partition.py:135-137
//  kd_moments — aggregate of [1, v, v**2] per label            partition.py:86-89
//  kd_counts  — aggregate of 2*(v[axis] < bounds) - 1          partition.py:60-63
//  kd_split   — filter(v[axis] >= boundary) -> next_label      partition.py:66-68
//  halo_members — DBSCAN._create_neighborhoods membership      dbscan.py:136-151
//
// The host keeps the reference's scalar arithmetic (mean, variance, the 7
// candidate bounds, argmin) in numpy; only the per-point passes live here.
// Every reduction is deterministic: per-block partials in a fixed order, then
// a fixed-order host sum.  HBM-bound streaming passes (one read of X each).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <cmath>
#include <cstring>
#include <vector>

#include "internal.hpp"
#include "stream.hpp"

namespace pd {
namespace {

constexpr int kRedBlocks = 1024;
constexpr int kGroup = 4;   // labels per moments pass (register budget)

// Point i's D consecutive coordinates starting at X (row stride ld): the
// passes below see a d-dimensional input as chunks of <= 4 axes.
template <typename T, int D>
__device__ __forceinline__ void load_pt(const T* __restrict__ X, uint64_t i, uint32_t ld,
                                        double (&v)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (double)X[i * ld + j];
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ double wave_min(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ double wave_max(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    return x;
}

// ---------------------------------------------------------------- bbox
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void bbox_kernel(const T* __restrict__ X, uint64_t n,
                                                      uint32_t ld, double* __restrict__ part) {
    double lo[D], hi[D];
    double bad = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        lo[j] = INFINITY;
        hi[j] = -INFINITY;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        double v[D];
        load_pt<T, D>(X, i, ld, v);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (!isfinite(v[j])) bad += 1;
            lo[j] = fmin(lo[j], v[j]);
            hi[j] = fmax(hi[j], v[j]);
        }
    }
    __shared__ double sm[kBlock / 64][2 * D + 1];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        double a = wave_min(lo[j]), b = wave_max(hi[j]);
        if (l == 0) {
            sm[w][j] = a;
            sm[w][D + j] = b;
        }
    }
    double bb = wave_sum(bad);
    if (l == 0) sm[w][2 * D] = bb;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 0; j < D; ++j) {
            double a = sm[0][j], b = sm[0][D + j];
            for (int q = 1; q < kBlock / 64; ++q) {
                a = fmin(a, sm[q][j]);
                b = fmax(b, sm[q][D + j]);
            }
            part[blockIdx.x * (2 * D + 1) + j] = a;
            part[blockIdx.x * (2 * D + 1) + D + j] = b;
        }
        double s = 0;
        for (int q = 0; q < kBlock / 64; ++q) s += sm[q][2 * D];
        part[blockIdx.x * (2 * D + 1) + 2 * D] = s;
    }
}

// ---------------------------------------------------------------- moments
// Squares are taken in the input precision then widened, as numpy does for
// ``vector[1] ** 2`` of an fp32 vector (R:dbscan/partition.py:88).
// Sums are double-double (error-free TwoSum per term, dd merges in the
// reductions), so the result is the correctly rounded sum — independent of
// thread/block/device order.  The reference's sequential fold can differ in
// the last bits; with exact ties (e.g. StandardScaler output, where every
// axis has variance 1) only the exact value makes the argmax well defined.
struct DD {
    double hi, lo;
};

__device__ __host__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

__device__ __host__ __forceinline__ DD dd_add(DD a, DD b) {
    double s, e;
    two_sum(a.hi, b.hi, s, e);
    e += a.lo + b.lo;
    DD r;
    r.hi = s + e;
    r.lo = e - (r.hi - s);
    return r;
}

__device__ __forceinline__ void dd_acc(DD& a, double x) {
    double s, e;
    two_sum(a.hi, x, s, e);
    a.hi = s;
    a.lo += e;
}

__device__ __forceinline__ DD wave_dd(DD a) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        DD b;
        b.hi = __shfl_xor(a.hi, o, 64);
        b.lo = __shfl_xor(a.lo, o, 64);
        a = dd_add(a, b);
    }
    return a;
}

template <typename T, int D>
__global__ __launch_bounds__(kBlock) void moments_kernel(const T* __restrict__ X, uint64_t n,
                                                         uint32_t ld,
                                                         const int32_t* __restrict__ labels,
                                                         int4 sel, double* __restrict__ part) {
    double c[kGroup];
    DD s[kGroup][D], q[kGroup][D];
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
        c[g] = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) s[g][j] = q[g][j] = DD{0.0, 0.0};
    }
    const int sl[kGroup] = {sel.x, sel.y, sel.z, sel.w};
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const int lab = labels[i];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) {
            if (lab == sl[g]) {
                c[g] += 1.0;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const T v = X[i * ld + j];
                    const T vv = v * v;
                    dd_acc(s[g][j], (double)v);
                    dd_acc(q[g][j], (double)vv);
                }
            }
        }
    }
    // per block: kGroup x [count, (s.hi, s.lo) x D, (q.hi, q.lo) x D]
    constexpr int G = 1 + 4 * D;
    constexpr int W = kGroup * G;
    __shared__ double sm[kBlock / 64][W];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
        double x = wave_sum(c[g]);
        if (l == 0) sm[w][g * G] = x;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const DD a = wave_dd(s[g][j]);
            const DD b = wave_dd(q[g][j]);
            if (l == 0) {
                sm[w][g * G + 1 + 2 * j] = a.hi;
                sm[w][g * G + 2 + 2 * j] = a.lo;
                sm[w][g * G + 1 + 2 * D + 2 * j] = b.hi;
                sm[w][g * G + 2 + 2 * D + 2 * j] = b.lo;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < kGroup * (1 + 2 * D)) {
        // one thread per (group, quantity): fixed-order dd merge over waves
        const int g = threadIdx.x / (1 + 2 * D), qd = threadIdx.x % (1 + 2 * D);
        if (qd == 0) {
            double acc = 0;
            for (int k = 0; k < kBlock / 64; ++k) acc += sm[k][g * G];
            part[(uint64_t)blockIdx.x * W + g * G] = acc;
        } else {
            const int off = g * G + 1 + 2 * (qd - 1);
            DD acc{0.0, 0.0};
            for (int k = 0; k < kBlock / 64; ++k) acc = dd_add(acc, DD{sm[k][off], sm[k][off + 1]});
            part[(uint64_t)blockIdx.x * W + off] = acc.hi;
            part[(uint64_t)blockIdx.x * W + off + 1] = acc.lo;
        }
    }
}

// Reference-order variant (PD_OPT_SEQUENTIAL_MOMENTS): one lane per
// (label, axis, moment) stream folds the points left to right in index order,
// i.e. exactly ``partition.aggregate(zeros, x + [1, v, v**2], add)`` over a
// single slice (R:dbscan/partition.py:86-89).  O(n) serial per lane: a
// compatibility mode for bit-identical split boundaries, not the fast path.
template <typename T, int D>
__global__ void moments_seq_kernel(const T* __restrict__ X, uint64_t n, uint32_t ld,
                                   const int32_t* __restrict__ labels, int4 sel,
                                   double* __restrict__ out) {
    const int lane = threadIdx.x;
    if (lane >= kGroup * 2 * D) return;
    const int g = lane / (2 * D), rem = lane % (2 * D), j = rem % D, sq = rem / D;
    const int want = (&sel.x)[g];
    double acc = 0.0, cnt = 0.0;
    for (uint64_t i = 0; i < n; ++i) {
        if (labels[i] != want) continue;
        const T v = X[i * ld + j];
        const T vv = v * v;
        acc = acc + (sq ? (double)vv : (double)v);
        cnt += 1.0;
    }
    constexpr int G = 1 + 4 * D;
    // same layout as moments_kernel's block partial (lo words = 0), block 0
    out[g * G + 1 + 2 * D * sq + 2 * j] = acc;
    out[g * G + 2 + 2 * D * sq + 2 * j] = 0.0;
    if (rem == 0) out[g * G] = cnt;
}

// ---------------------------------------------------------------- fused level pass
// One streaming read of X per BFS level does everything the level can do
// without a host decision: apply the previous level's splits
// (R:dbscan/partition.py:66-68), then accumulate this level's moments
// (:86-89) over the new labels, and on the first level the bbox
// (:135-137).  Each lane takes four consecutive points per step with 16-byte
// loads (D float4 / 2D double2 per four points) and the four labels as one
// int4; split results are written back only where a label changed.
struct SplitTab {
    const int32_t* slot_of;
    int ntab;
    const int32_t* axis;
    const double* boundary;
    const int32_t* newlab;
    int nsplit;
};

// Label / split tables staged in LDS by the level kernels (larger levels
// take the one-point-per-lane kernels).
constexpr int kTabLds = 256;
// kd_pass_kernel: up to this many labels are summed per lane without the
// LDS regroup
constexpr int kDirectMax = 1;
// more labels: regroup each wave's points by label in its own LDS region
// (false: one block-wide counting sort per tile, each wave summing one label)
constexpr bool kWaveRegroup = false;   // measured slower on C2: 0.69 / 1.00 vs 0.61 / 0.82 ms

// Label replay (kd_build, round 6): instead of reading and
// writing an int32 label per point per pass, a pass recomputes each point's
// label by replaying the BFS splits decided so far on its coordinates (level
// l, the label's slot: v[axis] >= boundary moves it to the new label,
// R:dbscan/partition.py:66-68) — the halo pass's tree_owner, from tables in
// LDS.  Levels 0 .. nl-1; per level the label -> slot table and per split
// (axis, new label, boundary), the axes and boundaries as the device decided
// them (kdb_axes_kernel / kdb_boundary_kernel).
constexpr int kMaxLevels = 16, kRSlots = 512, kRSplits = 256;
struct ReplayTab {
    int nl = 0;
    int ntab[kMaxLevels], nsplit[kMaxLevels], toff[kMaxLevels], eoff[kMaxLevels];
    const int32_t* slot[kMaxLevels];
    const int32_t* axis[kMaxLevels];
    const int32_t* newlab[kMaxLevels];
    const double* boundary[kMaxLevels];
};
struct ReplayLds {
    int32_t slot[kRSlots];
    int32_t axis[kRSplits], newlab[kRSplits];
    double bd[kRSplits];
};

__device__ __forceinline__ void replay_stage(ReplayLds& R, const ReplayTab& rp, int tid, int nt) {
    for (int l = 0; l < rp.nl; ++l) {
        for (int k = tid; k < rp.ntab[l]; k += nt) R.slot[rp.toff[l] + k] = rp.slot[l][k];
        for (int k = tid; k < rp.nsplit[l]; k += nt) {
            R.axis[rp.eoff[l] + k] = rp.axis[l][k];
            R.newlab[rp.eoff[l] + k] = rp.newlab[l][k];
            R.bd[rp.eoff[l] + k] = rp.boundary[l][k];
        }
    }
}

template <typename T, int D>
__device__ __forceinline__ int replay_label(const ReplayLds& R, const ReplayTab& rp,
                                            const T (&v)[D]) {
    int lab = 0;
    for (int l = 0; l < rp.nl; ++l) {
        if (lab >= rp.ntab[l]) continue;
        const int sl = R.slot[rp.toff[l] + lab];
        if (sl < 0) continue;
        const int e = rp.eoff[l] + sl;
        if ((double)pick_axis<T, D>(v, R.axis[e]) >= R.bd[e]) lab = R.newlab[e];
    }
    return lab;
}

// NG = labels whose moments this pass accumulates (0: none); LAB: labels are
// read (false: every point has label 0, the first level); SP: the previous
// level's splits are applied first; BB: bbox + non-finite count.
//
// Moments without per-label masking: a block takes a tile of 4·K·256
// consecutive points (K four-point chunks per lane), applies the splits,
// then regroups the tile in LDS by label slot (a counting sort from wave
// ballots, deterministic) so that every wave accumulates ONE slot: wave w
// sums slot w % NG, items sub·64 + lane + k·64·(4 / NG).  The double-double
// work per point is then that of one label, whatever NG is.
// Block partials: NG x [count, (sum hi, lo) x D, (sumsq hi, lo) x D], then
// the bbox [lo x D, hi x D, bad].
// RP: labels replayed from the split tree (rp), none read or written (LAB
// and SP unused).
template <typename T, int D, bool LAB, bool SP, int NG, bool BB, bool RP = false>
__global__ __launch_bounds__(kBlock) void kd_pass_kernel(const T* __restrict__ X, uint64_t n,
                                                         int32_t* __restrict__ labels, SplitTab sp,
                                                         int4 sel, double* __restrict__ part,
                                                         ReplayTab rp) {
    constexpr int K = (sizeof(T) * D <= 16) ? 2 : 1;
    constexpr int TP = 4 * K * kBlock;   // points per tile
    constexpr int NW = kBlock / 64;
    constexpr int NGa = NG > 0 ? NG : 1;
    static_assert(NW == 4 && (NG == 0 || NG == 1 || NG == 2 || NG == 4), "wave/slot mapping");
    __shared__ T s_val[(NG > kDirectMax) ? TP * D : 1];
    __shared__ int s_wcnt[NW][NGa];
    __shared__ int s_slot[SP ? kTabLds : 1], s_ax[SP ? kTabLds : 1], s_nl[SP ? kTabLds : 1];
    __shared__ double s_bd[SP ? kTabLds : 1];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    __shared__ std::conditional_t<RP, ReplayLds, char> s_rp;
    if constexpr (RP) {
        replay_stage(s_rp, rp, tid, kBlock);
        __syncthreads();
    } else if constexpr (SP) {
        for (int k = tid; k < sp.ntab; k += kBlock) s_slot[k] = sp.slot_of[k];
        for (int k = tid; k < sp.nsplit; k += kBlock) {
            s_ax[k] = sp.axis[k];
            s_bd[k] = sp.boundary[k];
            s_nl[k] = sp.newlab[k];
        }
        __syncthreads();
    }
    const int sl[4] = {sel.x, sel.y, sel.z, sel.w};
    const int wslot = w % NGa, sub = w / NGa, nsub = NW / NGa;
    double cnt = 0;
    DD s[D], q2[D];
#pragma unroll
    for (int j = 0; j < D; ++j) s[j] = q2[j] = DD{0.0, 0.0};
    constexpr bool kDirect = NG >= 1 && NG <= kDirectMax;
    constexpr bool kWave = NG > kDirectMax && kWaveRegroup;   // wave-local regroup
    constexpr int ND = (kDirect || kWave) ? NG : 1;
    double dc[ND];
    DD ds[ND][D], dq[ND][D];
#pragma unroll
    for (int g = 0; g < ND; ++g) {
        dc[g] = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) ds[g][j] = dq[g][j] = DD{0.0, 0.0};
    }
    double lo[D], hi[D], bad = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        lo[j] = INFINITY;
        hi[j] = -INFINITY;
    }
    const uint64_t nch = (n + 3) / 4;
    const uint64_t ntile = (n + TP - 1) / TP;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        T v[K][4][D];
        int slot[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t ch = t * (TP / 4) + (uint64_t)k * kBlock + tid;
            int m = 0;
            if (ch < nch) {
                m = load_chunk<T, D, true>(X, n, ch, v[k]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < D; ++j) v[k][q][j] = T(0);
            }
            int lab[4] = {0, 0, 0, 0};
            if constexpr (RP) {
#pragma unroll
                for (int q = 0; q < 4; ++q) lab[q] = replay_label<T, D>(s_rp, rp, v[k][q]);
            } else if constexpr (LAB) {
                if (m) load_labels4<true>(labels, ch, m, lab);
            }
            if constexpr (SP && !RP) {
                bool changed = false;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int L = lab[q];
                    if (q >= m || L < 0 || L >= sp.ntab) continue;
                    const int a = s_slot[L];
                    if (a < 0) continue;
                    const double x = (double)pick_axis<T, D>(v[k][q], s_ax[a]);
                    if (x >= s_bd[a]) {
                        lab[q] = s_nl[a];
                        changed = true;
                    }
                }
                // (!LAB: every point starts in label 0 and every label is
                // written — the caller's array need not be initialised)
                if (changed || !LAB) store_labels4<true>(labels, ch, m, lab);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                int g = -1;
#pragma unroll
                for (int h = NGa - 1; h >= 0; --h) g = (NG > 0 && lab[q] == sl[h]) ? h : g;
                slot[k][q] = q < m ? g : -1;
            }
            if constexpr (BB) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q >= m) continue;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const double x = (double)v[k][q][j];
                        if (!isfinite(x)) bad += 1;
                        lo[j] = fmin(lo[j], x);
                        hi[j] = fmax(hi[j], x);
                    }
                }
            }
        }
        if constexpr (NG >= 1 && NG <= kDirectMax) {
            // few labels: every lane sums its own points into one accumulator
            // per label (adding 0.0 to the others' is exact), no regroup
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int g = 0; g < NG; ++g) {
                        const bool on = slot[k][q] == g;
                        if (NG == 1 && !on) continue;
                        dc[g] += on ? 1.0 : 0.0;
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            const T x = on ? v[k][q][j] : T(0);
                            const T xx = x * x;   // squared in the input precision (numpy)
                            dd_acc(ds[g][j], (double)x);
                            dd_acc(dq[g][j], (double)xx);
                        }
                    }
                }
        } else if constexpr (kWave) {
            // each wave regroups its own 4·K·64 points by slot in its LDS
            // region (ballot counting sort, no block barrier), then sums each
            // slot's run into that slot's accumulators: one set of
            // double-double sums per point, no cross-wave imbalance
            constexpr int WP = 4 * K * 64;
            T* wv = s_val + (size_t)w * WP * D;
            int wc[NG], run[NG];
#pragma unroll
            for (int g = 0; g < NG; ++g) wc[g] = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int g = 0; g < NG; ++g) wc[g] += __popcll(__ballot(slot[k][q] == g));
            int acc0 = 0;
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                run[g] = acc0;
                acc0 += wc[g];
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int g = 0; g < NG; ++g) {
                        const unsigned long long b = __ballot(slot[k][q] == g);
                        if (slot[k][q] == g) {
                            const int pos = run[g] + __popcll(b & lt);
#pragma unroll
                            for (int j = 0; j < D; ++j) wv[pos * D + j] = v[k][q][j];
                        }
                        run[g] += __popcll(b);
                    }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int start = 0;
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                for (int i = lane; i < wc[g]; i += 64) {
                    const T* p = wv + (size_t)(start + i) * D;
                    dc[g] += 1.0;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const T x = p[j];
                        const T xx = x * x;   // squared in the input precision (numpy)
                        dd_acc(ds[g][j], (double)x);
                        dd_acc(dq[g][j], (double)xx);
                    }
                }
                start += wc[g];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else if constexpr (NG > 0) {
            // counting sort of the tile by slot: wave tallies, then positions
            int wc[NGa];
#pragma unroll
            for (int g = 0; g < NGa; ++g) wc[g] = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int g = 0; g < NGa; ++g) wc[g] += __popcll(__ballot(slot[k][q] == g));
            if (lane == 0)
#pragma unroll
                for (int g = 0; g < NGa; ++g) s_wcnt[w][g] = wc[g];
            __syncthreads();
            int run[NGa], seg[NGa];
            int acc = 0;
#pragma unroll
            for (int g = 0; g < NGa; ++g) {
                seg[g] = acc;
                int before = 0;
#pragma unroll
                for (int u = 0; u < NW; ++u) {
                    before += u < w ? s_wcnt[u][g] : 0;
                    acc += s_wcnt[u][g];
                }
                run[g] = seg[g] + before;
            }
            const int total = s_wcnt[0][wslot] + s_wcnt[1][wslot] + s_wcnt[2][wslot] +
                              s_wcnt[3][wslot];
            const int start = seg[wslot];
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int g = 0; g < NGa; ++g) {
                        const unsigned long long b = __ballot(slot[k][q] == g);
                        if (slot[k][q] == g) {
                            const int pos = run[g] + __popcll(b & lt);
#pragma unroll
                            for (int j = 0; j < D; ++j) s_val[pos * D + j] = v[k][q][j];
                        }
                        run[g] += __popcll(b);
                    }
                }
            __syncthreads();
            for (int i = sub * 64 + lane; i < total; i += nsub * 64) {
                const T* p = s_val + (size_t)(start + i) * D;
                cnt += 1.0;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const T x = p[j];
                    const T xx = x * x;   // squared in the input precision (numpy)
                    dd_acc(s[j], (double)x);
                    dd_acc(q2[j], (double)xx);
                }
            }
            __syncthreads();
        }
    }
    constexpr int G = 1 + 4 * D;
    constexpr int WM = NG * G;
    constexpr int WB = BB ? 2 * D + 1 : 0;
    constexpr int W = WM + WB;
    if constexpr (kDirect || kWave) {
        // every wave holds all NG slots: fold them into the regroup layout
        // (slot g in wave g's row) through LDS, waves in order
        __shared__ double sd[NW][NG][G];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const double x = wave_sum(dc[g]);
            if (lane == 0) sd[w][g][0] = x;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const DD a = wave_dd(ds[g][j]);
                const DD b = wave_dd(dq[g][j]);
                if (lane == 0) {
                    sd[w][g][1 + 2 * j] = a.hi;
                    sd[w][g][2 + 2 * j] = a.lo;
                    sd[w][g][1 + 2 * D + 2 * j] = b.hi;
                    sd[w][g][2 + 2 * D + 2 * j] = b.lo;
                }
            }
        }
        __syncthreads();
        if (w < NG) {   // wave g carries slot g (the others stay empty)
            const int g = w;
            if (lane == 0) {
                for (int u = 0; u < NW; ++u) {
                    cnt += sd[u][g][0];
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        s[j] = dd_add(s[j], DD{sd[u][g][1 + 2 * j], sd[u][g][2 + 2 * j]});
                        q2[j] = dd_add(q2[j], DD{sd[u][g][1 + 2 * D + 2 * j], sd[u][g][2 + 2 * D + 2 * j]});
                    }
                }
            }
        }
    }
    __shared__ double sm[NW][G + WB];
    if constexpr (NG > 0) {
        const double x = wave_sum(cnt);
        if (lane == 0) sm[w][0] = x;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const DD a = wave_dd(s[j]);
            const DD b = wave_dd(q2[j]);
            if (lane == 0) {
                sm[w][1 + 2 * j] = a.hi;
                sm[w][2 + 2 * j] = a.lo;
                sm[w][1 + 2 * D + 2 * j] = b.hi;
                sm[w][2 + 2 * D + 2 * j] = b.lo;
            }
        }
    }
    if constexpr (BB) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const double a = wave_min(lo[j]), b = wave_max(hi[j]);
            if (lane == 0) {
                sm[w][G + j] = a;
                sm[w][G + D + j] = b;
            }
        }
        const double bb = wave_sum(bad);
        if (lane == 0) sm[w][G + 2 * D] = bb;
    }
    if constexpr (W > 0) {
        __syncthreads();
        double* out = part + (uint64_t)blockIdx.x * W;
        // moments: slot g = waves g, g + NG, ... merged in that order
        for (int k = tid; k < W; k += kBlock) {
            if (k < WM) {
                const int g = k / G, r = k % G;
                if (r == 0) {
                    double a = 0;
                    for (int u = g; u < NW; u += NGa) a += sm[u][0];
                    out[k] = a;
                } else if ((r - 1) % 2 == 0) {
                    DD a{0.0, 0.0};
                    for (int u = g; u < NW; u += NGa) a = dd_add(a, DD{sm[u][r], sm[u][r + 1]});
                    out[k] = a.hi;
                    out[k + 1] = a.lo;
                }
            } else {
                const int b = k - WM;
                double a = sm[0][G + b];
                for (int u = 1; u < NW; ++u)
                    a = b < D ? fmin(a, sm[u][G + b])
                              : (b < 2 * D ? fmax(a, sm[u][G + b]) : a + sm[u][G + b]);
                out[k] = a;
            }
        }
    }
}

// Deterministic finish of kd_pass_kernel's block partials: per quantity,
// lane t folds blocks t, t + 256, ... in order, then a fixed-shape tree over
// the lanes (dd sums / counts / min / max).  out[W] as one block's layout.
// One block per quantity (grid W; a lo word's block leaves at once — its hi
// word's block writes both): the quantities reduce in parallel, each in the
// same fixed order as before (round 6: 111 -> ~10 us for 16 x 13 moments).
__global__ __launch_bounds__(kBlock) void kd_finish_kernel(const double* __restrict__ part, int nb,
                                                           int WM, int G, int D, int W,
                                                           double* __restrict__ out) {
    __shared__ double sh[kBlock], sl[kBlock];
    for (int k = blockIdx.x; k < W; k += gridDim.x) {
        const bool mom = k < WM;
        const int r = mom ? k % G : 0;
        if (mom && r != 0 && (r - 1) % 2 == 1) continue;   // lo word: handled with its hi
        const bool is_dd = mom && r != 0;
        const int b = mom ? -1 : k - WM;   // bbox: 0..D-1 min, D..2D-1 max, 2D bad
        DD acc{0.0, 0.0};
        double x = mom || b == 2 * D ? 0.0 : (b < D ? INFINITY : -INFINITY);
        for (int i = threadIdx.x; i < nb; i += kBlock) {
            const double* p = part + (uint64_t)i * W;
            if (is_dd)
                acc = dd_add(acc, DD{p[k], p[k + 1]});
            else if (mom || b == 2 * D)
                x += p[k];
            else
                x = b < D ? fmin(x, p[k]) : fmax(x, p[k]);
        }
        sh[threadIdx.x] = is_dd ? acc.hi : x;
        sl[threadIdx.x] = acc.lo;
        __syncthreads();
        for (int o = kBlock / 2; o > 0; o >>= 1) {
            if (threadIdx.x < o) {
                const int t = threadIdx.x;
                if (is_dd) {
                    const DD a = dd_add(DD{sh[t], sl[t]}, DD{sh[t + o], sl[t + o]});
                    sh[t] = a.hi;
                    sl[t] = a.lo;
                } else if (mom || b == 2 * D) {
                    sh[t] += sh[t + o];
                } else {
                    sh[t] = b < D ? fmin(sh[t], sh[t + o]) : fmax(sh[t], sh[t + o]);
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            out[k] = sh[0];
            if (is_dd) out[k + 1] = sl[0];
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- counts
// counts[slot][i] = #points of the slot's label with v[axis] < bounds[slot][i].
// mono (every slot's bounds non-decreasing, as mean + (i-3)*0.3*std is for
// std >= 0, or all NaN): v < b_i holds exactly for i >= 7 - c with c = #true,
// so one histogram bump of c per point carries all seven answers (the host
// sums the tail); the histograms are replicated per lane & (kRep-1) so a wave
// spreads its LDS atomics.  !mono: one atomic per true compare.
constexpr int kRep = 8;

template <typename T>
__global__ __launch_bounds__(kBlock) void counts_kernel(
    const T* __restrict__ X, uint64_t n, uint32_t ld, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ slot_of, int n_label_tab, const int32_t* __restrict__ axis,
    const double* __restrict__ bounds, int n_sel, int mono, int rep,
    unsigned long long* __restrict__ out) {
    extern __shared__ unsigned int lcnt[];   // rep * n_sel * 8
    for (int k = threadIdx.x; k < rep * n_sel * 8; k += kBlock) lcnt[k] = 0;
    __syncthreads();
    unsigned int* mine = lcnt + (threadIdx.x & (rep - 1)) * n_sel * 8;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const int lab = labels[i];
        if (lab < 0 || lab >= n_label_tab) continue;
        const int sl = slot_of[lab];
        if (sl < 0) continue;
        const double v = (double)X[i * ld + axis[sl]];
        if (mono) {
            int c = 0;
#pragma unroll
            for (int b = 0; b < 7; ++b) c += v < bounds[sl * 7 + b] ? 1 : 0;
            atomicAdd(&mine[sl * 8 + c], 1u);
        } else {
            for (int b = 0; b < 7; ++b)
                if (v < bounds[sl * 7 + b]) atomicAdd(&mine[sl * 8 + b], 1u);
            atomicAdd(&mine[sl * 8 + 7], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n_sel * 8; k += kBlock) {
        unsigned int v = 0;
        for (int q = 0; q < rep; ++q) v += lcnt[q * n_sel * 8 + k];
        if (v) atomicAdd(&out[k], (unsigned long long)v);
    }
}

// d <= 4: four points per lane per step (16-byte loads), the label tables
// and bounds staged in LDS (n_label_tab, n_sel <= kTabLds).
template <typename T, int D>
__global__ __launch_bounds__(kBlock) void counts4_kernel(
    const T* __restrict__ X, uint64_t n, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ slot_of, int n_label_tab, const int32_t* __restrict__ axis,
    const double* __restrict__ bounds, int n_sel, int mono, int rep,
    unsigned long long* __restrict__ out, ReplayTab rp) {
    extern __shared__ unsigned int lcnt[];   // rep * n_sel * 8
    __shared__ ReplayLds s_rp;   // (rp.nl > 0: labels replayed instead of read)
    replay_stage(s_rp, rp, threadIdx.x, kBlock);
    __shared__ int s_slot[kTabLds], s_ax[kTabLds];
    __shared__ double s_bd[kTabLds * 7];
    for (int k = threadIdx.x; k < rep * n_sel * 8; k += kBlock) lcnt[k] = 0;
    for (int k = threadIdx.x; k < n_label_tab; k += kBlock) s_slot[k] = slot_of[k];
    for (int k = threadIdx.x; k < n_sel; k += kBlock) s_ax[k] = axis[k];
    for (int k = threadIdx.x; k < n_sel * 7; k += kBlock) s_bd[k] = bounds[k];
    __syncthreads();
    unsigned int* mine = lcnt + (threadIdx.x & (rep - 1)) * n_sel * 8;
    const uint64_t nch = (n + 3) / 4;
    for (uint64_t ch = (uint64_t)blockIdx.x * kBlock + threadIdx.x; ch < nch;
         ch += (uint64_t)gridDim.x * kBlock) {
        T v[4][D];
        const int m = load_chunk<T, D, true>(X, n, ch, v);
        int lab[4];
        if (rp.nl) {
#pragma unroll
            for (int q = 0; q < 4; ++q) lab[q] = replay_label<T, D>(s_rp, rp, v[q]);
        } else {
            load_labels4<true>(labels, ch, m, lab);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q >= m || lab[q] < 0 || lab[q] >= n_label_tab) continue;
            const int sl = s_slot[lab[q]];
            if (sl < 0) continue;
            const double x = (double)pick_axis<T, D>(v[q], s_ax[sl]);
            const double* b = s_bd + sl * 7;
            if (mono) {
                int cc = 0;
#pragma unroll
                for (int i = 0; i < 7; ++i) cc += x < b[i] ? 1 : 0;
                atomicAdd(&mine[sl * 8 + cc], 1u);
            } else {
                for (int i = 0; i < 7; ++i)
                    if (x < b[i]) atomicAdd(&mine[sl * 8 + i], 1u);
                atomicAdd(&mine[sl * 8 + 7], 1u);
            }
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n_sel * 8; k += kBlock) {
        unsigned int v = 0;
        for (int q = 0; q < rep; ++q) v += lcnt[q * n_sel * 8 + k];
        if (v) atomicAdd(&out[k], (unsigned long long)v);
    }
}

// n_sel <= 4 (NS slots): per-lane register counters instead of LDS atomics
// (a wave's lanes mostly hit the same few bins, so shared counters
// serialise): c[s][i] = #points of slot s with v[axis] < bound i, c[s][7] =
// #points of slot s; one wave reduction and one LDS atomic per counter and
// wave at the end.  Labels < kTabLds.
template <typename T, int D, int NS, bool RP = false>
__global__ __launch_bounds__(kBlock) void counts_reg_kernel(
    const T* __restrict__ X, uint64_t n, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ slot_of, int n_label_tab, const int32_t* __restrict__ axis,
    const double* __restrict__ bounds, int n_sel, unsigned long long* __restrict__ out,
    ReplayTab rp) {
    __shared__ std::conditional_t<RP, ReplayLds, char> s_rp;
    if constexpr (RP) replay_stage(s_rp, rp, threadIdx.x, kBlock);
    __shared__ int s_slot[kTabLds];
    __shared__ unsigned int s_cnt[NS * 8];
    for (int k = threadIdx.x; k < n_label_tab; k += kBlock) s_slot[k] = slot_of[k];
    for (int k = threadIdx.x; k < NS * 8; k += kBlock) s_cnt[k] = 0;
    int ax[NS];
    double b[NS][7];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        ax[q] = q < n_sel ? axis[q] : 0;
#pragma unroll
        for (int i = 0; i < 7; ++i) b[q][i] = q < n_sel ? bounds[q * 7 + i] : 0.0;
    }
    __syncthreads();
    uint32_t c[NS][8];
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) c[q][i] = 0;
    const uint64_t nch = (n + 3) / 4;
    for (uint64_t ch = (uint64_t)blockIdx.x * kBlock + threadIdx.x; ch < nch;
         ch += (uint64_t)gridDim.x * kBlock) {
        T v[4][D];
        const int m = load_chunk<T, D, true>(X, n, ch, v);
        int lab[4] = {0, 0, 0, 0};   // labels == nullptr: every point in label 0
        if constexpr (RP) {
#pragma unroll
            for (int p = 0; p < 4; ++p) lab[p] = replay_label<T, D>(s_rp, rp, v[p]);
        } else if (labels) {
            load_labels4<true>(labels, ch, m, lab);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int L = lab[p];
            const int sl = (p < m && L >= 0 && L < n_label_tab) ? s_slot[L] : -1;
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                if (sl != q) continue;
                const double x = (double)pick_axis<T, D>(v[p], ax[q]);
                ++c[q][7];
#pragma unroll
                for (int i = 0; i < 7; ++i) c[q][i] += x < b[q][i] ? 1u : 0u;
            }
        }
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t t = c[q][i];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) t += (uint32_t)__shfl_xor((int)t, o, 64);
            if (lane == 0 && t) atomicAdd(&s_cnt[q * 8 + i], t);
        }
    __syncthreads();
    for (int k = threadIdx.x; k < n_sel * 8 && k < NS * 8; k += kBlock)
        if (s_cnt[k]) atomicAdd(&out[k], (unsigned long long)s_cnt[k]);
}

// ---------------------------------------------------------------- fused level pass 2
// Counts and the NEXT level's moments in one read of X (kd_build; VERDICT
// r05 #6): apply the previous level's split (SP, R:dbscan/partition.py:66-68;
// labels written back where they change, or all of them when none were
// written yet, !LAB), count this level's seven candidate compares per split
// (:60-63, counts_reg_kernel's register counters: c[s][i] = #(v[axis] <
// bound i), c[s][7] = #points) and, MOM, the double-double moments (:86-89)
// of every (split, interval) pair — interval q = #{i : v[axis] >= bound i}
// in 0..7.  The bounds mean + (i - 3) 0.3 std are non-decreasing, so the
// child a boundary i* makes is a run of intervals: left (v < bound i*) is q
// <= i*, right (v >= bound i*, the split's predicate) is q > i*.  The next
// level's moments are then dd sums of whole intervals (kdb_children_kernel),
// with no moments pass of their own; exact double-double sums do not depend
// on grouping, so they equal that pass's totals.
// MOM tiles: a counting sort of the tile by interval slot in LDS, then wave
// w sums slots w, w + NW, ... (NS * 8 / NW slots per wave, in registers).
template <typename T, int D, bool LAB, bool SP, int NS, bool MOM, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(
    (MOM && NS == 1 && sizeof(T) * D <= 12) ? 4 : 1))) void kdf_kernel(
    const T* __restrict__ X, uint64_t n, int32_t* __restrict__ labels, SplitTab sp,
    const int32_t* __restrict__ slot_of, int ntab, const int32_t* __restrict__ axis,
    const double* __restrict__ bounds, int n_sel, unsigned long long* __restrict__ cnt_out,
    double* __restrict__ part) {
    constexpr int NT = 64 * NW;
    constexpr int K = (sizeof(T) * D <= 16) ? 2 : 1;
    constexpr int TP = 4 * K * NT;   // points per tile
    constexpr int NI = NS * 8;       // interval slots
    constexpr int SPW = MOM ? NI / NW : 1;
    constexpr int G = 1 + 4 * D;
    static_assert(!MOM || (NI % NW == 0 && SPW >= 1), "slots per wave");
    __shared__ T s_val[MOM ? TP * D : 1];
    // per (wave, slot): running ranks, then the wave's first position; per
    // slot: the tile's total and first position
    __shared__ int s_lcnt[MOM ? NW : 1][MOM ? NI : 1], s_woff[MOM ? NW : 1][MOM ? NI : 1];
    __shared__ int s_tot[MOM ? NI : 1], s_seg[MOM ? NI : 1];
    // MOM: this level's axes and bounds by slot (one lookup per point, no
    // per-slot branches) and the block's points per (slot, interval) — the
    // counts follow from them: v < bound i  <=>  interval <= i
    __shared__ int s_axc[MOM ? NS : 1];
    __shared__ double s_bnd[MOM ? NS * 7 : 1];
    __shared__ unsigned int s_icnt[MOM ? NI : 1];
    __shared__ int s_slot[SP ? kTabLds : 1], s_ax[SP ? kTabLds : 1], s_nl[SP ? kTabLds : 1];
    __shared__ double s_bd[SP ? kTabLds : 1];
    __shared__ int s_cur[kTabLds];
    __shared__ unsigned int s_cnt[NS * 8];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if constexpr (SP) {
        for (int k = tid; k < sp.ntab; k += NT) s_slot[k] = sp.slot_of[k];
        for (int k = tid; k < sp.nsplit; k += NT) {
            s_ax[k] = sp.axis[k];
            s_bd[k] = sp.boundary[k];
            s_nl[k] = sp.newlab[k];
        }
    }
    for (int k = tid; k < ntab; k += NT) s_cur[k] = slot_of[k];
    for (int k = tid; k < NS * 8; k += NT) s_cnt[k] = 0;
    if constexpr (MOM) {
        for (int k = tid; k < NW * NI; k += NT) (&s_lcnt[0][0])[k] = 0;
        for (int k = tid; k < NI; k += NT) s_icnt[k] = 0;
        for (int k = tid; k < NS; k += NT) s_axc[k] = k < n_sel ? axis[k] : 0;
        for (int k = tid; k < NS * 7; k += NT) s_bnd[k] = k < n_sel * 7 ? bounds[k] : 0.0;
    }
    int ax[NS];
    double b[NS][7];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        ax[q] = q < n_sel ? axis[q] : 0;
#pragma unroll
        for (int i = 0; i < 7; ++i) b[q][i] = q < n_sel ? bounds[q * 7 + i] : 0.0;
    }
    __syncthreads();
    uint32_t c[NS][8];
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) c[q][i] = 0;
    double ac[SPW];
    DD as[SPW][D], aq[SPW][D];
#pragma unroll
    for (int o = 0; o < SPW; ++o) {
        ac[o] = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) as[o][j] = aq[o][j] = DD{0.0, 0.0};
    }
    const uint64_t nch = (n + 3) / 4;
    const uint64_t ntile = (n + TP - 1) / TP;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        T v[K][4][D];
        int slot[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t ch = t * (TP / 4) + (uint64_t)k * NT + tid;
            int m = 0;
            if (ch < nch) {
                m = load_chunk<T, D, true>(X, n, ch, v[k]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < D; ++j) v[k][q][j] = T(0);
            }
            int lab[4] = {0, 0, 0, 0};
            if constexpr (LAB) {
                if (m) load_labels4<true>(labels, ch, m, lab);
            }
            if constexpr (SP) {
                bool changed = false;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int L = lab[q];
                    if (q >= m || L < 0 || L >= sp.ntab) continue;
                    const int a = s_slot[L];
                    if (a < 0) continue;
                    const double x = (double)pick_axis<T, D>(v[k][q], s_ax[a]);
                    if (x >= s_bd[a]) {
                        lab[q] = s_nl[a];
                        changed = true;
                    }
                }
                if (m && (changed || !LAB)) store_labels4<true>(labels, ch, m, lab);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int L = lab[q];
                const int sl = (q < m && L >= 0 && L < ntab) ? s_cur[L] : -1;
                slot[k][q] = -1;
                if constexpr (MOM) {
                    if (sl >= 0) {
                        const double x = (double)pick_axis<T, D>(v[k][q], s_axc[sl]);
                        int qi = 0;
#pragma unroll
                        for (int i = 0; i < 7; ++i) qi += x >= s_bnd[sl * 7 + i] ? 1 : 0;
                        slot[k][q] = sl * 8 + qi;
                    }
                } else {
#pragma unroll
                    for (int sI = 0; sI < NS; ++sI) {
                        if (sl != sI) continue;
                        const double x = (double)pick_axis<T, D>(v[k][q], ax[sI]);
                        ++c[sI][7];
#pragma unroll
                        for (int i = 0; i < 7; ++i) c[sI][i] += x < b[sI][i] ? 1u : 0u;
                    }
                }
            }
        }
        if constexpr (MOM) {
            // counting sort of the tile by interval slot: each item's rank
            // among its wave's items of the slot (5-ballot peer mask, running
            // per-(wave, slot) counters in LDS, as rsort's pass_kernel ranks
            // digits), then the slots' and waves' starts, then the staging
            int rk[K][4];
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int sl = slot[k][q];
                    const unsigned u5 = sl < 0 ? 31u : (unsigned)sl;
                    unsigned long long mk = ~0ull;
#pragma unroll
                    for (int bt = 0; bt < 5; ++bt) {
                        const unsigned long long bb = __ballot((u5 >> bt) & 1u);
                        mk &= ((u5 >> bt) & 1u) ? bb : ~bb;
                    }
                    const int base = sl >= 0 ? s_lcnt[w][sl] : 0;
                    rk[k][q] = base + __popcll(mk & lt);
                    if (sl >= 0 && (mk & lt) == 0) s_lcnt[w][sl] = base + __popcll(mk);
                }
            __syncthreads();
            if (tid < NI) {
                int a = 0;
#pragma unroll
                for (int u = 0; u < NW; ++u) a += s_lcnt[u][tid];
                s_tot[tid] = a;
                s_icnt[tid] += (unsigned int)a;
            }
            __syncthreads();
            if (tid < NI) {
                int a = 0;
                for (int h = 0; h < tid; ++h) a += s_tot[h];
                s_seg[tid] = a;
#pragma unroll
                for (int u = 0; u < NW; ++u) {
                    s_woff[u][tid] = a;
                    a += s_lcnt[u][tid];
                    s_lcnt[u][tid] = 0;   // (restarted for the next tile)
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int sl = slot[k][q];
                    if (sl < 0) continue;
                    const int pos = s_woff[w][sl] + rk[k][q];
#pragma unroll
                    for (int j = 0; j < D; ++j) s_val[pos * D + j] = v[k][q][j];
                }
            __syncthreads();
#pragma unroll
            for (int o = 0; o < SPW; ++o) {
                const int g = w + o * NW;
                const int start = s_seg[g], len = s_tot[g];
                for (int i = lane; i < len; i += 64) {
                    const T* p = s_val + (size_t)(start + i) * D;
                    ac[o] += 1.0;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const T x = p[j];
                        const T xx = x * x;   // squared in the input precision (numpy)
                        dd_acc(as[o][j], (double)x);
                        dd_acc(aq[o][j], (double)xx);
                    }
                }
            }
            __syncthreads();
        }
    }
    if constexpr (!MOM) {
        // counts: one wave reduction and one LDS atomic per counter and wave
#pragma unroll
        for (int q = 0; q < NS; ++q)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t x = c[q][i];
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
                if (lane == 0 && x) atomicAdd(&s_cnt[q * 8 + i], x);
            }
    } else {
        // counts from the intervals: #(v < bound i) = points in intervals
        // <= i (bounds non-decreasing; NaN bounds: v < NaN never holds)
        __syncthreads();
        if (tid < NS * 8) {
            const int sI = tid >> 3, i = tid & 7;
            unsigned int x = 0;
            for (int q = 0; q < 8; ++q) x += (i == 7 || q <= i) ? s_icnt[sI * 8 + q] : 0u;
            if (i < 7 && isnan(s_bnd[sI * 7 + i])) x = 0;
            s_cnt[tid] = x;
        }
    }
    if constexpr (MOM) {
        // each slot has one owner wave: its lane 0 writes the block partial
        double* out = part + (uint64_t)blockIdx.x * NI * G;
#pragma unroll
        for (int o = 0; o < SPW; ++o) {
            const int g = w + o * NW;
            const double x = wave_sum(ac[o]);
            if (lane == 0) out[g * G] = x;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const DD a = wave_dd(as[o][j]);
                const DD q2 = wave_dd(aq[o][j]);
                if (lane == 0) {
                    out[g * G + 1 + 2 * j] = a.hi;
                    out[g * G + 2 + 2 * j] = a.lo;
                    out[g * G + 1 + 2 * D + 2 * j] = q2.hi;
                    out[g * G + 2 + 2 * D + 2 * j] = q2.lo;
                }
            }
        }
    }
    __syncthreads();
    for (int k = tid; k < n_sel * 8 && k < NS * 8; k += NT)
        if (s_cnt[k]) atomicAdd(&cnt_out[k], (unsigned long long)s_cnt[k]);
}

// ---------------------------------------------------------------- split
template <typename T>
__global__ __launch_bounds__(kBlock) void split_kernel(
    const T* __restrict__ X, uint64_t n, uint32_t ld, int32_t* __restrict__ labels,
    const int32_t* __restrict__ slot_of, int n_label_tab, const int32_t* __restrict__ axis,
    const double* __restrict__ boundary, const int32_t* __restrict__ newlab) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const int lab = labels[i];
        if (lab < 0 || lab >= n_label_tab) continue;
        const int sl = slot_of[lab];
        if (sl < 0) continue;
        const double v = (double)X[i * ld + axis[sl]];
        if (v >= boundary[sl]) labels[i] = newlab[sl];
    }
}

// ---------------------------------------------------------------- radix select
// One pass of an MSD radix select over v[axis] of each selected label
// (median_search_split, R:dbscan/partition.py:23-26: sortBy(v[axis]) then
// sorted_values[len/2]).  Values are widened to fp64 and mapped to an
// order-preserving u64 key (-0.0 folded onto +0.0: the reference's sort
// compares them equal).  hist[slot][b] = #points whose key agrees with the
// slot's prefix above bit (shift + 8) and whose digit at `shift` is b.
__device__ __forceinline__ uint64_t order_key(double v) {
    uint64_t b = (uint64_t)__double_as_longlong(v);
    if (b == 0x8000000000000000ull) b = 0;   // -0.0 == +0.0
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void radix_hist_kernel(
    const T* __restrict__ X, uint64_t n, uint32_t ld, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ slot_of, int n_label_tab, const int32_t* __restrict__ axis,
    const uint64_t* __restrict__ prefix, int shift, int n_sel, int lds,
    unsigned int* __restrict__ out) {
    extern __shared__ unsigned int lh[];   // n_sel * 256 when lds
    if (lds) {
        for (int k = threadIdx.x; k < n_sel * 256; k += kBlock) lh[k] = 0;
        __syncthreads();
    }
    unsigned int* h = lds ? lh : out;
    const int top = shift + 8;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const int lab = labels[i];
        if (lab < 0 || lab >= n_label_tab) continue;
        const int sl = slot_of[lab];
        if (sl < 0) continue;
        const uint64_t key = order_key((double)X[i * ld + axis[sl]]);
        if (top < 64 && (key >> top) != prefix[sl]) continue;
        atomicAdd(&h[sl * 256 + (int)((key >> shift) & 255u)], 1u);
    }
    if (lds) {
        __syncthreads();
        for (int k = threadIdx.x; k < n_sel * 256; k += kBlock)
            if (lh[k]) atomicAdd(&out[k], lh[k]);
    }
}

// ---------------------------------------------------------------- halo membership
template <typename T, int D>
struct InBox {
    const T* X;
    const double* box;   // lo[D], hi[D]
    __device__ bool operator()(int64_t i) const {
        bool in = true;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const double v = (double)X[i * D + j];
            in &= (box[j] <= v) & (box[D + j] >= v);
        }
        return in;
    }
};

// Any d (the dense high-dimensional path): runtime loop over the axes.
template <typename T>
struct InBoxDyn {
    const T* X;
    const double* box;   // lo[d], hi[d]
    int d;
    __device__ bool operator()(int64_t i) const {
        bool in = true;
        for (int j = 0; j < d; ++j) {
            const double v = (double)X[i * d + j];
            in &= (box[j] <= v) & (box[d + j] >= v);
        }
        return in;
    }
};

template <typename F>
void dispatch_d(int d, F&& f) {
    switch (d) {
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: f(std::integral_constant<int, 3>{}); break;
        case 4: f(std::integral_constant<int, 4>{}); break;
        default: throw Error(-1, "axis chunk must have 1..4 axes");
    }
}

template <typename F>
void dispatch_t(int dtype, F&& f) {
    if (dtype == 0)
        f((float*)nullptr);
    else if (dtype == 1)
        f((double*)nullptr);
    else
        throw Error(-1, "dtype must be 0 (float32) or 1 (float64)");
}

// f(T*, D, a0) for each chunk of <= 4 consecutive axes [a0, a0 + D).
template <typename F>
void dispatch_chunks(int dtype, int d, F&& f) {
    dispatch_t(dtype, [&](auto tp) {
        for (int a0 = 0; a0 < d; a0 += 4)
            dispatch_d(std::min(4, d - a0), [&](auto Dc) { f(tp, Dc, a0); });
    });
}

struct LabelTables {
    int32_t* slot_of;
    int32_t* axis;
    double* dbl;
    int32_t* newlab;
    int ntab;
};

// Upload the (label -> slot) map and the per-slot tables.  Pinned staging is
// safe to reuse because every KD entry point synchronises before returning.
LabelTables upload_tables(Ctx& ctx, int n_sel, const int32_t* sel, const int32_t* axis,
                          const double* dbl, int dbl_per, const int32_t* newlab,
                          hipStream_t s) {
    int ntab = 1;
    for (int k = 0; k < n_sel; ++k) ntab = std::max(ntab, sel[k] + 1);
    const size_t bytes = sizeof(int32_t) * (ntab + 2 * n_sel) + sizeof(double) * n_sel * dbl_per;
    char* h = (char*)pinned(ctx, bytes + 64);
    int32_t* h_slot = (int32_t*)h;
    for (int k = 0; k < ntab; ++k) h_slot[k] = -1;
    for (int k = 0; k < n_sel; ++k) h_slot[sel[k]] = k;
    int32_t* h_axis = h_slot + ntab;
    int32_t* h_new = h_axis + n_sel;
    for (int k = 0; k < n_sel; ++k) {
        h_axis[k] = axis ? axis[k] : 0;
        h_new[k] = newlab ? newlab[k] : 0;
    }
    size_t off_d = ((sizeof(int32_t) * (ntab + 2 * n_sel)) + 7) & ~size_t(7);
    double* h_d = (double*)(h + off_d);
    if (dbl) std::memcpy(h_d, dbl, sizeof(double) * n_sel * dbl_per);
    char* dmem = ctx.arena.get<char>("kd_tables", off_d + sizeof(double) * n_sel * dbl_per + 64);
    PD_HIP(hipMemcpyAsync(dmem, h, off_d + sizeof(double) * n_sel * dbl_per,
                          hipMemcpyHostToDevice, s));
    LabelTables t;
    t.slot_of = (int32_t*)dmem;
    t.axis = t.slot_of + ntab;
    t.newlab = t.axis + n_sel;
    t.dbl = (double*)(dmem + off_d);
    t.ntab = ntab;
    return t;
}

}  // namespace

void bbox(Ctx& ctx, const void* X, int dtype, int64_t n, int d, double* lohi, int64_t* bad,
          hipStream_t s) {
    const int nb = (int)std::min<int64_t>(kRedBlocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
    double* part = ctx.arena.get<double>("bbox_part", (size_t)nb * 9);
    double nbad = 0;
    dispatch_chunks(dtype, d, [&](auto tp, auto Dc, int a0) {
        using T = std::remove_pointer_t<decltype(tp)>;
        constexpr int D = decltype(Dc)::value;
        constexpr int W = 2 * D + 1;
        hipLaunchKernelGGL((bbox_kernel<T, D>), dim3(nb), dim3(kBlock), 0, s, (const T*)X + a0,
                           (uint64_t)n, (uint32_t)d, part);
        PD_HIP(hipGetLastError());
        double* h = (double*)pinned(ctx, sizeof(double) * nb * W);
        PD_HIP(hipMemcpyAsync(h, part, sizeof(double) * nb * W, hipMemcpyDeviceToHost, s));
        sync(s);
        for (int j = 0; j < D; ++j) {
            double lo = INFINITY, hi = -INFINITY;
            for (int k = 0; k < nb; ++k) {
                lo = std::fmin(lo, h[k * W + j]);
                hi = std::fmax(hi, h[k * W + D + j]);
            }
            lohi[a0 + j] = lo;
            lohi[d + a0 + j] = hi;
        }
        for (int k = 0; k < nb; ++k) nbad += h[k * W + 2 * D];
    });
    if (bad) *bad = (int64_t)nbad;
}

namespace {
// Moments of the selected labels, kGroup labels x <= 4 axes per pass.
void moments_impl(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                  int n_sel, const int32_t* sel, double* out, bool dd_out, hipStream_t s) {
    const int nb = (int)std::min<int64_t>(kRedBlocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
    const int nbk = ctx.seq_moments ? 1 : nb;
    const int Gd = 1 + 4 * d;
    double* part = ctx.arena.get<double>("mom_part", (size_t)nb * kGroup * (1 + 4 * 4));
    for (int g0 = 0; g0 < n_sel; g0 += kGroup) {
        int4 sl = make_int4(-2, -2, -2, -2);
        int* sp = &sl.x;
        for (int g = 0; g < kGroup && g0 + g < n_sel; ++g) sp[g] = sel[g0 + g];
        // per label of the group: count, dd sums and dd sums of squares per axis
        std::vector<double> cnt(kGroup, 0.0);
        std::vector<DD> sum((size_t)kGroup * d, DD{0.0, 0.0}), sq((size_t)kGroup * d, DD{0.0, 0.0});
        dispatch_chunks(dtype, d, [&](auto tp, auto Dc, int a0) {
            using T = std::remove_pointer_t<decltype(tp)>;
            constexpr int D = decltype(Dc)::value;
            constexpr int G = 1 + 4 * D;
            constexpr int W = kGroup * G;
            if (ctx.seq_moments)
                hipLaunchKernelGGL((moments_seq_kernel<T, D>), dim3(1), dim3(64), 0, s,
                                   (const T*)X + a0, (uint64_t)n, (uint32_t)d, labels, sl, part);
            else
                hipLaunchKernelGGL((moments_kernel<T, D>), dim3(nb), dim3(kBlock), 0, s,
                                   (const T*)X + a0, (uint64_t)n, (uint32_t)d, labels, sl, part);
            PD_HIP(hipGetLastError());
            double* h = (double*)pinned(ctx, sizeof(double) * nbk * W);
            PD_HIP(hipMemcpyAsync(h, part, sizeof(double) * nbk * W, hipMemcpyDeviceToHost, s));
            sync(s);
            for (int g = 0; g < kGroup; ++g)
                for (int k = 0; k < nbk; ++k) {
                    const double* p = h + (size_t)k * W + g * G;
                    if (a0 == 0) cnt[g] += p[0];
                    for (int j = 0; j < D; ++j) {
                        DD& su = sum[(size_t)g * d + a0 + j];
                        DD& sqq = sq[(size_t)g * d + a0 + j];
                        su = dd_add(su, DD{p[1 + 2 * j], p[2 + 2 * j]});
                        sqq = dd_add(sqq, DD{p[1 + 2 * D + 2 * j], p[2 + 2 * D + 2 * j]});
                    }
                }
        });
        for (int g = 0; g < kGroup && g0 + g < n_sel; ++g) {
            // out layout per selected label: [3][d] = count row, sum row, sumsq row;
            // dd_out: [1 + 4d] = count, (hi, lo) per axis of the sums, then of the squares
            double* o = out + (size_t)(g0 + g) * (dd_out ? Gd : 3 * d);
            const DD* su = &sum[(size_t)g * d];
            const DD* sqq = &sq[(size_t)g * d];
            if (dd_out) {
                o[0] = cnt[g];
                for (int j = 0; j < d; ++j) {
                    o[1 + 2 * j] = su[j].hi;
                    o[2 + 2 * j] = su[j].lo;
                    o[1 + 2 * d + 2 * j] = sqq[j].hi;
                    o[2 + 2 * d + 2 * j] = sqq[j].lo;
                }
                continue;
            }
            for (int j = 0; j < d; ++j) {
                o[j] = cnt[g];
                o[d + j] = su[j].hi + su[j].lo;
                o[2 * d + j] = sqq[j].hi + sqq[j].lo;
            }
        }
    }
}
}  // namespace

namespace {
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// The fused four-point kernels need d <= 4 and 16-byte aligned X and labels
// (torch allocations are); anything else takes the one-point-per-lane kernels.
inline bool vec_ok(int d, const void* X, const void* labels) {
    return d <= kMaxDim && aligned16(X) && (!labels || aligned16(labels));
}

// ... and LDS-sized label tables: labels < kTabLds, <= kTabLds slots.
inline bool tabs_ok(int n_sel, const int32_t* sel) {
    if (n_sel > kTabLds) return false;
    for (int k = 0; k < n_sel; ++k)
        if (sel[k] >= kTabLds) return false;
    return true;
}

template <typename F>
void dispatch_ng(int ng, F&& f) {
    switch (ng) {
        case 0: f(std::integral_constant<int, 0>{}); break;
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        default: f(std::integral_constant<int, 4>{}); break;
    }
}

// One launch of kd_pass_kernel + its deterministic finish; returns the
// finished quantities (NG x G moments, then the bbox) in `res` (host).
template <typename T, int D, bool LAB, bool SP, int NG, bool BB>
void run_pass(Ctx& ctx, const T* X, int64_t n, int32_t* labels, const SplitTab& sp, int4 sel,
              std::vector<double>& res, hipStream_t s) {
    constexpr int G = 1 + 4 * D, WM = NG * G, W = WM + (BB ? 2 * D + 1 : 0);
    constexpr int TP = 4 * kBlock * ((sizeof(T) * D <= 16) ? 2 : 1);   // kd_pass_kernel tile
    // one wave of resident blocks: a second, partial round would leave most
    // CUs idle at the end (LDS limits residency to a few blocks per CU)
    static int resident = 0;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        PD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&kd_pass_kernel<T, D, LAB, SP, NG, BB>), kBlock, 0));
        PD_HIP(hipGetDevice(&dev));
        PD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        resident = std::max(1, per_cu) * std::max(1, cus);
    }
    const int nb = (int)std::min<int64_t>(resident, std::max<int64_t>(1, (n + TP - 1) / TP));
    double* part = ctx.arena.get<double>("pass_part", (size_t)nb * (W > 0 ? W : 1));
    hipLaunchKernelGGL((kd_pass_kernel<T, D, LAB, SP, NG, BB>), dim3(nb), dim3(kBlock), 0, s,
                       X, (uint64_t)n, labels, sp, sel, part, ReplayTab{});
    PD_HIP(hipGetLastError());
    res.assign(W, 0.0);
    if constexpr (W > 0) {
        double* fin = ctx.arena.get<double>("pass_fin", W);
        hipLaunchKernelGGL(kd_finish_kernel, dim3(W), dim3(kBlock), 0, s, part, nb, WM, G, D, W,
                           fin);
        PD_HIP(hipGetLastError());
        double* h = (double*)pinned(ctx, sizeof(double) * W);
        PD_HIP(hipMemcpyAsync(h, fin, sizeof(double) * W, hipMemcpyDeviceToHost, s));
        sync(s);
        std::memcpy(res.data(), h, sizeof(double) * W);
    }
}
}  // namespace

void kd_pass(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
             bool labels_zero, int n_split, const int32_t* ssel, const int32_t* saxis,
             const double* sbound, const int32_t* snew, int n_sel, const int32_t* sel,
             double* out_dd, double* lohi, int64_t* bad, hipStream_t s) {
    const bool lab_first = labels_zero && n_split == 0;
    if (n_sel == 0 && !lohi) {
        if (n_split) kd_split(ctx, X, dtype, n, d, labels, n_split, ssel, saxis, sbound, snew, s);
        return;
    }
    if (!vec_ok(d, X, labels) || ctx.seq_moments || !tabs_ok(n_split, ssel)) {
        // generic passes (any d, unaligned inputs)
        if (n_split) kd_split(ctx, X, dtype, n, d, labels, n_split, ssel, saxis, sbound, snew, s);
        if (n_sel) moments_impl(ctx, X, dtype, n, d, labels, n_sel, sel, out_dd, true, s);
        if (lohi) bbox(ctx, X, dtype, n, d, lohi, bad, s);
        return;
    }
    SplitTab st{nullptr, 0, nullptr, nullptr, nullptr, 0};
    if (n_split) {
        LabelTables t = upload_tables(ctx, n_split, ssel, saxis, sbound, 1, snew, s);
        st = SplitTab{t.slot_of, t.ntab, t.axis, t.dbl, t.newlab, n_split};
    }
    const int Gd = 1 + 4 * d;
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        dispatch_d(d, [&](auto Dc) {
            constexpr int D = decltype(Dc)::value;
            constexpr int G = 1 + 4 * D;
            std::vector<double> res;
            // the first launch: splits, the first group of labels, the bbox
            const int ng0 = std::min(n_sel, kGroup);
            int4 sl = make_int4(-2, -2, -2, -2);
            for (int g = 0; g < ng0; ++g) (&sl.x)[g] = sel[g];
            auto take = [&](int g0, int ng) {
                for (int g = 0; g < ng; ++g) std::memcpy(out_dd + (size_t)(g0 + g) * Gd,
                                                         res.data() + (size_t)g * G,
                                                         sizeof(double) * G);
            };
            if (lohi) {
                if (!lab_first) throw Error(-1, "kd_pass: bbox only on the first level");
                run_pass<T, D, false, false, 1, true>(ctx, (const T*)X, n, labels, st, sl, res, s);
                take(0, 1);
                for (int j = 0; j < 2 * D; ++j) lohi[j] = res[G + j];
                if (bad) *bad = (int64_t)res[G + 2 * D];
                if (n_sel > 1) throw Error(-1, "kd_pass: one label on the first level");
                return;
            }
            dispatch_ng(ng0, [&](auto NGc) {
                constexpr int NG = decltype(NGc)::value;
                if (lab_first)
                    run_pass<T, D, false, false, NG, false>(ctx, (const T*)X, n, labels, st, sl,
                                                            res, s);
                else if (n_split)
                    run_pass<T, D, true, true, NG, false>(ctx, (const T*)X, n, labels, st, sl,
                                                          res, s);
                else
                    run_pass<T, D, true, false, NG, false>(ctx, (const T*)X, n, labels, st, sl,
                                                           res, s);
            });
            take(0, ng0);
            for (int g0 = kGroup; g0 < n_sel; g0 += kGroup) {
                const int ng = std::min(n_sel - g0, kGroup);
                sl = make_int4(-2, -2, -2, -2);
                for (int g = 0; g < ng; ++g) (&sl.x)[g] = sel[g0 + g];
                dispatch_ng(ng, [&](auto NGc) {
                    constexpr int NG = decltype(NGc)::value;
                    run_pass<T, D, true, false, NG, false>(ctx, (const T*)X, n, labels, st, sl,
                                                           res, s);
                });
                take(g0, ng);
            }
        });
    });
}

void kd_moments(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                int n_sel, const int32_t* sel, double* out, hipStream_t s) {
    moments_impl(ctx, X, dtype, n, d, labels, n_sel, sel, out, false, s);
}

void kd_moments_dd(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                   int n_sel, const int32_t* sel, double* out, hipStream_t s) {
    if (ctx.seq_moments) throw Error(-5, "double-double partials need exact (non-sequential) sums");
    moments_impl(ctx, X, dtype, n, d, labels, n_sel, sel, out, true, s);
}

void kd_counts(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
               int n_sel, const int32_t* sel, const int32_t* axis, const double* bounds,
               int64_t* out, hipStream_t s) {
    if (n_sel <= 0) return;
    LabelTables t = upload_tables(ctx, n_sel, sel, axis, bounds, 7, nullptr, s);
    unsigned long long* dcnt = ctx.arena.get<unsigned long long>("kd_cnt", (size_t)n_sel * 8);
    PD_HIP(hipMemsetAsync(dcnt, 0, sizeof(unsigned long long) * n_sel * 8, s));
    bool mono = true;
    for (int k = 0; k < n_sel; ++k) {
        const double* b = bounds + (size_t)k * 7;
        bool all_nan = true, ordered = true;
        for (int i = 0; i < 7; ++i) {
            all_nan &= std::isnan(b[i]);
            if (i) ordered &= b[i - 1] <= b[i];
        }
        mono &= all_nan || ordered;
    }
    int rep = kRep;
    while (rep > 1 && (size_t)rep * n_sel * 8 * sizeof(unsigned int) > 48 * 1024) rep >>= 1;
    if ((size_t)n_sel * 8 * sizeof(unsigned int) > 60 * 1024)
        throw Error(-5, "too many splits in one KD level (> 1920)");
    const unsigned nb = grid_for(n, 2048);
    if (n_sel <= 4 && vec_ok(d, X, labels) && tabs_ok(n_sel, sel)) {
        // direct less-than counts in registers
        dispatch_t(dtype, [&](auto tp) {
            using T = std::remove_pointer_t<decltype(tp)>;
            dispatch_d(d, [&](auto Dc) {
                constexpr int D = decltype(Dc)::value;
                const unsigned nb4 = grid_for((n + 3) / 4, 2048);
                auto go = [&](auto NSc) {
                    constexpr int NS = decltype(NSc)::value;
                    hipLaunchKernelGGL((counts_reg_kernel<T, D, NS>), dim3(nb4), dim3(kBlock), 0, s,
                                       (const T*)X, (uint64_t)n, labels, t.slot_of, t.ntab, t.axis,
                                       t.dbl, n_sel, dcnt, ReplayTab{});
                };
                if (n_sel == 1)
                    go(std::integral_constant<int, 1>{});
                else if (n_sel == 2)
                    go(std::integral_constant<int, 2>{});
                else
                    go(std::integral_constant<int, 4>{});
            });
        });
        mono = false;   // the counters are already n_less / n_total
    } else if (vec_ok(d, X, labels) && tabs_ok(n_sel, sel)) {
        dispatch_t(dtype, [&](auto tp) {
            using T = std::remove_pointer_t<decltype(tp)>;
            dispatch_d(d, [&](auto Dc) {
                constexpr int D = decltype(Dc)::value;
                const unsigned nb4 = grid_for((n + 3) / 4, 2048);
                hipLaunchKernelGGL((counts4_kernel<T, D>), dim3(nb4), dim3(kBlock),
                                   sizeof(unsigned int) * rep * n_sel * 8, s, (const T*)X,
                                   (uint64_t)n, labels, t.slot_of, t.ntab, t.axis, t.dbl, n_sel,
                                   mono ? 1 : 0, rep, dcnt, ReplayTab{});
            });
        });
    } else
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        hipLaunchKernelGGL((counts_kernel<T>), dim3(nb), dim3(kBlock),
                           sizeof(unsigned int) * rep * n_sel * 8, s, (const T*)X, (uint64_t)n,
                           (uint32_t)d, labels, t.slot_of, t.ntab, t.axis, t.dbl, n_sel,
                           mono ? 1 : 0, rep, dcnt);
    });
    PD_HIP(hipGetLastError());
    unsigned long long* h = (unsigned long long*)pinned(ctx, sizeof(unsigned long long) * n_sel * 8);
    PD_HIP(hipMemcpyAsync(h, dcnt, sizeof(unsigned long long) * n_sel * 8, hipMemcpyDeviceToHost, s));
    sync(s);
    // out[slot][0..6] = n_less per bound, out[slot][7] = n_total
    if (!mono) {
        for (int k = 0; k < n_sel * 8; ++k) out[k] = (int64_t)h[k];
        return;
    }
    for (int k = 0; k < n_sel; ++k) {   // h[k][c] = #points with c true compares
        const unsigned long long* hc = h + (size_t)k * 8;
        int64_t tot = 0;
        for (int c = 0; c < 8; ++c) tot += (int64_t)hc[c];
        for (int i = 0; i < 7; ++i) {
            int64_t less = 0;
            for (int c = 7 - i; c < 8; ++c) less += (int64_t)hc[c];
            out[(size_t)k * 8 + i] = less;
        }
        out[(size_t)k * 8 + 7] = tot;
    }
}

void kd_split(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels, int n_sel,
              const int32_t* sel, const int32_t* axis, const double* boundary,
              const int32_t* newlab, hipStream_t s) {
    if (n_sel <= 0) return;
    LabelTables t = upload_tables(ctx, n_sel, sel, axis, boundary, 1, newlab, s);
    if (vec_ok(d, X, labels) && tabs_ok(n_sel, sel)) {
        const SplitTab st{t.slot_of, t.ntab, t.axis, t.dbl, t.newlab, n_sel};
        dispatch_t(dtype, [&](auto tp) {
            using T = std::remove_pointer_t<decltype(tp)>;
            dispatch_d(d, [&](auto Dc) {
                constexpr int D = decltype(Dc)::value;
                std::vector<double> res;
                run_pass<T, D, true, true, 0, false>(ctx, (const T*)X, n, labels, st,
                                                     make_int4(-2, -2, -2, -2), res, s);
            });
        });
        sync(s);
        return;
    }
    const unsigned nb = grid_for(n, 4096);
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        hipLaunchKernelGGL((split_kernel<T>), dim3(nb), dim3(kBlock), 0, s, (const T*)X,
                           (uint64_t)n, (uint32_t)d, labels, t.slot_of, t.ntab, t.axis, t.dbl,
                           t.newlab);
    });
    PD_HIP(hipGetLastError());
    sync(s);
}

// ---------------------------------------------------------------- device-decided KD
// The whole min_var BFS of one device as one chain of launches with a single
// host sync at the end (R:dbscan/partition.py:139-183): the level decisions
// the host made between passes — the largest-variance axis and the seven
// candidate bounds (R:dbscan/partition.py:86-95, 58-59), the first bound that
// minimises |#left - #right| (:60-65) — run as one-thread-per-split kernels
// with the host's fp64 operation order (partition.level_axes /
// level_boundaries: same divisions, products and argmax/argmin tie rules),
// so the splits equal the host path's bit for bit.
// trace per split: axis, mean, var, cnt[8] (n_less per bound, n), cand, boundary.
constexpr int kTrace = 13;

__global__ void kdb_axes_kernel(const double* __restrict__ mom, int S, int D, int G,
                                int32_t* __restrict__ axis, double* __restrict__ bounds,
                                double* __restrict__ trace,
                                unsigned long long* __restrict__ zero_cnt) {
    // zero_cnt (nullable): the level's count slots (S x 8), zeroed here for
    // the counts pass that follows (one launch, one block: no fill)
    if (zero_cnt)
        for (int i = threadIdx.x; i < S * 8; i += blockDim.x) zero_cnt[i] = 0ull;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= S) return;
    const double* p = mom + (size_t)k * G;
    const double c = p[0];
    int a = 0;
    double best = 0.0, ma = 0.0, va = 0.0;
    for (int j = 0; j < D; ++j) {
        // partition.round_dd: hi + lo; level_axes: m = s / c, v = q / c - m * m
        const double sj = __dadd_rn(p[1 + 2 * j], p[2 + 2 * j]);
        const double qj = __dadd_rn(p[1 + 2 * D + 2 * j], p[2 + 2 * D + 2 * j]);
        const double m = __ddiv_rn(sj, c);
        const double v = __dsub_rn(__ddiv_rn(qj, c), __dmul_rn(m, m));
        // np.argmax: the first NaN if any, else the first maximum
        const bool take = j == 0 || (!isnan(best) && (isnan(v) || v > best));
        if (take) {
            best = v;
            a = j;
            ma = m;
            va = v;
        }
    }
    // partition._bounds: std = sqrt(v) (0 for v < 0, NaN stays NaN);
    // bound i = mean + ((i - 3) * 0.3) * std
    const double sd = isnan(va) ? va : (va >= 0.0 ? __dsqrt_rn(va) : 0.0);
    for (int i = 0; i < 7; ++i)
        bounds[(size_t)k * 7 + i] = __dadd_rn(ma, __dmul_rn(__dmul_rn((double)(i - 3), 0.3), sd));
    axis[k] = a;
    double* t = trace + (size_t)k * kTrace;
    t[0] = (double)a;
    t[1] = ma;
    t[2] = va;
}

__global__ void kdb_boundary_kernel(const unsigned long long* __restrict__ cnt, int S,
                                    const double* __restrict__ bounds,
                                    double* __restrict__ boundary, double* __restrict__ trace) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= S) return;
    const unsigned long long* c = cnt + (size_t)k * 8;
    const double tot = (double)c[7];
    // level_boundaries: |2.0 * n_less - n|, np.argmin (first minimum)
    int bi = 0;
    double best = fabs(__dsub_rn(__dmul_rn(2.0, (double)c[0]), tot));
    for (int i = 1; i < 7; ++i) {
        const double v = fabs(__dsub_rn(__dmul_rn(2.0, (double)c[i]), tot));
        if (v < best) {
            best = v;
            bi = i;
        }
    }
    boundary[k] = bounds[(size_t)k * 7 + bi];
    double* t = trace + (size_t)k * kTrace;
    for (int i = 0; i < 8; ++i) t[3 + i] = (double)c[i];
    t[11] = (double)bi;
    t[12] = boundary[k];
}

// The next level's moments from this level's interval moments (kdf_kernel):
// split k's left child is its intervals q <= i* (i* = the chosen candidate,
// trace[11]), the right child q > i*; dst[2k + side] = the child's slot in the
// next level (-1: not split there).  Counts are exact integers; the sums are
// double-double additions of whole intervals (exact, so equal to a moments
// pass over the child).
// Labels from a finished split tree (pd_kd_labels): replay every level per
// point, tables read through the caches (a one-off pass on request).
struct TreeG {
    int nl;
    int ntab[kMaxLevels], toff[kMaxLevels], eoff[kMaxLevels];
    const int32_t* slot;     // concatenated per level: label -> split index in the level (-1)
    const int32_t* ax_new;   // per split: axis, new label
    const double* bound;     // per split
};

template <typename T, int D>
__global__ __launch_bounds__(kBlock) void kd_label_kernel(const T* __restrict__ X, uint64_t n,
                                                          int32_t* __restrict__ labels, TreeG t) {
    const uint64_t nch = (n + 3) / 4;
    for (uint64_t ch = (uint64_t)blockIdx.x * kBlock + threadIdx.x; ch < nch;
         ch += (uint64_t)gridDim.x * kBlock) {
        T v[4][D];
        const int m = load_chunk<T, D, true>(X, n, ch, v);
        int lab[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int L = 0;
            for (int l = 0; l < t.nl; ++l) {
                if (L >= t.ntab[l]) continue;
                const int sl = t.slot[t.toff[l] + L];
                if (sl < 0) continue;
                const int e = t.eoff[l] + sl;
                if ((double)pick_axis<T, D>(v[q], t.ax_new[2 * e]) >= t.bound[e]) L = t.ax_new[2 * e + 1];
            }
            lab[q] = L;
        }
        store_labels4<true>(labels, ch, m, lab);
    }
}

__global__ void kdb_children_kernel(const double* __restrict__ fin, int S, int G,
                                    const double* __restrict__ trace,
                                    const int32_t* __restrict__ dst, double* __restrict__ mom) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = idx >> 1, side = idx & 1;
    if (k >= S) return;
    const int j = dst[2 * k + side];
    if (j < 0) return;
    const int bi = (int)trace[(size_t)k * kTrace + 11];
    const int q0 = side ? bi + 1 : 0, q1 = side ? 7 : bi;
    double* o = mom + (size_t)j * G;
    double c = 0.0;
    for (int q = q0; q <= q1; ++q) c += fin[((size_t)k * 8 + q) * G];
    o[0] = c;
    for (int r = 1; r < G; r += 2) {
        DD a{0.0, 0.0};
        for (int q = q0; q <= q1; ++q) {
            const double* p = fin + ((size_t)k * 8 + q) * G;
            a = dd_add(a, DD{p[r], p[r + 1]});
        }
        o[r] = a.hi;
        o[r + 1] = a.lo;
    }
}

namespace {
// run_pass without the host sync: the finished quantities stay on the device
// (fin: NG x G moments, then the bbox; may be null when the pass has none).
// RP: labels replayed from rp (kd_pass_kernel), none read or written.
template <typename T, int D, bool LAB, bool SP, int NG, bool BB, bool RP = false>
void run_pass_dev(Ctx& ctx, const T* X, int64_t n, int32_t* labels, const SplitTab& sp, int4 sel,
                  double* fin, hipStream_t s, const ReplayTab& rp = ReplayTab{}) {
    constexpr int G = 1 + 4 * D, WM = NG * G, W = WM + (BB ? 2 * D + 1 : 0);
    constexpr int TP = 4 * kBlock * ((sizeof(T) * D <= 16) ? 2 : 1);
    static int resident = 0;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        PD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&kd_pass_kernel<T, D, LAB, SP, NG, BB, RP>), kBlock, 0));
        PD_HIP(hipGetDevice(&dev));
        PD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        resident = std::max(1, per_cu) * std::max(1, cus);
    }
    const int nb = (int)std::min<int64_t>(resident, std::max<int64_t>(1, (n + TP - 1) / TP));
    double* part = ctx.arena.get<double>("pass_part", (size_t)nb * (W > 0 ? W : 1));
    hipLaunchKernelGGL((kd_pass_kernel<T, D, LAB, SP, NG, BB, RP>), dim3(nb), dim3(kBlock), 0, s,
                       X, (uint64_t)n, labels, sp, sel, part, rp);
    PD_HIP(hipGetLastError());
    if constexpr (W > 0) {
        hipLaunchKernelGGL(kd_finish_kernel, dim3(W), dim3(kBlock), 0, s, part, nb, WM, G, D, W,
                           fin);
        PD_HIP(hipGetLastError());
    }
}
}  // namespace

// final_mode: 0 leave the labels at the last level's labels (its split not
// applied), 1 apply the last split too, 2 the caller needs no labels at all
// (it replays the split tree itself: pd_train_tree, pd_kd_labels) — the
// levels then replay the splits instead of reading and writing labels
// (ctx.kd_replay, the tables fitting ReplayLds).
void kd_labels(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
               int n_levels, const int32_t* sizes, const int32_t* cur, const int32_t* axis,
               const double* bound, const int32_t* newl, hipStream_t s) {
    if (n <= 0) return;
    if (!vec_ok(d, X, labels)) throw Error(-5, "kd_labels: d <= 4, 16-byte aligned inputs only");
    if (n_levels > kMaxLevels) throw Error(-5, "kd_labels: more than 16 levels");
    TreeG t{};
    t.nl = n_levels;
    std::vector<int32_t> ints;
    std::vector<double> bd;
    int ne = 0, nslot = 0;
    for (int l = 0; l < n_levels; ++l) {
        int nt = 1;
        for (int k = 0; k < sizes[l]; ++k) nt = std::max(nt, cur[ne + k] + 1);
        t.ntab[l] = nt;
        t.toff[l] = nslot;
        t.eoff[l] = ne;
        nslot += nt;
        ne += sizes[l];
    }
    ints.assign((size_t)nslot + 2 * ne, -1);
    bd.assign(std::max(ne, 1), 0.0);
    for (int l = 0; l < n_levels; ++l)
        for (int k = 0; k < sizes[l]; ++k) {
            const int e = t.eoff[l] + k, L = cur[e];
            if (L < 0 || L >= t.ntab[l] || axis[e] < 0 || axis[e] >= d || newl[e] < 0)
                throw Error(-1, "kd_labels: bad split tree");
            ints[t.toff[l] + L] = k;
            ints[nslot + 2 * e] = axis[e];
            ints[nslot + 2 * e + 1] = newl[e];
            bd[e] = bound[e];
        }
    const size_t ib = (sizeof(int32_t) * ints.size() + 7) & ~size_t(7);
    char* h = (char*)pinned(ctx, ib + sizeof(double) * bd.size());
    std::memcpy(h, ints.data(), sizeof(int32_t) * ints.size());
    std::memcpy(h + ib, bd.data(), sizeof(double) * bd.size());
    char* dt = ctx.arena.get<char>("kdl_tables", ib + sizeof(double) * bd.size());
    PD_HIP(hipMemcpyAsync(dt, h, ib + sizeof(double) * bd.size(), hipMemcpyHostToDevice, s));
    t.slot = (const int32_t*)dt;
    t.ax_new = (const int32_t*)dt + nslot;
    t.bound = (const double*)(dt + ib);
    const unsigned nb = grid_for((n + 3) / 4, 4096);
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        dispatch_d(d, [&](auto Dc) {
            constexpr int D = decltype(Dc)::value;
            hipLaunchKernelGGL((kd_label_kernel<T, D>), dim3(nb), dim3(kBlock), 0, s, (const T*)X,
                               (uint64_t)n, labels, t);
        });
    });
    PD_HIP(hipGetLastError());
    sync(s);   // (the pinned block is reused by the next upload)
}

void kd_build(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels, int n_levels,
              const int32_t* sizes, const int32_t* cur, const int32_t* newl, int final_mode,
              double* trace_out, double* lohi, int64_t* bad, hipStream_t s) {
    const bool final_split = final_mode == 1;
    if (n <= 0 || n_levels <= 0) throw Error(-1, "kd_build: no points or no levels");
    if (ctx.seq_moments || !vec_ok(d, X, labels))
        throw Error(-5, "kd_build: d <= 4, 16-byte aligned inputs and exact sums only");
    // per level: slot_of[ntab] | axis[S] | newlab[S] | (pad 8) bounds[7 S] | boundary[S]
    std::vector<size_t> off(n_levels + 1, 0), off_d(n_levels, 0), first(n_levels, 0);
    std::vector<int> ntab(n_levels, 1);
    int total = 0;
    for (int l = 0; l < n_levels; ++l) {
        const int S = sizes[l];
        if (S < 1 || S > kTabLds) throw Error(-5, "kd_build: level too wide");
        first[l] = total;
        for (int k = 0; k < S; ++k) {
            const int L = cur[total + k], N = newl[total + k];
            if (L < 0 || L >= kTabLds || N < 0) throw Error(-5, "kd_build: labels beyond the LDS tables");
            ntab[l] = std::max(ntab[l], L + 1);
        }
        const size_t ints = (size_t)ntab[l] + 2 * S;
        off_d[l] = off[l] + ((sizeof(int32_t) * ints + 7) & ~size_t(7));
        off[l + 1] = off_d[l] + sizeof(double) * 8 * S;
        total += S;
    }
    char* h = (char*)pinned(ctx, off[n_levels] + sizeof(double) * ((size_t)total * kTrace + 16));
    std::memset(h, 0, off[n_levels]);
    for (int l = 0; l < n_levels; ++l) {
        int32_t* slot = (int32_t*)(h + off[l]);
        const int S = sizes[l];
        for (int k = 0; k < ntab[l]; ++k) slot[k] = -1;
        for (int k = 0; k < S; ++k) {
            slot[cur[first[l] + k]] = k;
            slot[ntab[l] + S + k] = newl[first[l] + k];   // newlab after axis
        }
    }
    char* dt = ctx.arena.get<char>("kdb_tables", off[n_levels] + 64);
    PD_HIP(hipMemcpyAsync(dt, h, off[n_levels], hipMemcpyHostToDevice, s));
    struct Lv {
        int32_t *slot, *axis, *newlab;
        double *bounds, *boundary;
    };
    std::vector<Lv> lv(n_levels);
    for (int l = 0; l < n_levels; ++l) {
        const int S = sizes[l];
        lv[l].slot = (int32_t*)(dt + off[l]);
        lv[l].axis = lv[l].slot + ntab[l];
        lv[l].newlab = lv[l].axis + S;
        lv[l].bounds = (double*)(dt + off_d[l]);
        lv[l].boundary = lv[l].bounds + 7 * S;
    }
    double* trace = ctx.arena.get<double>("kdb_trace", (size_t)total * kTrace);
    unsigned long long* dcnt = ctx.arena.get<unsigned long long>("kdb_cnt", (size_t)kTabLds * 8);
    // Fused levels (kdf_kernel): a level of <= 2 splits whose
    // children are exactly the next level's splits counts its candidates and
    // sums its (split, interval) moments in one pass; the next level's
    // moments come from those (kdb_children_kernel) and its own counting pass
    // applies this level's split.  dst[l]: per split of level l, the slot of
    // its left / right child in level l + 1 (-1: not split there).
    // label replay: every level's tables in ReplayLds
    bool replay = final_mode == 2 && ctx.kd_replay && n_levels <= kMaxLevels;
    ReplayTab rpt;
    {
        int so = 0, eo = 0;
        for (int l = 0; l < n_levels && l < kMaxLevels; ++l) {
            rpt.ntab[l] = ntab[l];
            rpt.nsplit[l] = sizes[l];
            rpt.toff[l] = so;
            rpt.eoff[l] = eo;
            so += ntab[l];
            eo += sizes[l];
        }
        replay = replay && so <= kRSlots && eo <= kRSplits;
    }
    std::vector<char> fuse(n_levels, 0);
    std::vector<std::vector<int32_t>> dst(n_levels);
    for (int l = 0; ctx.kd_fuse && !replay && l + 1 < n_levels; ++l) {
        const int S = sizes[l], S1 = sizes[l + 1];
        if (S > 2 || S1 > 4) continue;
        std::vector<int32_t> dd(2 * S, -1);
        int found = 0;
        for (int j = 0; j < S1; ++j) {
            const int X = cur[first[l + 1] + j];
            for (int k = 0; k < S; ++k) {
                if (cur[first[l] + k] == X && dd[2 * k] < 0) { dd[2 * k] = j; ++found; break; }
                if (newl[first[l] + k] == X && dd[2 * k + 1] < 0) { dd[2 * k + 1] = j; ++found; break; }
            }
        }
        if (found != S1) continue;   // a split of level l + 1 is not a child of level l
        fuse[l] = 1;
        dst[l] = dd;
    }
    int32_t* ddst = ctx.arena.get<int32_t>("kdb_dst", (size_t)n_levels * 8);
    {
        std::vector<int32_t> hd((size_t)n_levels * 8, -1);
        for (int l = 0; l < n_levels; ++l)
            for (size_t i = 0; i < dst[l].size(); ++i) hd[(size_t)l * 8 + i] = dst[l][i];
        int32_t* hp = (int32_t*)(h + off[n_levels]);   // (the trace's block: read back only later)
        std::memcpy(hp, hd.data(), sizeof(int32_t) * hd.size());
        PD_HIP(hipMemcpyAsync(ddst, hp, sizeof(int32_t) * hd.size(), hipMemcpyHostToDevice, s));
    }
    for (int l = 0; replay && l < n_levels; ++l) {
        rpt.slot[l] = lv[l].slot;
        rpt.axis[l] = lv[l].axis;
        rpt.newlab[l] = lv[l].newlab;
        rpt.boundary[l] = lv[l].boundary;
    }
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        dispatch_d(d, [&](auto Dc) {
            constexpr int D = decltype(Dc)::value;
            constexpr int G = 1 + 4 * D;
            const T* Xt = (const T*)X;
            double* fin0 = ctx.arena.get<double>("kdb_fin0", G + 2 * D + 1);
            double* mom = ctx.arena.get<double>("kdb_mom", (size_t)kTabLds * G);
            double* momc = ctx.arena.get<double>("kdb_momc", (size_t)2 * 8 * G);   // children's
            double* ifin = ctx.arena.get<double>("kdb_ifin", (size_t)2 * 8 * G);   // interval moments
            const SplitTab none{nullptr, 0, nullptr, nullptr, nullptr, 0};
            run_pass_dev<T, D, false, false, 1, true>(ctx, Xt, n, labels, none,
                                                      make_int4(cur[0], -2, -2, -2), fin0, s);
            bool labels_written = false;   // some pass wrote the labels
            for (int l = 0; l < n_levels; ++l) {
                const int S = sizes[l];
                const int32_t* sel = cur + first[l];
                const double* m = fin0;
                // this level's counting pass still has the previous split to apply
                const bool pending = l > 0 && fuse[l - 1];
                ReplayTab rpl = rpt;   // the levels decided so far
                rpl.nl = l;
                if (l > 0 && pending) {
                    m = momc;
                } else if (l > 0 && replay) {
                    for (int g0 = 0; g0 < S; g0 += kGroup) {
                        const int ng = std::min(S - g0, kGroup);
                        int4 sl = make_int4(-2, -2, -2, -2);
                        for (int g = 0; g < ng; ++g) (&sl.x)[g] = sel[g0 + g];
                        dispatch_ng(ng, [&](auto NGc) {
                            constexpr int NG = decltype(NGc)::value;
                            run_pass_dev<T, D, false, false, NG, false, true>(
                                ctx, Xt, n, labels, none, sl, mom + (size_t)g0 * G, s, rpl);
                        });
                    }
                    m = mom;
                } else if (l > 0) {
                    const Lv& p = lv[l - 1];
                    const SplitTab sp{p.slot, ntab[l - 1], p.axis, p.boundary, p.newlab, sizes[l - 1]};
                    for (int g0 = 0; g0 < S; g0 += kGroup) {
                        const int ng = std::min(S - g0, kGroup);
                        int4 sl = make_int4(-2, -2, -2, -2);
                        for (int g = 0; g < ng; ++g) (&sl.x)[g] = sel[g0 + g];
                        dispatch_ng(ng, [&](auto NGc) {
                            constexpr int NG = decltype(NGc)::value;
                            if (g0 == 0 && !labels_written)   // labels all 0 so far: not read
                                run_pass_dev<T, D, false, true, NG, false>(ctx, Xt, n, labels, sp, sl,
                                                                           mom, s);
                            else if (g0 == 0)
                                run_pass_dev<T, D, true, true, NG, false>(ctx, Xt, n, labels, sp, sl,
                                                                          mom, s);
                            else
                                run_pass_dev<T, D, true, false, NG, false>(
                                    ctx, Xt, n, labels, none, sl, mom + (size_t)g0 * G, s);
                        });
                    }
                    labels_written = true;
                    m = mom;
                }
                double* tr = trace + (size_t)first[l] * kTrace;
                hipLaunchKernelGGL(kdb_axes_kernel, dim3(1), dim3(kTabLds), 0, s, m, S, D, G,
                                   lv[l].axis, lv[l].bounds, tr, dcnt);
                const unsigned nb4 = grid_for((n + 3) / 4, 2048);
                if (fuse[l] || pending) {
                    // kdf_kernel: the previous split (pending), the counts, and
                    // (fuse) the children's interval moments
                    const Lv* pv = pending ? &lv[l - 1] : nullptr;
                    const SplitTab sp = pending ? SplitTab{pv->slot, ntab[l - 1], pv->axis, pv->boundary,
                                                           pv->newlab, sizes[l - 1]}
                                                : none;
                    auto go = [&](auto LABc, auto SPc, auto NSc, auto MOMc) {
                        constexpr bool LAB_ = decltype(LABc)::value, SP_ = decltype(SPc)::value,
                                       MOM_ = decltype(MOMc)::value;
                        constexpr int NS_ = decltype(NSc)::value;
                        constexpr int NW_ = (MOM_ && NS_ == 2) ? 8 : 4;
                        constexpr int TP_ = 4 * ((sizeof(T) * D <= 16) ? 2 : 1) * 64 * NW_;
                        static int resident = 0;
                        if (!resident) {
                            int per_cu = 0, dev = 0, cus = 0;
                            PD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                &per_cu,
                                reinterpret_cast<const void*>(&kdf_kernel<T, D, LAB_, SP_, NS_, MOM_, NW_>),
                                64 * NW_, 0));
                            PD_HIP(hipGetDevice(&dev));
                            PD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
                            resident = std::max(1, per_cu) * std::max(1, cus);
                        }
                        const int nb = (int)std::min<int64_t>(resident, std::max<int64_t>(1, (n + TP_ - 1) / TP_));
                        double* part = MOM_ ? ctx.arena.get<double>("pass_part", (size_t)nb * NS_ * 8 * G)
                                            : nullptr;
                        hipLaunchKernelGGL((kdf_kernel<T, D, LAB_, SP_, NS_, MOM_, NW_>), dim3(nb),
                                           dim3(64 * NW_), 0, s, Xt, (uint64_t)n, labels, sp, lv[l].slot,
                                           ntab[l], lv[l].axis, lv[l].bounds, S, dcnt, part);
                        PD_HIP(hipGetLastError());
                        if constexpr (MOM_) {
                            hipLaunchKernelGGL(kd_finish_kernel, dim3(NS_ * 8 * G), dim3(kBlock), 0, s, part, nb,
                                               NS_ * 8 * G, G, D, NS_ * 8 * G, ifin);
                            PD_HIP(hipGetLastError());
                        }
                    };
                    using TT = std::true_type;
                    using FF = std::false_type;
                    auto ns = [&](auto LABc, auto SPc, auto MOMc) {
                        if (S == 1) go(LABc, SPc, std::integral_constant<int, 1>{}, MOMc);
                        else if (S == 2) go(LABc, SPc, std::integral_constant<int, 2>{}, MOMc);
                        else if constexpr (!decltype(MOMc)::value)
                            go(LABc, SPc, std::integral_constant<int, 4>{}, MOMc);
                    };
                    if (S > 4 || (fuse[l] && S > 2)) throw Error(-1, "kd_build: fused level too wide");
                    if (fuse[l]) {
                        if (!pending) ns(FF{}, FF{}, TT{});   // level 0: labels all 0, nothing to apply
                        else if (!labels_written) ns(FF{}, TT{}, TT{});
                        else ns(TT{}, TT{}, TT{});
                    } else {
                        if (!labels_written) ns(FF{}, TT{}, FF{});
                        else ns(TT{}, TT{}, FF{});
                    }
                    if (pending) labels_written = true;
                } else if (S <= 4) {
                    auto go = [&](auto NSc) {
                        constexpr int NS = decltype(NSc)::value;
                        if (replay && l > 0)
                            hipLaunchKernelGGL((counts_reg_kernel<T, D, NS, true>), dim3(nb4),
                                               dim3(kBlock), 0, s, Xt, (uint64_t)n, nullptr,
                                               lv[l].slot, ntab[l], lv[l].axis, lv[l].bounds, S,
                                               dcnt, rpl);
                        else
                            hipLaunchKernelGGL((counts_reg_kernel<T, D, NS>), dim3(nb4), dim3(kBlock), 0,
                                               s, Xt, (uint64_t)n, labels_written ? labels : nullptr,
                                               lv[l].slot, ntab[l], lv[l].axis, lv[l].bounds, S, dcnt,
                                               ReplayTab{});
                    };
                    if (S == 1)
                        go(std::integral_constant<int, 1>{});
                    else if (S == 2)
                        go(std::integral_constant<int, 2>{});
                    else
                        go(std::integral_constant<int, 4>{});
                } else {
                    int rep = kRep;
                    while (rep > 1 && (size_t)rep * S * 8 * sizeof(unsigned int) > 48 * 1024) rep >>= 1;
                    hipLaunchKernelGGL((counts4_kernel<T, D>), dim3(nb4), dim3(kBlock),
                                       sizeof(unsigned int) * rep * S * 8, s, Xt, (uint64_t)n, labels,
                                       lv[l].slot, ntab[l], lv[l].axis, lv[l].bounds, S, 0, rep,
                                       dcnt, replay ? rpl : ReplayTab{});
                }
                PD_HIP(hipGetLastError());
                hipLaunchKernelGGL(kdb_boundary_kernel, dim3(1), dim3(kTabLds), 0, s, dcnt, S,
                                   lv[l].bounds, lv[l].boundary, tr);
                PD_HIP(hipGetLastError());
                if (fuse[l]) {
                    hipLaunchKernelGGL(kdb_children_kernel, dim3(1), dim3(64), 0, s, ifin, S, G, tr,
                                       ddst + (size_t)l * 8, momc);
                    PD_HIP(hipGetLastError());
                }
            }
            // the last level's split alone (or left to the caller: pd_train_tree
            // replays the split tree, the labels are then applied lazily)
            if (final_split) {
                const Lv& p = lv[n_levels - 1];
                const SplitTab sp{p.slot, ntab[n_levels - 1], p.axis, p.boundary, p.newlab,
                                  sizes[n_levels - 1]};
                if (!labels_written)   // no level pass wrote the labels yet
                    run_pass_dev<T, D, false, true, 0, false>(ctx, Xt, n, labels, sp,
                                                              make_int4(-2, -2, -2, -2), nullptr, s);
                else
                    run_pass_dev<T, D, true, true, 0, false>(ctx, Xt, n, labels, sp,
                                                             make_int4(-2, -2, -2, -2), nullptr, s);
            }
            // one copy back: the trace and the bbox
            double* ht = (double*)(h + off[n_levels]);
            PD_HIP(hipMemcpyAsync(ht, trace, sizeof(double) * total * kTrace, hipMemcpyDeviceToHost, s));
            PD_HIP(hipMemcpyAsync(ht + (size_t)total * kTrace, fin0 + G, sizeof(double) * (2 * D + 1),
                                  hipMemcpyDeviceToHost, s));
            sync(s);
            std::memcpy(trace_out, ht, sizeof(double) * total * kTrace);
            for (int j = 0; j < 2 * D; ++j) lohi[j] = ht[(size_t)total * kTrace + j];
            if (bad) *bad = (int64_t)ht[(size_t)total * kTrace + 2 * D];
        });
    });
}

// ---------------------------------------------------------------- sharded device-decided KD
// pd_kd_build split at its collectives: every rank runs the same level chain
// on its slice, and between the passes the caller all-gathers the moment
// partials (rank order) and all-reduces the counts on the device, so a level
// costs no host round trip.  The partials of all ranks are added with the
// host path's double-double fold (distributed.dd_combine: dd_add in rank
// order from zero), then kdb_axes_kernel / kdb_boundary_kernel decide as
// pd_kd_build does — the splits equal the host-decided sharded path's and the
// single-device ones bit for bit.
namespace {
// out[k] for k < S*G: the rank-order fold of gathered[w][k] (counts: sums; dd
// pairs: dd_add); level 0 also folds the bbox (min / max / non-finite sum).
__global__ void kdx_combine_kernel(const double* __restrict__ g, int W, int len, int SG, int G,
                                   int D, double* __restrict__ mom, double* __restrict__ bbox) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= len) return;
    if (k < SG) {
        const int r = k % G;
        if (r == 0) {
            double c = 0.0;
            for (int w = 0; w < W; ++w) c = __dadd_rn(c, g[(size_t)w * len + k]);
            mom[k] = c;
        } else if ((r - 1) % 2 == 0) {
            DD a{0.0, 0.0};
            for (int w = 0; w < W; ++w)
                a = dd_add(a, DD{g[(size_t)w * len + k], g[(size_t)w * len + k + 1]});
            mom[k] = a.hi;
            mom[k + 1] = a.lo;
        }
        return;
    }
    const int b = k - SG;
    double x = b < D ? INFINITY : (b < 2 * D ? -INFINITY : 0.0);
    for (int w = 0; w < W; ++w) {
        const double v = g[(size_t)w * len + k];
        x = b < D ? fmin(x, v) : (b < 2 * D ? fmax(x, v) : __dadd_rn(x, v));
    }
    bbox[b] = x;
}

// An empty slice's partials: zero moments, an empty bbox.
__global__ void kdx_empty_kernel(double* __restrict__ out, int SG, int len, int D) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= len) return;
    const int b = k - SG;
    out[k] = k < SG ? 0.0 : (b < D ? INFINITY : (b < 2 * D ? -INFINITY : 0.0));
}

struct KdxLv {
    int32_t *slot, *axis, *newlab;
    double *bounds, *boundary;
};

KdxLv kdx_level(const KdxState& k, int l) {
    const int S = k.sizes[l];
    KdxLv v;
    v.slot = (int32_t*)(k.tables + k.off[l]);
    v.axis = v.slot + k.ntab[l];
    v.newlab = v.axis + S;
    v.bounds = (double*)(k.tables + k.off_d[l]);
    v.boundary = v.bounds + 7 * S;
    return v;
}

void kdx_check(const Ctx& ctx, int level) {
    if (!ctx.kdx.valid) throw Error(-1, "pd_kdx_*: no pd_kdx_begin on this context");
    if (level < 0 || level >= ctx.kdx.n_levels) throw Error(-1, "pd_kdx_*: level out of range");
}
}  // namespace

void kdx_begin(Ctx& ctx, int d, int n_levels, const int32_t* sizes, const int32_t* cur,
               const int32_t* newl, hipStream_t s) {
    KdxState& k = ctx.kdx;
    k = KdxState{};
    if (n_levels <= 0 || n_levels > 16) throw Error(-5, "pd_kdx_begin: 1..16 levels");
    if (d < 1 || d > kMaxDim) throw Error(-5, "pd_kdx_begin: d <= 4");
    k.n_levels = n_levels;
    k.d = d;
    k.sizes.assign(sizes, sizes + n_levels);
    k.first.assign(n_levels, 0);
    k.ntab.assign(n_levels, 1);
    k.off.assign(n_levels + 1, 0);
    k.off_d.assign(n_levels, 0);
    int total = 0;
    for (int l = 0; l < n_levels; ++l) {
        const int S = sizes[l];
        if (S < 1 || S > kTabLds) throw Error(-5, "pd_kdx_begin: level too wide");
        k.first[l] = total;
        for (int q = 0; q < S; ++q) {
            const int L = cur[total + q], N = newl[total + q];
            if (L < 0 || L >= kTabLds || N < 0)
                throw Error(-5, "pd_kdx_begin: labels beyond the LDS tables");
            k.ntab[l] = std::max(k.ntab[l], L + 1);
        }
        const size_t ints = (size_t)k.ntab[l] + 2 * S;
        k.off_d[l] = k.off[l] + ((sizeof(int32_t) * ints + 7) & ~size_t(7));
        k.off[l + 1] = k.off_d[l] + sizeof(double) * 8 * S;
        total += S;
    }
    k.total = total;
    k.cur.assign(cur, cur + total);
    char* h = (char*)pinned(ctx, k.off[n_levels]);
    std::memset(h, 0, k.off[n_levels]);
    for (int l = 0; l < n_levels; ++l) {
        int32_t* slot = (int32_t*)(h + k.off[l]);
        const int S = sizes[l];
        for (int q = 0; q < k.ntab[l]; ++q) slot[q] = -1;
        for (int q = 0; q < S; ++q) {
            slot[cur[k.first[l] + q]] = q;
            slot[k.ntab[l] + S + q] = newl[k.first[l] + q];
        }
    }
    k.tables = ctx.arena.get<char>("kdx_tables", k.off[n_levels] + 64);
    PD_HIP(hipMemcpyAsync(k.tables, h, k.off[n_levels], hipMemcpyHostToDevice, s));
    sync(s);   // the pinned block is reused by later calls
    k.trace = ctx.arena.get<double>("kdx_trace", (size_t)total * kTrace);
    k.bbox = ctx.arena.get<double>("kdx_bbox", 2 * kMaxDim + 1);
    k.mom = ctx.arena.get<double>("kdx_mom", (size_t)kTabLds * (1 + 4 * kMaxDim));
    k.valid = true;
}

void kdx_moments(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels, int level,
                 double* out, hipStream_t s) {
    kdx_check(ctx, level);
    const KdxState& k = ctx.kdx;
    if (d != k.d) throw Error(-1, "pd_kdx_moments: d differs from pd_kdx_begin");
    const int S = k.sizes[level], G = 1 + 4 * d;
    const int len = S * G + (level == 0 ? 2 * d + 1 : 0);
    if (n == 0) {
        hipLaunchKernelGGL(kdx_empty_kernel, dim3((len + 255) / 256), dim3(256), 0, s, out, S * G,
                           len, d);
        PD_HIP(hipGetLastError());
        return;
    }
    if (ctx.seq_moments || !vec_ok(d, X, labels))
        throw Error(-5, "pd_kdx_moments: d <= 4, 16-byte aligned inputs and exact sums only");
    const int32_t* sel = k.cur.data() + k.first[level];
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        dispatch_d(d, [&](auto Dc) {
            constexpr int D = decltype(Dc)::value;
            constexpr int Gc = 1 + 4 * D;
            const T* Xt = (const T*)X;
            const SplitTab none{nullptr, 0, nullptr, nullptr, nullptr, 0};
            if (level == 0) {   // bbox + the root's moments, labels not read
                run_pass_dev<T, D, false, false, 1, true>(ctx, Xt, n, labels, none,
                                                          make_int4(sel[0], -2, -2, -2), out, s);
                return;
            }
            const KdxLv p = kdx_level(k, level - 1);
            const SplitTab sp{p.slot, k.ntab[level - 1], p.axis, p.boundary, p.newlab,
                              k.sizes[level - 1]};
            for (int g0 = 0; g0 < S; g0 += kGroup) {
                const int ng = std::min(S - g0, kGroup);
                int4 sl = make_int4(-2, -2, -2, -2);
                for (int g = 0; g < ng; ++g) (&sl.x)[g] = sel[g0 + g];
                dispatch_ng(ng, [&](auto NGc) {
                    constexpr int NG = decltype(NGc)::value;
                    if (g0 == 0)
                        run_pass_dev<T, D, true, true, NG, false>(ctx, Xt, n, labels, sp, sl, out, s);
                    else
                        run_pass_dev<T, D, true, false, NG, false>(ctx, Xt, n, labels, none, sl,
                                                                   out + (size_t)g0 * Gc, s);
                });
            }
        });
    });
}

void kdx_axes(Ctx& ctx, const double* gathered, int n_ranks, int level, hipStream_t s) {
    kdx_check(ctx, level);
    const KdxState& k = ctx.kdx;
    if (n_ranks < 1) throw Error(-1, "pd_kdx_axes: n_ranks < 1");
    const int d = k.d, S = k.sizes[level], G = 1 + 4 * d;
    const int len = S * G + (level == 0 ? 2 * d + 1 : 0);
    hipLaunchKernelGGL(kdx_combine_kernel, dim3((len + 255) / 256), dim3(256), 0, s, gathered,
                       n_ranks, len, S * G, G, d, k.mom, k.bbox);
    const KdxLv v = kdx_level(k, level);
    hipLaunchKernelGGL(kdb_axes_kernel, dim3(1), dim3(kTabLds), 0, s, k.mom, S, d, G, v.axis,
                       v.bounds, k.trace + (size_t)k.first[level] * kTrace,
                       (unsigned long long*)nullptr);
    PD_HIP(hipGetLastError());
}

void kdx_counts(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                int level, unsigned long long* out, hipStream_t s) {
    kdx_check(ctx, level);
    const KdxState& k = ctx.kdx;
    const int S = k.sizes[level];
    PD_HIP(hipMemsetAsync(out, 0, sizeof(unsigned long long) * S * 8, s));
    if (n == 0) return;
    if (!vec_ok(d, X, labels)) throw Error(-5, "pd_kdx_counts: 16-byte aligned inputs only");
    const KdxLv v = kdx_level(k, level);
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        dispatch_d(d, [&](auto Dc) {
            constexpr int D = decltype(Dc)::value;
            const T* Xt = (const T*)X;
            const unsigned nb4 = grid_for((n + 3) / 4, 2048);
            if (S <= 4) {
                auto go = [&](auto NSc) {
                    constexpr int NS = decltype(NSc)::value;
                    hipLaunchKernelGGL((counts_reg_kernel<T, D, NS>), dim3(nb4), dim3(kBlock), 0, s,
                                       Xt, (uint64_t)n, labels, v.slot, k.ntab[level], v.axis,
                                       v.bounds, S, out, ReplayTab{});
                };
                if (S == 1)
                    go(std::integral_constant<int, 1>{});
                else if (S == 2)
                    go(std::integral_constant<int, 2>{});
                else
                    go(std::integral_constant<int, 4>{});
            } else {
                int rep = kRep;
                while (rep > 1 && (size_t)rep * S * 8 * sizeof(unsigned int) > 48 * 1024) rep >>= 1;
                hipLaunchKernelGGL((counts4_kernel<T, D>), dim3(nb4), dim3(kBlock),
                                   sizeof(unsigned int) * rep * S * 8, s, Xt, (uint64_t)n, labels,
                                   v.slot, k.ntab[level], v.axis, v.bounds, S, 0, rep, out, ReplayTab{});
            }
        });
    });
    PD_HIP(hipGetLastError());
}

void kdx_boundary(Ctx& ctx, const unsigned long long* cnt, int level, hipStream_t s) {
    kdx_check(ctx, level);
    const KdxState& k = ctx.kdx;
    const KdxLv v = kdx_level(k, level);
    hipLaunchKernelGGL(kdb_boundary_kernel, dim3(1), dim3(kTabLds), 0, s, cnt, k.sizes[level],
                       v.bounds, v.boundary, k.trace + (size_t)k.first[level] * kTrace);
    PD_HIP(hipGetLastError());
}

void kdx_end(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
             bool final_split, double* trace_out, double* lohi, int64_t* bad, hipStream_t s) {
    KdxState& k = ctx.kdx;
    if (!k.valid) throw Error(-1, "pd_kdx_end: no pd_kdx_begin on this context");
    if (d != k.d) throw Error(-1, "pd_kdx_end: d differs from pd_kdx_begin");
    const int nl = k.n_levels;
    if (final_split && n > 0) {
        if (!vec_ok(d, X, labels)) throw Error(-5, "pd_kdx_end: 16-byte aligned inputs only");
        const KdxLv p = kdx_level(k, nl - 1);
        const SplitTab sp{p.slot, k.ntab[nl - 1], p.axis, p.boundary, p.newlab, k.sizes[nl - 1]};
        dispatch_t(dtype, [&](auto tp) {
            using T = std::remove_pointer_t<decltype(tp)>;
            dispatch_d(d, [&](auto Dc) {
                constexpr int D = decltype(Dc)::value;
                run_pass_dev<T, D, true, true, 0, false>(ctx, (const T*)X, n, labels, sp,
                                                         make_int4(-2, -2, -2, -2), nullptr, s);
            });
        });
    }
    double* h = (double*)pinned(ctx, sizeof(double) * ((size_t)k.total * kTrace + 2 * kMaxDim + 8));
    PD_HIP(hipMemcpyAsync(h, k.trace, sizeof(double) * k.total * kTrace, hipMemcpyDeviceToHost, s));
    PD_HIP(hipMemcpyAsync(h + (size_t)k.total * kTrace, k.bbox, sizeof(double) * (2 * d + 1),
                          hipMemcpyDeviceToHost, s));
    sync(s);
    std::memcpy(trace_out, h, sizeof(double) * k.total * kTrace);
    for (int j = 0; j < 2 * d; ++j) lohi[j] = h[(size_t)k.total * kTrace + j];
    if (bad) *bad = (int64_t)h[(size_t)k.total * kTrace + 2 * d];
    k.valid = false;
}

void kd_radix_hist(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                   int n_sel, const int32_t* sel, const int32_t* axis, const uint64_t* prefix,
                   int shift, int64_t* out, hipStream_t s) {
    if (n_sel <= 0) return;
    // the u64 prefixes travel in the tables' fp64 slots (bit copies)
    LabelTables t = upload_tables(ctx, n_sel, sel, axis, reinterpret_cast<const double*>(prefix),
                                  1, nullptr, s);
    unsigned int* dh = ctx.arena.get<unsigned int>("kd_rhist", (size_t)n_sel * 256);
    PD_HIP(hipMemsetAsync(dh, 0, sizeof(unsigned int) * n_sel * 256, s));
    const int lds = n_sel <= 48 ? 1 : 0;   // <= 48 KiB of LDS histograms per block
    const unsigned nb = grid_for(n, 2048);
    dispatch_t(dtype, [&](auto tp) {
        using T = std::remove_pointer_t<decltype(tp)>;
        hipLaunchKernelGGL((radix_hist_kernel<T>), dim3(nb), dim3(kBlock),
                           lds ? sizeof(unsigned int) * n_sel * 256 : 0, s, (const T*)X,
                           (uint64_t)n, (uint32_t)d, labels, t.slot_of, t.ntab, t.axis,
                           reinterpret_cast<const uint64_t*>(t.dbl), shift, n_sel, lds, dh);
    });
    PD_HIP(hipGetLastError());
    unsigned int* h = (unsigned int*)pinned(ctx, sizeof(unsigned int) * n_sel * 256);
    PD_HIP(hipMemcpyAsync(h, dh, sizeof(unsigned int) * n_sel * 256, hipMemcpyDeviceToHost, s));
    sync(s);
    for (int k = 0; k < n_sel * 256; ++k) out[k] = (int64_t)h[k];
}

void halo_members(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P,
                  const double* ebox, int64_t* counts, int64_t* members, int64_t cap,
                  hipStream_t s) {
    double* dbox = ctx.arena.get<double>("halo_box", (size_t)P * 2 * d);
    double* hbox = (double*)pinned(ctx, sizeof(double) * P * 2 * d + sizeof(int64_t));
    std::memcpy(hbox, ebox, sizeof(double) * P * 2 * d);
    PD_HIP(hipMemcpyAsync(dbox, hbox, sizeof(double) * P * 2 * d, hipMemcpyHostToDevice, s));
    int64_t* dsel = ctx.arena.get<int64_t>("halo_nsel", 1);
    int64_t* scratch = members ? nullptr : ctx.arena.get<int64_t>("halo_scratch", (size_t)n);
    int64_t used = 0;
    for (int L = 0; L < P; ++L) {
        int64_t* outp = members ? members + used : scratch;
        auto run_select = [&](auto pred) {
            rocprim::counting_iterator<int64_t> it(0);
            size_t tb = 0;
            PD_HIP(rocprim::select(nullptr, tb, it, outp, dsel, (size_t)n, pred, s));
            void* tmp = ctx.arena.get<char>("halo_tmp", tb);
            PD_HIP(rocprim::select(tmp, tb, it, outp, dsel, (size_t)n, pred, s));
        };
        dispatch_t(dtype, [&](auto tp) {
            using T = std::remove_pointer_t<decltype(tp)>;
            if (d <= kMaxDim)
                dispatch_d(d, [&](auto Dc) {
                    constexpr int D = decltype(Dc)::value;
                    run_select(InBox<T, D>{(const T*)X, dbox + (size_t)L * 2 * D});
                });
            else
                run_select(InBoxDyn<T>{(const T*)X, dbox + (size_t)L * 2 * d, d});
        });
        int64_t* h = (int64_t*)pinned(ctx, sizeof(int64_t));
        PD_HIP(hipMemcpyAsync(h, dsel, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        sync(s);
        counts[L] = *h;
        used += *h;
        if (members && used > cap) throw Error(-1, "halo_members: members buffer too small");
    }
}

}  // namespace pd
