// Stable LSD radix sort of (key, 32-bit value) pairs, one pass per 8-bit
// digit, each pass ONE kernel (the "onesweep" scheme): a tile of the input
// ranks its items by digit in LDS, learns how many items of each digit the
// tiles before it hold from their published counts (decoupled look-back),
// and writes its items out as digit runs through an LDS staging copy, so
// the global writes are contiguous per digit.  The digit histograms of all
// passes come from one counting pass over the keys first.
//
// Written for gfx950: 64-wide waves rank 64 items per step with eight
// ballots (a lane's peers = the lanes whose digit has the same 8 bits), one
// LDS counter per (wave, digit) keeps the running ranks, no LDS atomics.
// Tile t takes its index from a ticket counter, so the tile it waits for
// (t - 1) was dispatched before it and never waits for it: forward progress
// without assuming any dispatch order.  The look-back words carry a pass
// epoch, so no buffer is cleared between passes or calls.
#pragma once

#include <algorithm>
#include <utility>

#include "common.hpp"

namespace pd {
namespace rsort {

constexpr int kThreads = 256;   // histogram kernels
constexpr int kRadix = 256;

template <typename K>
struct Tile {
    // u32 keys: 512 threads x 16 items (8192-item tiles, 72 KB of LDS, 2
    // blocks per CU): 2.40 ms for 1e8 pairs (256 x 32: 2.57, 1024 x 12:
    // 2.58, 256 x 16: 3.18; rocPRIM 3.02).  u64 keys: 256 x 24 (6144-item
    // tiles, 78 KB): 7.76 ms for 2e8 37-bit pairs (1024 x 8: 8.24, 512 x
    // 12: 9.96; rocPRIM 8.25).  tools/sort_probe.hip
    static constexpr int kThreads = sizeof(K) == 4 ? 512 : 256;
    static constexpr int kItems = sizeof(K) == 4 ? 16 : 24;
    static constexpr int kSize = kThreads * kItems;
};
template <typename K>
constexpr int default_items() { return Tile<K>::kItems; }

__device__ __forceinline__ uint32_t digit_of(uint32_t k, int shift) { return (k >> shift) & 0xFFu; }
__device__ __forceinline__ uint32_t digit_of(uint64_t k, int shift) {
    return (uint32_t)(k >> shift) & 0xFFu;
}

// Digit histograms of `places` passes (place p: bits [8p + begin, +8), the
// last place's digit masked by last_mask so only the sorted bits count), one
// read of the keys (16-byte loads), each wave counting into its own LDS copy
// (no atomics between waves).  hist: places x 256 uint32, zeroed by the caller.
template <typename K>
__global__ __launch_bounds__(kThreads) void hist_kernel(const K* __restrict__ keys, uint64_t n,
                                                        int begin, int places, int vec,
                                                        uint32_t last_mask,
                                                        uint32_t* __restrict__ hist) {
    constexpr int NW = kThreads / 64, V = 16 / sizeof(K);   // keys per 16-byte load
    __shared__ uint32_t h[NW][8][kRadix];
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < NW * 8 * kRadix; i += kThreads) (&h[0][0][0])[i] = 0;
    __syncthreads();
    const uint64_t nv = vec ? n / V : 0;   // (vec: keys 16-byte aligned)
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < nv;
         i += (uint64_t)gridDim.x * kThreads) {
        const uint4 q = kv[i];
        K k[V];
        __builtin_memcpy(k, &q, 16);
#pragma unroll
        for (int u = 0; u < V; ++u)
            for (int p = 0; p < places; ++p)
                atomicAdd(&h[w][p][digit_of(k[u], begin + 8 * p) & (p == places - 1 ? last_mask : 0xFFu)], 1u);
    }
    // the tail (< V keys; every key when unaligned)
    for (uint64_t i = nv * V + (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kThreads) {
        const K k = keys[i];
        for (int p = 0; p < places; ++p)
            atomicAdd(&h[w][p][digit_of(k, begin + 8 * p) & (p == places - 1 ? last_mask : 0xFFu)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < places * kRadix; i += kThreads) {
        uint32_t c = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) c += (&h[u][0][0])[i];
        if (c) atomicAdd(hist + i, c);
    }
}

// hist (places x 256) -> exclusive digit offsets per place, in place; also
// starts the sort's tile ticket at 0 (pass p's tiles take p * tiles ..).
__global__ __launch_bounds__(kRadix) void hist_scan_kernel(uint32_t* __restrict__ hist, int places,
                                                           unsigned long long* __restrict__ ticket) {
    __shared__ uint32_t ws[kRadix / 64];
    const int d = threadIdx.x, lane = d & 63, w = d >> 6;
    if (d == 0) *ticket = 0ull;
    for (int p = 0; p < places; ++p) {
        const uint32_t v = hist[p * kRadix + d];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[w] = x;
        __syncthreads();
        uint32_t before = 0;
#pragma unroll
        for (int u = 0; u < kRadix / 64; ++u) before += u < w ? ws[u] : 0u;
        hist[p * kRadix + d] = before + x - v;
        __syncthreads();
    }
}

// Look-back words are self-contained (tag and count in one 64-bit word,
// written whole), so relaxed device-scope atomics suffice: no other data is
// published through them.  (Acquire / release here cost a cache invalidate
// or write-back per step of the look-back: 20x slower.)
__device__ __forceinline__ uint64_t ld_lb(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_lb(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One pass over bits [shift, shift + 8) & dmask (dmask < 0xFF on the last
// pass when the key width is not a multiple of 8: the bits above it are not
// sorted, as rocPRIM's begin/end bits).  goff: this place's exclusive digit
// offsets; look: ntiles x 256 look-back words (tag << 32 | count; tag =
// 2 epoch + 1 aggregate of the tile alone, 2 epoch + 2 inclusive of all tiles
// up to it; older tags read as not yet published); ticket: 64-bit counter,
// tile = atomicAdd(ticket, 1) - tick0 (the sort's p-th pass: tick0 = p tiles).
template <typename K, int I = Tile<K>::kItems, int NT = Tile<K>::kThreads>
__global__ __launch_bounds__(NT) void pass_kernel(const K* __restrict__ kin,
                                                  const uint32_t* __restrict__ vin,
                                                  K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                  uint64_t n, int shift, uint32_t dmask,
                                                  const uint32_t* __restrict__ goff,
                                                  uint64_t* __restrict__ look, uint32_t epoch,
                                                  unsigned long long* __restrict__ ticket,
                                                  unsigned long long tick0) {
    // NT threads (NT / 64 waves) rank the tile; the first 256 also carry one
    // digit each through the count / scan / look-back phase
    constexpr int T = NT * I, NW = NT / 64;
    static_assert(NT >= kRadix && NT % 64 == 0, "one thread per digit");
    __shared__ K sk[T];
    __shared__ uint32_t sv[T];
    __shared__ uint32_t wcnt[NW][kRadix];
    __shared__ uint32_t dbase[kRadix];
    __shared__ uint32_t gbase[kRadix];
    __shared__ uint32_t ws[kRadix / 64];
    __shared__ uint32_t s_tile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tick0);
    for (int d = lane; d < kRadix; d += 64) wcnt[w][d] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * T;
    const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)T ? n - t0 : (uint64_t)T);
    // wave w holds items [w I 64, (w + 1) I 64) of the tile, slot j lane l =
    // item w I 64 + 64 j + l: (w, j, l) order is index order (stable)
    K k[I];
    uint32_t v[I], rk[I];
    const uint32_t wbase = (uint32_t)w * I * 64;
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t i = wbase + 64 * j + lane;
        const bool ok = i < tn;
        k[j] = ok ? kin[t0 + i] : K(0);
        v[j] = ok ? vin[t0 + i] : 0u;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t i = wbase + 64 * j + lane;
        const bool ok = i < tn;
        const uint32_t d = digit_of(k[j], shift) & dmask;
        unsigned long long m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t base = wcnt[w][d];
        rk[j] = base + (uint32_t)__popcll(m & lt);
        if (ok && (m & lt) == 0) wcnt[w][d] = base + (uint32_t)__popcll(m);
    }
    __syncthreads();
    const bool dig = tid < kRadix;
    const int d = tid & (kRadix - 1);
    // per digit: the tile's count, the waves' exclusive prefixes (in place)
    uint32_t h = 0;
    uint64_t* lk = look + (uint64_t)tile * kRadix + d;
    const uint64_t agg_tag = (uint64_t)(2u * epoch + 1u) << 32, inc_tag = (uint64_t)(2u * epoch + 2u) << 32;
    uint32_t x = 0;
    if (dig) {
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            const uint32_t c = wcnt[u][d];
            wcnt[u][d] = h;
            h += c;
        }
        // publish the tile's own count first (tile 0: already inclusive)
        st_lb(lk, (tile == 0 ? inc_tag : agg_tag) | h);
        // tile-local exclusive digit starts
        x = h;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[w] = x;
    }
    __syncthreads();
    if (dig) {
        uint32_t before = 0;
#pragma unroll
        for (int u = 0; u < kRadix / 64; ++u) before += u < w ? ws[u] : 0u;
        dbase[d] = before + x - h;
        // look back: items of digit d in the tiles before this one (one
        // dependent load per step; reading 8 words per step measured the
        // same, 2.57 ms for 1e8 pairs: the walk is short)
        uint32_t excl = 0;
        if (tile > 0) {
            int64_t t = (int64_t)tile - 1;
            while (t >= 0) {
                const uint64_t sw = ld_lb(look + (uint64_t)t * kRadix + d);
                const uint32_t tag = (uint32_t)(sw >> 32);
                if (tag < 2u * epoch + 1u) continue;   // not published yet: spin
                excl += (uint32_t)sw;
                if (tag == 2u * epoch + 2u) break;
                --t;
            }
            st_lb(lk, inc_tag | (excl + h));
        }
        gbase[d] = goff[d] + excl;
    }
    __syncthreads();
    // stage the tile in digit order
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t i = wbase + 64 * j + lane;
        if (i < tn) {
            const uint32_t dj = digit_of(k[j], shift) & dmask;
            const uint32_t p = dbase[dj] + wcnt[w][dj] + rk[j];
            sk[p] = k[j];
            sv[p] = v[j];
        }
    }
    __syncthreads();
    // contiguous runs per digit
    for (uint32_t i = tid; i < tn; i += NT) {
        const K key = sk[i];
        const uint32_t dk = digit_of(key, shift) & dmask;
        const uint64_t g = (uint64_t)gbase[dk] + (i - dbase[dk]);
        kout[g] = key;
        vout[g] = sv[i];
    }
}

// State of the sorts run on one stream: the look-back words (zeroed when
// allocated, then tagged by the host's pass epoch), the digit histograms and
// the tile ticket (restarted by every sort).
struct State {
    uint64_t* look = nullptr;            // look_tiles x 256
    uint64_t look_tiles = 0;
    uint32_t* hist = nullptr;            // 8 x 256
    unsigned long long* ticket = nullptr;
    uint32_t epoch = 0;
};

inline uint64_t tiles_for(uint64_t n, int key_bytes) {
    const uint64_t T = key_bytes == 4 ? Tile<uint32_t>::kSize : Tile<uint64_t>::kSize;
    return (n + T - 1) / T;
}

// Sort (k0, v0) by key bits [0, bits) through the double buffer (k1, v1); the
// sorted pairs end in (*kres, *vres), one of the two.  Stable; bits at and
// above `bits` are ignored (pairs equal in [0, bits) keep their input order).
// st.look must hold tiles_for(n) tiles; st.hist 8 x 256; st.ticket one counter.
// hist_zeroed: the caller already zeroed st.hist (8 x 256) on the stream.
template <typename K, int I = Tile<K>::kItems, int NT = Tile<K>::kThreads>
void sort_pairs(State& st, K* k0, uint32_t* v0, K* k1, uint32_t* v1, uint64_t n, int bits,
                hipStream_t s, K** kres, uint32_t** vres, bool hist_zeroed) {
    *kres = k0;
    *vres = v0;
    if (n == 0 || bits <= 0) return;
    const int places = (bits + 7) / 8;
    if (places > 8 || bits > 8 * (int)sizeof(K)) throw Error(-5, "rsort: key bits beyond the key");
    const uint32_t last_mask = (bits % 8) ? (1u << (bits % 8)) - 1u : 0xFFu;
    if (!hist_zeroed) PD_HIP(hipMemsetAsync(st.hist, 0, sizeof(uint32_t) * kRadix * places, s));
    const unsigned hb = (unsigned)std::min<uint64_t>(2048, (n + kThreads - 1) / kThreads);
    const int vec = ((uintptr_t)k0 & 15) == 0 ? 1 : 0;
    hipLaunchKernelGGL((hist_kernel<K>), dim3(hb), dim3(kThreads), 0, s, k0, n, 0, places, vec,
                       last_mask, st.hist);
    hipLaunchKernelGGL(hist_scan_kernel, dim3(1), dim3(kRadix), 0, s, st.hist, places, st.ticket);
    const uint64_t tiles = (n + (uint64_t)NT * I - 1) / ((uint64_t)NT * I);
    if (tiles > st.look_tiles) throw Error(-5, "rsort: look-back buffer too small");
    K* ki = k0;
    uint32_t* vi = v0;
    K* ko = k1;
    uint32_t* vo = v1;
    for (int p = 0; p < places; ++p) {
        if (st.epoch >= 0x7FFFFFF0u) {   // tags would overflow: start over from zeroed words
            PD_HIP(hipMemsetAsync(st.look, 0, sizeof(uint64_t) * kRadix * st.look_tiles, s));
            st.epoch = 0;
        }
        // (the epoch is consumed before the launch: a pass that fails never
        // leaves words a later pass could take for its own)
        const uint32_t ep = st.epoch++;
        hipLaunchKernelGGL((pass_kernel<K, I, NT>), dim3((unsigned)tiles), dim3(NT), 0, s, ki, vi, ko,
                           vo, n, 8 * p, p == places - 1 ? last_mask : 0xFFu,
                           st.hist + p * kRadix, st.look, ep, st.ticket,
                           (unsigned long long)p * tiles);
        PD_HIP(hipGetLastError());
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    *kres = ki;
    *vres = vi;
}

}  // namespace rsort
}  // namespace pd
