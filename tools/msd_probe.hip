// Probe for the two-level bucketed sort (round 5): how fast can one MSD
// scatter pass move 24-B records (u32 key, u32 val, float4 coordinates, SoA)
// into B buckets, staged through LDS (runs written by consecutive threads)
// or scattered directly; and how fast does a one-workgroup LDS radix sort of
// <= 16k-record segments (rocprim block_radix_sort) write them out in order?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/msd_probe.hip -o tools/msd_probe
// Result on one MI355X (profiles/r05_v1_msd_probe.txt, 1e8 records): one
// staged scatter pass 2.0-2.8 ms (1.7-2.4 TB/s of 48 B per record) for 256 to
// 4096 buckets, 1.0-1.2 TB/s scattered directly; the final LDS sort 2.4-4.1
// ms.  The full bucketed sort built from them (round 5, later removed) took
// C2 8.76 ms against the onesweep + gather's 5.91 ms
// (profiles/r05_v1_ab_bucket_sort.txt).
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

constexpr int kThreads = 1024, kPer = 16, kTile = kThreads * kPer;   // records per tile

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void gen_kernel(uint32_t* key, uint32_t* val, float4* xyz, uint32_t R, uint32_t kmask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    key[i] = hash32(i * 2654435761u + 17u) & kmask;
    val[i] = i;
    xyz[i] = make_float4((float)i, (float)(i ^ 5), (float)(i * 3), 0.0f);
}

// per tile: bucket histogram, one column of the bucket-major matrix
__global__ __launch_bounds__(kThreads) void hist_kernel(const uint32_t* __restrict__ key, uint32_t R,
                                                        int shift, int B, uint32_t ntiles,
                                                        uint32_t* __restrict__ hist) {
    extern __shared__ uint32_t h[];
    for (int b = threadIdx.x; b < B; b += kThreads) h[b] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kThreads + threadIdx.x;
        if (r < R) atomicAdd(&h[key[r] >> shift], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += kThreads) hist[(uint64_t)b * ntiles + blockIdx.x] = h[b];
}

// staged scatter: the tile's records counting-sorted by bucket in LDS, each
// field written out by consecutive threads (runs of a bucket contiguous)
template <int B>
__global__ __launch_bounds__(kThreads) void scatter_staged(
    const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
    const float4* __restrict__ xyz, uint32_t R, int shift, uint32_t ntiles,
    const uint32_t* __restrict__ off, uint32_t* __restrict__ okey, uint32_t* __restrict__ oval,
    float4* __restrict__ oxyz) {
    __shared__ uint32_t cnt[B], gb[B];   // cnt: counts, then the local offsets
    __shared__ uint32_t dst[kTile];
    __shared__ uint32_t stage[kTile];   // one u32 field, or a quarter of the tile's float4s
    uint32_t* loff = cnt;
    uint32_t* wsum = stage;             // (before the staging starts)
    const int tid = threadIdx.x;
    for (int b = tid; b < B; b += kThreads) cnt[b] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
    uint32_t k[kPer], rk[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kThreads + tid;
        k[i] = r < R ? key[r] : 0xFFFFFFFFu;
        rk[i] = r < R ? atomicAdd(&cnt[k[i] >> shift], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of cnt (B / kThreads per thread)
    constexpr int PT = (B + kThreads - 1) / kThreads;
    uint32_t c[PT], s = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        const int b = tid * PT + q;
        c[q] = b < B ? cnt[b] : 0u;
        s += c[q];
    }
    uint32_t incl = s;
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t wb = 0;
    for (int u = 0; u < w; ++u) wb += wsum[u];
    uint32_t ex = wb + incl - s;
    __syncthreads();   // every count read before loff overwrites it, wsum read before staging
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        const int b = tid * PT + q;
        if (b < B) {
            loff[b] = ex;
            gb[b] = off[(uint64_t)b * ntiles + blockIdx.x];
        }
        ex += c[q];
    }
    __syncthreads();
    uint32_t sp[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kThreads + tid;
        if (r < R) {
            const uint32_t b = k[i] >> shift;
            sp[i] = loff[b] + rk[i];
            dst[sp[i]] = gb[b] + rk[i];
            stage[sp[i]] = k[i];
        } else {
            sp[i] = 0xFFFFFFFFu;
        }
    }
    const uint32_t n = (uint32_t)((R - t0) < (uint64_t)kTile ? (R - t0) : kTile);
    __syncthreads();
    for (uint32_t p = tid; p < n; p += kThreads) okey[dst[p]] = stage[p];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kThreads + tid;
        if (r < R) stage[sp[i]] = val[r];
    }
    __syncthreads();
    for (uint32_t p = tid; p < n; p += kThreads) oval[dst[p]] = stage[p];
    float4* st4 = reinterpret_cast<float4*>(stage);
    for (int qt = 0; qt < 4; ++qt) {
        __syncthreads();
        const uint32_t lo = qt * (kTile / 4), hi = lo + kTile / 4;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint64_t r = t0 + (uint64_t)i * kThreads + tid;
            if (sp[i] >= lo && sp[i] < hi) st4[sp[i] - lo] = xyz[r];
        }
        __syncthreads();
        for (uint32_t p = lo + tid; p < hi && p < n; p += kThreads) oxyz[dst[p]] = st4[p - lo];
    }
}

// direct scatter: the same destinations, each thread writes its own records
template <int B>
__global__ __launch_bounds__(kThreads) void scatter_direct(
    const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
    const float4* __restrict__ xyz, uint32_t R, int shift, uint32_t ntiles,
    const uint32_t* __restrict__ off, uint32_t* __restrict__ okey, uint32_t* __restrict__ oval,
    float4* __restrict__ oxyz) {
    __shared__ uint32_t cnt[B];
    const int tid = threadIdx.x;
    for (int b = tid; b < B; b += kThreads) cnt[b] = off[(uint64_t)b * ntiles + blockIdx.x];
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
#pragma unroll 4
    for (int i = 0; i < kPer; ++i) {
        const uint64_t r = t0 + (uint64_t)i * kThreads + tid;
        if (r >= R) continue;
        const uint32_t kk = key[r];
        const uint32_t d = atomicAdd(&cnt[kk >> shift], 1u);
        okey[d] = kk;
        oval[d] = val[r];
        oxyz[d] = xyz[r];
    }
}

// final level: one workgroup per segment of m <= kTile records; stable LDS
// radix sort of (rel key, index), then each output position gathers its
// record from the (L2-hot) segment and writes it coalesced
template <int IPT>
__global__ __launch_bounds__(kThreads) void seg_sort_kernel(
    const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
    const float4* __restrict__ xyz, const uint32_t* __restrict__ seg_start, uint32_t seg_mask,
    int bits, uint32_t* __restrict__ okey, uint32_t* __restrict__ oval, float4* __restrict__ oxyz) {
    using sort_t = rocprim::block_radix_sort<uint32_t, kThreads, IPT, uint32_t>;
    __shared__ typename sort_t::storage_type st;
    const uint32_t s0 = seg_start[blockIdx.x], s1 = seg_start[blockIdx.x + 1];
    const uint32_t m = s1 - s0;
    uint32_t kk[IPT], ix[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t p = threadIdx.x * IPT + i;   // blocked
        kk[i] = p < m ? (key[s0 + p] & seg_mask) : 0xFFFFFFFFu;
        ix[i] = p;
    }
    sort_t().sort_to_striped(kk, ix, st, 0, bits);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t p = i * kThreads + threadIdx.x;   // striped
        if (p < m) {
            const uint32_t src = s0 + ix[i];
            okey[s0 + p] = key[src];
            oval[s0 + p] = val[src];
            oxyz[s0 + p] = xyz[src];
        }
    }
}

int main(int argc, char** argv) {
    const uint32_t R = argc > 1 ? (uint32_t)atol(argv[1]) : 100000000u;
    uint32_t *key, *val, *okey, *oval, *hist, *off;
    float4 *xyz, *oxyz;
    CK(hipMalloc(&key, 4ull * R)); CK(hipMalloc(&val, 4ull * R)); CK(hipMalloc(&xyz, 16ull * R));
    CK(hipMalloc(&okey, 4ull * R)); CK(hipMalloc(&oval, 4ull * R)); CK(hipMalloc(&oxyz, 16ull * R));
    const uint32_t ntiles = (R + kTile - 1) / kTile;
    CK(hipMalloc(&hist, 4ull * 8192 * ntiles + 4)); CK(hipMalloc(&off, 4ull * 8192 * ntiles + 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = 48.0 * R;   // 24 B read + 24 B written per record
    auto timeit = [&](auto&& f, int reps) {
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    gen_kernel<<<(R + 255) / 256, 256>>>(key, val, xyz, R, 0x7FFFFFFFu);
    CK(hipDeviceSynchronize());
    void* tmp = nullptr;
    size_t tb = 0;
    CK(rocprim::exclusive_scan(nullptr, tb, hist, off, 0u, (size_t)8192 * ntiles, rocprim::plus<uint32_t>()));
    CK(hipMalloc(&tmp, tb));
    auto run = [&](auto Bc) {
        constexpr int B = decltype(Bc)::value;
        int lb = 0;
        while ((1 << lb) < B) ++lb;
        const int shift = 31 - lb;
        const size_t nh = (size_t)B * ntiles;
        auto prep = [&]() {
            hist_kernel<<<ntiles, kThreads, B * 4>>>(key, R, shift, B, ntiles, hist);
            size_t t2 = tb;
            CK(rocprim::exclusive_scan(tmp, t2, hist, off, 0u, nh, rocprim::plus<uint32_t>()));
        };
        const float th = timeit([&] { hist_kernel<<<ntiles, kThreads, B * 4>>>(key, R, shift, B, ntiles, hist); }, 5);
        const float tp = timeit(prep, 5);
        prep();
        const float ts = timeit([&] {
            scatter_staged<B><<<ntiles, kThreads>>>(key, val, xyz, R, shift, ntiles, off, okey, oval, oxyz);
        }, 5);
        // check: bucket-sorted output
        std::vector<uint32_t> hk(R);
        CK(hipMemcpy(hk.data(), okey, 4ull * R, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (uint32_t i = 1; i < R; ++i) bad += (hk[i] >> shift) < (hk[i - 1] >> shift);
        const float td = timeit([&] {
            scatter_direct<B><<<ntiles, kThreads>>>(key, val, xyz, R, shift, ntiles, off, okey, oval, oxyz);
        }, 5);
        std::printf("B=%5d hist %.3f ms, hist+scan %.3f ms | staged %.3f ms (%.2f TB/s) | direct %.3f ms "
                    "(%.2f TB/s) | order violations %zu\n",
                    B, th, tp, ts, bytes / ts / 1e9, td, bytes / td / 1e9, bad);
    };
    run(std::integral_constant<int, 256>{});
    run(std::integral_constant<int, 1024>{});
    run(std::integral_constant<int, 2048>{});
    run(std::integral_constant<int, 4096>{});
    // final level: segments of m records (keys random within 20 bits)
    for (uint32_t m : {4096u, 8192u, 12288u, 16384u}) {
        const uint32_t nseg = R / m;
        std::vector<uint32_t> hs(nseg + 1);
        for (uint32_t i = 0; i <= nseg; ++i) hs[i] = i * m;
        uint32_t* dseg;
        CK(hipMalloc(&dseg, 4ull * (nseg + 1)));
        CK(hipMemcpy(dseg, hs.data(), 4ull * (nseg + 1), hipMemcpyHostToDevice));
        const uint32_t Rm = nseg * m;
        float t;
        if (m <= 4096)
            t = timeit([&] { seg_sort_kernel<4><<<nseg, kThreads>>>(key, val, xyz, dseg, 0xFFFFFu, 20, okey, oval, oxyz); }, 5);
        else if (m <= 8192)
            t = timeit([&] { seg_sort_kernel<8><<<nseg, kThreads>>>(key, val, xyz, dseg, 0xFFFFFu, 20, okey, oval, oxyz); }, 5);
        else
            t = timeit([&] { seg_sort_kernel<16><<<nseg, kThreads>>>(key, val, xyz, dseg, 0xFFFFFu, 20, okey, oval, oxyz); }, 5);
        std::vector<uint32_t> hk(Rm);
        CK(hipMemcpy(hk.data(), okey, 4ull * Rm, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (uint32_t i = 1; i < Rm; ++i)
            if (i % m) bad += (hk[i] & 0xFFFFFu) < (hk[i - 1] & 0xFFFFFu);
        std::printf("seg sort m=%5u: %.3f ms (%.2f TB/s over %u records), order violations %zu\n", m, t,
                    48.0 * Rm / t / 1e9, Rm, bad);
        CK(hipFree(dseg));
    }
    return 0;
}
