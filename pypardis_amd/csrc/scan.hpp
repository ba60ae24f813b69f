// Block-level scan helpers for the ordered passes (two-pass tile scans:
// per-tile counts, a device-wide scan of the counts, then the write pass).
#pragma once

#include "common.hpp"

namespace pd {

// Block-wide exclusive scan of one u32 per thread (NT threads); returns
// the thread's exclusive prefix within the block and the block total.
template <int NT = kBlock>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t& total) {
    __shared__ uint32_t wsum[NT / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < NT / 64; ++u) {
        before += u < w ? wsum[u] : 0u;
        tot += wsum[u];
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

}  // namespace pd
