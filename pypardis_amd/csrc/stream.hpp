// Streaming helpers shared by the per-point passes: four consecutive points
// per lane per step with 16-byte loads (d <= 4; X and labels 16-byte aligned,
// as torch allocations and the arena are).
#pragma once

#include <type_traits>

#include "common.hpp"

namespace pd {

template <typename T, int D, bool VEC>
__device__ __forceinline__ int load_chunk(const T* __restrict__ X, uint64_t n, uint64_t c,
                                          T (&v)[4][D]) {
    const uint64_t i0 = c * 4;
    const int m = n - i0 >= 4 ? 4 : (int)(n - i0);
    if (VEC && m == 4) {
        T t[4 * D];
        if constexpr (sizeof(T) == 4) {
            const float4* p = reinterpret_cast<const float4*>(X + i0 * D);
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const float4 f = p[k];
                t[4 * k] = f.x;
                t[4 * k + 1] = f.y;
                t[4 * k + 2] = f.z;
                t[4 * k + 3] = f.w;
            }
        } else {
            const double2* p = reinterpret_cast<const double2*>(X + i0 * D);
#pragma unroll
            for (int k = 0; k < 2 * D; ++k) {
                const double2 f = p[k];
                t[2 * k] = f.x;
                t[2 * k + 1] = f.y;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < D; ++j) v[q][j] = t[q * D + j];
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < D; ++j) v[q][j] = q < m ? X[(i0 + q) * D + j] : T(0);
    }
    return m;
}

template <bool VEC>
__device__ __forceinline__ void load_labels4(const int32_t* __restrict__ L, uint64_t c, int m,
                                             int (&lab)[4]) {
    if (VEC && m == 4) {
        const int4 v = reinterpret_cast<const int4*>(L)[c];
        lab[0] = v.x;
        lab[1] = v.y;
        lab[2] = v.z;
        lab[3] = v.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) lab[q] = q < m ? L[c * 4 + q] : -1;
    }
}

template <bool VEC>
__device__ __forceinline__ void store_labels4(int32_t* __restrict__ L, uint64_t c, int m,
                                              const int (&lab)[4]) {
    if (VEC && m == 4) {
        reinterpret_cast<int4*>(L)[c] = make_int4(lab[0], lab[1], lab[2], lab[3]);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < m) L[c * 4 + q] = lab[q];
    }
}

// v[ax] for a per-lane ax, as a bitwise select over the D values: written as
// a select chain, the compiler turns it into an indexed load from a stack copy
// of v (a scratch round trip per point with a full vmcnt wait, 112 bytes of
// scratch per lane in the KD split passes).
template <typename T, int D>
__device__ __forceinline__ T pick_axis(const T (&v)[D], int ax) {
    using U = std::conditional_t<sizeof(T) == 4, uint32_t, uint64_t>;
    U r = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        U b;
        __builtin_memcpy(&b, &v[j], sizeof(T));
        r |= b & (U)0 - (U)(ax == j);
    }
    T out;
    __builtin_memcpy(&out, &r, sizeof(T));
    return out;
}

}  // namespace pd
