// Lock-free union-find shared by the grid engine (engine.hip) and the dense
// tile engine (dense.hip).
//
// Invariant parent[x] <= x: links always hook the larger root under the
// smaller, so a component's root is its minimum element and every stale
// (older) parent value is still an ancestor — plain path halving is safe
// without locks (ECL-CC style).
#pragma once

#include "common.hpp"

namespace pd {
namespace {

__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t uf_find(uint32_t* par, uint32_t x) {
    uint32_t p = ld_rlx(par + x);
    while (p != x) {
        uint32_t g = ld_rlx(par + p);
        if (g == p) return p;
        st_rlx(par + x, g);
        x = g;
        p = ld_rlx(par + x);
    }
    return x;
}

__device__ __forceinline__ void uf_unite(uint32_t* par, uint32_t a, uint32_t b) {
    a = uf_find(par, a);
    b = uf_find(par, b);
    while (a != b) {
        if (a > b) {
            uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t expected = b;
        if (__hip_atomic_compare_exchange_strong(par + b, &expected, a, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        b = uf_find(par, expected);
        a = uf_find(par, a);
    }
}

}  // namespace
}  // namespace pd
