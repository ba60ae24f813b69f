// Shared device/host helpers for libpardis (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace pd {

// Launch geometry: 256-thread blocks (4 waves), grid-stride beyond this.
constexpr int kBlock = 256;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kOwnerBit = 0x80000000u;   // record value: point id | flags
constexpr uint32_t kDupBit = 0x40000000u;     // point lies in >= 2 neighbourhoods
constexpr uint32_t kIdMask = 0x3FFFFFFFu;     // => n < 2^30 points per device
constexpr int kMaxDim = 4;                    // grid path; d > 4 is the tile path
constexpr int kMaxParts = 64;                 // one bit per neighbourhood in the halo mask
constexpr int kMaxLdsParts = 64;              // neighbourhood grids staged in LDS up to this

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PD_HIP(expr)                                                                 \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess)                                                        \
            throw ::pd::Error(-3, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

inline unsigned grid_for(int64_t n, int64_t cap = 256 * 64) {
    int64_t b = (n + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

// Per-neighbourhood grid: cell side = eps * (1 + 2^-20) so that any pair the
// fp64 predicate can accept lies in adjacent rows; axis 0 (the row axis) is
// cut finer (eps/xsub) so a row's candidate range can follow the eps-ball's
// chord at the query point.  Origin and extent clipped
// to the data's tight bbox (the reference's root box can reach to ±0 through
// the float_info.min sentinel, R:dbscan/geometry.py:28-29).
struct PartGrid {
    double lo[kMaxDim];     // origin (fp64)
    double inv[kMaxDim];    // 1 / cell side per axis (axis 0 is split into xsub sub-cells)
    double cs[kMaxDim];     // cell side per axis
    int64_t nc[kMaxDim];    // cells per axis (0 => empty neighbourhood)
    uint64_t base;          // first key of this neighbourhood
    double elo[kMaxDim];    // expanded box (halo membership test), inclusive
    double ehi[kMaxDim];    // (empty neighbourhood: +inf / -inf, a box nothing is in)
    float flo[kMaxDim];     // the same test for fp32 coordinates in fp32: the smallest
    float fhi[kMaxDim];     // float >= elo, the largest float <= ehi (exact equivalence)
};

// XCD-aware block remap (cdna_hip_programming.md T1, bijective form): blocks
// b and b+8 share an XCD, so give each XCD a contiguous run of block ids —
// neighbouring records (which read the same cells) then share one L2.
__device__ __forceinline__ unsigned xcd_block(unsigned bid, unsigned nblk) {
    const unsigned q = nblk / 8, r = nblk % 8, x = bid % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <typename T> struct Vec;
template <> struct Vec<float> { using type = float; };
template <> struct Vec<double> { using type = double; };

}  // namespace pd
