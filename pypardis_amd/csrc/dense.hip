// The high-dimensional path (d > 4): DBSCAN from dense distance tiles on the
// matrix cores (BASELINE config C3, 64-D embeddings).  An eps-grid is useless
// there (3^d neighbour cells), so the neighbour test of sklearn's radius query
// (SK:cluster/_dbscan.py:410-434; the reference calls it per partition in
// R:dbscan/dbscan.py:28-30) becomes a Gram-matrix tile:
//
//   d2~(i, j) = |x_i|^2 + |x_j|^2 - 2 <x_i, x_j>
//
// with <.,.> from split-bf16 MFMA (x = hi + lo, hi = bf16(x), lo = bf16(x -
// hi); hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_bf16, fp32 accumulation)
// and a rigorous error band |d2~ - d2| <= c (|x_i|^2 + |x_j|^2), c = 2^-13:
// the split drops <= 3 * 2^-18 |x||y|, the fp32 accumulation over K <= 128
// adds <= 2^-17 |x||y|, fp32 rounding of the coordinates and of d2~ itself
// < 2^-21 (|x|^2 + |y|^2), and 2|x||y| <= |x|^2 + |y|^2 — a > 4x margin.
// Pairs outside the band are decided exactly by the bound; pairs inside it
// are re-tested with sklearn's kd_tree leaf predicate (fp64, per axis in
// order, no FMA; SK:metrics/_dist_metrics.pxd.tp:39-49).  So counts, core
// flags and labels are bit-exact, as on the grid path (engine.hip).
//
// Stages (sklearn DBSCAN.fit semantics, same keys and numbering as engine.hip):
//   count   all x all tiles              -> neighbour counts (self included)
//   link    core x core tiles, j > i     -> union-find -> components
//   border  non-core-with-neighbour x core tiles -> smallest adjacent key
//   labels  rank of the keys (rank_labels_async, engine.hip)
// Cityblock, and d > 128, take an exact fp64 VALU tile instead of the MFMA.
//
// Layout in HBM: points centred on the bbox midpoint and scaled by a power of
// two (the exact recheck reads the caller's X), split into bf16 hi / lo
// arrays in "fragment-major" order so one 16-byte load per lane is an MFMA
// operand: row group g (32 rows), k-step s (16 dims) is a 1 KiB block of 64
// lanes x 8 bf16 where lane 32h + r holds dims 16s + 8h .. 16s + 8h + 7 of
// row 32g + r — the A[row][k] / B[k][col] maps of 32x32x16 (the Gram matrix
// needs the same layout for both operands).  Norms |x|^2 in fp32.  Per wave:
// 64 query points (B operand, held in registers) against a stream of 64-point
// tiles of the other set (A operand); C/D: col = lane & 31 is the query,
// rows = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5) the streamed points.
#include <cstring>   // before rocprim (its texture_cache_iterator uses memset)
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <string>
#include <vector>

#include "internal.hpp"
#include "uf.hpp"

namespace pd {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));   // 32 e4m3 values

enum { kCount = 0, kLink = 1, kBorder = 2 };
constexpr int kTile = 64;                 // points per wave tile (2 MFMA tiles of 32)
constexpr float kBandC = 1.0f / 8192.0f;  // error band c (see header)
// Count pass screen: hi.hi alone (one MFMA per k-step instead of three) is
// within 2^-8 (1 + 2^-10) |x||y| + 2^-17 s of the dot product (bf16 rounds
// each coordinate by <= 2^-9 of itself; products exact, fp32 accumulation
// over <= 128 terms), i.e. d2 within 2^-8 * 1.01 s.  A tile where no pair
// passes the band c' = 2^-7 holds no neighbour (a 1.9x margin), so only
// tiles that can hold one fetch the lo fragments and finish the split
// product; C3 pairs lie ~100 eps^2 apart, so most tiles stop at the screen.
constexpr float kScreenC = 1.0f / 128.0f;
// e4m3 screen (PD_OPT_DENSE_SCREEN = 1, the default for the count pass):
// v_mfma_f32_32x32x64_f8f6f4 on coordinates scaled by 2^8 (|v| <= 256 <=
// 448) and rounded to OCP e4m3 (round-to-nearest-even, subnormals kept:
// tools/fp8x64_probe.hip).  Per coordinate |q - x| <= 2^-4 |x| + 2^-18 (the
// subnormal spacing 2^-9 over the 2^8 scale, halved), so with a = 2^-18
// sqrt(d_pad): |<qx,qy> - <x,y>| <= (2^-3 + 2^-8)|x||y| + 1.125 a (|x| + |y|)
// + a^2; products of e4m3 values are exact and the fp32 accumulation of <= 128
// of them adds <= 2^-17 |qx||qy|.  d2 is therefore within (2^-3 + 2^-8 +
// 2^-17) s + 4.5 a sqrt(max|x|^2) + 2 a^2 of the truth; the band below, c8 =
// 2^-3 + 2^-7, keeps 0.004 s of slack for the fp32 epilogue.  A tile where no
// pair passes it holds no neighbour; the others compute the split-bf16
// product from scratch (hi and lo from global memory).  Half the staged bytes
// of the hi.hi screen, and one 32x32x64 MFMA (64 cycles) per 64 dims where the
// bf16 screen issues four 32x32x16 (32 cycles each).  At C3's distances the
// same tiles pass (clustered pairs lie within 0.05 of each other, the rest
// beyond 0.88 in d2; the band adds 0.27).
constexpr float kScreen8C = 1.0f / 8.0f + 1.0f / 128.0f;
constexpr float kF8Scale = 256.0f;        // coordinates -> e4m3 range
constexpr float kF8Acc = kF8Scale * kF8Scale;
constexpr float kPadNorm = 1.0e30f;       // norm of padding rows: never a neighbour

inline unsigned nblocks(uint64_t n, unsigned per = kBlock) {
    return n ? (unsigned)((n + per - 1) / per) : 1u;
}
// rows padded to a whole wave's query block (4 x 32 with kCountQT = 4)
inline uint32_t pad_rows(uint32_t m) { return (m + 2 * kTile - 1) / (2 * kTile) * (2 * kTile); }

// A point set in MFMA fragment layout.
struct FragSet {
    const bf16x8* hi;
    const bf16x8* lo;
    const i32x8* f8;       // e4m3 fragments (count pass screen) or null: row group g,
                           // k8-step s (64 dims) is 64 lanes x 32 bytes, lane 32h + r holding
                           // dims 64s + 32h .. +31 of row 32g + r
    const float* norm;     // [rows_pad]
    const float* nmax;     // max norm over the valid rows (device scalar)
    const uint32_t* idx;   // row -> point id (null: identity)
    uint32_t m;            // valid rows
};

// sklearn kd_tree leaf predicate (exact, as engine.hip's `within`), any d.
template <typename T, int M>
__device__ __noinline__ bool exact_within(const T* __restrict__ X, int d, uint32_t p, uint32_t q,
                                          double eps, double eps2) {
    const T* a = X + (uint64_t)p * d;
    const T* b = X + (uint64_t)q * d;
    double acc = 0.0;
    for (int k = 0; k < d; ++k) {
        const double t = __dadd_rn((double)a[k], -(double)b[k]);
        acc = M == 0 ? __dadd_rn(acc, __dmul_rn(t, t)) : __dadd_rn(acc, fabs(t));
    }
    return M == 0 ? (acc <= eps2) : (acc <= eps);
}

// ---------------------------------------------------------------- data prep
// One thread per (row, k-step, lane half): 8 dims -> bf16 hi and lo.
template <typename T>
__global__ __launch_bounds__(kBlock) void prep_kernel(const T* __restrict__ X, int d,
                                                      const uint32_t* __restrict__ idx, uint32_t m,
                                                      uint32_t rows_pad, int KS,
                                                      const double* __restrict__ center,
                                                      double scale, bf16x8* __restrict__ Fh,
                                                      bf16x8* __restrict__ Fl) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (uint64_t)rows_pad * KS * 2) return;
    const int h = (int)(t & 1);
    const int s = (int)((t >> 1) % KS);
    const uint32_t r = (uint32_t)((t >> 1) / KS);
    bf16x8 vh, vl;
    const uint32_t p = r < m ? (idx ? idx[r] : r) : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * h + j;
        float v = 0.0f;
        if (r < m && k < d) v = (float)(((double)X[(uint64_t)p * d + k] - center[k]) * scale);
        const __bf16 bh = (__bf16)v;
        vh[j] = bh;
        vl[j] = (__bf16)(v - (float)bh);
    }
    const uint64_t o = ((uint64_t)(r >> 5) * KS + s) * 64 + 32 * h + (r & 31);
    Fh[o] = vh;
    Fl[o] = vl;
}

// One thread per (row, k8-step, lane half): 32 dims -> e4m3 (scaled by 2^8).
// The k order inside a lane is the same for both MFMA operands (a Gram tile),
// so any consistent (h, j) -> k map computes the same products.
template <typename T>
__global__ __launch_bounds__(kBlock) void prep8_kernel(const T* __restrict__ X, int d,
                                                       const uint32_t* __restrict__ idx, uint32_t m,
                                                       uint32_t rows_pad, int KS8,
                                                       const double* __restrict__ center,
                                                       double scale, i32x8* __restrict__ F8) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (uint64_t)rows_pad * KS8 * 2) return;
    const int h = (int)(t & 1);
    const int s = (int)((t >> 1) % KS8);
    const uint32_t r = (uint32_t)((t >> 1) / KS8);
    const uint32_t p = r < m ? (idx ? idx[r] : r) : 0u;
    i32x8 v;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        float f[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = 64 * s + 32 * h + 4 * w + q;
            // the bf16 path's fp32 value, then the exact power-of-two scale
            f[q] = (r < m && k < d)
                       ? (float)(((double)X[(uint64_t)p * d + k] - center[k]) * scale) * kF8Scale
                       : 0.0f;
        }
        int x = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
        x = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], x, true);
        v[w] = x;
    }
    F8[((uint64_t)(r >> 5) * KS8 + s) * 64 + 32 * h + (r & 31)] = v;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void norm_kernel(const T* __restrict__ X, int d,
                                                      const uint32_t* __restrict__ idx, uint32_t m,
                                                      uint32_t rows_pad,
                                                      const double* __restrict__ center,
                                                      double scale, float* __restrict__ norm,
                                                      uint32_t* __restrict__ nmax) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    float nr = 0.0f;   // norms are >= 0: their bits order as uint32
    if (r < m) {
        const uint32_t p = idx ? idx[r] : r;
        double acc = 0.0;
        for (int k = 0; k < d; ++k) {
            const double v = (double)(float)(((double)X[(uint64_t)p * d + k] - center[k]) * scale);
            acc += v * v;
        }
        nr = (float)acc;
        norm[r] = nr;
    } else if (r < rows_pad) {
        norm[r] = kPadNorm;
    }
    uint32_t w = __float_as_uint(nr);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w = max(w, (uint32_t)__shfl_xor((int)w, o, 64));
    if ((threadIdx.x & 63) == 0 && w) atomicMax(nmax, w);
}

// ---------------------------------------------------------------- tiles
template <typename T>
struct TileArgs {
    FragSet I, J;
    const T* X;
    int d;
    double eps, eps2;      // exact predicate, caller's units
    float elo, ehi;        // scaled eps^2 thresholds, rounded outward
    uint32_t* cnt;         // kCount: neighbours per I row
    uint32_t* par;         // kLink: union-find over the (I = J) rows
    const uint32_t* keyJ;  // kBorder: cluster key per J row
    uint32_t* best;        // kBorder: smallest adjacent key per I row
    // projection pruning (count pass, I = J) over three coordinates p1, p2,
    // p3: rows in bands of `band` rows by their p1 rank, each band in
    // sub-bands of `sub` rows by p2 rank, sorted by p3 within a sub-band.  A
    // pair whose p1, p2 or p3 differ by more than win cannot be within eps
    // (|x_k - y_k| <= |x - y|), so a block streams, per sub-band whose p1
    // and p2 ranges meet its own widened by win, only the run of rows whose
    // p3 lies within win of its rows' p3 range.  p3: null = no pruning.
    const double* p3;           // [m] p3 of each row
    const double* bp1;          // [2 * nband] p1 range (lo, hi) of each band
    const double* bp2;          // [2 * nband * nsub] p2 range of each sub-band
    uint32_t band, nband, sub, nsub;
    uint32_t whole_bands;       // 1: one run per band (the overflow path), for tests
    double win;
    unsigned long long* tiles;  // [2]: wave tiles computed, of which refined past the
                                // count screen (null: not counted)
    float f8_a;                 // e4m3 screen: 2^-18 sqrt(d_pad), the subnormal term
    // sharded train: this device computes the I rows of the chunks
    // (kShardChunk rows each) c with c % shard_world == shard_rank
    uint32_t shard_rank, shard_world;
};

// Rows per shard chunk: a multiple of every block's query rows (256) and of
// the pruned count's sub-band (2048), so a block lies in one chunk and the
// chunks dealt round-robin give every rank a slice of every band (balanced
// windows, and one sub-band per band per XCD at 8 ranks).
constexpr uint32_t kShardChunk = 2048;
__device__ __forceinline__ bool not_my_rows(uint32_t row0, uint32_t rank, uint32_t world) {
    return world > 1 && (row0 / kShardChunk) % world != rank;
}

constexpr int kMaxBand = 256;   // bands (host keeps nband <= this)
constexpr int kMaxSeg = 1024;
constexpr bool kSubWindow = false;  // count pass: one p3 window per sub-band (measured 109 vs
                                     // 74 ms on C3: 0.35 vs 0.22 of the tiles)   // sub-band segments a block keeps (else one per band)

// First index in the ascending p[lo, hi) with p[k] >= v (upper: > v).
__device__ __forceinline__ uint32_t p_bound(const double* __restrict__ p, uint32_t lo, uint32_t hi,
                                            double v, bool upper) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const double x = p[mid];
        if (upper ? (x <= v) : (x < v))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

template <typename T, int MODE>
__device__ __forceinline__ void tile_hit(const TileArgs<T>& A, uint32_t i, uint32_t j, uint32_t& cnt,
                                         uint32_t& best) {
    if constexpr (MODE == kCount) {
        ++cnt;
    } else if constexpr (MODE == kLink) {
        uf_unite(A.par, i, j);
    } else {
        const uint32_t k = A.keyJ[j];
        best = k < best ? k : best;
    }
}

// One block = 4 waves x 64 query points; the streamed 64-point tiles of the
// other set are shared by the 4 waves through LDS (double-buffered, the next
// tile prefetched into registers while the current one is computed).
//
// Epilogue: with s = |x_i|^2 + |x_j|^2 and acc = <x_i, x_j>~,
//   in    <=>  d2~ + c s <= elo  <=>  acc - ta_j >= ai := ((1+c)|x_i|^2 - elo)/2
//   maybe <=>  d2~ - c s <= ehi  <=>  acc - ta_j >= ((1-c)|x_i|^2 - ehi)/2 - c |x_j|^2
// with ta_j = (1+c)|x_j|^2/2.  The row term -ta_j is the MFMA's C operand
// (the accumulation starts from it), so `in` is one compare against a column
// constant; `maybe` is widened to the column constant bi := ((1-c)|x_i|^2 -
// ehi)/2 - c max_j |x_j|^2 (a superset: more pairs re-tested, none missed).
// The fp32 rounding of the rearrangement is < 2^-22 s, inside the band's
// margin.  The count pass tallies in and maybe per lane and builds the band
// bits (maybe && !in, re-tested exactly) only for tiles where they differ.
// Threads per tile block: 4 waves share each streamed tile.  (8 waves per
// block halve the streamed bytes per MFMA but measured slower on C3: 125 vs
// 110 ms — an 8-wave barrier per tile, one block per CU.)
constexpr int kCountWaves = 4;   // waves per count-pass block (each staged tile feeds them all; 8:
                                 // 41.4 vs 36.1 ms on C3 — wider windows per block, more tiles)
constexpr int tile_threads(int, int mode) { return mode == kCount ? 64 * kCountWaves : 256; }
constexpr int kCountQT = 2;   // query tiles (of 32) per wave in the count pass (4: one
                              // wave per SIMD, measured 125 vs 74 ms on C3)

// LO: the lo fragments are staged too (link / border); the count pass
// stages hi only and reads lo from global memory for the tiles its screen
// keeps (half the streamed bytes per tile).
template <int KS, bool LO>
struct TileLds {
    bf16x8 hi[2][2][KS][64];   // [buffer][row group][k-step][lane]
    bf16x8 lo[LO ? 2 : 1][LO ? 2 : 1][LO ? KS : 1][LO ? 64 : 1];
    float nta[2][kTile];       // -ta_j = -(1+c)|x_j|^2 / 2
};
// e4m3 screen: the staged tile is the e4m3 fragments only (4 KiB per 64 rows
// of up to 64 dims)
template <int KS8, int NB = 2>
struct TileLds8 {
    i32x8 f8[NB][2][KS8][64];   // [buffer][row group][k8-step][lane]
    float nta[NB][kTile];
};
// All of a tile block's LDS in one object (staging buffers and the segment
// list of its projection window).
template <typename TL>
struct TileShared {
    TL t;
    uint32_t seg_lo[kMaxSeg], seg_hi[kMaxSeg];
    uint32_t bk_lo[kMaxBand], bk_off[kMaxBand + 1];
    uint32_t nseg, fallback;
};

// QT: 32-query groups per wave (B operand tiles held in registers).  QT = 4
// doubles the MFMA work per streamed byte (each staged tile feeds 2 x 4 x 3 x
// KS MFMAs per wave) at one wave per SIMD.
#ifndef PD_F8_WAVES
#define PD_F8_WAVES 3
#endif
#ifndef PD_F8_QT
#define PD_F8_QT 2
#endif
constexpr int kF8Waves = PD_F8_WAVES;   // e4m3 count pass: waves per SIMD (no bf16 query fragments held)
constexpr int kF8QT = PD_F8_QT;         // e4m3 count pass: query tiles (of 32) per wave

// The e4m3 count pass streams each tile through two register stages ahead of
// a double-buffered LDS tile.  (Measured and retired in round 4: an LDS-DMA
// ring of 4 or 8 buffers — 29.9 ms vs 21.3 at 2 waves/SIMD, depth never
// mattered — and blocks of 1 or 2 waves — 38.2 / 24.7 ms; DESIGN.md §6.
// Round 5: a depth-4 tree of maxima for the screen instead of the linear
// v_max3 fold — C3 count 24.5 vs 24.1 ms, rejected: the screen's hot path is
// ds_read -> 4 MFMAs -> max fold -> vote with no spills, and the fold is not
// the limiter; profiles/r05_v3_ab_dense_max_tree.txt.)
template <typename T, int MODE, int KS, int QT, bool F8>
__global__ __launch_bounds__(tile_threads(KS, MODE)) __attribute__((amdgpu_waves_per_eu(F8 ? (KS >= 8 ? 1 : kF8Waves) : ((KS >= 8 || QT > 2) ? 1 : 2)))) void tile_kernel(TileArgs<T> A) {
    constexpr int NB = 2;                        // LDS tile buffers
    constexpr int TB = tile_threads(KS, MODE);
    constexpr int QW = 32 * QT;                  // query rows per wave
    constexpr int KS8 = (KS + 3) / 4;            // e4m3 k-steps of 64 dims
    static_assert(!F8 || MODE == kCount, "the e4m3 screen is the count pass's");
    // every mode screens with hi.hi and reads lo from global memory for the
    // tiles it keeps (link / border too: their core x core and border x core
    // pairs are as far apart as the count pass's); LO = true would stage lo
    constexpr bool LO = false;
    // 16-byte chunks per staged tile (e4m3: two per lane fragment)
    constexpr int NC = F8 ? 2 * KS8 * 64 * 2 : (LO ? 2 : 1) * 2 * KS * 64;
    constexpr int NCH = (NC + TB - 1) / TB;      // per thread
    __shared__ TileShared<std::conditional_t<F8, TileLds8<KS8, NB>, TileLds<KS, LO>>> SH;
    auto& S = SH.t;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // block -> query rows.  Pruned count: bands are dealt round-robin to the
    // 8 XCDs (dispatch puts block id b on XCD b % 8), a band's blocks kept
    // together on one XCD (its L2 serves their overlapping windows); bands
    // near the middle of the first axis have larger windows, so contiguous
    // runs of bands per XCD would leave the XCDs unbalanced (106 -> 88 ms on
    // C3; handing bands out centre-first measured 91 ms).
    uint32_t lblk;
    if (A.p3) {
        const uint32_t bpb = A.band / ((TB / 64) * QW);   // blocks per band
        const uint32_t x = blockIdx.x % 8u, k = blockIdx.x / 8u;
        lblk = (x + 8u * (k / bpb)) * bpb + k % bpb;
    } else {
        lblk = xcd_block(blockIdx.x, gridDim.x);
    }
    const uint32_t blk_i0 = lblk * (TB / 64) * QW;
    // spare block of the pruned grid, or another rank's rows (whole block, no
    // barrier yet)
    if (blk_i0 >= A.I.m || not_my_rows(blk_i0, A.shard_rank, A.shard_world)) return;
    const uint32_t i0 = blk_i0 + wave * QW;
    const bool wave_ok = i0 < A.I.m;
    const int col = lane & 31, h = lane >> 5;
    const float nJmax = *A.J.nmax;
    // the wave's 32 QT query points: B operand fragments, kept in registers
    // (e4m3 screen: the bf16 query fragments are re-read for the few kept
    // tiles instead of held, 64 registers fewer)
    bf16x8 bh[F8 ? 1 : QT][F8 ? 1 : KS], bl[F8 ? 1 : QT][F8 ? 1 : KS];
    i32x8 bq8[F8 ? QT : 1][F8 ? KS8 : 1];
    uint32_t iq[QT];
    float ai[QT], bi[QT], bc[QT];
    bool ok[QT];
    // e4m3 screen's absolute term (subnormals), over max |x_j|^2 for both rows
    const float a8 = A.f8_a;
    const float abs8 = 4.5f * a8 * __builtin_sqrtf(nJmax) * 1.001f + 2.0f * a8 * a8;
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        if constexpr (!F8) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint64_t o = ((uint64_t)((wave_ok ? i0 : 0) / 32 + t) * KS + s) * 64 + lane;
                bh[t][s] = A.I.hi[o];
                bl[t][s] = A.I.lo[o];
            }
        } else {
#pragma unroll
            for (int s = 0; s < KS8; ++s)
                bq8[t][s] = A.I.f8[((uint64_t)((wave_ok ? i0 : 0) / 32 + t) * KS8 + s) * 64 + lane];
        }
        iq[t] = i0 + 32 * t + col;
        ok[t] = wave_ok && iq[t] < A.I.m;
        const float nI = wave_ok ? A.I.norm[iq[t]] : kPadNorm;
        ai[t] = ((1.0f + kBandC) * nI - A.elo) * 0.5f;
        bi[t] = ((1.0f - kBandC) * nI - A.ehi) * 0.5f - kBandC * 1.001f * nJmax;
        // screen: acc_hh - ta_j >= ((1-c')|x_i|^2 - ehi)/2 - ((c'+c)/2)|x_j|^2,
        // widened by max |x_j|^2
        bc[t] = ((1.0f - kScreenC) * nI - A.ehi) * 0.5f -
                (0.5f * (kScreenC + kBandC)) * 1.001f * nJmax;
        if constexpr (F8)   // in the e4m3 accumulator's units (x 2^16, exact)
            bc[t] = kF8Acc * (((1.0f - kScreen8C) * nI - A.ehi - abs8) * 0.5f -
                              (0.5f * (kScreen8C + kBandC)) * 1.001f * nJmax);
    }
    uint32_t cnt[QT], best[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        cnt[t] = 0u;
        best[t] = kNone;
    }

    // streamed segments [seg_lo, seg_hi) of J rows (tile-aligned starts):
    // all of J, from the diagonal (link), or one per band in the window
    uint32_t(&seg_lo)[kMaxSeg] = SH.seg_lo;
    uint32_t(&seg_hi)[kMaxSeg] = SH.seg_hi;
    uint32_t& nseg_s = SH.nseg;
    uint32_t(&bk_lo)[kMaxBand] = SH.bk_lo;
    uint32_t(&bk_off)[kMaxBand + 1] = SH.bk_off;
    uint32_t& fallback_s = SH.fallback;
    if (A.p3 && blk_i0 < A.I.m) {
        const uint32_t b = blk_i0 / A.band;                 // a block lies in one band
        const uint32_t k = (blk_i0 - b * A.band) / A.sub;   // ... and one sub-band
        const uint32_t last = min(blk_i0 + (uint32_t)(TB / 64) * QW, A.I.m) - 1u;
        const double lo1 = A.bp1[2 * b] - A.win, hi1 = A.bp1[2 * b + 1] + A.win;
        const uint64_t kb = (uint64_t)b * A.nsub + k;
        const double lo2 = A.bp2[2 * kb] - A.win, hi2 = A.bp2[2 * kb + 1] + A.win;
        // the sub-band's p3 range (not only this block's rows): the blocks of
        // a sub-band then stream the same tiles in the same order, so the ones
        // resident together on an XCD share them in its L2
        const uint32_t sb0 = b * A.band + k * A.sub;
        const uint32_t sb1 = min(sb0 + A.sub, min(b * A.band + A.band, A.I.m)) - 1u;
        const double lo3 = (kSubWindow ? A.p3[sb0] : A.p3[blk_i0]) - A.win;
        const double hi3 = (kSubWindow ? A.p3[sb1] : A.p3[last]) + A.win;
        // bands are p1-ordered, sub-bands p2-ordered: both ends of their
        // ranges ascend
        uint32_t blo, bhi;
        {
            uint32_t l = 0, h = A.nband;
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                if (A.bp1[2 * mid + 1] < lo1) l = mid + 1; else h = mid;
            }
            blo = l;
            h = A.nband;
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                if (A.bp1[2 * mid] <= hi1) l = mid + 1; else h = mid;
            }
            bhi = l;
        }
        const uint32_t ns = bhi - blo;   // <= nband <= kMaxBand
        // (1) per candidate band: its candidate sub-bands [klo, khi)
        for (uint32_t t = threadIdx.x; t < ns; t += TB) {
            const uint32_t bb = blo + t;
            const uint32_t r0 = bb * A.band, r1 = min(r0 + A.band, A.J.m);
            const uint32_t nsb = (r1 - r0 + A.sub - 1) / A.sub;
            const double* q = A.bp2 + 2ull * bb * A.nsub;
            uint32_t l = 0, h = nsb;
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                if (q[2 * mid + 1] < lo2) l = mid + 1; else h = mid;
            }
            const uint32_t klo = l;
            h = nsb;
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                if (q[2 * mid] <= hi2) l = mid + 1; else h = mid;
            }
            bk_lo[t] = klo;
            bk_off[t + 1] = l - klo;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            bk_off[0] = 0;
            for (uint32_t t = 0; t < ns; ++t) {
                acc += bk_off[t + 1];
                bk_off[t + 1] = acc;
            }
            const bool fb = acc > (uint32_t)kMaxSeg || A.whole_bands;
            fallback_s = fb ? 1u : 0u;
            nseg_s = fb ? ns : acc;
        }
        __syncthreads();
        if (!fallback_s) {
            // (2) one segment per candidate sub-band: its rows within the p3 window
            const uint32_t total = nseg_s;
            for (uint32_t sg = threadIdx.x; sg < total; sg += TB) {
                uint32_t l = 0, h = ns;   // band slot t: bk_off[t] <= sg < bk_off[t + 1]
                while (l < h) {
                    const uint32_t mid = (l + h) >> 1;
                    if (bk_off[mid + 1] <= sg) l = mid + 1; else h = mid;
                }
                const uint32_t bb = blo + l, kk = bk_lo[l] + (sg - bk_off[l]);
                const uint32_t bend = min(bb * A.band + A.band, A.J.m);
                const uint32_t r0 = bb * A.band + kk * A.sub, r1 = min(r0 + A.sub, bend);
                const uint32_t sl = p_bound(A.p3, r0, r1, lo3, false);
                const uint32_t sh = p_bound(A.p3, sl, r1, hi3, true);
                seg_lo[sg] = sl < sh ? (sl & ~(uint32_t)(kTile - 1)) : sh;
                seg_hi[sg] = sh;
            }
        } else {
            // too many: the candidate sub-bands of each band as one run
            for (uint32_t t = threadIdx.x; t < ns; t += TB) {
                const uint32_t bb = blo + t, n_k = bk_off[t + 1] - bk_off[t];
                const uint32_t bend = min(bb * A.band + A.band, A.J.m);
                const uint32_t r0 = bb * A.band + bk_lo[t] * A.sub;
                const uint32_t r1 = min(r0 + n_k * A.sub, bend);
                seg_lo[t] = n_k ? r0 : r1;
                seg_hi[t] = r1;
            }
        }
    } else if (threadIdx.x == 0) {
        seg_lo[0] = MODE == kLink ? blk_i0 : 0u;
        seg_hi[0] = A.J.m;
        nseg_s = 1;
    }
    __syncthreads();
    const uint32_t nseg = nseg_s;
    uint32_t ntiles = 0, nrefined = 0;
    // cursor over the tiles of the segments; false at the end
    auto seg_at = [&](const uint32_t* p) -> uint32_t { return *p; };
    auto seek = [&](uint32_t& sg, uint32_t& j) -> bool {
        while (sg < nseg) {
            if (j < seg_at(&seg_hi[sg])) return true;
            if (++sg < nseg) j = seg_at(&seg_lo[sg]);
        }
        return false;
    };
    // staging: thread k moves 16-byte chunks c = k + q * TB of the tile
    // (hi then lo), plus one norm per thread < 64
    // Two register stages: the tile two ahead is in flight while the next
    // one is committed (a streamed tile often misses L2 under pruning)
    struct Stage {
        bf16x8 v[NCH];
        float n;
    };
    Stage stA, stB;
    auto fetch = [&](Stage& st, uint32_t j0) {
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            const int c = threadIdx.x + q * TB;        // [0, 2 * 2 * KS * 64)
            if (NC % TB != 0 && c >= NC) break;
            if constexpr (F8) {   // the tile's e4m3 fragments are contiguous
                const bf16x8* src = reinterpret_cast<const bf16x8*>(A.J.f8) +
                                    (uint64_t)(j0 / 32) * KS8 * 64 * 2;
                st.v[q] = src[c];
            } else {
                const int half = c / (2 * KS * 64);            // 0 hi, 1 lo
                const int w = c % (2 * KS * 64);               // (row group, k-step, lane)
                const uint64_t o = (uint64_t)(j0 / 32) * KS * 64 + w;
                st.v[q] = (LO && half) ? A.J.lo[o] : A.J.hi[o];
            }
        }
        if (threadIdx.x < kTile) st.n = A.J.norm[j0 + threadIdx.x];
    };
    auto commit = [&](const Stage& st, int buf) {
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            const int c = threadIdx.x + q * TB;
            if (NC % TB != 0 && c >= NC) break;
            if constexpr (F8) {
                reinterpret_cast<bf16x8*>(&S.f8[buf][0][0][0])[c] = st.v[q];
            } else {
                const int half = c / (2 * KS * 64);
                const int w = c % (2 * KS * 64);
                bf16x8* dst = (LO && half) ? &S.lo[LO ? buf : 0][0][0][0] : &S.hi[buf][0][0][0];
                dst[w] = st.v[q];
            }
        }
        // (e4m3 screen: in the x 2^16 units of its products, exact)
        if (threadIdx.x < kTile)
            S.nta[buf][threadIdx.x] = -((1.0f + kBandC) * 0.5f) * st.n * (F8 ? kF8Acc : 1.0f);
    };
    uint32_t j0 = 0;
    int buf = 0;
    // one streamed tile (rows j0.., staged in LDS buffer buf) against the
    // wave's queries
    auto work = [&]() {
        // link: only j > i; tiles wholly below this wave's diagonal are skipped
        const bool compute = wave_ok && !(MODE == kLink && j0 + kTile <= i0);   // i0: first query
        if (compute) {
            ++ntiles;
            // C operand: -ta of the tile's rows, element 4q + e = row 32u + 8q + 4h + e
            // (read where it is used: the e4m3 screen re-reads it for a kept tile
            // rather than holding 32 registers across the screen)
            auto nt_of = [&](int u) {
                f32x16 v16;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v =
                        *reinterpret_cast<const float4*>(&S.nta[buf][32 * u + 8 * q + 4 * h]);
                    v16[4 * q + 0] = v.x;
                    v16[4 * q + 1] = v.y;
                    v16[4 * q + 2] = v.z;
                    v16[4 * q + 3] = v.w;
                }
                return v16;
            };
            f32x16 nt[2];
            if constexpr (!F8) {
                nt[0] = nt_of(0);
                nt[1] = nt_of(1);
            }
            f32x16 acc[2][QT];
            bool refine = true;
            if constexpr (LO) {
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    bf16x8 ah[2], al[2];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        ah[u] = S.hi[buf][u][s][lane];
                        al[u] = S.lo[LO ? buf : 0][LO ? u : 0][LO ? s : 0][LO ? lane : 0];
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int t = 0; t < QT; ++t) {
                            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                ah[u], bh[t][s], s == 0 ? nt[u] : acc[u][t], 0, 0, 0);
                            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[u], bl[t][s],
                                                                                acc[u][t], 0, 0, 0);
                            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[u], bh[t][s],
                                                                                acc[u][t], 0, 0, 0);
                        }
                }
            } else if constexpr (F8) {
                // count pass, e4m3 screen (kScreen8C, in the x 2^16 units of
                // the e4m3 products); a kept tile recomputes the split-bf16
                // product from scratch, hi and lo from global memory
#pragma unroll
                for (int s = 0; s < KS8; ++s) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const i32x8 a8 = S.f8[buf][u][s][lane];
#pragma unroll
                        for (int t = 0; t < QT; ++t)
                            acc[u][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                                a8, bq8[t][s],
                                s == 0 ? nt_of(u) : acc[u][t], 0, 0,
                                0, 0, 0, 0);
                    }
                }
                bool mb = false;
#pragma unroll
                for (int t = 0; t < QT; ++t) {
                    float m0 = fmaxf(acc[0][t][0], acc[1][t][0]);
#pragma unroll
                    for (int r = 1; r < 16; ++r) m0 = fmaxf(fmaxf(m0, acc[0][t][r]), acc[1][t][r]);
                    mb |= m0 >= bc[t];
                }
                refine = __any(mb);
                nrefined += refine ? 1u : 0u;
                if (refine) {
                    const uint32_t iw = (wave_ok ? i0 : 0) / 32;
#pragma unroll
                    for (int u = 0; u < 2; ++u)   // exact
                        nt[u] = nt_of(u) * (1.0f / kF8Acc);
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        bf16x8 ah[2], al[2], qh[QT], ql[QT];
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const uint64_t o = ((uint64_t)(j0 / 32 + u) * KS + s) * 64 + lane;
                            ah[u] = A.J.hi[o];
                            al[u] = A.J.lo[o];
                        }
#pragma unroll
                        for (int t = 0; t < QT; ++t) {
                            const uint64_t o = ((uint64_t)(iw + t) * KS + s) * 64 + lane;
                            qh[t] = A.I.hi[o];
                            ql[t] = A.I.lo[o];
                        }
#pragma unroll
                        for (int u = 0; u < 2; ++u)
#pragma unroll
                            for (int t = 0; t < QT; ++t) {
                                acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    ah[u], qh[t], s == 0 ? nt[u] : acc[u][t], 0, 0, 0);
                                acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    ah[u], ql[t], acc[u][t], 0, 0, 0);
                                acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    al[u], qh[t], acc[u][t], 0, 0, 0);
                            }
                    }
                }
            } else {
                // count pass: the hi.hi screen (kScreenC), then the rest of the
                // split product only where the screen leaves a candidate pair
#pragma unroll
                for (int s = 0; s < KS; ++s) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const bf16x8 ah = S.hi[buf][u][s][lane];
#pragma unroll
                        for (int t = 0; t < QT; ++t)
                            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                ah, bh[t][s], s == 0 ? nt[u] : acc[u][t], 0, 0, 0);
                    }
                }
                // per query column t one maximum over the tile's 32 rows
                // (3-input max: half the VALU work of a compare per element;
                // the accumulators are finite), then one compare
                bool mb = false;
#pragma unroll
                for (int t = 0; t < QT; ++t) {
                    float m0 = fmaxf(acc[0][t][0], acc[1][t][0]);
#pragma unroll
                    for (int r = 1; r < 16; ++r) m0 = fmaxf(fmaxf(m0, acc[0][t][r]), acc[1][t][r]);
                    mb |= m0 >= bc[t];
                }
                refine = __any(mb);
                nrefined += refine ? 1u : 0u;
                if (refine) {
                    bf16x8 al[2][KS];
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int s = 0; s < KS; ++s)
                            al[u][s] = A.J.lo[((uint64_t)(j0 / 32 + u) * KS + s) * 64 + lane];
#pragma unroll
                    for (int s = 0; s < KS; ++s)
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const bf16x8 ah = S.hi[buf][u][s][lane];
#pragma unroll
                            for (int t = 0; t < QT; ++t) {
                                acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    ah, bl[t][s], acc[u][t], 0, 0, 0);
                                acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    al[u][s], bh[t][s], acc[u][t], 0, 0, 0);
                            }
                        }
                }
            }
            // element e of block q of m-tile u: row j = j0 + 32u + 8q + 4h + e
            uint64_t band[QT];
#pragma unroll
            for (int t = 0; t < QT; ++t) band[t] = 0ull;
            bool walk = refine;
            if constexpr (MODE == kCount) {
              if (refine) {
                uint32_t ci[QT], cm[QT];
#pragma unroll
                for (int t = 0; t < QT; ++t) ci[t] = cm[t] = 0u;
#pragma unroll
                for (int r = 0; r < 16; ++r)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int t = 0; t < QT; ++t) {
                            ci[t] += acc[u][t][r] >= ai[t] ? 1u : 0u;
                            cm[t] += acc[u][t][r] >= bi[t] ? 1u : 0u;
                        }
                bool differ = false;
#pragma unroll
                for (int t = 0; t < QT; ++t) {
                    cnt[t] += ci[t];
                    differ |= ci[t] != cm[t];
                }
                walk = __any(differ);
                if (walk) {
                    // fresh compares (keeps the masks above from living across)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int t = 0; t < QT; ++t) asm volatile("" : "+v"(acc[u][t]));
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int u = 0; u < 2; ++u)
#pragma unroll
                            for (int t = 0; t < QT; ++t) {
                                const float v = acc[u][t][r];
                                const bool b = v >= bi[t] && !(v >= ai[t]);
                                band[t] |= b ? (1ull << (16 * u + r)) : 0ull;
                            }
                }
              }
            } else if (refine) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int t = 0; t < QT; ++t) {
                            const float v = acc[u][t][r];
                            const int bit = 16 * u + r;
                            band[t] |= v >= bi[t] ? (1ull << bit) : 0ull;   // hits + band
                            if (v >= ai[t]) band[t] |= 1ull << (32 + bit);
                        }
            }
            // hits (link / border) and band pairs (all modes), lane-divergent
#pragma unroll
            for (int t = 0; t < QT && walk; ++t) {
                uint32_t m = (uint32_t)band[t];
                while (m) {
                    const int bit = __builtin_ctz(m);
                    m &= m - 1;
                    const int u = bit >> 4, q = (bit >> 2) & 3, e = bit & 3;
                    const uint32_t j = j0 + 32 * u + 8 * q + 4 * h + e;
                    if (!ok[t] || j >= A.J.m) continue;
                    if (MODE == kLink && j <= iq[t]) continue;
                    bool in = MODE != kCount && ((band[t] >> (32 + bit)) & 1ull);
                    if (!in) {
                        const uint32_t p = A.I.idx ? A.I.idx[iq[t]] : iq[t];
                        const uint32_t qj = A.J.idx ? A.J.idx[j] : j;
                        in = exact_within<T, 0>(A.X, A.d, p, qj, A.eps, A.eps2);
                    }
                    if (in) tile_hit<T, MODE>(A, iq[t], j, cnt[t], best[t]);
                }
            }
        }
    };
    // cursors: current tile (in LDS buf), next (in `ready`), the one after
    uint32_t sg = 0;
    j0 = seg_lo[0];
    bool have = seek(sg, j0);
    if (have) {
        fetch(stA, j0);
        commit(stA, 0);
    }
    uint32_t sn = sg, jn = j0 + kTile;
    bool more = have && seek(sn, jn);
    if (more) fetch(stB, jn);
    __syncthreads();
    auto step = [&](Stage& ready, Stage& spare) {
        uint32_t sf = sn, jf = jn + kTile;
        const bool far = more && seek(sf, jf);
        if (far) fetch(spare, jf);
        work();
        if (more) commit(ready, buf ^ 1);
        __syncthreads();
        sg = sn;
        j0 = jn;
        have = more;
        sn = sf;
        jn = jf;
        more = far;
        buf ^= 1;
    };
    while (have) {
        step(stB, stA);
        if (!have) break;
        step(stA, stB);
    }
    if (A.tiles && lane == 0 && ntiles) {
        atomicAdd(A.tiles, (unsigned long long)ntiles);
        if (nrefined) atomicAdd(A.tiles + 1, (unsigned long long)nrefined);
    }
    // lanes l and l + 32 hold the same query column
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        if constexpr (MODE == kCount) {
            cnt[t] += (uint32_t)__shfl_xor((int)cnt[t], 32, 64);
            if (h == 0 && ok[t]) A.cnt[iq[t]] = cnt[t];
        } else if constexpr (MODE == kBorder) {
            const uint32_t o = (uint32_t)__shfl_xor((int)best[t], 32, 64);
            best[t] = o < best[t] ? o : best[t];
            if (h == 0 && ok[t]) A.best[iq[t]] = best[t];
        }
    }
}

// Exact fp64 VALU tiles (cityblock; euclidean with d > 128 or an extreme
// scale): one lane per query, the streamed point broadcast to the wave.
template <typename T, int MODE, int M>
__global__ __launch_bounds__(kBlock) void brute_kernel(TileArgs<T> A) {
    if (not_my_rows(blockIdx.x * kBlock, A.shard_rank, A.shard_world)) return;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const bool ok = i < A.I.m;
    const uint32_t p = ok ? (A.I.idx ? A.I.idx[i] : i) : 0u;
    uint32_t cnt = 0, best = kNone;
    const uint32_t jbeg = MODE == kLink ? __builtin_amdgcn_readfirstlane(blockIdx.x * kBlock) : 0u;
    for (uint32_t j = jbeg; j < A.J.m; ++j) {
        if (!ok || (MODE == kLink && j <= i)) continue;
        const uint32_t q = A.J.idx ? A.J.idx[j] : j;
        if (exact_within<T, M>(A.X, A.d, p, q, A.eps, A.eps2)) tile_hit<T, MODE>(A, i, j, cnt, best);
    }
    if (!ok) return;
    if constexpr (MODE == kCount) A.cnt[i] = cnt;
    if constexpr (MODE == kBorder) A.best[i] = best;
}

// ---------------------------------------------------------------- small kernels
__global__ __launch_bounds__(kBlock) void iota_kernel(uint32_t* __restrict__ p, uint32_t m) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k < m) p[k] = k;
}

__global__ __launch_bounds__(kBlock) void flatten_keys_kernel(uint32_t* __restrict__ par,
                                                              const uint32_t* __restrict__ list,
                                                              uint32_t m,
                                                              uint32_t* __restrict__ keyc,
                                                              uint32_t* __restrict__ key_out) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    // root = smallest core row of the component = smallest core point id
    // (the list is ascending): sklearn's cluster order (engine.hip gmin)
    const uint32_t key = list[uf_find(par, k)];
    keyc[k] = key;
    key_out[list[k]] = key;
}

__global__ __launch_bounds__(kBlock) void scatter_best_kernel(const uint32_t* __restrict__ best,
                                                              const uint32_t* __restrict__ list,
                                                              uint32_t m,
                                                              uint32_t* __restrict__ key_out) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b < m) key_out[list[b]] = best[b];
}

// Sharded link: the union of every rank's forest over the core rows (each
// forest's edges i -> parent[i] carry its rank's connectivity).
__global__ __launch_bounds__(kBlock) void merge_forests_kernel(uint32_t* __restrict__ par,
                                                               const uint32_t* __restrict__ f,
                                                               uint32_t m, uint64_t total) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= total) return;
    const uint32_t i = (uint32_t)(t % m), p = f[t];
    if (p != i && p < m) uf_unite(par, i, p);
}

// Border keys in the exchange format (int32, none = INT32_MAX: a MIN
// all-reduce over the ranks picks the smallest adjacent key) and back.
__global__ __launch_bounds__(kBlock) void best_to_i32_kernel(const uint32_t* __restrict__ b,
                                                             uint32_t m, int32_t* __restrict__ o) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k < m) o[k] = b[k] == kNone ? INT32_MAX : (int32_t)b[k];
}
__global__ __launch_bounds__(kBlock) void best_from_i32_kernel(const int32_t* __restrict__ o,
                                                               uint32_t m, uint32_t* __restrict__ b) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k < m) b[k] = o[k] == INT32_MAX ? kNone : (uint32_t)o[k];
}

__global__ __launch_bounds__(kBlock) void outputs_kernel(const uint32_t* __restrict__ cnt,
                                                         uint64_t n, uint32_t ms, int full,
                                                         uint8_t* __restrict__ core,
                                                         uint32_t* __restrict__ counts) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = cnt[i];
    if (core) core[i] = c >= ms ? 1 : 0;
    if (counts) counts[i] = full ? c : (c < ms ? c : ms);
}

// Projection pruning: sort rows by one coordinate (order-preserving u64 of
// its fp64 value, -0.0 folded onto +0.0).
__device__ __forceinline__ unsigned long long proj_okey(double v) {
    unsigned long long b = (unsigned long long)__double_as_longlong(v);
    if (b == 0x8000000000000000ull) b = 0ull;
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void proj_key_kernel(const T* __restrict__ X, int d, int ax,
                                                          uint32_t n,
                                                          unsigned long long* __restrict__ key,
                                                          uint32_t* __restrict__ id) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    key[i] = proj_okey((double)X[(uint64_t)i * d + ax]);
    id[i] = i;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void proj_gather_kernel(const T* __restrict__ X, int d, int ax,
                                                             const uint32_t* __restrict__ sid,
                                                             uint32_t n, double* __restrict__ p) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < n) p[r] = (double)X[(uint64_t)sid[r] * d + ax];
}

// band of each point = its p1 rank / band; band p1 ranges from the p1 order
__global__ __launch_bounds__(kBlock) void band_of_kernel(const uint32_t* __restrict__ sid1, uint32_t n,
                                                         uint32_t band,
                                                         uint32_t* __restrict__ band_of) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < n) band_of[sid1[r]] = r / band;
}

__global__ __launch_bounds__(kBlock) void band_key_kernel(const uint32_t* __restrict__ band_of,
                                                          const uint32_t* __restrict__ sid2,
                                                          uint32_t n, uint32_t* __restrict__ key) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < n) key[r] = band_of[sid2[r]];
}

__global__ __launch_bounds__(kBlock) void band_range_kernel(const double* __restrict__ p1s, uint32_t n,
                                                            uint32_t band, uint32_t nband,
                                                            double* __restrict__ bp1) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= nband) return;
    bp1[2 * b] = p1s[b * band];
    bp1[2 * b + 1] = p1s[min((b + 1) * band, n) - 1u];
}

// group (band * nsub + sub-band) of each point from its position in the
// (band, p2) order; sub-band p2 ranges from the same order
__global__ __launch_bounds__(kBlock) void sub_of_kernel(const uint32_t* __restrict__ sid, uint32_t n,
                                                        uint32_t band, uint32_t sub, uint32_t nsub,
                                                        uint32_t* __restrict__ grp) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= n) return;
    const uint32_t b = r / band;
    grp[sid[r]] = b * nsub + (r - b * band) / sub;
}

__global__ __launch_bounds__(kBlock) void sub_range_kernel(const double* __restrict__ p2s, uint32_t n,
                                                           uint32_t band, uint32_t sub,
                                                           uint32_t nsub, uint32_t nband,
                                                           double* __restrict__ bp2) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= nband * nsub) return;
    const uint32_t b = g / nsub, k = g % nsub;
    const uint32_t r0 = b * band + k * sub, bend = min(b * band + band, n);
    if (r0 >= bend) {   // past the last band's rows: never a candidate
        bp2[2 * g] = 0.0;
        bp2[2 * g + 1] = 0.0;
        return;
    }
    bp2[2 * g] = p2s[r0];
    bp2[2 * g + 1] = p2s[min(r0 + sub, bend) - 1u];
}

__global__ __launch_bounds__(kBlock) void scatter_cnt_kernel(const uint32_t* __restrict__ cs,
                                                             const uint32_t* __restrict__ sid,
                                                             uint32_t n, uint32_t* __restrict__ cnt) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < n) cnt[sid[r]] = cs[r];
}

struct CntAtLeast {
    const uint32_t* cnt;
    uint32_t v;
    __device__ bool operator()(uint32_t i) const { return cnt[i] >= v; }
};
struct BorderCand {   // not core, a neighbour besides itself
    const uint32_t* cnt;
    uint32_t ms;
    __device__ bool operator()(uint32_t i) const { return cnt[i] >= 2 && cnt[i] < ms; }
};

template <typename Pred>
uint32_t select_ids(Ctx& ctx, const char* name, uint32_t n, Pred pred, uint32_t** out,
                    hipStream_t s) {
    uint32_t* list = ctx.arena.get<uint32_t>(name, n);
    uint32_t* dcount = ctx.arena.get<uint32_t>("dsel_count", 4);
    rocprim::counting_iterator<uint32_t> it(0u);
    size_t tb = 0;
    PD_HIP(rocprim::select(nullptr, tb, it, list, dcount, (size_t)n, pred, s));
    void* tmp = ctx.arena.get<char>("dsel_tmp", tb);
    PD_HIP(rocprim::select(tmp, tb, it, list, dcount, (size_t)n, pred, s));
    uint32_t* h = (uint32_t*)pinned(ctx, sizeof(uint32_t));
    PD_HIP(hipMemcpyAsync(h, dcount, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    sync(s);
    *out = list;
    return *h;
}

// ---------------------------------------------------------------- driver
struct Geometry {
    int KS = 1;            // k-steps of 16 dims (1, 2, 4 or 8)
    double* center = nullptr;
    double scale = 1.0;
    float elo = 0, ehi = 0;
    bool mfma = false;
    bool f8 = false;       // also build the e4m3 fragments (count pass screen)
};

template <typename T>
FragSet make_frags(Ctx& ctx, const std::string& tag, const T* X, int d, const uint32_t* idx,
                   uint32_t m, const Geometry& G, hipStream_t s) {
    const uint32_t rp = pad_rows(m ? m : 1);
    FragSet F;
    F.m = m;
    F.idx = idx;
    F.f8 = nullptr;
    if (!G.mfma) {
        F.hi = F.lo = nullptr;
        F.norm = F.nmax = nullptr;
        return F;
    }
    if (G.f8) {
        const int KS8 = (G.KS + 3) / 4;
        i32x8* f8 = ctx.arena.get<i32x8>(tag + "_f8", (size_t)(rp / 32) * KS8 * 64);
        hipLaunchKernelGGL(prep8_kernel<T>, dim3(nblocks((uint64_t)rp * KS8 * 2)), dim3(kBlock), 0,
                           s, X, d, idx, m, rp, KS8, G.center, G.scale, f8);
        F.f8 = f8;
    }
    const size_t nfrag = (size_t)(rp / 32) * G.KS * 64;
    bf16x8* hi = ctx.arena.get<bf16x8>(tag + "_hi", nfrag);
    bf16x8* lo = ctx.arena.get<bf16x8>(tag + "_lo", nfrag);
    float* nrm = ctx.arena.get<float>(tag + "_norm", rp);
    uint32_t* nmax = ctx.arena.get<uint32_t>(tag + "_nmax", 1);
    PD_HIP(hipMemsetAsync(nmax, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(prep_kernel<T>, dim3(nblocks((uint64_t)rp * G.KS * 2)), dim3(kBlock), 0, s,
                       X, d, idx, m, rp, G.KS, G.center, G.scale, hi, lo);
    hipLaunchKernelGGL(norm_kernel<T>, dim3(nblocks(rp)), dim3(kBlock), 0, s, X, d, idx, m, rp,
                       G.center, G.scale, nrm, nmax);
    PD_HIP(hipGetLastError());
    F.hi = hi;
    F.lo = lo;
    F.norm = nrm;
    F.nmax = (const float*)nmax;
    return F;
}

template <typename T, int MODE>
void run_tiles(const TileArgs<T>& A, const Geometry& G, int metric, hipStream_t s) {
    if (A.I.m == 0 || A.J.m == 0) return;
    if (G.mfma) {
        auto launch = [&](auto ks) {
            constexpr int KS = decltype(ks)::value, TB = tile_threads(KS, MODE);
            // the count pass (the bulk of the MFMA work) takes 4 query tiles per
            // wave where the registers allow it
            constexpr int QT = (MODE == kCount && KS <= 4) ? kCountQT : 2;
            const unsigned waves = (A.I.m + 32 * QT - 1) / (32 * QT);
            // pruned count: 8 x ceil(bands / 8) x blocks per band (tile_kernel)
            const unsigned grid = A.p3 ? 8u * ((A.nband + 7u) / 8u) * (A.band / (TB / 64 * 32 * QT))
                                       : nblocks(waves, TB / 64);
            if constexpr (MODE == kCount) {
                if (A.I.f8 && A.J.f8) {
                    constexpr int QT8 = KS <= 4 ? kF8QT : 2;
                    const unsigned grid8 =
                        A.p3 ? 8u * ((A.nband + 7u) / 8u) * (A.band / (TB / 64 * 32 * QT8))
                             : nblocks((A.I.m + 32 * QT8 - 1) / (32 * QT8), TB / 64);
                    hipLaunchKernelGGL((tile_kernel<T, MODE, KS, QT8, true>), dim3(grid8),
                                       dim3(TB), 0, s, A);
                    return;
                }
            }
            hipLaunchKernelGGL((tile_kernel<T, MODE, KS, QT, false>), dim3(grid), dim3(TB), 0, s, A);
        };
        switch (G.KS) {
            case 1: launch(std::integral_constant<int, 1>{}); break;
            case 2: launch(std::integral_constant<int, 2>{}); break;
            case 4: launch(std::integral_constant<int, 4>{}); break;
            default: launch(std::integral_constant<int, 8>{});
        }
    } else if (metric == 0) {
        hipLaunchKernelGGL((brute_kernel<T, MODE, 0>), dim3(nblocks(A.I.m)), dim3(kBlock), 0, s, A);
    } else {
        hipLaunchKernelGGL((brute_kernel<T, MODE, 1>), dim3(nblocks(A.I.m)), dim3(kBlock), 0, s, A);
    }
    PD_HIP(hipGetLastError());
}

struct Ev {
    Ctx& ctx;
    hipStream_t s;
    int k = 0;
    Ev(Ctx& c, hipStream_t st) : ctx(c), s(st) {}
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

Geometry geometry_of(const DenseState& ds) {
    Geometry G;
    G.KS = ds.KS;
    G.center = ds.center;
    G.scale = ds.scale;
    G.elo = ds.elo;
    G.ehi = ds.ehi;
    G.mfma = ds.mfma;
    return G;
}

template <typename T>
TileArgs<T> base_args(const DenseState& ds) {
    TileArgs<T> A{};
    A.X = (const T*)ds.X;
    A.d = ds.d;
    A.eps = ds.eps;
    A.eps2 = ds.eps * ds.eps;
    A.elo = ds.elo;
    A.ehi = ds.ehi;
    A.shard_rank = (uint32_t)ds.rank;
    A.shard_world = (uint32_t)ds.world;
    return A;
}

// Stage 1: neighbour counts (all x all tiles; this rank's rows when world >
// 1, every other row's count left 0 so the ranks' arrays sum to the whole).
template <typename T>
void count_stage(Ctx& ctx, TrainArgs& a, int rank, int world) {
    hipStream_t s = a.stream;
    DenseState& ds = ctx.dn;
    ds = DenseState{};
    const T* X = (const T*)a.X;
    const uint32_t n = (uint32_t)a.n;
    const int d = a.d;
    ds.X = a.X;
    ds.dtype = a.dtype;
    ds.d = d;
    ds.metric = a.metric;
    ds.n = n;
    ds.min_samples = (uint32_t)a.min_samples;
    ds.eps = a.eps;
    ds.rank = rank;
    ds.world = world;

    // geometry: centre on the bbox midpoint, scale by a power of two
    ds.KS = d <= 16 ? 1 : d <= 32 ? 2 : d <= 64 ? 4 : 8;
    std::vector<double> hc(d);
    double span = 0.0;
    for (int k = 0; k < d; ++k) {
        const double lo = a.data_box[k], hi = a.data_box[d + k];
        hc[k] = 0.5 * lo + 0.5 * hi;
        span = std::max(span, std::max(std::fabs(lo - hc[k]), std::fabs(hi - hc[k])));
    }
    int e2 = 0;
    if (span > 0.0) std::frexp(span, &e2);
    ds.scale = std::ldexp(1.0, -e2);   // max |scaled coordinate| in [0.5, 1]
    const double eps2s = a.eps * a.eps * ds.scale * ds.scale;
    ds.mfma = a.metric == 0 && d <= 128 && std::isfinite(eps2s) && eps2s > 1e-30 && eps2s < 1e30;
    if (ds.mfma) {
        ds.elo = std::nextafter((float)(eps2s * (1.0 - 1.0 / 1048576.0)), 0.0f);
        ds.ehi = std::nextafter((float)(eps2s * (1.0 + 1.0 / 1048576.0)), INFINITY);
        ds.center = ctx.arena.get<double>("dn_center", d);
        double* h = (double*)pinned(ctx, sizeof(double) * d);
        std::memcpy(h, hc.data(), sizeof(double) * d);
        PD_HIP(hipMemcpyAsync(ds.center, h, sizeof(double) * d, hipMemcpyHostToDevice, s));
    }
    Geometry G = geometry_of(ds);
    G.f8 = G.mfma && ctx.dense_screen == 1;   // the count pass's e4m3 screen
    TileArgs<T> A = base_args<T>(ds);
    A.f8_a = (float)std::ldexp(std::sqrt(64.0 * ((ds.KS + 3) / 4)), -18);

    uint32_t* cnt = ctx.arena.get<uint32_t>("dn_cnt", n);
    unsigned long long* dtiles = nullptr;
    if (G.mfma && ctx.dense_prune) {
        // rows in bands of the widest axis' rank, sub-bands of the second
        // widest's rank, sorted by the third within a sub-band; each block
        // streams only the tiles of its projection window (TileArgs::p3).
        // The margin covers the fp64 predicate: a pruned pair has one squared
        // term above eps^2 by 2^-20, so sklearn's rounded sum exceeds eps^2 too.
        int ax[3] = {0, 1, 2};
        double amax = 0.0;
        {
            std::vector<std::pair<double, int>> wd;
            for (int k = 0; k < d; ++k) {
                const double lo = a.data_box[k], hi = a.data_box[d + k];
                wd.push_back({-(hi - lo), k});
                amax = std::max(amax, std::max(std::fabs(lo), std::fabs(hi)));
            }
            std::stable_sort(wd.begin(), wd.end());
            for (int q = 0; q < 3; ++q) ax[q] = wd[q].second;   // d > 4
        }
        uint32_t band = 16384;   // a multiple of every tile block's rows
        while ((n + band - 1) / band > (uint32_t)kMaxBand) band *= 2;
        const uint32_t nband = (n + band - 1) / band;
        // sub-band rows: C3 sweep 256 / 512 / 1024 / 2048 / 4096 -> 89.1 / 82.0 /
        // 81.9 / 77.3 / 85.1 ms (a narrower p2 range vs shorter p3 runs)
        const uint32_t subr = 2048, nsub = band / subr;
        unsigned long long* k0 = ctx.arena.get<unsigned long long>("dn_pk0", n);
        unsigned long long* k1 = ctx.arena.get<unsigned long long>("dn_pk1", n);
        uint32_t* i0 = ctx.arena.get<uint32_t>("dn_pi0", n);
        uint32_t* i1 = ctx.arena.get<uint32_t>("dn_pi1", n);
        uint32_t* bof = ctx.arena.get<uint32_t>("dn_band_of", n);
        uint32_t* grp = ctx.arena.get<uint32_t>("dn_grp", n);
        uint32_t* bk0 = ctx.arena.get<uint32_t>("dn_bk0", n);
        uint32_t* bk1 = ctx.arena.get<uint32_t>("dn_bk1", n);
        uint32_t* i2 = ctx.arena.get<uint32_t>("dn_pi2", n);
        uint32_t* i3 = ctx.arena.get<uint32_t>("dn_pi3", n);
        double* pv = ctx.arena.get<double>("dn_p1s", n);
        double* bp1 = ctx.arena.get<double>("dn_bp1", 2 * nband);
        double* bp2 = ctx.arena.get<double>("dn_bp2", 2ull * nband * nsub);
        auto sort64 = [&](int axis) {   // ids in the order of coordinate `axis`
            hipLaunchKernelGGL(proj_key_kernel<T>, dim3(nblocks(n)), dim3(kBlock), 0, s, X, d,
                               axis, n, k0, i0);
            rocprim::double_buffer<unsigned long long> kb(k0, k1);
            rocprim::double_buffer<uint32_t> vb(i0, i1);
            size_t tb = 0;
            PD_HIP(rocprim::radix_sort_pairs(nullptr, tb, kb, vb, (size_t)n, 0u, 64u, s));
            void* tmp = ctx.arena.get<char>("dn_sort_tmp", tb);
            PD_HIP(rocprim::radix_sort_pairs(tmp, tb, kb, vb, (size_t)n, 0u, 64u, s));
            return (const uint32_t*)vb.current();
        };
        // stable re-sort of `ids` by key[id] (`bits` wide): the group order
        auto regroup = [&](const uint32_t* ids, const uint32_t* key, unsigned bits) {
            hipLaunchKernelGGL(band_key_kernel, dim3(nblocks(n)), dim3(kBlock), 0, s, key, ids, n,
                               bk0);
            PD_HIP(hipMemcpyAsync(i2, ids, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s));
            rocprim::double_buffer<uint32_t> kb(bk0, bk1);
            rocprim::double_buffer<uint32_t> vb(i2, i3);
            size_t tb = 0;
            PD_HIP(rocprim::radix_sort_pairs(nullptr, tb, kb, vb, (size_t)n, 0u, bits, s));
            void* tmp = ctx.arena.get<char>("dn_sort_tmp2", tb);
            PD_HIP(rocprim::radix_sort_pairs(tmp, tb, kb, vb, (size_t)n, 0u, bits, s));
            return (const uint32_t*)vb.current();
        };
        auto bits_for = [](uint32_t v) {
            unsigned b = 1;
            while ((1ull << b) < v) ++b;
            return b;
        };
        // (1) p1 order -> band of each point, band p1 ranges
        const uint32_t* sid1 = sort64(ax[0]);
        hipLaunchKernelGGL(band_of_kernel, dim3(nblocks(n)), dim3(kBlock), 0, s, sid1, n, band, bof);
        hipLaunchKernelGGL(proj_gather_kernel<T>, dim3(nblocks(n)), dim3(kBlock), 0, s, X, d, ax[0],
                           sid1, n, pv);
        hipLaunchKernelGGL(band_range_kernel, dim3(nblocks(nband)), dim3(kBlock), 0, s, pv, n,
                           band, nband, bp1);
        // (2) p2 order within bands -> sub-band (group) of each point, p2 ranges
        const uint32_t* sid2 = regroup(sort64(ax[1]), bof, bits_for(nband));
        hipLaunchKernelGGL(sub_of_kernel, dim3(nblocks(n)), dim3(kBlock), 0, s, sid2, n, band, subr,
                           nsub, grp);
        hipLaunchKernelGGL(proj_gather_kernel<T>, dim3(nblocks(n)), dim3(kBlock), 0, s, X, d, ax[1],
                           sid2, n, pv);
        hipLaunchKernelGGL(sub_range_kernel, dim3(nblocks(nband * nsub)), dim3(kBlock), 0, s, pv,
                           n, band, subr, nsub, nband, bp2);
        // (3) p3 order within groups: the final row order
        const uint32_t* sid = regroup(sort64(ax[2]), grp, bits_for(nband * nsub));
        double* ps = ctx.arena.get<double>("dn_proj", n);
        hipLaunchKernelGGL(proj_gather_kernel<T>, dim3(nblocks(n)), dim3(kBlock), 0, s, X, d, ax[2],
                           sid, n, ps);
        PD_HIP(hipGetLastError());
        const FragSet Fs = make_frags<T>(ctx, "dn_all", X, d, sid, n, G, s);
        uint32_t* cs = ctx.arena.get<uint32_t>("dn_cnt_sorted", n);
        if (world > 1) PD_HIP(hipMemsetAsync(cs, 0, sizeof(uint32_t) * n, s));
        dtiles = ctx.arena.get<unsigned long long>("dn_tiles", 2);
        PD_HIP(hipMemsetAsync(dtiles, 0, 2 * sizeof(unsigned long long), s));
        A.I = A.J = Fs;
        A.p3 = ps;
        A.bp1 = bp1;
        A.bp2 = bp2;
        A.band = band;
        A.nband = nband;
        A.sub = subr;
        A.nsub = nsub;
        A.whole_bands = ctx.dense_prune == 2 ? 1u : 0u;
        A.win = a.eps * (1.0 + 1.0 / 1048576.0) + 16.0 * amax * DBL_EPSILON;
        A.tiles = dtiles;
        A.cnt = cs;
        // the roofline kernel's own time (events around the launch alone)
        if (ctx.timing) {
            for (int k = 14; k < 16; ++k)
                if (!ctx.ev[k]) PD_HIP(hipEventCreate(&ctx.ev[k]));
            PD_HIP(hipEventRecord(ctx.ev[14], s));
        }
        run_tiles<T, kCount>(A, G, a.metric, s);
        if (ctx.timing) PD_HIP(hipEventRecord(ctx.ev[15], s));
        hipLaunchKernelGGL(scatter_cnt_kernel, dim3(nblocks(n)), dim3(kBlock), 0, s, cs, sid, n,
                           cnt);
        PD_HIP(hipGetLastError());
    } else {
        const FragSet Fall = make_frags<T>(ctx, "dn_all", X, d, nullptr, n, G, s);
        if (world > 1) PD_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * n, s));
        A.I = A.J = Fall;
        A.cnt = cnt;
        run_tiles<T, kCount>(A, G, a.metric, s);
    }
    ds.cnt = cnt;
    ds.tiles = dtiles;
    ds.stage = 1;
}

// Stage 2: core list from the (whole) counts; union-find over the core x
// core tiles j > i of this rank's rows.
template <typename T>
void link_stage(Ctx& ctx, hipStream_t s) {
    DenseState& ds = ctx.dn;
    const Geometry G = geometry_of(ds);
    uint32_t* clist = nullptr;
    const uint32_t mc = select_ids(ctx, "dn_core", ds.n, CntAtLeast{ds.cnt, ds.min_samples}, &clist, s);
    ds.n_core = mc;
    ds.clist = clist;
    ds.par = ctx.arena.get<uint32_t>("dn_par", mc + 1);
    ds.keyc = ctx.arena.get<uint32_t>("dn_keyc", mc + 1);
    if (mc) {
        hipLaunchKernelGGL(iota_kernel, dim3(nblocks(mc)), dim3(kBlock), 0, s, ds.par, mc);
        const FragSet Fcore = make_frags<T>(ctx, "dn_cf", (const T*)ds.X, ds.d, clist, mc, G, s);
        ds.cf[0] = Fcore.hi;
        ds.cf[1] = Fcore.lo;
        ds.cf[2] = Fcore.norm;
        ds.cf[3] = Fcore.nmax;
        TileArgs<T> A = base_args<T>(ds);
        A.I = A.J = Fcore;
        A.par = ds.par;
        run_tiles<T, kLink>(A, G, ds.metric, s);
    }
    ds.stage = 2;
}

// Stage 3: components (the union of `n_forests` forests when sharded), keys,
// border candidates' smallest adjacent core key over this rank's rows.
template <typename T>
void border_stage(Ctx& ctx, const uint32_t* forests, int n_forests, hipStream_t s) {
    DenseState& ds = ctx.dn;
    const Geometry G = geometry_of(ds);
    const uint32_t n = ds.n, mc = ds.n_core;
    ds.key_out = ctx.arena.get<uint32_t>("dn_key", n);
    PD_HIP(hipMemsetAsync(ds.key_out, 0xFF, sizeof(uint32_t) * n, s));
    ds.n_border = 0;
    if (mc) {
        if (forests && n_forests > 0) {
            const uint64_t total = (uint64_t)mc * (uint64_t)n_forests;
            hipLaunchKernelGGL(iota_kernel, dim3(nblocks(mc)), dim3(kBlock), 0, s, ds.par, mc);
            hipLaunchKernelGGL(merge_forests_kernel, dim3(nblocks(total)), dim3(kBlock), 0, s,
                               ds.par, forests, mc, total);
        }
        hipLaunchKernelGGL(flatten_keys_kernel, dim3(nblocks(mc)), dim3(kBlock), 0, s, ds.par,
                           ds.clist, mc, ds.keyc, ds.key_out);
        PD_HIP(hipGetLastError());
        uint32_t* blist = nullptr;
        const uint32_t mb = select_ids(ctx, "dn_border", n, BorderCand{ds.cnt, ds.min_samples},
                                       &blist, s);
        ds.n_border = mb;
        ds.blist = blist;
        if (mb) {
            ds.best = ctx.arena.get<uint32_t>("dn_best", mb);
            if (ds.world > 1) PD_HIP(hipMemsetAsync(ds.best, 0xFF, sizeof(uint32_t) * mb, s));
            FragSet Fcore;
            Fcore.hi = (const bf16x8*)ds.cf[0];
            Fcore.lo = (const bf16x8*)ds.cf[1];
            Fcore.norm = (const float*)ds.cf[2];
            Fcore.nmax = (const float*)ds.cf[3];
            Fcore.idx = ds.clist;
            Fcore.m = mc;
            TileArgs<T> A = base_args<T>(ds);
            A.I = make_frags<T>(ctx, "dn_bf", (const T*)ds.X, ds.d, blist, mb, G, s);
            A.J = Fcore;
            A.keyJ = ds.keyc;
            A.best = ds.best;
            run_tiles<T, kBorder>(A, G, ds.metric, s);
        }
    }
    ds.stage = 3;
}

// Stage 4: border keys into the key array, core flags / counts, labels.
void finish_stage(Ctx& ctx, int32_t* labels, uint8_t* core, uint32_t* counts, hipStream_t s) {
    DenseState& ds = ctx.dn;
    if (ds.n_border)
        hipLaunchKernelGGL(scatter_best_kernel, dim3(nblocks(ds.n_border)), dim3(kBlock), 0, s,
                           ds.best, ds.blist, ds.n_border, ds.key_out);
    hipLaunchKernelGGL(outputs_kernel, dim3(nblocks(ds.n)), dim3(kBlock), 0, s, ds.cnt,
                       (uint64_t)ds.n, ds.min_samples, ctx.full_counts ? 1 : 0, core, counts);
    PD_HIP(hipGetLastError());
    rank_labels_async(ctx, ds.key_out, ds.n, labels, s);   // count: rank_labels_count
}

template <typename T>
void run_dense(Ctx& ctx, TrainArgs& a) {
    hipStream_t s = a.stream;
    Ev ev(ctx, s);
    ev.mark();   // 0
    count_stage<T>(ctx, a, 0, 1);
    ev.mark();   // 1
    link_stage<T>(ctx, s);
    ev.mark();   // 2 (flatten of the components and the border tiles: border)
    border_stage<T>(ctx, nullptr, 0, s);
    ev.mark();   // 3
    finish_stage(ctx, a.labels, a.core, a.counts, s);
    ev.mark();   // 4
    a.n_clusters = rank_labels_count(ctx, s);
    DenseState& ds = ctx.dn;
    ctx.t.records = ds.n;
    ctx.t.core_records = ds.n_core;
    // dense (timing on): cells_n = wave tiles the count pass computed,
    // grid_cells = those its hi.hi screen passed on to the full split product
    ctx.t.cells_n = 0;
    ctx.t.grid_cells = 0;
    if (ds.tiles && ctx.timing) {
        unsigned long long nt[2] = {0, 0};
        PD_HIP(hipMemcpy(nt, ds.tiles, sizeof(nt), hipMemcpyDeviceToHost));
        ctx.t.cells_n = (int64_t)nt[0];
        ctx.t.grid_cells = (int64_t)nt[1];
    }
    ctx.t.count_kernel = 0;
    if (ctx.timing && ds.tiles && ctx.ev[14] && ctx.ev[15]) {
        float ms = 0;
        PD_HIP(hipEventElapsedTime(&ms, ctx.ev[14], ctx.ev[15]));
        ctx.t.count_kernel = ms;
    }
    if (ctx.timing) {
        ctx.t.count = ev.span(0, 1);
        ctx.t.link = ev.span(1, 2);
        ctx.t.border = ev.span(2, 3);
        ctx.t.label = ev.span(3, 4);
        ctx.t.total = ev.span(0, 4);
    }
}

template <typename F>
void by_dtype(int dtype, F&& f) {
    if (dtype == 0)
        f(float{});
    else if (dtype == 1)
        f(double{});
    else
        throw Error(-1, "dtype must be 0 (float32) or 1 (float64)");
}

}  // namespace

void dense_train(Ctx& ctx, TrainArgs& a) {
    if (a.phase != 0)
        throw Error(-5, "the grid phases (pd_train_begin/end) are d <= 4; d > 4 shards with pd_dense_*");
    if (!a.data_box) throw Error(-1, "dense path needs the data bbox");
    if (a.n >= 0xFFFFFFFFll) throw Error(-5, "dense path: n must be < 2^32 - 1");
    ctx.st.valid = false;
    by_dtype(a.dtype, [&](auto t) { run_dense<decltype(t)>(ctx, a); });
}

void dense_count(Ctx& ctx, TrainArgs& a, int rank, int world, uint32_t* counts_out) {
    if (!a.data_box) throw Error(-1, "dense path needs the data bbox");
    if (a.n >= 0x7FFFFFFFll) throw Error(-5, "sharded dense path: n must be < 2^31 - 1");
    if (world < 1 || rank < 0 || rank >= world) throw Error(-1, "bad rank / world");
    ctx.st.valid = false;
    ctx.t = Timings{};
    by_dtype(a.dtype, [&](auto t) { count_stage<decltype(t)>(ctx, a, rank, world); });
    if (a.n)
        PD_HIP(hipMemcpyAsync(counts_out, ctx.dn.cnt, sizeof(uint32_t) * a.n,
                              hipMemcpyDeviceToDevice, a.stream));
    if (ctx.timing && ctx.dn.tiles && ctx.ev[14] && ctx.ev[15]) {
        // this rank's share of the count pass (PD_T_COUNT / PD_T_COUNT_KERNEL)
        sync(a.stream);
        float ms = 0;
        PD_HIP(hipEventElapsedTime(&ms, ctx.ev[14], ctx.ev[15]));
        unsigned long long nt[2] = {0, 0};
        PD_HIP(hipMemcpy(nt, ctx.dn.tiles, sizeof(nt), hipMemcpyDeviceToHost));
        ctx.t.count = ctx.t.count_kernel = ms;
        ctx.t.records = a.n;
        ctx.t.cells_n = (int64_t)nt[0];
        ctx.t.grid_cells = (int64_t)nt[1];
    }
}

uint32_t dense_link(Ctx& ctx, const uint32_t* counts, uint32_t* forest_out, hipStream_t s) {
    DenseState& ds = ctx.dn;
    if (ds.stage != 1) throw Error(-1, "pd_dense_link: call pd_dense_count first");
    if (ds.n)
        PD_HIP(hipMemcpyAsync(ds.cnt, counts, sizeof(uint32_t) * ds.n, hipMemcpyDeviceToDevice, s));
    by_dtype(ds.dtype, [&](auto t) { link_stage<decltype(t)>(ctx, s); });
    if (ds.n_core)
        PD_HIP(hipMemcpyAsync(forest_out, ds.par, sizeof(uint32_t) * ds.n_core,
                              hipMemcpyDeviceToDevice, s));
    return ds.n_core;
}

uint32_t dense_border(Ctx& ctx, const uint32_t* forests, int n_forests, int32_t* best_out,
                      hipStream_t s) {
    DenseState& ds = ctx.dn;
    if (ds.stage != 2) throw Error(-1, "pd_dense_border: call pd_dense_link first");
    by_dtype(ds.dtype, [&](auto t) { border_stage<decltype(t)>(ctx, forests, n_forests, s); });
    if (ds.n_border) {
        hipLaunchKernelGGL(best_to_i32_kernel, dim3(nblocks(ds.n_border)), dim3(kBlock), 0, s,
                           ds.best, ds.n_border, best_out);
        PD_HIP(hipGetLastError());
    }
    return ds.n_border;
}

int64_t dense_finish(Ctx& ctx, const int32_t* best, int32_t* labels, uint8_t* core,
                     uint32_t* counts, hipStream_t s) {
    DenseState& ds = ctx.dn;
    if (ds.stage != 3) throw Error(-1, "pd_dense_finish: call pd_dense_border first");
    if (ds.n_border) {
        hipLaunchKernelGGL(best_from_i32_kernel, dim3(nblocks(ds.n_border)), dim3(kBlock), 0, s,
                           best, ds.n_border, ds.best);
        PD_HIP(hipGetLastError());
    }
    finish_stage(ctx, labels, core, counts, s);
    const int64_t ncl = rank_labels_count(ctx, s);
    ds.stage = 0;
    return ncl;
}

}  // namespace pd
