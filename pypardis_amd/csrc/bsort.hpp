// Bucketed sort of the halo records by (neighbourhood, eps-cell) key that
// carries the coordinates (round 5; the partitionBy shuffle,
// R:dbscan/dbscan.py:116-118, with the coordinate gather folded in).
//
// Included by engine.hip inside its anonymous namespace (it uses Stride<D>,
// wave_append and the arena helpers defined there).
//
// The rocPRIM onesweep sort of (key, id) pairs followed by a gather of the
// coordinates read the 1.2 GB input at random 12-byte rows (C2: 7 GB of
// 64-byte requests for 1.6 GB of coordinates) and moved the 8-byte pairs
// through four or five full passes.  Here records move as whole records —
// key, value (point id | flags) and the padded coordinate row — through a
// most-significant-digit bucket sort:
//
//   level 1   the records in input order (halo_write's output, coordinates
//             read from X at the record's point: consecutive records are
//             consecutive points) are scattered by the top <= 10 key bits;
//   level l   every bucket still larger than kBsCap records is scattered by
//             its next digit (fan-out sized to the bucket: ~kBsTarget records
//             per child), the rest stop here;
//   final     each bucket of <= kBsCap records is sorted in LDS by one
//             workgroup (rocprim block_radix_sort on its remaining <= 32 key
//             bits, stable) and written to its final place in order; a bucket
//             whose remaining bits are all used (a single key: one dense
//             cell) is copied as it is.
//
// Every scatter is a two-pass tile scan without atomics on global memory:
// bs_hist_kernel writes each tile's digit histogram as one column of a
// bucket-major matrix, one device-wide exclusive scan gives every (digit,
// tile) run its global offset, and bs_scatter_kernel counting-sorts the tile
// by digit in LDS and writes each field out by consecutive threads, so a
// digit's run is written as contiguous lines.  Positions are global: a bucket
// occupies the same index range [gpos, gpos + count) in every buffer, so the
// final pass reads a bucket wherever its last scatter left it.  Within one
// key the order is the LDS arrival order (not deterministic); every output of
// the train is independent of it (labels, core flags and counts are defined
// per point).

// Scatter tiles: 512 threads x 16 records, 72 KiB of LDS, so two tiles run
// per CU and one's loads overlap the other's stores (tools/msd_probe.hip:
// one 1024-thread tile per CU ran its load and store phases back to back,
// 2.0-2.4 TB/s).
constexpr int kBsThreads = 512;
constexpr int kBsPer = 16;
constexpr uint32_t kBsTile = kBsThreads * kBsPer;   // records per scatter tile
constexpr int kBsMaxBits = 10;            // fan-out <= 1024 per scatter
constexpr int kBsMaxFan = 1 << kBsMaxBits;
constexpr uint32_t kBsStage = 32768;      // LDS bytes staged per field round
constexpr uint32_t kBsCap = 8192;         // final-sort capacity (records per bucket)
constexpr uint32_t kBsTarget = 2048;      // aimed-at records per child bucket

template <typename T, int S>
struct alignas(sizeof(T) * S >= 16 ? 16 : sizeof(T) * S) BsRow {
    T v[S];
};

struct BsTile {
    uint64_t start;    // first record of the tile (input order on level 1, else global)
    uint32_t count;    // records of the tile
    uint32_t hbase;    // the segment's first histogram entry
    uint32_t nt;       // tiles of the segment
    uint32_t ti;       // this tile's index within its segment
    uint32_t shift;    // digit = (key >> shift) & (2^bits - 1)
    uint32_t bits;
    uint32_t cbase;    // the segment's first child-total entry
    uint32_t pad;
    int64_t delta;     // global position = scanned offset + delta
};

struct BsFin {
    uint64_t gpos;     // first record (global position)
    uint32_t count;
    uint32_t rem;      // key bits below the segment's common prefix (<= 32)
};

template <typename K>
__device__ __forceinline__ uint32_t bs_digit(K k, uint32_t shift, uint32_t bits) {
    return (uint32_t)((uint64_t)k >> shift) & ((1u << bits) - 1u);
}

// Per tile: its digit histogram as one column of the segment's bucket-major
// matrix (entry hbase + digit * nt + ti), and the digit totals of the
// segment (child totals, one atomic per non-empty digit and tile).
template <typename K>
__global__ __launch_bounds__(kBsThreads) void bs_hist_kernel(const K* __restrict__ keys,
                                                             const BsTile* __restrict__ tiles,
                                                             uint32_t* __restrict__ hist,
                                                             uint32_t* __restrict__ ctot) {
    __shared__ uint32_t h[kBsMaxFan];
    const BsTile t = tiles[blockIdx.x];
    const uint32_t F = 1u << t.bits;
    for (uint32_t b = threadIdx.x; b < F; b += kBsThreads) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kBsPer; ++i) {
        const uint32_t p = (uint32_t)i * kBsThreads + threadIdx.x;
        if (p < t.count) atomicAdd(&h[bs_digit(keys[t.start + p], t.shift, t.bits)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < F; b += kBsThreads) {
        const uint32_t c = h[b];
        hist[(uint64_t)t.hbase + (uint64_t)b * t.nt + t.ti] = c;
        if (c) atomicAdd(ctot + t.cbase + b, c);
    }
}

// One field of the tile's records written out in digit order: positions
// [lo, lo + per) of the tile's sorted order go through LDS (stage), then
// consecutive threads write consecutive sorted positions to their global
// slots dst[p] — a digit's run lands as contiguous lines.  value(i) is read
// in the round that needs it (loads of the later fields overlap the stores).
template <typename E, typename F>
__device__ __forceinline__ void bs_field_out(uint32_t n, const uint32_t (&sp)[kBsPer],
                                             const uint32_t* __restrict__ dst, char* stage,
                                             E* __restrict__ out, F&& value) {
    constexpr uint32_t per = kBsStage / sizeof(E);   // positions per round
    E* st = reinterpret_cast<E*>(stage);
    for (uint32_t lo = 0; lo < n; lo += per) {
        __syncthreads();   // the previous round's (or field's) readers are done
#pragma unroll
        for (int i = 0; i < kBsPer; ++i)
            if (sp[i] - lo < per) st[sp[i] - lo] = value(i);
        __syncthreads();
        const uint32_t hi = n < lo + per ? n : lo + per;
        for (uint32_t p = lo + threadIdx.x; p < hi; p += kBsThreads) out[dst[p]] = st[p - lo];
    }
}

// Scatter of one level: every tile's records to their children's global
// positions.  FROM_X (level 1): the records are in input order and their
// coordinates come from the points (X, D values per point); otherwise from
// the previous level's row buffer.
template <typename T, int D, typename K, bool FROM_X>
__global__ __launch_bounds__(kBsThreads) void bs_scatter_kernel(
    const T* __restrict__ X, const K* __restrict__ keys, const uint32_t* __restrict__ vals,
    const BsRow<T, Stride<D>::v>* __restrict__ rows, const BsTile* __restrict__ tiles,
    const uint32_t* __restrict__ scan, K* __restrict__ okeys, uint32_t* __restrict__ ovals,
    BsRow<T, Stride<D>::v>* __restrict__ orows) {
    constexpr int S = Stride<D>::v;
    using Row = BsRow<T, S>;
    __shared__ uint32_t cnt[kBsMaxFan];   // digit counts, then the tile-local offsets
    __shared__ uint32_t gb[kBsMaxFan];    // the digit's global offset for this tile
    __shared__ uint32_t dst[kBsTile];     // sorted position -> global position
    __shared__ __attribute__((aligned(16))) char stage[kBsStage];
    const BsTile t = tiles[blockIdx.x];
    const uint32_t F = 1u << t.bits;
    for (uint32_t b = threadIdx.x; b < F; b += kBsThreads) cnt[b] = 0;
    __syncthreads();
    K k[kBsPer];
    uint32_t sp[kBsPer];   // digit, then the rank within it, then the sorted position
#pragma unroll
    for (int i = 0; i < kBsPer; ++i) {
        const uint32_t p = (uint32_t)i * kBsThreads + threadIdx.x;
        k[i] = p < t.count ? keys[t.start + p] : K(0);
    }
    uint32_t rk[kBsPer];
#pragma unroll
    for (int i = 0; i < kBsPer; ++i) {
        const uint32_t p = (uint32_t)i * kBsThreads + threadIdx.x;
        sp[i] = bs_digit(k[i], t.shift, t.bits);
        rk[i] = p < t.count ? atomicAdd(&cnt[sp[i]], 1u) : 0u;
    }
    __syncthreads();
    // tile-local exclusive scan of the digit counts (two per thread)
    {
        const uint32_t b0 = 2 * threadIdx.x, b1 = b0 + 1;
        const uint32_t c0 = b0 < F ? cnt[b0] : 0u, c1 = b1 < F ? cnt[b1] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan<kBsThreads>(c0 + c1, total);
        if (b0 < F) {
            cnt[b0] = ex;
            gb[b0] = (uint32_t)((int64_t)scan[(uint64_t)t.hbase + (uint64_t)b0 * t.nt + t.ti] + t.delta);
        }
        if (b1 < F) {
            cnt[b1] = ex + c0;
            gb[b1] = (uint32_t)((int64_t)scan[(uint64_t)t.hbase + (uint64_t)b1 * t.nt + t.ti] + t.delta);
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kBsPer; ++i) {
        const uint32_t p = (uint32_t)i * kBsThreads + threadIdx.x;
        if (p < t.count) {
            const uint32_t d = sp[i];
            sp[i] = cnt[d] + rk[i];
            dst[sp[i]] = gb[d] + rk[i];
        } else {
            sp[i] = 0xFFFFFFFFu;
        }
    }
    const uint32_t n = t.count;
    const uint64_t r0 = t.start + threadIdx.x;
    bs_field_out<K>(n, sp, dst, stage, okeys, [&](int i) { return k[i]; });
    bs_field_out<uint32_t>(n, sp, dst, stage, ovals,
                           [&](int i) { return vals[r0 + (uint64_t)i * kBsThreads]; });
    bs_field_out<Row>(n, sp, dst, stage, orows, [&](int i) {
        if constexpr (FROM_X) {
            const uint64_t pt = vals[r0 + (uint64_t)i * kBsThreads] & kIdMask;
            Row row;
#pragma unroll
            for (int j = 0; j < S; ++j) row.v[j] = j < D ? X[pt * D + j] : T(0);
            return row;
        } else {
            return rows[r0 + (uint64_t)i * kBsThreads];
        }
    });
}

// Final level: one workgroup per bucket of <= NT * IPT records.  A stable LDS
// radix sort of (key bits below the bucket's prefix, index), then output
// position p takes record idx[p] of the bucket (re-read from the L2-hot
// source) and is written in order; the records of points in several
// neighbourhoods are listed for the merge (dup list) and their points' merge
// representative (rep) starts at kNone.
template <typename T, int D, typename K, int NT, int IPT>
__global__ __launch_bounds__(NT) void bs_final_kernel(
    const K* __restrict__ keys, const uint32_t* __restrict__ vals,
    const BsRow<T, Stride<D>::v>* __restrict__ rows, const BsFin* __restrict__ fins,
    K* __restrict__ okeys, uint32_t* __restrict__ ovals, BsRow<T, Stride<D>::v>* __restrict__ orows,
    uint32_t* __restrict__ dup_list, uint32_t* __restrict__ dup_count, uint32_t* __restrict__ rep) {
    using sort_t = rocprim::block_radix_sort<uint32_t, NT, IPT, uint16_t>;
    __shared__ typename sort_t::storage_type st;
    const BsFin f = fins[blockIdx.x];
    const uint32_t m = f.count;
    const uint64_t mask = f.rem >= 32 ? 0xFFFFFFFFull : ((1ull << f.rem) - 1ull);
    uint32_t kk[IPT];
    uint16_t ix[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t p = threadIdx.x * IPT + i;   // blocked
        kk[i] = p < m ? (uint32_t)((uint64_t)keys[f.gpos + p] & mask) : 0xFFFFFFFFu;
        ix[i] = (uint16_t)p;
    }
    // the padding keys (0xFFFFFFFF) sort last: bits [0, 32) whenever padded
    const int end_bit = (m < (uint32_t)(NT * IPT) || f.rem >= 32) ? 32 : (int)f.rem;
    sort_t().sort_to_striped(kk, ix, st, 0, end_bit);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t p = (uint32_t)i * NT + threadIdx.x;   // striped
        uint32_t v = 0;
        if (p < m) {
            const uint64_t src = f.gpos + ix[i], o = f.gpos + p;
            okeys[o] = keys[src];
            v = vals[src];
            ovals[o] = v;
            orows[o] = rows[src];
            if (rep && (v & kDupBit)) rep[v & kIdMask] = kNone;
        }
        wave_append(dup_list, dup_count, p < m && (v & kDupBit), (uint32_t)(f.gpos + p));
    }
}

// A bucket of one key (more than kBsCap records of one dense cell): copied
// as it is, several workgroups per bucket.
template <typename T, int D, typename K>
__global__ __launch_bounds__(kBlock) void bs_copy_kernel(
    const K* __restrict__ keys, const uint32_t* __restrict__ vals,
    const BsRow<T, Stride<D>::v>* __restrict__ rows, const BsFin* __restrict__ cps, uint32_t ncp,
    K* __restrict__ okeys, uint32_t* __restrict__ ovals, BsRow<T, Stride<D>::v>* __restrict__ orows,
    uint32_t* __restrict__ dup_list, uint32_t* __restrict__ dup_count, uint32_t* __restrict__ rep) {
    for (uint32_t c = 0; c < ncp; ++c) {   // uniform loop over the (few) copy buckets
        const BsFin f = cps[c];
        for (uint32_t b = blockIdx.x * kBlock; b < f.count; b += gridDim.x * kBlock) {
            const uint32_t p = b + threadIdx.x;
            uint32_t v = 0;
            if (p < f.count) {
                const uint64_t o = f.gpos + p;
                okeys[o] = keys[o];
                v = vals[o];
                ovals[o] = v;
                orows[o] = rows[o];
                if (rep && (v & kDupBit)) rep[v & kIdMask] = kNone;
            }
            wave_append(dup_list, dup_count, p < f.count && (v & kDupBit), (uint32_t)(f.gpos + p));
        }
    }
}

// Host side: grow-only pinned staging for the level lists (tiles, child
// totals, final / copy lists).  A level's lists are written only after the
// previous level's last upload has left the block (ctx.bs_ev).
struct BsHost {
    std::vector<BsTile> tiles;
    std::vector<BsFin> fin_s, fin_m, fin_l, copies;
};

inline char* bs_pinned(Ctx& ctx, size_t bytes) {
    if (ctx.bs_pinned_bytes < bytes) {
        if (ctx.bs_pinned) {
            PD_HIP(hipDeviceSynchronize());
            PD_HIP(hipHostFree(ctx.bs_pinned));
            ctx.bs_pinned = nullptr;
            ctx.bs_pinned_bytes = 0;
        }
        const size_t want = std::max<size_t>(bytes + bytes / 4, 4 << 20);
        void* p = nullptr;
        PD_HIP(hipHostMalloc(&p, want, hipHostMallocDefault));
        ctx.bs_pinned = p;
        ctx.bs_pinned_bytes = want;
    }
    return (char*)ctx.bs_pinned;
}

// Sort the R records (keys_in, vals_in: input order; coordinates at X[point])
// into (okeys, ovals, orows), ascending key.  keys_in / vals_in are
// overwritten (they double as the second level buffer).  Stats: levels run.
template <typename T, int D, typename K>
int bucket_sort(Ctx& ctx, hipStream_t s, uint32_t R, int key_bits, const T* X, K* keys_in,
                uint32_t* vals_in, K* okeys, uint32_t* ovals, T* oxs, uint32_t* dup_list,
                uint32_t* dup_count, uint32_t* rep) {
    constexpr int S = Stride<D>::v;
    using Row = BsRow<T, S>;
    constexpr uint32_t TILE = kBsTile;
    if (!R) return 0;
    Row* orows = reinterpret_cast<Row*>(oxs);
    // level buffers: A, and B = the input pairs (dead after level 1) + rows
    K* kA = ctx.arena.get<K>("bs_keysA", R);
    uint32_t* vA = ctx.arena.get<uint32_t>("bs_valsA", R);
    Row* rA = ctx.arena.get<Row>("bs_rowsA", R);
    K* kB = keys_in;
    uint32_t* vB = vals_in;
    Row* rB = nullptr;   // allocated when a third level needs it

    struct Seg {
        uint64_t gpos;
        uint32_t count, rem;
    };
    std::vector<Seg> active{{0, R, (uint32_t)std::max(key_bits, 1)}};
    BsHost H;
    int level = 0;
    // source of the current level: (keys, vals, rows); level 1 reads X
    const K* sk = keys_in;
    const uint32_t* sv = vals_in;
    const Row* sr = nullptr;
    K* dk = kA;
    uint32_t* dv = vA;
    Row* dr = rA;
    bool upload_pending = false;
    while (!active.empty()) {
        if (upload_pending) PD_HIP(hipEventSynchronize(ctx.bs_ev));
        upload_pending = false;
        // ---- the level's tiles and digit widths
        H.tiles.clear();
        std::vector<uint32_t> seg_bits(active.size()), seg_cbase(active.size());
        uint64_t hent = 0, cent = 0, act_prefix = 0;
        for (size_t si = 0; si < active.size(); ++si) {
            const Seg& g = active[si];
            uint32_t want = 1;
            while (want < (uint32_t)kBsMaxBits && ((uint64_t)g.count >> want) > kBsTarget) ++want;
            const uint32_t bits = std::min<uint32_t>(want, g.rem);
            const uint32_t nt = (g.count + TILE - 1) / TILE;
            seg_bits[si] = bits;
            seg_cbase[si] = (uint32_t)cent;
            for (uint32_t ti = 0; ti < nt; ++ti) {
                BsTile t{};
                t.start = (level == 0 ? 0 : g.gpos) + (uint64_t)ti * TILE;
                t.count = std::min<uint32_t>(TILE, g.count - ti * TILE);
                t.hbase = (uint32_t)hent;
                t.nt = nt;
                t.ti = ti;
                t.shift = g.rem - bits;
                t.bits = bits;
                t.cbase = (uint32_t)cent;
                t.delta = (int64_t)g.gpos - (int64_t)act_prefix;
                H.tiles.push_back(t);
            }
            hent += (uint64_t)nt << bits;
            cent += 1ull << bits;
            act_prefix += g.count;
        }
        if (hent >= 0xFFFFFFF0ull) throw Error(-5, "bucket sort: histogram too large");
        const size_t ntl = H.tiles.size();
        // pinned: [tiles | child totals]
        const size_t tb = sizeof(BsTile) * ntl, cb = sizeof(uint32_t) * cent;
        char* hp = bs_pinned(ctx, tb + cb + 64);
        std::memcpy(hp, H.tiles.data(), tb);
        BsTile* dtiles = ctx.arena.get<BsTile>("bs_tiles", ntl);
        PD_HIP(hipMemcpyAsync(dtiles, hp, tb, hipMemcpyHostToDevice, s));
        uint32_t* hist = ctx.arena.get<uint32_t>("bs_hist", hent + 1);
        uint32_t* scan = ctx.arena.get<uint32_t>("bs_scan", hent + 1);
        uint32_t* ctot = ctx.arena.get<uint32_t>("bs_ctot", cent);
        PD_HIP(hipMemsetAsync(ctot, 0, cb, s));
        hipLaunchKernelGGL((bs_hist_kernel<K>), dim3((unsigned)ntl), dim3(kBsThreads), 0, s,
                           sk, dtiles, hist, ctot);
        {
            size_t tmpb = 0;
            PD_HIP(rocprim::exclusive_scan(nullptr, tmpb, hist, scan, 0u, (size_t)hent,
                                           rocprim::plus<uint32_t>(), s));
            void* tmp = ctx.arena.get<char>("bs_scan_tmp", tmpb);
            PD_HIP(rocprim::exclusive_scan(tmp, tmpb, hist, scan, 0u, (size_t)hent,
                                           rocprim::plus<uint32_t>(), s));
        }
        if (level == 0)
            hipLaunchKernelGGL((bs_scatter_kernel<T, D, K, true>), dim3((unsigned)ntl),
                               dim3(kBsThreads), 0, s, X, sk, sv, (const Row*)nullptr, dtiles,
                               scan, dk, dv, dr);
        else
            hipLaunchKernelGGL((bs_scatter_kernel<T, D, K, false>), dim3((unsigned)ntl),
                               dim3(kBsThreads), 0, s, X, sk, sv, sr, dtiles, scan, dk, dv, dr);
        PD_HIP(hipGetLastError());
        uint32_t* hc = (uint32_t*)(hp + ((tb + 15) & ~size_t(15)));
        PD_HIP(hipMemcpyAsync(hc, ctot, cb, hipMemcpyDeviceToHost, s));
        sync(s);
        // ---- children: final (sorted in LDS), copied (one key), or the next level
        std::vector<Seg> next;
        H.fin_s.clear();
        H.fin_m.clear();
        H.fin_l.clear();
        H.copies.clear();
        for (size_t si = 0; si < active.size(); ++si) {
            const Seg& g = active[si];
            const uint32_t bits = seg_bits[si], F = 1u << bits, rem = g.rem - bits;
            uint64_t pos = g.gpos;
            for (uint32_t c = 0; c < F; ++c) {
                const uint32_t m = hc[seg_cbase[si] + c];
                if (!m) continue;
                if (m <= kBsCap && rem <= 32) {
                    const BsFin f{pos, m, rem};
                    (m <= 1024 ? H.fin_s : m <= 4096 ? H.fin_m : H.fin_l).push_back(f);
                } else if (rem == 0) {
                    H.copies.push_back(BsFin{pos, m, 0});
                } else {
                    next.push_back(Seg{pos, m, rem});
                }
                pos += m;
            }
            if (pos != g.gpos + g.count) throw Error(-3, "bucket sort: child totals disagree");
        }
        // ---- finish the buckets that stop here (source: this level's output)
        const size_t nf = H.fin_s.size() + H.fin_m.size() + H.fin_l.size() + H.copies.size();
        if (nf) {
            char* fp = bs_pinned(ctx, tb + cb + 64 + sizeof(BsFin) * nf + 64) + tb + cb + 64;
            fp = (char*)(((uintptr_t)fp + 15) & ~uintptr_t(15));
            BsFin* hf = (BsFin*)fp;
            size_t o = 0;
            for (auto* L : {&H.fin_s, &H.fin_m, &H.fin_l, &H.copies})
                for (const BsFin& f : *L) hf[o++] = f;
            BsFin* df = ctx.arena.get<BsFin>("bs_fins", nf);
            PD_HIP(hipMemcpyAsync(df, hf, sizeof(BsFin) * nf, hipMemcpyHostToDevice, s));
            if (!ctx.bs_ev) PD_HIP(hipEventCreateWithFlags(&ctx.bs_ev, hipEventDisableTiming));
            PD_HIP(hipEventRecord(ctx.bs_ev, s));
            upload_pending = true;
            size_t at = 0;
            if (!H.fin_s.empty())
                hipLaunchKernelGGL((bs_final_kernel<T, D, K, 256, 4>), dim3((unsigned)H.fin_s.size()),
                                   dim3(256), 0, s, dk, dv, dr, df + at, okeys, ovals, orows, dup_list,
                                   dup_count, rep);
            at += H.fin_s.size();
            if (!H.fin_m.empty())
                hipLaunchKernelGGL((bs_final_kernel<T, D, K, 512, 8>), dim3((unsigned)H.fin_m.size()),
                                   dim3(512), 0, s, dk, dv, dr, df + at, okeys, ovals, orows, dup_list,
                                   dup_count, rep);
            at += H.fin_m.size();
            if (!H.fin_l.empty())
                hipLaunchKernelGGL((bs_final_kernel<T, D, K, 512, 16>),
                                   dim3((unsigned)H.fin_l.size()), dim3(512), 0, s, dk, dv, dr,
                                   df + at, okeys, ovals, orows, dup_list, dup_count, rep);
            at += H.fin_l.size();
            if (!H.copies.empty())
                hipLaunchKernelGGL((bs_copy_kernel<T, D, K>), dim3(1024), dim3(kBlock), 0, s, dk, dv,
                                   dr, df + at, (uint32_t)H.copies.size(), okeys, ovals, orows,
                                   dup_list, dup_count, rep);
            PD_HIP(hipGetLastError());
        }
        active.swap(next);
        ++level;
        if (active.empty()) break;
        if (level > 12) throw Error(-3, "bucket sort: too many levels");
        // the next level reads this level's output and writes the other buffer
        if (!rB) rB = ctx.arena.get<Row>("bs_rowsB", R);
        sk = dk;
        sv = dv;
        sr = dr;
        const bool toB = dk == kA;
        dk = toB ? kB : kA;
        dv = toB ? vB : vA;
        dr = toB ? rB : rA;
        // (the final kernels of this level read sk/sv/sr; the next scatter
        // writes the other buffer, so they do not race)
    }
    return level;
}
