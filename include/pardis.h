/*
 * libpardis — C ABI of the MI355X DBSCAN engine (drop-in for the pyParDis
 * per-partition clustering path).
 *
 * Every entry point takes plain pointers and sizes.  X / labels / owner /
 * core / counts / members are DEVICE pointers (caller-owned, e.g. a torch
 * tensor's data_ptr()); arrays named *_host are host memory.  `stream` is a
 * hipStream_t (NULL = default stream).  Calls are stream-ordered; functions
 * that return a host result synchronise the stream before returning.
 * Return value: PD_OK (0) or a negative PD_E* code; pd_last_error() gives the
 * message for the calling thread.  No C++ exception crosses this boundary.
 *
 * Reference interfaces replaced (R: = mathematiguy/pypardis, SK: = sklearn 1.7.2):
 *   pd_bbox          R:dbscan/partition.py:135-137  data.aggregate(BoundingBox(k), union)
 *   pd_kd_moments    R:dbscan/partition.py:86-89    min_var_split moments aggregate
 *   pd_kd_counts     R:dbscan/partition.py:60-63    mean_var_split 7-bound counts aggregate
 *   pd_kd_split      R:dbscan/partition.py:66-68    filter(v[axis] >= boundary) relabel
 *                    (also :27-29, the median_search_split filters)
 *   pd_kd_radix_hist R:dbscan/partition.py:23-26    sortBy(v[axis]).collect()[len/2] (rotation)
 *   pd_kd_pass       R:dbscan/partition.py:66-68 + 86-89 (+ 135-137): one level's split of
 *                    the previous level fused with this level's moments aggregate
 *   pd_halo_members  R:dbscan/dbscan.py:136-151     _create_neighborhoods filter(contains)
 *   pd_cluster       R:dbscan/dbscan.py:28-30       skc.DBSCAN(**params).fit_predict(x),
 *                                                   core_sample_indices_  (SK:cluster/_dbscan.py:369-446)
 *   pd_train         R:dbscan/dbscan.py:114-126     halo + partitionBy + mapPartitions(dbscan_partition)
 *                                                   + _remap_cluster_ids (dbscan.py:153-165,
 *                                                   aggregator.py:9-73) fused on one device
 */
#ifndef PARDIS_H
#define PARDIS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PD_ABI_VERSION 3

enum pd_status {
    PD_OK = 0,
    PD_EINVAL = -1,       /* bad argument (also: NaN/inf input, like sklearn's ValueError) */
    PD_EOOM = -2,         /* device allocation failed */
    PD_EHIP = -3,         /* HIP runtime error */
    PD_ERCCL = -4,        /* RCCL error (multi-device merge) */
    PD_EUNSUPPORTED = -5  /* shape/extent outside what this build implements */
};

enum pd_dtype { PD_F32 = 0, PD_F64 = 1 };

/* scipy.spatial.distance.euclidean / cityblock (R:dbscan/dbscan.py:74,82-91) */
enum pd_metric { PD_EUCLIDEAN = 0, PD_CITYBLOCK = 1 };

enum pd_option {
    PD_OPT_TIMING = 1,      /* record per-stage HIP events inside pd_train */
    PD_OPT_FULL_COUNTS = 2,  /* neighbour counts without the >= min_samples early exit */
    PD_OPT_SEQUENTIAL_MOMENTS = 3, /* pd_kd_moments folds points in index order, exactly as
                                      the reference's single-slice aggregate (slow; for
                                      bit-identical split boundaries).  Default: correctly
                                      rounded, order-independent double-double sums. */
    PD_OPT_XSUB = 6,        /* sub-cells per eps along axis 0 (default 2): finer rows follow
                               the eps-ball's chord more tightly, at 1/xsub the directory
                               density */
    PD_OPT_FP32_SCREEN = 7, /* fp32 inputs: decide pairs outside a 2^-18 band around eps with
                               fp32 arithmetic, the rest with the exact fp64 predicate
                               (default 1; results are identical with 0) */
    PD_OPT_SWEEP_STATS = 8, /* tally the neighbour sweeps' candidates and union-find outcomes
                               into the PD_T_S_* slots (instrumented kernels; default 0) */
    PD_OPT_DENSE_PRUNE = 11   /* d > 4 count pass: stream only the tiles inside the three-axis
                                projection window (exact; default 1; 0 = all n^2 pairs;
                                2 = per-band runs, the path a block takes when its segment
                                list overflows — for tests) */,
    PD_OPT_COUNT_ROTATE = 12  /* count sweep: a candidate list longer than this starts at
                                record (r & ~255) when that lies in the query's own row, and
                                wraps (dense cells: spreads the row-start hot spot; same
                                counts, same labels); default 1024, 0 = never */,
    PD_OPT_CENTRE_WINDOW = 13 /* link stage: records after each record tested by the window union
                                (2, 4, 8, 16, 32 or 64).  Default -1: by the records per
                                occupied cell — 2 up to 2.5, 8 up to 8, else 16.  A heuristic either way: the cell
                                verify proves or tests every core-core edge, so labels are the
                                same */,
    PD_OPT_DIR_BUDGET = 14    /* bytes the eps-grid directory may take (flat: 20 B per 64 cells;
                                paged: 16 B per 4096 cells + 40 B per point); beyond it every cell
                                grows by a common factor until it fits (exact at any width >= eps;
                                more candidates per record).
                                Default 32 GiB (PD_T_GRID_GROW reports the factor) */,
    PD_OPT_LABEL_BUCKETS = 15 /* single device: the labels reach input order through
                                coalesced passes (pairs bucketed by point id into 2^19-point
                                buckets, those split into 2^15-point ones, each placed in LDS
                                and written out with the core flags coalesced) instead of one
                                scattered write per record: 1 on, 0 off, -1 (default) from
                                2^22 points on, where it is faster (C2 1e8: border + label
                                4.35 -> 3.65 ms; C4 1e9: 30.3 -> 25.4 ms; C1 1e7: 0.33 ->
                                0.29 ms); 2: the round-4 form (2^19-point buckets scattered
                                inside one XCD's L2, then a key -> label pass).  Same labels
                                either way */,
    PD_OPT_DIR_PAGED = 17     /* eps-grid directory layout: 1 paged (pages of 4096 cells hold a
                                mask of their occupied 64-cell words; only occupied words are
                                stored: memory and build time follow the occupied cells, not the
                                extent), 0 flat (one word per 64 cells of the bounding box), -1
                                (default) paged when the grid has more words than points or the
                                flat one would pass PD_OPT_DIR_BUDGET.  Same results either way */,
    PD_OPT_DENSE_SCREEN = 18  /* d > 4 count pass: the tile screen that decides which tiles
                                compute the exact-banded split-bf16 product.  1 (default): e4m3
                                Gram tiles on v_mfma_f32_32x32x64_f8f6f4 (half the staged bytes,
                                twice the MFMA rate); 0: bf16 hi.hi.  Same counts either way */,
    PD_OPT_SHARD_CORE_BIT = 19 /* pd_train_end: 1 = the caller guarantees every global id is
                                < 2^31, so the core flags ride bit 31 of the keys and reach
                                core_out by one coalesced pass instead of a byte scattered per
                                owner record (default 0; same outputs).  pd_train_end checks
                                the guarantee on the device (every component key < 2^31) and
                                returns PD_EINVAL when a key breaks it */,
    PD_OPT_COUNT_REPLAY = 24  /* measurement only (tools/count_ceiling.py): after the grid train's
                                count sweep, run the same sweep again over this many replicas of
                                the records (lane i sweeps record i mod R; replicas write the
                                same values) and put its time in PD_T_COUNT_KERNEL — on a record
                                set small enough to stay in L2, the sweep's latency ceiling.
                                Default 0 (off) */,
    PD_OPT_HALO_PASSES = 25   /* grid train halo records: 2 (default) tile counts, scan, write
                                (two reads of the points); 1: one pass — each tile counts its
                                records, takes its offset by decoupled look-back and writes them
                                into buffers of a guessed capacity (a larger total reruns 2);
                                measured slower on C2 (halo 1.62 vs 1.31 ms), kept for A/B.
                                Same records either way */,
    PD_OPT_HALO_CAP = 26      /* single-pass halo record capacity (tests: force the overflow
                                path); 0 (default): n + n/8 + 4096 */,
    PD_OPT_KD_FUSE = 27       /* device-decided KD (pd_kd_build): 0 (default) a moments pass and
                                a counts pass per level; 1: a level of <= 2 splits counts its
                                candidates and sums the moments of each (split, candidate
                                interval) in one pass, so the next level's moments need no pass
                                of their own (4 passes over the points instead of 6 at
                                max_partitions = 8) — measured slower on C2 (the interval-slot
                                counting sort costs more than the pass it saves), kept for A/B.
                                Same splits either way */,
    PD_OPT_VERIFY_FUSED = 28  /* link stage cell verify: 0 (default) a screen pass flags the cells
                                whose forward rows hold another root, then the flagged cells are
                                listed and verified; 1: one pass over every cell with the screen
                                inline (no flags, list, scan or host read) — measured slower on
                                C2 (link 5.52 vs 5.32 ms: the flagged lanes' work diverges inside
                                every wave), kept for A/B.  Same labels */,
    PD_OPT_HALO_TREE = 29     /* grid train halo (two-pass form, split tree replayed, P <= 64):
                                0 (default) every point tests every expanded box; 1: a point
                                farther than 2 eps from every split plane on its KD path is in
                                its owner's expanded box only — one record, no box tests — and
                                the points near a plane are listed per tile for the full test;
                                measured slower (C2 halo 1.36 vs 1.19 ms, C4 11.3 vs 9.4 ms: the
                                dependent tree walk and the list cost more than the box tests),
                                kept for A/B.  Same records either way */,
    PD_OPT_KD_REPLAY = 30     /* pd_kd_build with final_split = 2 (DBSCAN.train's KD): 0 (default)
                                labels in HBM, read and rewritten by each level's passes; 1 each
                                pass recomputes the points' labels by replaying the splits
                                decided so far (tables in LDS) — no int32 label traffic, but the
                                walk costs more than it saves (KD C2 2.76 vs 2.55 ms, C4 18.7 vs
                                17.1 ms), kept for A/B.  Same splits either way */
    /* Retired in round 5 (measured A/Bs whose losing kernels were removed;
       pd_ctx_set_option returns PD_EINVAL for them, and the numbers are not
       reused): 4 LINK_MODE, 5 JUMP_ROUNDS, 9 SWEEP_VARIANT, 10 BORDER_ROOTS,
       16 SORT_PAYLOAD, 20 BORDER_LISTS, 21 LINK_JUMPS, 22 DENSE_PREFETCH,
       23 DENSE_WAVES.  DESIGN.md §6 keeps their measurements. */
};

/* pd_ctx_timings() slots (ms from HIP events on the call's stream; counters) */
enum pd_timing_slot {
    PD_T_HALO = 0, PD_T_SORT, PD_T_GATHER, PD_T_CELLS, PD_T_COUNT, PD_T_LINK, PD_T_MERGE,
    PD_T_ROOTS, PD_T_BORDER, PD_T_LABEL, PD_T_TOTAL, PD_T_RECORDS, PD_T_CELLS_N, PD_T_GRID_CELLS,
    PD_T_KEY_BITS, PD_T_CORE_RECORDS,
    /* PD_OPT_SWEEP_STATS counters */
    PD_T_S_COUNT_CAND, PD_T_S_LINK_CAND, PD_T_S_LINK_HIT, PD_T_S_LINK_CORE, PD_T_S_LINK_SAME,
    PD_T_S_LINK_FIND_SAME, PD_T_S_LINK_UNIONS, PD_T_S_VERIFY_PAIRS,
    PD_T_GRID_GROW,            /* cell width / eps of the last grid train (1 unless the
                                  directory budget made the cells grow) */
    PD_T_COUNT_KERNEL,         /* dense path: ms of the count pass's tile kernel alone
                                  (PD_T_COUNT includes its projection sorts) */
    PD_T_DIR_PAGED,            /* 1 if the last grid train used the paged directory */
    PD_T_DIR_WORDS,            /* directory words it allocated (paged: occupied + 1) */
    PD_T_S_COUNT_BATCHES,      /* count sweep (PD_OPT_SWEEP_STATS): wave batches swept */
    PD_T_S_COUNT_STAGED,       /*   (retired LDS-staged count sweep: always 0) */
    PD_T_HALO_FALLBACK,        /* 1 if the last single-pass halo overflowed its capacity and
                                  the two-pass form ran */
    PD_T_NSLOTS
};

typedef struct pd_ctx pd_ctx;

int32_t pd_abi_version(void);
const char* pd_last_error(void);

/* One context per (host thread, device): owns the device scratch arena. */
int32_t pd_ctx_create(int32_t device, pd_ctx** out);
int32_t pd_ctx_destroy(pd_ctx* ctx);
int32_t pd_ctx_set_option(pd_ctx* ctx, int32_t option, int64_t value);
int32_t pd_ctx_timings(pd_ctx* ctx, double* out_host, int32_t n_slots);

/* Tight bbox: lohi_host[0..d) = min, [d..2d) = max (fp64); nonfinite_host
 * (nullable) = number of NaN/inf coordinates. */
int32_t pd_bbox(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                double* lohi_host, int64_t* nonfinite_host, void* stream);

/* For each selected label sel_host[s]: moments_host[s][3][d] = {count, sum v,
 * sum v*v}, v*v rounded in the input precision, sums in fp64, deterministic. */
int32_t pd_kd_moments(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                      const int32_t* labels, int32_t n_sel, const int32_t* sel_host,
                      double* moments_host, void* stream);

/* counts_host[s][0..6] = #points of label sel_host[s] with v[axis_host[s]] <
 * bounds_host[s][i]; counts_host[s][7] = #points of that label. */
int32_t pd_kd_counts(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                     const int32_t* labels, int32_t n_sel, const int32_t* sel_host,
                     const int32_t* axis_host, const double* bounds_host, int64_t* counts_host,
                     void* stream);

/* labels[i] = new_host[s] where labels[i] == sel_host[s] and
 * v[axis_host[s]] >= boundary_host[s] (in place). */
int32_t pd_kd_split(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                    int32_t* labels, int32_t n_sel, const int32_t* sel_host,
                    const int32_t* axis_host, const double* boundary_host,
                    const int32_t* new_host, void* stream);

/* One pass of the radix select behind split_method='rotation'
 * (median_search_split, R:dbscan/partition.py:8-30: the value at index len/2
 * of sortBy(v[axis])).  key(v) = order-preserving u64 of (double)v[axis_host[s]]
 * (-0.0 taken as +0.0).  hist_host[s][b] = #points of label sel_host[s] with
 * key >> (shift + 8) == prefix_host[s] (no condition when shift == 56) and
 * (key >> shift) & 255 == b.  shift in {56, 48, .., 0}. */
int32_t pd_kd_radix_hist(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                         const int32_t* labels, int32_t n_sel, const int32_t* sel_host,
                         const int32_t* axis_host, const uint64_t* prefix_host, int32_t shift,
                         int64_t* hist_host, void* stream);

/* The record sort of pd_train on caller arrays (utility; exposed so the
 * kernel can be tested on its own): stable LSD radix sort of n (key, value)
 * pairs by key bits [0, key_bits), in place (bits at and above key_bits are
 * ignored: pairs whose keys agree below key_bits keep their input order).
 * keys: device uint32 (key_bytes
 * 4) or uint64 (8); vals: device uint32.  n < 2^32 - 1.  It is the shuffle
 * by neighbourhood that R:dbscan/dbscan.py:116-118 (partitionBy) performs,
 * keyed by (neighbourhood, cell). */
int32_t pd_sort_pairs(pd_ctx* ctx, void* keys, int32_t key_bytes, uint32_t* vals, int64_t n,
                      int32_t key_bits, void* stream);

/* ebox_host: P x [lo[d], hi[d]] (inclusive).  counts_host[P] = members per
 * box; if members != NULL it receives the ascending point ids of box 0, then
 * box 1, ... (capacity entries at most). */
int32_t pd_halo_members(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                        int32_t P, const double* ebox_host, int64_t* counts_host,
                        int64_t* members, int64_t capacity, void* stream);

/* sklearn DBSCAN(eps, min_samples, metric).fit_predict on one point set:
 * labels[n] (int32, -1 noise, equal to sklearn's labels_), core[n] (nullable),
 * counts[n] (nullable: neighbour counts incl. self, capped at min_samples
 * unless PD_OPT_FULL_COUNTS), *n_clusters_host. */
int32_t pd_cluster(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                   double eps, int32_t min_samples, int32_t metric, int32_t* labels,
                   uint8_t* core, uint32_t* counts, int64_t* n_clusters_host, void* stream);

/* The whole per-device train: P neighbourhoods given by their expanded boxes
 * (ebox_host, P x [lo[d], hi[d]], i.e. BoundingBox.expand(2*eps)), owner[n] =
 * KD label of each point (NULL when P == 1), data_box_host = tight bbox
 * (nullable).  Output as pd_cluster: global DBSCAN labels over all points. */
int32_t pd_train(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                 int32_t min_samples, int32_t metric, int32_t P, const double* ebox_host,
                 const double* data_box_host, const int32_t* owner, int32_t* labels,
                 uint8_t* core, uint32_t* counts, int64_t* n_clusters_host, void* stream);

/* pd_train with the KD split tree instead of the owner labels
 * (R:dbscan/partition.py:151-152 replayed per point inside the halo pass:
 * level l, a point whose label has a split moves to newlab when v[axis] >=
 * boundary): no owner array, no final split pass.  The tree in BFS order as
 * pd_kd_build's: level_sizes_host[l] splits, then per split cur / axis /
 * boundary / newlab (host).  d <= 4, <= 16 levels. */
int32_t pd_train_tree(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                      int32_t min_samples, int32_t metric, int32_t P, const double* ebox,
                      const double* data_box, int32_t n_levels, const int32_t* level_sizes_host,
                      const int32_t* cur_host, const int32_t* axis_host,
                      const double* boundary_host, const int32_t* newlab_host, int32_t* labels,
                      uint8_t* core, uint32_t* counts, int64_t* n_clusters, void* stream);

/* ---- sharded train (one process per device; the caller moves the buffers
 * between devices, e.g. torch.distributed over RCCL).  Replaces Spark's
 * partitionBy shuffle of the halo records (R:dbscan/dbscan.py:114-118) and the
 * driver-side ClusterAggregator merge (R:dbscan/dbscan.py:153-165,
 * R:dbscan/aggregator.py:9-73).  Global ids must stay below 2^32 - 1. */

/* pd_kd_moments with the double-double partial sums left unrounded, so that
 * devices can add them exactly: out_host[s][1 + 4d] = {count, (sum hi, sum
 * lo) per axis, (sumsq hi, sumsq lo) per axis}.  R:dbscan/partition.py:86-89 */
int32_t pd_kd_moments_dd(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                         const int32_t* labels, int32_t n_sel, const int32_t* sel_host,
                         double* out_host, void* stream);

/* One fused streaming pass of a KD BFS level (R:dbscan/partition.py:66-68 then
 * :86-89, and :135-137 on the first level), so a level costs two reads of X
 * (this pass and pd_kd_counts) instead of three:
 *   1. labels[i] = split_new_host[s] where labels[i] == split_sel_host[s] and
 *      v[split_axis_host[s]] >= split_boundary_host[s] (the previous level's
 *      splits; n_split may be 0);
 *   2. out_host[s][1 + 4d] = pd_kd_moments_dd of label sel_host[s] over the
 *      updated labels (n_sel may be 0);
 *   3. labels_zero != 0 (every label is 0; no split): labels are not read, and
 *      if lohi_host != NULL also the tight bbox as pd_bbox (n_sel must be 1).
 * Sums as pd_kd_moments_dd: correctly rounded double-double partials. */
int32_t pd_kd_pass(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                   int32_t* labels, int32_t labels_zero, int32_t n_split,
                   const int32_t* split_sel_host, const int32_t* split_axis_host,
                   const double* split_boundary_host, const int32_t* split_new_host,
                   int32_t n_sel, const int32_t* sel_host, double* out_host, double* lohi_host,
                   int64_t* nonfinite_host, void* stream);

/* mask[n] (device, u64): bit r set when some neighbourhood L with
 * part_rank_host[L] == r has an expanded box containing point i;
 * counts_host[r] = points routed to device r.  n_ranks <= 64. */
int32_t pd_route(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t P,
                 const double* ebox_host, const int32_t* part_rank_host, int32_t n_ranks,
                 uint64_t* mask, int64_t* counts_host, void* stream);

/* Pack the points routed to device `dest` (ascending local index): coords
 * (d values each, input dtype), gid = gid_base + local index, owner = index of
 * the point's KD partition kdlab[i] among dest's neighbourhoods
 * (local_index_host) when part_rank_host[kdlab[i]] == dest, else -1, xr = the
 * point was routed to more than one device.  *m_host = points packed. */
int32_t pd_pack(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                const uint64_t* mask, int32_t dest, const int32_t* kdlab, int32_t P,
                const int32_t* part_rank_host, const int32_t* local_index_host,
                uint32_t gid_base, void* coords, uint32_t* gid, int32_t* owner, uint8_t* xr,
                int64_t capacity, int64_t* m_host, void* stream);

/* Phase A on this device's neighbourhoods (arguments as pd_train; gid[n] =
 * global id of each local point (null: the identity, a one-rank group), xr[n]
 * = point also lives on another device (null: none does)).
 * *n_exports_host = number of (global id, component key) exports. */
int32_t pd_train_begin(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                       double eps, int32_t min_samples, int32_t metric, int32_t P,
                       const double* ebox_host, const double* data_box_host,
                       const int32_t* owner, const uint32_t* gid, const uint8_t* xr,
                       int64_t* n_exports_host, void* stream);

/* Copy the exports of the last pd_train_begin into device buffers. */
int32_t pd_train_exports(pd_ctx* ctx, uint32_t* gid, uint32_t* key, int64_t capacity,
                         void* stream);

/* Union of all devices' exports (gid[m], key[m]: every device's
 * pd_train_exports, gathered): ids[u] = the distinct ids the pairs name,
 * ascending; keys[u] = each one's global key (its component's smallest id).
 * Capacity of ids / keys: 2 m.  *u_host = u.  O(m log m): the id space is
 * never materialised.  Replaces the driver-side ClusterAggregator
 * (R:dbscan/dbscan.py:153-161, R:dbscan/aggregator.py:9-73). */
int32_t pd_merge_exports(pd_ctx* ctx, const uint32_t* gid, const uint32_t* key, int64_t m,
                         uint32_t* ids, uint32_t* keys, int64_t* u_host, void* stream);

/* Phase B: (map_ids, map_keys, n_map) from pd_merge_exports (n_map may be 0);
 * keys[n] = global cluster key of each owned point (0xFFFFFFFF = noise or not
 * owned here), core[n] (nullable) = owned core point. */
int32_t pd_train_end(pd_ctx* ctx, int64_t n, const uint32_t* map_ids, const uint32_t* map_keys,
                     int64_t n_map, uint32_t* keys, uint8_t* core, void* stream);

/* roots (device, capacity n) = global ids of owned points that are their
 * cluster's key, i.e. one id per cluster over all devices; *m_host = count. */
int32_t pd_select_roots(pd_ctx* ctx, const uint32_t* keys, const uint32_t* gid, int64_t n,
                        uint32_t* roots, int64_t* m_host, void* stream);

/* In-place ascending sort of n u32 (device). */
int32_t pd_sort_u32(pd_ctx* ctx, uint32_t* data, int64_t n, void* stream);

/* labels[i] = rank of keys[i] among the sorted roots (all devices' roots),
 * -1 for 0xFFFFFFFF — sklearn's numbering, as pd_train's labels.  A key that
 * is not among the roots (roots not gathered from every device) is an error:
 * PD_EINVAL.  Synchronises the stream. */
int32_t pd_rank_labels(pd_ctx* ctx, const uint32_t* keys, int64_t n, const uint32_t* roots,
                       int64_t n_roots, int32_t* labels, void* stream);

/* Results back to the devices that hold the points (R:dbscan/dbscan.py:162-164
 * result RDD): the owned records (owner[i] >= 0) of this device packed as
 * out[2 m] = (gid, (label + 1) | core << 31) pairs in ascending gid, and
 * counts_host[r] = how many fall in [gid_offsets_host[r],
 * gid_offsets_host[r + 1]) (device r's input slice).  The gids must ascend
 * (the pd_pack / all-to-all order); *m_host = m. */
int32_t pd_owned_results(pd_ctx* ctx, int64_t n, const int32_t* owner, const uint32_t* gid,
                         const int32_t* labels, const uint8_t* core, int32_t n_ranks,
                         const int64_t* gid_offsets_host, uint32_t* out, int64_t capacity,
                         int64_t* counts_host, int64_t* m_host, void* stream);

/* labels[gid - gid_base] / core[...] (nullable) from m received pairs of
 * pd_owned_results; m must equal n and every point must receive exactly one
 * result (PD_EINVAL otherwise). */
int32_t pd_scatter_results(pd_ctx* ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base,
                           int64_t n, int32_t* labels, uint8_t* core, void* stream);

/* ---- Sharded dense train (d > 4): the reference runs any k through the same
 * per-partition sklearn fit (R:dbscan/partition.py:131-133, R:dbscan/dbscan.py:
 * 123-124, SK:cluster/_dbscan.py:410-434); here every rank holds all n points
 * (an all-gather of the slices) and computes the distance tiles of its share
 * of the rows: row chunks of 2048 dealt round-robin over the ranks.  Four
 * stages with one collective between each (the caller's):
 *   pd_dense_count  -> counts: this rank's rows' neighbour counts (self
 *                      included), 0 elsewhere        [all-reduce SUM, u32]
 *   pd_dense_link   <- the summed counts; -> forest: this rank's union-find
 *                      over the core rows (*n_core)  [all-gather, n_ranks x n_core]
 *   pd_dense_border <- the gathered forests; -> best: smallest adjacent core
 *                      key per border candidate, INT32_MAX where none or not
 *                      this rank's row (*n_border)   [all-reduce MIN, i32]
 *   pd_dense_finish <- the reduced best; labels / core / counts of all n
 *                      points, *n_clusters — equal on every rank and to
 *                      pd_cluster's.
 * Calls on one context must follow this order; X must stay valid until
 * pd_dense_finish.  n < 2^31 - 1.  data_box: 2 x d tight bbox (host).
 * Single rank (rank 0 of 1): the stages chained without collectives equal
 * pd_cluster.  Buffers are device pointers sized n (counts, forest, best). */
int32_t pd_dense_count(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                       int32_t min_samples, int32_t metric, const double* data_box_host,
                       int32_t rank, int32_t n_ranks, uint32_t* counts, void* stream);
int32_t pd_dense_link(pd_ctx* ctx, const uint32_t* counts, uint32_t* forest, int64_t* n_core_host,
                      void* stream);
int32_t pd_dense_border(pd_ctx* ctx, const uint32_t* forests, int32_t n_forests, int32_t* best,
                        int64_t* n_border_host, void* stream);
int32_t pd_dense_finish(pd_ctx* ctx, const int32_t* best, int32_t* labels, uint8_t* core,
                        uint32_t* counts, int64_t* n_clusters_host, void* stream);

/* The whole KD partition of one device (R:dbscan/partition.py:139-183 with
 * min_var_split, exact sums) as one chain of launches and one host sync: the
 * per-level decisions (largest-variance axis, the seven bounds, the balanced
 * boundary — R:dbscan/partition.py:86-95,58-65) run on the device in the host
 * path's fp64 operation order, so the splits equal pd_kd_pass + pd_kd_counts
 * + host decisions bit for bit.  Levels of the BFS schedule: level l splits
 * level_sizes[l] labels, cur[] -> newlab[] (concatenated over levels, the
 * first level's single label 0).  labels (device int32[n]; need not be initialised
 * when n_levels >= 2 or final_split — every label is then written — else all 0)
 * end as the partition labels.  trace_host: 13 doubles per split — axis,
 * mean, variance, n_less for the 7 bounds, n, candidate index, boundary.
 * lohi_host: bbox (2 d); *bad_host: non-finite coordinates.  d <= 4, labels
 * < 256, 16-byte aligned X / labels; PD_EUNSUPPORTED otherwise (use the
 * per-pass entry points).  final_split = 0 leaves the last level's split
 * unapplied (labels then hold the previous level's; pd_train_tree replays
 * the tree itself, pd_kd_split applies it when the labels are wanted);
 * final_split = 2: the caller needs no labels (it replays the tree itself:
 * pd_train_tree, pd_kd_labels) — the passes then replay the splits decided
 * so far from tables in LDS instead of reading and writing an int32 label
 * per point (PD_OPT_KD_REPLAY; trees of <= 256 splits), and the labels array
 * is left unspecified. */
int32_t pd_kd_build(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                    int32_t* labels, int32_t n_levels, const int32_t* level_sizes_host,
                    const int32_t* cur_host, const int32_t* newlab_host, int32_t final_split,
                    double* trace_host, double* lohi_host, int64_t* bad_host, void* stream);

/* The KD labels of every point from a finished split tree (the
 * R:dbscan/partition.py:66-68 filters replayed per point: level l, a point
 * whose label has a split moves to newlab when v[axis] >= boundary) — the
 * labels of a pd_kd_build run with final_split = 2, on request.  The tree in
 * BFS order as pd_train_tree's: level_sizes_host[l] splits, then per split
 * cur / axis / boundary / newlab (host arrays).  labels: device int32[n]. */
int32_t pd_kd_labels(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                     int32_t* labels, int32_t n_levels, const int32_t* level_sizes_host,
                     const int32_t* cur_host, const int32_t* axis_host,
                     const double* boundary_host, const int32_t* newlab_host, void* stream);

/* ---- Sharded train, device-resident variant (no host round trip per KD
 * level, one ordered pass per exchange side).  The KD partition of
 * R:dbscan/partition.py:139-183 (min_var_split, exact sums) split at its
 * collectives: per level l of the BFS schedule (as pd_kd_build's)
 *   pd_kdx_moments  -> out: this slice's partials, S_l x (1 + 4d) doubles (+ the
 *                      bbox, 2d + 1 doubles, on level 0)  [caller: all-gather,
 *                      rank order -> n_ranks x len]
 *   pd_kdx_axes     <- the gathered partials: exact rank-order fold, the split
 *                      axes and 7 bounds (R:dbscan/partition.py:86-95,58-59)
 *   pd_kdx_counts   -> out: S_l x 8 u64 n_less / n of this slice
 *                      [caller: all-reduce SUM, u64]
 *   pd_kdx_boundary <- the summed counts: the balanced bound (:60-65)
 * then pd_kdx_end: the last level's split (final_split), the trace (13 doubles
 * per split, as pd_kd_build) and the global bbox to the host (one sync).  The
 * splits equal the single-device pd_kd_build's bit for bit.  Every rank calls
 * every step (an empty slice contributes zeros).  d <= 4. */
int32_t pd_kdx_begin(pd_ctx* ctx, int32_t d, int32_t n_levels, const int32_t* level_sizes_host,
                     const int32_t* cur_host, const int32_t* newlab_host, void* stream);
int32_t pd_kdx_moments(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                       int32_t* labels, int32_t level, double* out, void* stream);
int32_t pd_kdx_axes(pd_ctx* ctx, const double* gathered, int32_t n_ranks, int32_t level,
                    void* stream);
int32_t pd_kdx_counts(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                      const int32_t* labels, int32_t level, uint64_t* out, void* stream);
int32_t pd_kdx_boundary(pd_ctx* ctx, const uint64_t* counts, int32_t level, void* stream);
int32_t pd_kdx_end(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                   int32_t* labels, int32_t final_split, double* trace_host, double* lohi_host,
                   int64_t* bad_host, void* stream);

/* The partitionBy shuffle of the halo records (R:dbscan/dbscan.py:114-118) in
 * two ordered passes over the slice.  pd_route2: destination mask of every
 * point (kept in the context) and counts_host[2 r] = points routed to rank r,
 * counts_host[2 r + 1] = those of them rank r owns (kdlab's partition lives
 * there) — the sizes of the results that come back.  pd_pack2 (same context,
 * next call): every point written to each of its destinations in ascending
 * local index, into per-destination buffers given as host arrays of device
 * pointers (coords[r], gid[r], owner[r], xr[r]; null where nothing is routed):
 * pack the self block straight into the receive buffers and the rest into
 * the send buffers of pd_comm_exchange.  Fields as pd_pack. */
int32_t pd_route2(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t P,
                  const double* ebox_host, const int32_t* part_rank_host, const int32_t* kdlab,
                  int32_t n_ranks, int64_t* counts_host, void* stream);
int32_t pd_pack2(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                 const int32_t* kdlab, int32_t P, const int32_t* part_rank_host,
                 const int32_t* local_index_host, uint32_t gid_base, int32_t n_ranks,
                 void* const* coords_host, uint32_t* const* gid_host, int32_t* const* owner_host,
                 uint8_t* const* xr_host, void* stream);

/* Results back to the ranks holding the points (R:dbscan/dbscan.py:162-164):
 * after pd_train_end (keys) and the gathered, sorted roots of all ranks.  The
 * nr records arrived grouped by source rank (src_offsets_host[n_ranks + 1]);
 * the owned ones of this rank's own block are written straight into
 * labels[n_local] / core_out (gid - gid_base), the others compacted in order
 * as pairs (gid, (label + 1) | core << 31) — block by block, i.e. destination
 * by destination — expect_remote of them (the exchanged owned counts).  gid
 * may be null (identity: a one-rank group).  pd_results_scatter adds the
 * pairs received from the other ranks and checks (one sync) that every point
 * got exactly one label and every key has a root: PD_EINVAL otherwise. */
int32_t pd_results(pd_ctx* ctx, int64_t nr, const uint32_t* keys, const uint8_t* core,
                   const int32_t* owner, const uint32_t* gid, const uint32_t* roots,
                   int64_t n_roots, int64_t n_total, uint32_t gid_base, int64_t n_local,
                   int32_t n_ranks, int32_t rank, const int64_t* src_offsets_host,
                   int64_t expect_remote, int32_t* labels, uint8_t* core_out, uint32_t* pairs,
                   void* stream);
int32_t pd_results_scatter(pd_ctx* ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base,
                           int64_t n, int32_t* labels, uint8_t* core, void* stream);

/* ---- RCCL collectives of the sharded train (one rank per device).  They
 * replace Spark's data movement: partitionBy shuffle (R:dbscan/dbscan.py:
 * 114-118) -> pd_comm_all_to_all_v; collect / broadcast of the cluster-id map
 * (R:dbscan/dbscan.py:153-161) -> pd_comm_all_gather_v; the KD aggregates
 * (R:dbscan/partition.py:60-63,86-89,135-137) -> pd_comm_all_reduce.  Buffers
 * are device pointers, counts are elements; calls are stream-ordered. */
typedef struct pd_comm pd_comm;
#define PD_COMM_ID_BYTES 128
enum pd_elem { PD_E_U8 = 0, PD_E_I32 = 1, PD_E_U32 = 2, PD_E_I64 = 3, PD_E_U64 = 4,
               PD_E_F32 = 5, PD_E_F64 = 6 };
enum pd_reduce { PD_R_SUM = 0, PD_R_MAX = 1, PD_R_MIN = 2 };

/* ncclGetUniqueId: rank 0 creates the id, the caller hands the
 * PD_COMM_ID_BYTES bytes to every rank (any host channel). */
int32_t pd_comm_unique_id(uint8_t* id_host);
/* ncclCommInitRank on the context's device (collective over n_ranks). */
int32_t pd_comm_init(pd_ctx* ctx, int32_t n_ranks, int32_t rank, const uint8_t* id_host,
                     pd_comm** out);
/* One process driving n devices: out_host[i] = rank i on devices_host[i]
 * (ncclCommInitAll). */
int32_t pd_comm_init_all(int32_t n, const int32_t* devices_host, pd_comm** out_host);
int32_t pd_comm_destroy(pd_comm* comm);
int32_t pd_comm_all_reduce(pd_comm* comm, const void* send, void* recv, int64_t count,
                           int32_t elem, int32_t op, void* stream);
/* recv = concatenation over ranks r of counts_host[r] elements. */
int32_t pd_comm_all_gather_v(pd_comm* comm, const void* send, void* recv,
                             const int64_t* counts_host, int32_t elem, void* stream);
/* send grouped by destination rank, recv grouped by source rank. */
int32_t pd_comm_all_to_all_v(pd_comm* comm, const void* send, const int64_t* send_counts_host,
                             void* recv, const int64_t* recv_counts_host, int32_t elem,
                             void* stream);
int32_t pd_comm_broadcast(pd_comm* comm, void* buf, int64_t count, int32_t elem, int32_t root,
                          void* stream);
/* ncclCommCount / ncclCommUserRank: the rank count and this rank as RCCL
 * reports them (the executor count of the reference's fan-out,
 * R:dbscan/dbscan.py:116-126; bench.py's rccl_ranks). */
int32_t pd_comm_size(pd_comm* comm, int32_t* n_ranks, int32_t* rank);
/* n_fields buffers exchanged in ONE group (the halo-record fields of the
 * partitionBy shuffle): block r of field f = rec_bytes[f] * counts[r] bytes at
 * rec_bytes[f] * offsets[r] (send grouped by destination, recv by source;
 * all host arrays of n_ranks).  skip_self != 0: the self blocks are already in
 * place in recv (pd_pack2 wrote them). */
int32_t pd_comm_exchange(pd_comm* comm, int32_t n_fields, const void* const* send_host,
                         void* const* recv_host, const int64_t* rec_bytes_host,
                         const int64_t* send_counts_host, const int64_t* send_offsets_host,
                         const int64_t* recv_counts_host, const int64_t* recv_offsets_host,
                         int32_t skip_self, void* stream);
/* ncclCommAbort: releases every rank blocked on this communicator (a rank of
 * a one-process group failed); the communicator is unusable afterwards. */
int32_t pd_comm_abort(pd_comm* comm);
/* The check pd_comm_init / pd_comm_init_all run when n_ranks > 1 (unless
 * PD_COMM_SELF_CHECK=0): one all_to_all_v (uneven and zero-sized blocks) and
 * one all_gather_v with a known rank pattern, verified on the device;
 * PD_ERCCL on a mismatch.  Collective; callable at any n_ranks. */
int32_t pd_comm_self_check(pd_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* PARDIS_H */
