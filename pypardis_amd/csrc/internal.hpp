// Internal declarations shared by the libpardis translation units.
#pragma once

#include "common.hpp"

#include <map>
#include <vector>

namespace pd {

// Grow-only device scratch owned by a context (SURVEY.md §8(b) "Ownership":
// the ctx owns a reusable arena; no allocation crosses the ABI).
struct Arena {
    struct Buf {
        void* ptr = nullptr;
        size_t bytes = 0;
    };
    std::map<std::string, Buf> bufs;
    template <typename T>
    T* get(const std::string& name, size_t count) {
        size_t bytes = count * sizeof(T);
        if (bytes == 0) bytes = 16;
        Buf& b = bufs[name];
        if (b.bytes < bytes) {
            if (b.ptr) PD_HIP(hipFree(b.ptr));
            b.ptr = nullptr;
            size_t want = bytes + bytes / 8;   // headroom for slightly larger calls
            if (hipMalloc(&b.ptr, want) != hipSuccess) {
                (void)hipGetLastError();
                throw Error(-2, "device allocation of " + std::to_string(want) +
                                    " bytes failed for '" + name + "'");
            }
            b.bytes = want;
        }
        return static_cast<T*>(b.ptr);
    }
    void release() {
        for (auto& kv : bufs)
            if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        bufs.clear();
    }
};

struct Timings {
    // milliseconds of the last pd_train call, HIP events on the call's stream
    float halo = 0, sort = 0, gather = 0, cells = 0, count = 0, link = 0, merge = 0,
          roots = 0, border = 0, label = 0, total = 0;
    int64_t records = 0, cells_n = 0, grid_cells = 0, core_records = 0, key_bits = 0;
    int64_t halo_fallback = 0;   // single-pass halo overflowed its capacity: two passes ran
    // PD_OPT_SWEEP_STATS: count candidates; link candidates, predicate hits,
    // core hits, hits already under the root, finds that met the root, unions;
    // cell pairs tested record by record (link mode 3)
    int64_t sweep[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double grid_grow = 1.0;      // cell width / eps (PD_OPT_DIR_BUDGET)
    int64_t dir_words = 0;       // directory words allocated (paged: occupied + 1)
    int dir_paged = 0;           // the last train's directory layout
    float count_kernel = 0;      // dense path: the count pass's tile kernel alone (ms)
};

// Device state carried from phase A (local clustering) to phase B (border
// attach, keys).  The pointers are arena buffers; any other train call on the
// context invalidates it.
struct PhaseState {
    bool valid = false;
    uint32_t R = 0;
    uint64_t n = 0, G = 0;
    int P = 0, d = 0, dtype = 0, metric = 0, min_samples = 0, key_bits = 0;
    double eps = 0;
    float slo = -1.0f, shi = 0.0f;
    uint32_t ncells = 0;
    uint32_t n_exports = 0;
    uint32_t n_roots = 0;        // components on this device (single device: clusters)
    void* Xs = nullptr;
    void* parts = nullptr;
    uint32_t* part_start = nullptr;
    void* dir = nullptr;
    void* pages = nullptr;       // paged directory (null: flat)
    uint32_t* cstart = nullptr;
    uint32_t* vals = nullptr;
    uint8_t* core = nullptr;
    uint32_t* par = nullptr;
    uint32_t* gmin = nullptr;
    uint32_t* cnt_rec = nullptr;
    uint32_t* mn = nullptr;      // per record: the two smallest neighbours the count sweep saw
    uint32_t* exp_gid = nullptr;
    uint32_t* exp_key = nullptr;
};

// Dense path (d > 4, dense.hip) state carried between its stages: count ->
// link -> border -> finish.  Single device runs them back to back; the
// sharded dense train (pd_dense_*) runs each stage on every rank over its
// share of the tile rows, with a collective between stages.  Pointers are
// arena buffers (or the caller's X, which must stay alive until finish).
struct DenseState {
    int stage = 0;               // last stage run (0 none, 1 count, 2 link, 3 border)
    const void* X = nullptr;
    int dtype = 0, d = 0, metric = 0;
    uint32_t n = 0, min_samples = 1;
    double eps = 0;
    int rank = 0, world = 1;     // tile rows of chunk c belong to rank c % world
    // geometry (scaled bf16 split; see dense.hip)
    int KS = 1;
    bool mfma = false;
    double scale = 1.0;
    double* center = nullptr;
    float elo = 0, ehi = 0;
    uint32_t* cnt = nullptr;     // [n] neighbour counts, input order
    uint32_t n_core = 0, n_border = 0;
    uint32_t* clist = nullptr;   // core point ids, ascending
    uint32_t* par = nullptr;     // union-find over the core rows
    uint32_t* keyc = nullptr;    // cluster key per core row
    uint32_t* key_out = nullptr; // [n] cluster key per point
    uint32_t* blist = nullptr;   // border candidate ids, ascending
    uint32_t* best = nullptr;    // smallest adjacent core key per border candidate
    const void* cf[4] = {};      // core fragment set: hi, lo, norm, nmax
    unsigned long long* tiles = nullptr;
};

// Device-decided KD partition of a sharded train (pd_kdx_*, kd.hip): the
// level tables and decisions stay on the device between the per-level calls;
// the caller runs the collectives (all-gather of the moment partials,
// all-reduce of the counts) in between, stream-ordered, with no host sync.
struct KdxState {
    bool valid = false;
    int n_levels = 0, d = 0;
    std::vector<int> sizes, first, ntab;
    std::vector<int32_t> cur;
    std::vector<size_t> off, off_d;
    int total = 0;
    char* tables = nullptr;      // device: per level slot_of | axis | newlab | bounds | boundary
    double* trace = nullptr;     // device: 13 doubles per split
    double* bbox = nullptr;      // device: combined bbox (2d) + non-finite count
    double* mom = nullptr;       // device: combined moments of the current level
};

// Exchange state of a sharded train between pd_route2 and pd_pack2 (shard.hip).
struct RouteState {
    bool valid = false;
    int64_t n = 0;
    int n_ranks = 0;
    unsigned tiles = 0;
    uint64_t* mask = nullptr;    // device u64[n]: destination ranks of each point
    uint64_t* off = nullptr;     // device: dest-major exclusive scan of the per-tile counts
};

struct Ctx {
    int device = 0;
    Arena arena;
    void* pinned = nullptr;      // small pinned staging block for D2H scalars
    bool timing = false;
    bool full_counts = false;    // debug: count every neighbour (no early exit)
    bool seq_moments = false;    // reference-order (sequential) KD moment sums
    int xsub = 2;                // axis-0 sub-cells per eps
    int centre_window = -1;      // window union: records after each record tested (2..64);
                                 // < 0 (default): 2, 8 or 16 by records per occupied cell
    int count_rotate = 1024;     // count sweep: lists longer than this start near the query (0: off)
    int count_replay = 0;        // PD_OPT_COUNT_REPLAY: replicas of the count sweep to time (0: off)
    // the record sort's look-back words (rsort.hpp): zeroed when allocated,
    // then tagged with the pass epoch kept here
    uint64_t* rs_look = nullptr;
    uint64_t rs_look_tiles = 0;
    uint32_t rs_epoch = 0;
    // the single-pass halo's look-back words, ticket and total (zeroed when
    // allocated, then tagged / offset by the epoch and ticket base kept here)
    int halo_passes = 2;         // PD_OPT_HALO_PASSES: 2 tile counts + scan (default), 1 single
                                 // pass (look-back; measured slower on C2: halo 1.62 vs 1.31 ms)
    int64_t halo_cap = 0;        // PD_OPT_HALO_CAP: single-pass record capacity (0: n + n/8 + 4096)
    uint64_t* h1_look = nullptr;
    uint64_t h1_look_tiles = 0;
    unsigned long long* h1_tick = nullptr;
    unsigned long long h1_tick0 = 0;
    uint32_t h1_epoch = 0;
    double h1_ratio = 1.0;       // records per point of the last grid train (sizes the next cap)
    bool kd_fuse = false;        // PD_OPT_KD_FUSE: kd_build fuses counts + the children's moments
                                 // (measured slower on C2: outside the train 2.79-3.32 vs 2.61-2.96 ms)
    bool verify_fused = false;   // PD_OPT_VERIFY_FUSED: cell verify over every cell, screen inline
    bool halo_tree = false;      // PD_OPT_HALO_TREE: halo membership tests only near split planes
                                 // (measured slower: C2 halo 1.36 vs 1.19 ms, C4 11.3 vs 9.4 ms)
    bool kd_replay = false;      // PD_OPT_KD_REPLAY: KD passes replay the splits instead of labels
    bool screen = true;          // fp32 screening of fp32 inputs (exact either way)
    bool sweep_stats = false;    // tally sweep candidates / union-find outcomes
    int64_t dir_budget = 32ll << 30;   // eps-grid directory bytes before cells grow
    int dir_paged = -1;          // PD_OPT_DIR_PAGED: 1 paged, 0 flat, -1 paged when the grid has
                                 // more directory words than points
    int dense_prune = 1;         // dense count pass: projection-window tiles only (2: per-band runs)
    bool shard_core_bit = false; // PD_OPT_SHARD_CORE_BIT: sharded phase B keys carry the core flag
    int dense_screen = 1;        // dense count pass screen: 1 e4m3 (32x32x64), 0 bf16 hi.hi
    int label_buckets = -1;      // labels to input order by bucketed pair passes (PD_OPT_LABEL_BUCKETS;
                                 // -1: from 2^22 points on, where they beat the direct scatter;
                                 // 2: the round-4 L2-bucket scatter)
    Timings t;
    PhaseState st;
    DenseState dn;
    KdxState kdx;
    RouteState rt;
    hipEvent_t ev[16] = {};
};

struct TrainArgs {
    const void* X = nullptr;
    int dtype = 0;   // 0 fp32, 1 fp64
    int64_t n = 0;
    int d = 0;
    double eps = 0;
    int min_samples = 1;
    int metric = 0;  // 0 euclidean, 1 cityblock
    int P = 1;
    const double* ebox = nullptr;     // host, P x 2 x d (lo row then hi row)
    const double* data_box = nullptr; // host, 2 x d tight bbox (optional)
    const int32_t* owner = nullptr;   // device, KD label per point (nullable if P==1)
    int32_t* labels = nullptr;        // device out, n
    uint8_t* core = nullptr;          // device out, n (nullable)
    uint32_t* counts = nullptr;       // device out, n (nullable; owner-record counts)
    int64_t n_clusters = 0;           // out
    hipStream_t stream = nullptr;
    // sharded (multi-device) train: phase 1 = local clustering + exports,
    // phase 2 = key remap + border attach; phase 0 = both, single device
    int phase = 0;
    const uint32_t* gid = nullptr;    // device, global id per local point (null: identity)
    const uint8_t* xr = nullptr;      // device, point also lives on another device
    // device, phase 2: the merged exports (pd_merge_exports): ascending
    // distinct ids and each one's global key
    const uint32_t* map_ids = nullptr;
    const uint32_t* map_keys = nullptr;
    int64_t n_map = 0;
    uint32_t* keys_out = nullptr;     // device out, n: cluster key per owned point (phase 2)
    // pd_train_tree: the KD split tree instead of `owner` (host arrays, BFS
    // order: tree_sizes[l] splits at level l, cur -> new when v[axis] >= bound)
    int tree_levels = 0;
    const int32_t* tree_sizes = nullptr;
    const int32_t* tree_cur = nullptr;
    const int32_t* tree_axis = nullptr;
    const double* tree_bound = nullptr;
    const int32_t* tree_new = nullptr;
    int64_t n_exports = 0;            // out (phase 1)
    bool dir_paged = false;           // internal: directory layout of this train
};

void train(Ctx& ctx, TrainArgs& a);
// d > kMaxDim: dense distance tiles on the matrix cores (dense.hip)
void dense_train(Ctx& ctx, TrainArgs& a);
// sharded dense train (dense.hip): every rank holds all n points and runs
// each stage over its share of the tile rows (pd_dense_* in pardis.h)
void dense_count(Ctx& ctx, TrainArgs& a, int rank, int world, uint32_t* counts_out);
uint32_t dense_link(Ctx& ctx, const uint32_t* counts, uint32_t* forest_out, hipStream_t s);
uint32_t dense_border(Ctx& ctx, const uint32_t* forests, int n_forests, int32_t* best_out,
                      hipStream_t s);
int64_t dense_finish(Ctx& ctx, const int32_t* best, int32_t* labels, uint8_t* core,
                     uint32_t* counts, hipStream_t s);
// labels from cluster keys (engine.hip): async, then the cluster count (syncs)
// core_bit: keys carry the core flag in bit 30 (stripped; written to
// core_from_key when not null)
void rank_labels_async(Ctx& ctx, const uint32_t* key, uint64_t n, int32_t* labels, hipStream_t s,
                       int core_bit = 0, uint8_t* core_from_key = nullptr);
int64_t rank_labels_count(Ctx& ctx, hipStream_t s);

// KD partition stages (kd.hip)
void bbox(Ctx& ctx, const void* X, int dtype, int64_t n, int d, double* lohi_host,
          int64_t* nonfinite_host, hipStream_t s);
void kd_moments(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                int n_sel, const int32_t* sel_host, double* out_host, hipStream_t s);
void kd_counts(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
               int n_sel, const int32_t* sel_host, const int32_t* axis_host,
               const double* bounds_host, int64_t* out_host, hipStream_t s);
void kd_split(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
              int n_sel, const int32_t* sel_host, const int32_t* axis_host,
              const double* boundary_host, const int32_t* new_host, hipStream_t s);
void kd_radix_hist(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                   int n_sel, const int32_t* sel_host, const int32_t* axis_host,
                   const uint64_t* prefix_host, int shift, int64_t* hist_host, hipStream_t s);
// One fused streaming pass of a BFS level (kd.hip): apply the splits of the
// previous level (n_split > 0), then the double-double moment partials of the
// labels `sel` (out_dd: n_sel x (1 + 4d)), and on the first level (labels all
// zero, lohi != null) the bbox + non-finite count.
void kd_pass(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
             bool labels_zero, int n_split, const int32_t* ssel, const int32_t* saxis,
             const double* sbound, const int32_t* snew, int n_sel, const int32_t* sel,
             double* out_dd, double* lohi, int64_t* bad, hipStream_t s);
// The whole min_var BFS (exact sums) in one launch chain, the level
// decisions on the device; trace: 13 doubles per split (kd.hip kd_build).
void kd_build(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels, int n_levels,
              const int32_t* sizes, const int32_t* cur, const int32_t* newl, int final_mode,
              double* trace_out, double* lohi, int64_t* bad, hipStream_t s);
// The KD labels of every point by replaying a finished BFS split tree
// (host arrays: tree_sizes[l] splits at level l, cur -> new when v[axis] >=
// bound) — pd_kd_labels, for a pd_kd_build run in final mode 2.
void kd_labels(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
               int n_levels, const int32_t* sizes, const int32_t* cur, const int32_t* axis,
               const double* bound, const int32_t* newl, hipStream_t s);
void kd_moments_dd(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                   int n_sel, const int32_t* sel_host, double* out_host, hipStream_t s);
// Sharded device-decided KD (kd.hip): begin -> per level (moments -> [caller:
// all-gather] -> axes -> counts -> [caller: all-reduce] -> boundary) -> end.
void kdx_begin(Ctx& ctx, int d, int n_levels, const int32_t* sizes, const int32_t* cur,
               const int32_t* newl, hipStream_t s);
void kdx_moments(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels, int level,
                 double* out, hipStream_t s);
void kdx_axes(Ctx& ctx, const double* gathered, int n_ranks, int level, hipStream_t s);
void kdx_counts(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* labels,
                int level, unsigned long long* out, hipStream_t s);
void kdx_boundary(Ctx& ctx, const unsigned long long* cnt, int level, hipStream_t s);
void kdx_end(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int32_t* labels,
             bool final_split, double* trace_out, double* lohi, int64_t* bad, hipStream_t s);
// Sharded exchange (shard.hip): one ordered pass per side, every destination.
void route2(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P, const double* ebox_host,
            const int32_t* part_rank_host, const int32_t* kdlab, int n_ranks, int64_t* counts_host,
            hipStream_t s);
void pack2(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const int32_t* kdlab, int P,
           const int32_t* part_rank_host, const int32_t* local_index_host, uint32_t gid_base,
           int n_ranks, void* const* coords, uint32_t* const* gid, int32_t* const* owner,
           uint8_t* const* xr, hipStream_t s);
void results(Ctx& ctx, int64_t nr, const uint32_t* keys, const uint8_t* core, const int32_t* owner,
             const uint32_t* gid, const uint32_t* roots, int64_t n_roots, int64_t n_total,
             uint32_t gid_base, int64_t n_local, int n_ranks, int me, const int64_t* src_off_host,
             int64_t expect_remote, int32_t* labels, uint8_t* core_out, uint32_t* pairs,
             hipStream_t s);
void results_scatter(Ctx& ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base, int64_t n,
                     int32_t* labels, uint8_t* core, hipStream_t s);
void route(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P, const double* ebox_host,
           const int32_t* part_rank_host, int n_ranks, uint64_t* mask, int64_t* counts_host,
           hipStream_t s);
int64_t pack(Ctx& ctx, const void* X, int dtype, int64_t n, int d, const uint64_t* mask, int dest,
             const int32_t* kdlab, int P, const int32_t* part_rank_host,
             const int32_t* local_index_host, uint32_t gid_base, void* coords_out,
             uint32_t* gid_out, int32_t* owner_out, uint8_t* xr_out, int64_t cap, hipStream_t s);
void train_exports(Ctx& ctx, uint32_t* gid_out, uint32_t* key_out, int64_t cap, hipStream_t s);
int64_t merge_exports(Ctx& ctx, const uint32_t* gid, const uint32_t* key, int64_t m,
                      uint32_t* ids_out, uint32_t* keys_out, hipStream_t s);
int64_t select_roots(Ctx& ctx, const uint32_t* keys, const uint32_t* gid, int64_t n, uint32_t* out,
                     hipStream_t s);
void sort_u32(Ctx& ctx, uint32_t* data, int64_t n, hipStream_t s);
void rank_labels(Ctx& ctx, const uint32_t* keys, int64_t n, const uint32_t* roots, int64_t nr,
                 int32_t* labels, hipStream_t s);
int64_t owned_results(Ctx& ctx, int64_t n, const int32_t* owner, const uint32_t* gid,
                      const int32_t* labels, const uint8_t* core, int n_ranks,
                      const int64_t* gid_offsets_host, uint32_t* out, int64_t cap,
                      int64_t* counts_host, hipStream_t s);
void scatter_results(Ctx& ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base, int64_t n,
                     int32_t* labels, uint8_t* core, hipStream_t s);

// RCCL communicator (comm.hip): one rank of a device group
struct Comm;
Comm* comm_init(int device, int n_ranks, int rank, const uint8_t* id);
void comm_init_all(int n, const int32_t* devices, Comm** out);
void comm_destroy(Comm* c);
void comm_unique_id(uint8_t* id);
int comm_device(const Comm* c);
void comm_size(const Comm* c, int* n_ranks, int* rank);
void comm_all_reduce(Comm* c, const void* send, void* recv, int64_t count, int elem, int op,
                     hipStream_t s);
void comm_all_gather_v(Comm* c, const void* send, void* recv, const int64_t* counts, int elem,
                       hipStream_t s);
void comm_all_to_all_v(Comm* c, const void* send, const int64_t* send_counts, void* recv,
                       const int64_t* recv_counts, int elem, hipStream_t s);
void comm_broadcast(Comm* c, void* buf, int64_t count, int elem, int root, hipStream_t s);
// Field-wise all-to-all in ONE group (blocks in records; rec_bytes per field);
// skip_self: the self blocks are already in place in recv.
void comm_exchange(Comm* c, int nf, const void* const* send, void* const* recv,
                   const int64_t* rec_bytes, const int64_t* send_counts, const int64_t* send_off,
                   const int64_t* recv_counts, const int64_t* recv_off, bool skip_self,
                   hipStream_t s);
void comm_abort(Comm* c);
// W > 1: one all_to_all_v and one all_gather_v with a known rank pattern,
// verified on the device (throws on a mismatch); comms: every rank of one
// process (init_all) or just this rank's.
void comm_self_check(Comm* const* comms, int n);
void halo_members(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P,
                  const double* ebox_host, int64_t* counts_host, int64_t* members_dev,
                  int64_t members_cap, hipStream_t s);

// small helpers (api.hip)
void sort_pairs_inplace(Ctx& ctx, void* keys, int key_bytes, uint32_t* vals, uint64_t n,
                        int key_bits, hipStream_t s);
void* pinned(Ctx& ctx, size_t bytes);
void sync(hipStream_t s);

}  // namespace pd
