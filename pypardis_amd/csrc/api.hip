// C ABI (include/pardis.h): argument checks, error translation, contexts.
#include "../../include/pardis.h"

#include <cstring>
#include <string>
#include <vector>

#include "internal.hpp"

struct pd_ctx {
    pd::Ctx c;
};

namespace pd {

static thread_local std::string g_err;
void* pinned(Ctx& ctx, size_t bytes) {
    // One grow-only pinned block per context.  Callers never keep two views
    // alive across a stream synchronisation (see kd.hip / engine.hip); a grow
    // first drains the device so no async copy still reads the old block.
    struct Hdr {
        size_t bytes;
    };
    Hdr* h = (Hdr*)ctx.pinned;
    if (!h || h->bytes < bytes) {
        if (h) {
            PD_HIP(hipDeviceSynchronize());
            PD_HIP(hipHostFree(h));
            ctx.pinned = nullptr;
        }
        size_t want = std::max<size_t>(bytes + 64, 1 << 20);
        void* p = nullptr;
        PD_HIP(hipHostMalloc(&p, want + 64, hipHostMallocDefault));
        ctx.pinned = p;
        h = (Hdr*)p;
        h->bytes = want;
    }
    return (char*)h + 64;
}

void sync(hipStream_t s) { PD_HIP(hipStreamSynchronize(s)); }

template <typename F>
static int32_t guard(pd_ctx* ctx, F&& f) {
    try {
        if (ctx) PD_HIP(hipSetDevice(ctx->c.device));
        f();
        return PD_OK;
    } catch (const Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return PD_EINVAL;
    } catch (...) {
        g_err = "unknown error";
        return PD_EINVAL;
    }
}

static void check_common(pd_ctx* ctx, const void* X, int64_t n, int32_t d) {
    if (!ctx) throw Error(PD_EINVAL, "null context");
    if (n < 0) throw Error(PD_EINVAL, "n < 0");
    if (d < 1) throw Error(PD_EINVAL, "d < 1");
    if (n > 0 && !X) throw Error(PD_EINVAL, "null X");
}

}  // namespace pd

struct pd_comm {
    pd::Comm* c;
};

namespace pd {
template <typename F>
static int32_t comm_guard(pd_comm* comm, F&& f) {
    try {
        if (!comm || !comm->c) throw Error(PD_EINVAL, "null communicator");
        PD_HIP(hipSetDevice(comm_device(comm->c)));
        f();
        return PD_OK;
    } catch (const Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return PD_EINVAL;
    } catch (...) {
        g_err = "unknown error";
        return PD_EINVAL;
    }
}
}  // namespace pd

using namespace pd;

extern "C" {

int32_t pd_abi_version(void) { return PD_ABI_VERSION; }

const char* pd_last_error(void) { return g_err.c_str(); }

int32_t pd_ctx_create(int32_t device, pd_ctx** out) {
    return guard(nullptr, [&] {
        if (!out) throw Error(PD_EINVAL, "null out");
        int ndev = 0;
        PD_HIP(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev)
            throw Error(PD_EINVAL, "device " + std::to_string(device) + " not present (" +
                                       std::to_string(ndev) + " visible)");
        PD_HIP(hipSetDevice(device));
        pd_ctx* c = new pd_ctx();
        c->c.device = device;
        *out = c;
    });
}

int32_t pd_ctx_destroy(pd_ctx* ctx) {
    if (!ctx) return PD_OK;
    int32_t rc = guard(ctx, [&] {
        ctx->c.arena.release();
        if (ctx->c.pinned) (void)hipHostFree(ctx->c.pinned);
        for (auto& e : ctx->c.ev)
            if (e) (void)hipEventDestroy(e);
    });
    delete ctx;
    return rc;
}

int32_t pd_ctx_set_option(pd_ctx* ctx, int32_t option, int64_t value) {
    return guard(ctx, [&] {
        if (!ctx) throw Error(PD_EINVAL, "null context");
        if (option == PD_OPT_TIMING)
            ctx->c.timing = value != 0;
        else if (option == PD_OPT_FULL_COUNTS)
            ctx->c.full_counts = value != 0;
        else if (option == PD_OPT_SEQUENTIAL_MOMENTS)
            ctx->c.seq_moments = value != 0;
        else if (option == PD_OPT_FP32_SCREEN)
            ctx->c.screen = value != 0;
        else if (option == PD_OPT_SWEEP_STATS)
            ctx->c.sweep_stats = value != 0;
        else if (option == PD_OPT_DENSE_PRUNE) {
            if (value < 0 || value > 2) throw Error(PD_EINVAL, "dense prune is 0, 1 or 2");
            ctx->c.dense_prune = (int)value;
        } else if (option == PD_OPT_COUNT_ROTATE) {
            if (value < 0 || value > 0x7FFFFFFF) throw Error(PD_EINVAL, "count rotate must be >= 0");
            ctx->c.count_rotate = (int)value;
        } else if (option == PD_OPT_CENTRE_WINDOW) {
            if (value > 0x7FFFFFFF) throw Error(PD_EINVAL, "centre window too large");
            ctx->c.centre_window = value < 0 ? -1 : (int)value;   // < 0: automatic
        } else if (option == PD_OPT_DIR_BUDGET) {
            if (value < 16) throw Error(PD_EINVAL, "directory budget must be >= 16 bytes");
            ctx->c.dir_budget = value;
        } else if (option == PD_OPT_XSUB) {
            if (value < 1 || value > 16) throw Error(PD_EINVAL, "xsub must be in [1, 16]");
            ctx->c.xsub = (int)value;
        } else if (option == PD_OPT_LABEL_BUCKETS) {
            ctx->c.label_buckets = value < 0 ? -1 : (value == 2 ? 2 : (value ? 1 : 0));
        } else if (option == PD_OPT_DIR_PAGED) {
            ctx->c.dir_paged = value < 0 ? -1 : (value ? 1 : 0);
        } else if (option == PD_OPT_DENSE_SCREEN) {
            if (value < 0 || value > 1) throw Error(PD_EINVAL, "dense screen is 0 or 1");
            ctx->c.dense_screen = (int)value;
        } else if (option == PD_OPT_SHARD_CORE_BIT) {
            ctx->c.shard_core_bit = value != 0;
        } else if (option == PD_OPT_HALO_PASSES) {
            if (value != 1 && value != 2) throw Error(PD_EINVAL, "halo passes is 1 or 2");
            ctx->c.halo_passes = (int)value;
        } else if (option == PD_OPT_KD_REPLAY) {
            ctx->c.kd_replay = value != 0;
        } else if (option == PD_OPT_HALO_TREE) {
            ctx->c.halo_tree = value != 0;
        } else if (option == PD_OPT_VERIFY_FUSED) {
            ctx->c.verify_fused = value != 0;
        } else if (option == PD_OPT_KD_FUSE) {
            ctx->c.kd_fuse = value != 0;
        } else if (option == PD_OPT_HALO_CAP) {
            if (value < 0) throw Error(PD_EINVAL, "halo capacity must be >= 0");
            ctx->c.halo_cap = value;
        } else if (option == PD_OPT_COUNT_REPLAY) {
            if (value < 0 || value > 65536) throw Error(PD_EINVAL, "count replay must be in [0, 65536]");
            ctx->c.count_replay = (int)value;
        } else if (option == 4 || option == 5 || option == 9 || option == 10 || option == 16 ||
                   (option >= 20 && option <= 23)) {
            // retired tuning knobs (round 5): measured A/Bs whose losing
            // kernels were removed; pardis.h lists them
            throw Error(PD_EINVAL, "option " + std::to_string(option) +
                                       " was retired (see pardis.h, pd_option)");
        } else
            throw Error(PD_EINVAL, "unknown option");
    });
}

int32_t pd_ctx_timings(pd_ctx* ctx, double* out, int32_t n) {
    return guard(ctx, [&] {
        if (!ctx || !out) throw Error(PD_EINVAL, "null argument");
        const Timings& t = ctx->c.t;
        const double v[PD_T_NSLOTS] = {t.halo,    t.sort,   t.gather, t.cells,
                                       t.count,   t.link,   t.merge,  t.roots,  t.border,
                                       t.label,   t.total,  (double)t.records,
                                       (double)t.cells_n, (double)t.grid_cells,
                                       (double)t.key_bits, (double)t.core_records,
                                       (double)t.sweep[0], (double)t.sweep[1],
                                       (double)t.sweep[2], (double)t.sweep[3],
                                       (double)t.sweep[4], (double)t.sweep[5],
                                       (double)t.sweep[6], (double)t.sweep[7], t.grid_grow,
                                       (double)t.count_kernel, (double)t.dir_paged,
                                       (double)t.dir_words, (double)t.sweep[8],
                                       (double)t.sweep[9], (double)t.halo_fallback};
        for (int i = 0; i < n && i < PD_T_NSLOTS; ++i) out[i] = v[i];
    });
}

int32_t pd_bbox(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double* lohi,
                int64_t* bad, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!lohi) throw Error(PD_EINVAL, "null lohi");
        if (n == 0) throw Error(PD_EINVAL, "bbox of an empty set");
        bbox(ctx->c, X, dtype, n, d, lohi, bad, (hipStream_t)stream);
    });
}

int32_t pd_kd_moments(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                      const int32_t* labels, int32_t n_sel, const int32_t* sel, double* out,
                      void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_sel < 0 || (n_sel && (!sel || !out)) || (n && !labels))
            throw Error(PD_EINVAL, "bad selection");
        if (n == 0) {
            std::memset(out, 0, sizeof(double) * 3 * d * n_sel);
            return;
        }
        kd_moments(ctx->c, X, dtype, n, d, labels, n_sel, sel, out, (hipStream_t)stream);
    });
}

int32_t pd_kd_counts(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                     const int32_t* labels, int32_t n_sel, const int32_t* sel,
                     const int32_t* axis, const double* bounds, int64_t* out, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_sel < 0 || (n_sel && (!sel || !axis || !bounds || !out)) || (n && !labels))
            throw Error(PD_EINVAL, "bad selection");
        for (int s = 0; s < n_sel; ++s)
            if (axis[s] < 0 || axis[s] >= d || sel[s] < 0) throw Error(PD_EINVAL, "bad axis/label");
        if (n == 0) {
            std::memset(out, 0, sizeof(int64_t) * 8 * n_sel);
            return;
        }
        kd_counts(ctx->c, X, dtype, n, d, labels, n_sel, sel, axis, bounds, out,
                  (hipStream_t)stream);
    });
}

int32_t pd_kd_split(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                    int32_t* labels, int32_t n_sel, const int32_t* sel, const int32_t* axis,
                    const double* boundary, const int32_t* newlab, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_sel < 0 || (n_sel && (!sel || !axis || !boundary || !newlab)) || (n && !labels))
            throw Error(PD_EINVAL, "bad selection");
        for (int s = 0; s < n_sel; ++s)
            if (axis[s] < 0 || axis[s] >= d || sel[s] < 0) throw Error(PD_EINVAL, "bad axis/label");
        if (n == 0) return;
        kd_split(ctx->c, X, dtype, n, d, labels, n_sel, sel, axis, boundary, newlab,
                 (hipStream_t)stream);
    });
}

int32_t pd_kd_radix_hist(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                         const int32_t* labels, int32_t n_sel, const int32_t* sel,
                         const int32_t* axis, const uint64_t* prefix, int32_t shift,
                         int64_t* hist, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_sel < 0 || (n_sel && (!sel || !axis || !prefix || !hist)) || (n && !labels))
            throw Error(PD_EINVAL, "bad selection");
        if (shift < 0 || shift > 56 || shift % 8) throw Error(PD_EINVAL, "shift must be 0, 8, .., 56");
        for (int s = 0; s < n_sel; ++s)
            if (axis[s] < 0 || axis[s] >= d || sel[s] < 0) throw Error(PD_EINVAL, "bad axis/label");
        if (n == 0) {
            std::memset(hist, 0, sizeof(int64_t) * 256 * n_sel);
            return;
        }
        kd_radix_hist(ctx->c, X, dtype, n, d, labels, n_sel, sel, axis, prefix, shift, hist,
                      (hipStream_t)stream);
    });
}

int32_t pd_sort_pairs(pd_ctx* ctx, void* keys, int32_t key_bytes, uint32_t* vals, int64_t n,
                      int32_t key_bits, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || n < 0 || (n && (!keys || !vals))) throw Error(PD_EINVAL, "bad arrays");
        if (key_bytes != 4 && key_bytes != 8) throw Error(PD_EINVAL, "key_bytes must be 4 or 8");
        if (key_bits < 1 || key_bits > 8 * key_bytes) throw Error(PD_EINVAL, "bad key_bits");
        if (n >= 0xFFFFFFFFll) throw Error(PD_EINVAL, "n >= 2^32 - 1");
        sort_pairs_inplace(ctx->c, keys, key_bytes, vals, (uint64_t)n, key_bits,
                           (hipStream_t)stream);
    });
}

int32_t pd_halo_members(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                        int32_t P, const double* ebox, int64_t* counts, int64_t* members,
                        int64_t capacity, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (P < 1 || !ebox || !counts) throw Error(PD_EINVAL, "bad boxes");
        if (n == 0) {
            std::memset(counts, 0, sizeof(int64_t) * P);
            return;
        }
        halo_members(ctx->c, X, dtype, n, d, P, ebox, counts, members, capacity,
                     (hipStream_t)stream);
    });
}

int32_t pd_train(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                 int32_t min_samples, int32_t metric, int32_t P, const double* ebox,
                 const double* data_box, const int32_t* owner, int32_t* labels, uint8_t* core,
                 uint32_t* counts, int64_t* n_clusters, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!ebox) throw Error(PD_EINVAL, "null ebox");
        if (P > 1 && n > 0 && !owner) throw Error(PD_EINVAL, "owner labels required for P > 1");
        TrainArgs a;
        a.X = X;
        a.dtype = dtype;
        a.n = n;
        a.d = d;
        a.eps = eps;
        a.min_samples = min_samples;
        a.metric = metric;
        a.P = P;
        a.ebox = ebox;
        a.data_box = data_box;
        a.owner = owner;
        a.labels = labels;
        a.core = core;
        a.counts = counts;
        a.stream = (hipStream_t)stream;
        train(ctx->c, a);
        if (n_clusters) *n_clusters = a.n_clusters;
    });
}

int32_t pd_train_tree(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                      int32_t min_samples, int32_t metric, int32_t P, const double* ebox,
                      const double* data_box, int32_t n_levels, const int32_t* level_sizes,
                      const int32_t* cur, const int32_t* axis, const double* boundary,
                      const int32_t* newlab, int32_t* labels, uint8_t* core, uint32_t* counts,
                      int64_t* n_clusters, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!ebox) throw Error(PD_EINVAL, "null ebox");
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "pd_train_tree: d > 4 (use pd_train)");
        if (n_levels < 0 || n_levels > 16 ||
            (n_levels && (!level_sizes || !cur || !axis || !boundary || !newlab)))
            throw Error(PD_EINVAL, "bad split tree");
        if (P > 1 && n_levels == 0) throw Error(PD_EINVAL, "P > 1 needs the split tree");
        TrainArgs a;
        a.X = X;
        a.dtype = dtype;
        a.n = n;
        a.d = d;
        a.eps = eps;
        a.min_samples = min_samples;
        a.metric = metric;
        a.P = P;
        a.ebox = ebox;
        a.data_box = data_box;
        a.tree_levels = n_levels;
        a.tree_sizes = level_sizes;
        a.tree_cur = cur;
        a.tree_axis = axis;
        a.tree_bound = boundary;
        a.tree_new = newlab;
        a.labels = labels;
        a.core = core;
        a.counts = counts;
        a.stream = (hipStream_t)stream;
        train(ctx->c, a);
        if (n_clusters) *n_clusters = a.n_clusters;
    });
}

int32_t pd_cluster(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                   int32_t min_samples, int32_t metric, int32_t* labels, uint8_t* core,
                   uint32_t* counts, int64_t* n_clusters, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        TrainArgs a;
        a.X = X;
        a.dtype = dtype;
        a.n = n;
        a.d = d;
        a.eps = eps;
        a.min_samples = min_samples;
        a.metric = metric;
        a.P = 1;
        a.labels = labels;
        a.core = core;
        a.counts = counts;
        a.stream = (hipStream_t)stream;
        std::vector<double> box(2 * (size_t)d, 0.0);
        if (n > 0) {
            int64_t bad = 0;
            bbox(ctx->c, X, dtype, n, d, box.data(), &bad, a.stream);
            if (bad) throw Error(PD_EINVAL, "input contains NaN or infinity");
        }
        a.ebox = box.data();
        a.data_box = box.data();
        train(ctx->c, a);
        if (n_clusters) *n_clusters = a.n_clusters;
    });
}

// ---------------------------------------------------------------- sharded train

int32_t pd_kd_moments_dd(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                         const int32_t* labels, int32_t n_sel, const int32_t* sel, double* out,
                         void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_sel < 0 || (n_sel && (!sel || !out)) || (n && !labels))
            throw Error(PD_EINVAL, "bad selection");
        if (n == 0) {
            std::memset(out, 0, sizeof(double) * (1 + 4 * d) * n_sel);
            return;
        }
        kd_moments_dd(ctx->c, X, dtype, n, d, labels, n_sel, sel, out, (hipStream_t)stream);
    });
}

int32_t pd_kd_pass(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                   int32_t* labels, int32_t labels_zero, int32_t n_split, const int32_t* ssel,
                   const int32_t* saxis, const double* sbound, const int32_t* snew, int32_t n_sel,
                   const int32_t* sel, double* out, double* lohi, int64_t* bad, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n_split < 0 || n_sel < 0) throw Error(PD_EINVAL, "bad selection");
        if (n_split && (!ssel || !saxis || !sbound || !snew)) throw Error(PD_EINVAL, "null split table");
        if (n_sel && (!sel || !out)) throw Error(PD_EINVAL, "null selection");
        if (n && !labels) throw Error(PD_EINVAL, "null labels");
        for (int s = 0; s < n_split; ++s)
            if (saxis[s] < 0 || saxis[s] >= d || ssel[s] < 0) throw Error(PD_EINVAL, "bad axis/label");
        if (lohi && (!labels_zero || n_split || n_sel != 1))
            throw Error(PD_EINVAL, "the bbox is fused into the first level only (one label, no split)");
        if (n == 0) {
            if (n_sel) std::memset(out, 0, sizeof(double) * (1 + 4 * d) * n_sel);
            if (lohi) throw Error(PD_EINVAL, "bbox of an empty set");
            return;
        }
        kd_pass(ctx->c, X, dtype, n, d, labels, labels_zero != 0, n_split, ssel, saxis, sbound, snew,
                n_sel, sel, out, lohi, bad, (hipStream_t)stream);
    });
}

int32_t pd_route(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t P,
                 const double* ebox, const int32_t* part_rank, int32_t n_ranks, uint64_t* mask,
                 int64_t* counts, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "d > 4");
        if (!ebox || !part_rank || !counts || (n && !mask)) throw Error(PD_EINVAL, "null argument");
        route(ctx->c, X, dtype, n, d, P, ebox, part_rank, n_ranks, mask, counts,
              (hipStream_t)stream);
    });
}

int32_t pd_pack(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                const uint64_t* mask, int32_t dest, const int32_t* kdlab, int32_t P,
                const int32_t* part_rank, const int32_t* local_index, uint32_t gid_base,
                void* coords, uint32_t* gid, int32_t* owner, uint8_t* xr, int64_t capacity,
                int64_t* m, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "d > 4");
        if (P < 1 || !part_rank || !local_index || !m) throw Error(PD_EINVAL, "null argument");
        if (n && (!mask || !kdlab)) throw Error(PD_EINVAL, "null argument");
        if (capacity > 0 && (!coords || !gid || !owner || !xr))
            throw Error(PD_EINVAL, "null output buffer");
        *m = pack(ctx->c, X, dtype, n, d, mask, dest, kdlab, P, part_rank, local_index, gid_base,
                  coords, gid, owner, xr, capacity, (hipStream_t)stream);
    });
}

int32_t pd_train_begin(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                       double eps, int32_t min_samples, int32_t metric, int32_t P,
                       const double* ebox, const double* data_box, const int32_t* owner,
                       const uint32_t* gid, const uint8_t* xr, int64_t* n_exports, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!ebox) throw Error(PD_EINVAL, "null ebox");
        // gid null: identity (one rank); xr null: no point lives on another rank
        if (n > 0 && !owner) throw Error(PD_EINVAL, "owner required");
        TrainArgs a;
        a.X = X;
        a.dtype = dtype;
        a.n = n;
        a.d = d;
        a.eps = eps;
        a.min_samples = min_samples;
        a.metric = metric;
        a.P = P;
        a.ebox = ebox;
        a.data_box = data_box;
        a.owner = owner;
        a.gid = gid;
        a.xr = xr;
        a.phase = 1;
        a.stream = (hipStream_t)stream;
        train(ctx->c, a);
        if (n_exports) *n_exports = a.n_exports;
    });
}

int32_t pd_train_exports(pd_ctx* ctx, uint32_t* gid, uint32_t* key, int64_t capacity,
                         void* stream) {
    return guard(ctx, [&] {
        if (!ctx) throw Error(PD_EINVAL, "null context");
        if (capacity > 0 && (!gid || !key)) throw Error(PD_EINVAL, "null output buffer");
        train_exports(ctx->c, gid, key, capacity, (hipStream_t)stream);
    });
}

int32_t pd_merge_exports(pd_ctx* ctx, const uint32_t* gid, const uint32_t* key, int64_t m,
                         uint32_t* ids, uint32_t* keys, int64_t* u, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !u) throw Error(PD_EINVAL, "null argument");
        if (m < 0 || (m && (!gid || !key || !ids || !keys))) throw Error(PD_EINVAL, "null argument");
        *u = merge_exports(ctx->c, gid, key, m, ids, keys, (hipStream_t)stream);
    });
}

int32_t pd_train_end(pd_ctx* ctx, int64_t n, const uint32_t* map_ids, const uint32_t* map_keys,
                     int64_t n_map, uint32_t* keys, uint8_t* core, void* stream) {
    return guard(ctx, [&] {
        if (!ctx) throw Error(PD_EINVAL, "null context");
        if (n_map < 0 || n_map > (int64_t)0xFFFFFFFE || (n_map && (!map_ids || !map_keys)))
            throw Error(PD_EINVAL, "bad key map");
        TrainArgs a;
        a.n = n;
        a.map_ids = map_ids;
        a.map_keys = map_keys;
        a.n_map = n_map;
        a.keys_out = keys;
        a.core = core;
        a.phase = 2;
        a.stream = (hipStream_t)stream;
        train(ctx->c, a);
    });
}

int32_t pd_select_roots(pd_ctx* ctx, const uint32_t* keys, const uint32_t* gid, int64_t n,
                        uint32_t* roots, int64_t* m, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !m || n < 0 || (n && (!keys || !roots))) throw Error(PD_EINVAL, "bad argument");
        *m = select_roots(ctx->c, keys, gid, n, roots, (hipStream_t)stream);
    });
}

int32_t pd_sort_u32(pd_ctx* ctx, uint32_t* data, int64_t n, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || n < 0 || (n && !data)) throw Error(PD_EINVAL, "bad argument");
        sort_u32(ctx->c, data, n, (hipStream_t)stream);
    });
}

int32_t pd_rank_labels(pd_ctx* ctx, const uint32_t* keys, int64_t n, const uint32_t* roots,
                       int64_t n_roots, int32_t* labels, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || n < 0 || n_roots < 0 || (n && (!keys || !labels)) || (n_roots && !roots))
            throw Error(PD_EINVAL, "bad argument");
        rank_labels(ctx->c, keys, n, roots, n_roots, labels, (hipStream_t)stream);
    });
}

int32_t pd_owned_results(pd_ctx* ctx, int64_t n, const int32_t* owner, const uint32_t* gid,
                         const int32_t* labels, const uint8_t* core, int32_t n_ranks,
                         const int64_t* gid_offsets, uint32_t* out, int64_t capacity,
                         int64_t* counts, int64_t* m, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !gid_offsets || !counts || !m || n < 0) throw Error(PD_EINVAL, "bad argument");
        if (n && (!owner || !gid || !labels)) throw Error(PD_EINVAL, "null argument");
        if (capacity > 0 && !out) throw Error(PD_EINVAL, "null output buffer");
        *m = owned_results(ctx->c, n, owner, gid, labels, core, n_ranks, gid_offsets, out, capacity,
                           counts, (hipStream_t)stream);
    });
}

int32_t pd_scatter_results(pd_ctx* ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base,
                           int64_t n, int32_t* labels, uint8_t* core, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || m < 0 || n < 0 || (m && !pairs) || (n && !labels))
            throw Error(PD_EINVAL, "bad argument");
        scatter_results(ctx->c, pairs, m, gid_base, n, labels, core, (hipStream_t)stream);
    });
}

int32_t pd_kd_build(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t* labels,
                    int32_t n_levels, const int32_t* sizes, const int32_t* cur, const int32_t* newlab,
                    int32_t final_split, double* trace, double* lohi, int64_t* bad, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n == 0) throw Error(PD_EINVAL, "kd_build of an empty set");
        if (!labels || n_levels < 1 || !sizes || !cur || !newlab || !trace || !lohi)
            throw Error(PD_EINVAL, "null argument");
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "kd_build: d > 4");
        if (final_split < 0 || final_split > 2) throw Error(PD_EINVAL, "final_split is 0, 1 or 2");
        kd_build(ctx->c, X, dtype, n, d, labels, n_levels, sizes, cur, newlab, final_split,
                 trace, lohi, bad, (hipStream_t)stream);
    });
}

int32_t pd_kd_labels(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                     int32_t* labels, int32_t n_levels, const int32_t* sizes, const int32_t* cur,
                     const int32_t* axis, const double* boundary, const int32_t* newlab,
                     void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (n && !labels) throw Error(PD_EINVAL, "null labels");
        if (n_levels < 0 || n_levels > 16 || (n_levels && (!sizes || !cur || !axis || !boundary || !newlab)))
            throw Error(PD_EINVAL, "bad split tree");
        if (n == 0) return;
        kd_labels(ctx->c, X, dtype, n, d, labels, n_levels, sizes, cur, axis, boundary, newlab,
                  (hipStream_t)stream);
    });
}

// ---------------------------------------------------------------- sharded device-decided KD
int32_t pd_kdx_begin(pd_ctx* ctx, int32_t d, int32_t n_levels, const int32_t* sizes,
                     const int32_t* cur, const int32_t* newlab, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !sizes || !cur || !newlab) throw Error(PD_EINVAL, "null argument");
        kdx_begin(ctx->c, d, n_levels, sizes, cur, newlab, (hipStream_t)stream);
    });
}

int32_t pd_kdx_moments(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                       int32_t* labels, int32_t level, double* out, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!out || (n && !labels)) throw Error(PD_EINVAL, "null argument");
        kdx_moments(ctx->c, X, dtype, n, d, labels, level, out, (hipStream_t)stream);
    });
}

int32_t pd_kdx_axes(pd_ctx* ctx, const double* gathered, int32_t n_ranks, int32_t level,
                    void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !gathered) throw Error(PD_EINVAL, "null argument");
        kdx_axes(ctx->c, gathered, n_ranks, level, (hipStream_t)stream);
    });
}

int32_t pd_kdx_counts(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                      const int32_t* labels, int32_t level, uint64_t* out, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!out || (n && !labels)) throw Error(PD_EINVAL, "null argument");
        kdx_counts(ctx->c, X, dtype, n, d, labels, level, (unsigned long long*)out,
                   (hipStream_t)stream);
    });
}

int32_t pd_kdx_boundary(pd_ctx* ctx, const uint64_t* counts, int32_t level, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !counts) throw Error(PD_EINVAL, "null argument");
        kdx_boundary(ctx->c, (const unsigned long long*)counts, level, (hipStream_t)stream);
    });
}

int32_t pd_kdx_end(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t* labels,
                   int32_t final_split, double* trace, double* lohi, int64_t* bad, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (!trace || !lohi || (n && !labels)) throw Error(PD_EINVAL, "null argument");
        kdx_end(ctx->c, X, dtype, n, d, labels, final_split != 0, trace, lohi, bad,
                (hipStream_t)stream);
    });
}

// ---------------------------------------------------------------- one-pass exchange, results
int32_t pd_route2(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, int32_t P,
                  const double* ebox, const int32_t* part_rank, const int32_t* kdlab,
                  int32_t n_ranks, int64_t* counts, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "d > 4");
        if (!ebox || !part_rank || !counts || (n && !kdlab)) throw Error(PD_EINVAL, "null argument");
        route2(ctx->c, X, dtype, n, d, P, ebox, part_rank, kdlab, n_ranks, counts,
               (hipStream_t)stream);
    });
}

int32_t pd_pack2(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d,
                 const int32_t* kdlab, int32_t P, const int32_t* part_rank,
                 const int32_t* local_index, uint32_t gid_base, int32_t n_ranks,
                 void* const* coords, uint32_t* const* gid, int32_t* const* owner,
                 uint8_t* const* xr, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (d > kMaxDim) throw Error(PD_EUNSUPPORTED, "d > 4");
        if (P < 1 || !part_rank || !local_index || !coords || !gid || !owner || !xr ||
            (n && !kdlab))
            throw Error(PD_EINVAL, "null argument");
        pack2(ctx->c, X, dtype, n, d, kdlab, P, part_rank, local_index, gid_base, n_ranks, coords,
              gid, owner, xr, (hipStream_t)stream);
    });
}

int32_t pd_results(pd_ctx* ctx, int64_t nr, const uint32_t* keys, const uint8_t* core,
                   const int32_t* owner, const uint32_t* gid, const uint32_t* roots, int64_t n_roots,
                   int64_t n_total, uint32_t gid_base, int64_t n_local, int32_t n_ranks,
                   int32_t rank, const int64_t* src_offsets, int64_t expect_remote,
                   int32_t* labels, uint8_t* core_out, uint32_t* pairs, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !src_offsets || nr < 0 || n_local < 0 || n_roots < 0 || expect_remote < 0)
            throw Error(PD_EINVAL, "bad argument");
        if (nr && (!keys || !owner)) throw Error(PD_EINVAL, "null argument");
        if (n_roots && !roots) throw Error(PD_EINVAL, "null roots");
        if (n_local && !labels) throw Error(PD_EINVAL, "null labels");
        if (expect_remote && !pairs) throw Error(PD_EINVAL, "null pairs");
        results(ctx->c, nr, keys, core, owner, gid, roots, n_roots, n_total, gid_base, n_local,
                n_ranks, rank, src_offsets, expect_remote, labels, core_out, pairs,
                (hipStream_t)stream);
    });
}

int32_t pd_results_scatter(pd_ctx* ctx, const uint32_t* pairs, int64_t m, uint32_t gid_base,
                           int64_t n, int32_t* labels, uint8_t* core, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || m < 0 || n < 0 || (m && !pairs) || (n && !labels))
            throw Error(PD_EINVAL, "bad argument");
        results_scatter(ctx->c, pairs, m, gid_base, n, labels, core, (hipStream_t)stream);
    });
}

// ---------------------------------------------------------------- sharded dense train

int32_t pd_dense_count(pd_ctx* ctx, const void* X, int32_t dtype, int64_t n, int32_t d, double eps,
                       int32_t min_samples, int32_t metric, const double* data_box, int32_t rank,
                       int32_t n_ranks, uint32_t* counts, void* stream) {
    return guard(ctx, [&] {
        check_common(ctx, X, n, d);
        if (d <= kMaxDim) throw Error(PD_EINVAL, "pd_dense_* is the d > 4 path (pd_train for d <= 4)");
        if (!data_box) throw Error(PD_EINVAL, "null data_box");
        if (n > 0 && !counts) throw Error(PD_EINVAL, "null counts");
        if (n_ranks < 1 || rank < 0 || rank >= n_ranks) throw Error(PD_EINVAL, "bad rank / n_ranks");
        TrainArgs a;
        a.X = X;
        a.dtype = dtype;
        a.n = n;
        a.d = d;
        a.eps = eps;
        a.min_samples = min_samples;
        a.metric = metric;
        a.data_box = data_box;
        a.stream = (hipStream_t)stream;
        dense_count(ctx->c, a, rank, n_ranks, counts);
    });
}

int32_t pd_dense_link(pd_ctx* ctx, const uint32_t* counts, uint32_t* forest, int64_t* n_core,
                      void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !n_core) throw Error(PD_EINVAL, "null argument");
        if (ctx->c.dn.n && (!counts || !forest)) throw Error(PD_EINVAL, "null buffer");
        *n_core = dense_link(ctx->c, counts, forest, (hipStream_t)stream);
    });
}

int32_t pd_dense_border(pd_ctx* ctx, const uint32_t* forests, int32_t n_forests, int32_t* best,
                        int64_t* n_border, void* stream) {
    return guard(ctx, [&] {
        if (!ctx || !n_border || n_forests < 0) throw Error(PD_EINVAL, "bad argument");
        if (ctx->c.dn.n && !best) throw Error(PD_EINVAL, "null best");
        if (n_forests && ctx->c.dn.n_core && !forests) throw Error(PD_EINVAL, "null forests");
        *n_border = dense_border(ctx->c, forests, n_forests, best, (hipStream_t)stream);
    });
}

int32_t pd_dense_finish(pd_ctx* ctx, const int32_t* best, int32_t* labels, uint8_t* core,
                        uint32_t* counts, int64_t* n_clusters, void* stream) {
    return guard(ctx, [&] {
        if (!ctx) throw Error(PD_EINVAL, "null context");
        if (ctx->c.dn.n && !labels) throw Error(PD_EINVAL, "null labels");
        if (ctx->c.dn.n_border && !best) throw Error(PD_EINVAL, "null best");
        const int64_t ncl = dense_finish(ctx->c, best, labels, core, counts, (hipStream_t)stream);
        if (n_clusters) *n_clusters = ncl;
    });
}

// ---------------------------------------------------------------- RCCL

int32_t pd_comm_unique_id(uint8_t* id) {
    return guard(nullptr, [&] {
        if (!id) throw Error(PD_EINVAL, "null id");
        comm_unique_id(id);
    });
}

int32_t pd_comm_init(pd_ctx* ctx, int32_t n_ranks, int32_t rank, const uint8_t* id, pd_comm** out) {
    return guard(ctx, [&] {
        if (!ctx || !id || !out) throw Error(PD_EINVAL, "null argument");
        pd::Comm* c = comm_init(ctx->c.device, n_ranks, rank, id);
        *out = new pd_comm{c};
    });
}

int32_t pd_comm_init_all(int32_t n, const int32_t* devices, pd_comm** out) {
    return guard(nullptr, [&] {
        if (n < 1 || !devices || !out) throw Error(PD_EINVAL, "bad argument");
        std::vector<pd::Comm*> cs(n, nullptr);
        comm_init_all(n, devices, cs.data());
        for (int i = 0; i < n; ++i) out[i] = new pd_comm{cs[i]};
    });
}

int32_t pd_comm_destroy(pd_comm* comm) {
    if (!comm) return PD_OK;
    comm_destroy(comm->c);
    delete comm;
    return PD_OK;
}

int32_t pd_comm_all_reduce(pd_comm* comm, const void* send, void* recv, int64_t count, int32_t elem,
                           int32_t op, void* stream) {
    return comm_guard(comm, [&] {
        if (count < 0 || (count && (!send || !recv))) throw Error(PD_EINVAL, "bad buffer");
        comm_all_reduce(comm->c, send, recv, count, elem, op, (hipStream_t)stream);
    });
}

int32_t pd_comm_all_gather_v(pd_comm* comm, const void* send, void* recv, const int64_t* counts,
                             int32_t elem, void* stream) {
    return comm_guard(comm, [&] {
        if (!counts) throw Error(PD_EINVAL, "null counts");
        comm_all_gather_v(comm->c, send, recv, counts, elem, (hipStream_t)stream);
    });
}

int32_t pd_comm_all_to_all_v(pd_comm* comm, const void* send, const int64_t* send_counts,
                             void* recv, const int64_t* recv_counts, int32_t elem, void* stream) {
    return comm_guard(comm, [&] {
        if (!send_counts || !recv_counts) throw Error(PD_EINVAL, "null counts");
        comm_all_to_all_v(comm->c, send, send_counts, recv, recv_counts, elem, (hipStream_t)stream);
    });
}

int32_t pd_comm_exchange(pd_comm* comm, int32_t n_fields, const void* const* send,
                         void* const* recv, const int64_t* rec_bytes, const int64_t* send_counts,
                         const int64_t* send_offsets, const int64_t* recv_counts,
                         const int64_t* recv_offsets, int32_t skip_self, void* stream) {
    return comm_guard(comm, [&] {
        if (n_fields < 1 || n_fields > 16 || !send || !recv || !rec_bytes || !send_counts ||
            !send_offsets || !recv_counts || !recv_offsets)
            throw Error(PD_EINVAL, "bad argument");
        comm_exchange(comm->c, n_fields, send, recv, rec_bytes, send_counts, send_offsets,
                      recv_counts, recv_offsets, skip_self != 0, (hipStream_t)stream);
    });
}

int32_t pd_comm_abort(pd_comm* comm) {
    if (!comm) return PD_OK;
    comm_abort(comm->c);
    return PD_OK;
}

int32_t pd_comm_self_check(pd_comm* comm) {
    return comm_guard(comm, [&] { comm_self_check(&comm->c, 1); });
}

int32_t pd_comm_size(pd_comm* comm, int32_t* n_ranks, int32_t* rank) {
    return comm_guard(comm, [&] {
        if (!n_ranks || !rank) throw Error(PD_EINVAL, "null argument");
        int n = 0, r = 0;
        comm_size(comm->c, &n, &r);
        *n_ranks = n;
        *rank = r;
    });
}

int32_t pd_comm_broadcast(pd_comm* comm, void* buf, int64_t count, int32_t elem, int32_t root,
                          void* stream) {
    return comm_guard(comm, [&] {
        if (count < 0 || (count && !buf)) throw Error(PD_EINVAL, "bad buffer");
        comm_broadcast(comm->c, buf, count, elem, root, (hipStream_t)stream);
    });
}

}  // extern "C"
