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

#define PD_ABI_VERSION 1

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
    PD_OPT_LINK_MODE = 4,  /* union strategy (tuning): 0 (default) initial forest from the count
                              pass's smallest neighbour + pointer jumping, then lock-free union
                              over core-core edges; 2 the union pass alone */
    PD_OPT_JUMP_ROUNDS = 5, /* pointer-jumping rounds for link mode 0 (default 4) */
    PD_OPT_XSUB = 6,        /* sub-cells per eps along axis 0 (default 2): finer rows follow
                               the eps-ball's chord more tightly, at 1/xsub the directory
                               density */
    PD_OPT_FP32_SCREEN = 7  /* fp32 inputs: decide pairs outside a 2^-18 band around eps with
                               fp32 arithmetic, the rest with the exact fp64 predicate
                               (default 1; results are identical with 0) */
};

/* pd_ctx_timings() slots (ms from HIP events on the call's stream; counters) */
enum pd_timing_slot {
    PD_T_HALO = 0, PD_T_SORT, PD_T_GATHER, PD_T_CELLS, PD_T_COUNT, PD_T_LINK, PD_T_MERGE,
    PD_T_ROOTS, PD_T_BORDER, PD_T_LABEL, PD_T_TOTAL, PD_T_RECORDS, PD_T_CELLS_N, PD_T_GRID_CELLS,
    PD_T_KEY_BITS, PD_T_NSLOTS
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

#ifdef __cplusplus
}
#endif
#endif /* PARDIS_H */
