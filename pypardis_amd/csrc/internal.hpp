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
};

struct Ctx {
    int device = 0;
    Arena arena;
    void* pinned = nullptr;      // small pinned staging block for D2H scalars
    bool timing = false;
    bool full_counts = false;    // debug: count every neighbour (no early exit)
    bool seq_moments = false;    // reference-order (sequential) KD moment sums
    int link_mode = 0;           // 0 init forest + jumps + union; 2 union only; 1 diagnostic
    int jump_rounds = 4;
    int xsub = 2;                // axis-0 sub-cells per eps
    bool screen = true;          // fp32 screening of fp32 inputs (exact either way)
    Timings t;
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
};

void train(Ctx& ctx, TrainArgs& a);

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
void halo_members(Ctx& ctx, const void* X, int dtype, int64_t n, int d, int P,
                  const double* ebox_host, int64_t* counts_host, int64_t* members_dev,
                  int64_t members_cap, hipStream_t s);

// small helpers (api.hip)
void* pinned(Ctx& ctx, size_t bytes);
void sync(hipStream_t s);

}  // namespace pd
