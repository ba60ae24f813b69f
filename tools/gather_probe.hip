// Gather probe (measurement only, not part of the library): the train's
// coordinate gather (Xs[r] = X[id[r]], 3-D f32 rows padded to 16 B) for R
// records with random ids over n points — C2's shape — as the library does it
// and in id-chunked passes (pass c moves only the records whose id falls in
// the c-th of k id ranges, so each pass's random reads stay within an
// X slice of 1.2 GB / k: does a slice that fits the 256 MB MALL beat HBM?).
// Median of 7 timed runs after 2 warm-ups; every variant checked against the
// first.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_probe.hip -o tools/gather_probe
//   tools/gather_probe [n=100000000] [R=101084014]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__global__ void fill_kernel(float* X, uint32_t* ids, size_t n, size_t R, uint64_t seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n * 3) X[i] = (float)(i % 1000003) * 1e-3f;
    if (i < R) {
        uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        ids[i] = (uint32_t)(x % n);
    }
}

// the library's form: three 4-B loads, four 4-B stores
__global__ __launch_bounds__(256) void g_base(const float* __restrict__ X, size_t R,
                                              const uint32_t* __restrict__ ids,
                                              float* __restrict__ Xs) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const size_t i = ids[r];
#pragma unroll
    for (int j = 0; j < 4; ++j) Xs[r * 4 + j] = j < 3 ? X[i * 3 + j] : 0.f;
}

// one 16-B store
__global__ __launch_bounds__(256) void g_vec(const float* __restrict__ X, size_t R,
                                             const uint32_t* __restrict__ ids,
                                             float* __restrict__ Xs) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const size_t i = ids[r];
    float4 o;
    o.x = X[i * 3];
    o.y = X[i * 3 + 1];
    o.z = X[i * 3 + 2];
    o.w = 0.f;
    reinterpret_cast<float4*>(Xs)[r] = o;
}

// one id range per launch
__global__ __launch_bounds__(256) void g_chunk(const float* __restrict__ X, size_t R,
                                               const uint32_t* __restrict__ ids,
                                               float* __restrict__ Xs, uint32_t lo, uint32_t hi) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const uint32_t i = ids[r];
    if (i < lo || i >= hi) return;
    float4 o;
    o.x = X[(size_t)i * 3];
    o.y = X[(size_t)i * 3 + 1];
    o.z = X[(size_t)i * 3 + 2];
    o.w = 0.f;
    reinterpret_cast<float4*>(Xs)[r] = o;
}

// each lane handles 4 records (4 independent loads in flight per lane)
__global__ __launch_bounds__(256) void g_ilp(const float* __restrict__ X, size_t R,
                                             const uint32_t* __restrict__ ids,
                                             float* __restrict__ Xs) {
    const size_t b = (size_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t id[4];
    float4 o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) id[q] = b + 256 * q < R ? ids[b + 256 * q] : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        o[q].x = X[(size_t)id[q] * 3];
        o[q].y = X[(size_t)id[q] * 3 + 1];
        o[q].z = X[(size_t)id[q] * 3 + 2];
        o[q].w = 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (b + 256 * q < R) reinterpret_cast<float4*>(Xs)[b + 256 * q] = o[q];
}

__global__ void diff_kernel(const float* a, const float* b, size_t m, unsigned* bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && a[i] != b[i]) atomicAdd(bad, 1u);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000000ull;
    const size_t R = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 101084014ull;
    float *X, *Xs, *ref;
    uint32_t* ids;
    unsigned* bad;
    CK(hipMalloc(&X, n * 12));
    CK(hipMalloc(&ids, R * 4));
    CK(hipMalloc(&Xs, R * 16));
    CK(hipMalloc(&ref, R * 16));
    CK(hipMalloc(&bad, 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const size_t fm = std::max(n * 3, R);
    hipLaunchKernelGGL(fill_kernel, dim3((fm + 255) / 256), dim3(256), 0, s, X, ids, n, R, 12345ull);
    const unsigned gb = (unsigned)((R + 255) / 256);
    hipLaunchKernelGGL(g_base, dim3(gb), dim3(256), 0, s, X, R, ids, ref);
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("n %zu  R %zu  X %.2f GB\n", n, R, n * 12 / 1e9);
    auto time = [&](const char* name, auto launch) {
        std::vector<float> t;
        for (int it = 0; it < 9; ++it) {
            CK(hipMemsetAsync(Xs, 0xFF, R * 16, s));
            CK(hipEventRecord(e0, s));
            launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        CK(hipMemsetAsync(bad, 0, 4, s));
        hipLaunchKernelGGL(diff_kernel, dim3((R * 4 + 255) / 256), dim3(256), 0, s, Xs, ref, R * 4, bad);
        unsigned hb = 0;
        CK(hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        std::printf("%-28s median %.3f ms  min %.3f  mismatches %u\n", name, t[t.size() / 2], t[0], hb);
        std::fflush(stdout);
    };
    time("base (3 ld, 4 st)", [&] {
        hipLaunchKernelGGL(g_base, dim3(gb), dim3(256), 0, s, X, R, ids, Xs);
    });
    time("vec store", [&] {
        hipLaunchKernelGGL(g_vec, dim3(gb), dim3(256), 0, s, X, R, ids, Xs);
    });
    time("4 records per lane", [&] {
        hipLaunchKernelGGL(g_ilp, dim3((unsigned)((R + 1023) / 1024)), dim3(256), 0, s, X, R, ids, Xs);
    });
    for (int k : {2, 4, 6, 8, 16}) {
        char name[64];
        std::snprintf(name, sizeof name, "id chunks k=%d (%.0f MB)", k, n * 12.0 / k / 1e6);
        time(name, [&] {
            for (int c = 0; c < k; ++c) {
                const uint32_t lo = (uint32_t)(n * c / k), hi = (uint32_t)(n * (c + 1) / k);
                hipLaunchKernelGGL(g_chunk, dim3(gb), dim3(256), 0, s, X, R, ids, Xs, lo, hi);
            }
        });
    }
    std::printf("done\n");
    return 0;
}
