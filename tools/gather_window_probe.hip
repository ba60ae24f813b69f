// Gather window probe (measurement only, not part of the library): how fast
// is the train's coordinate gather (Xs[r] = row[id[r]], R records) when the
// source rows are not in random order but grouped so that consecutive
// records read from a window of B rows (a coarse spatial layout: B = n/8 is
// "grouped by KD leaf", smaller B a finer bucket order)?  ids[r] = window of r
// (windows in order, R/ (n/B) records each) + a hash of r inside the window.
// Rows are 12-B (x, y, z: the library's X) or 16-B (x, y, z, id: one 16-B
// load carrying the point id).  Median of 7 timed runs after 2 warm-ups.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_window_probe.hip -o tools/gather_window_probe
//   tools/gather_window_probe [n=100000000] [R=101084014]
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

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x;
}

__global__ void fill_rows(float* X3, float4* X4, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = (float)(i % 1000003) * 1e-3f, b = a + 1.f, c = a + 2.f;
    X3[i * 3] = a;
    X3[i * 3 + 1] = b;
    X3[i * 3 + 2] = c;
    X4[i] = make_float4(a, b, c, __uint_as_float((uint32_t)i));
}

// B = window rows (0: uniformly random over n)
__global__ void fill_ids(uint32_t* ids, size_t n, size_t R, size_t B, uint64_t seed) {
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const uint64_t h = mix((r + 1) * 0x9E3779B97F4A7C15ull ^ seed);
    if (B == 0 || B >= n) {
        ids[r] = (uint32_t)(h % n);
        return;
    }
    const size_t nw = n / B;
    const size_t w = r * nw / R;
    ids[r] = (uint32_t)(w * B + h % B);
}

__global__ __launch_bounds__(256) void g12(const float* __restrict__ X, size_t R,
                                           const uint32_t* __restrict__ ids,
                                           float4* __restrict__ Xs) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const size_t i = ids[r];
    Xs[r] = make_float4(X[i * 3], X[i * 3 + 1], X[i * 3 + 2], 0.f);
}

__global__ __launch_bounds__(256) void g16(const float4* __restrict__ X, size_t R,
                                           const uint32_t* __restrict__ ids,
                                           float4* __restrict__ Xs, uint32_t* __restrict__ idout) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const float4 v = X[ids[r]];
    Xs[r] = make_float4(v.x, v.y, v.z, 0.f);
    idout[r] = __float_as_uint(v.w);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000000ull;
    const size_t R = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 101084014ull;
    float* X3;
    float4 *X4, *Xs;
    uint32_t *ids, *idout;
    CK(hipMalloc(&X3, n * 12));
    CK(hipMalloc(&X4, n * 16));
    CK(hipMalloc(&ids, R * 4));
    CK(hipMalloc(&idout, R * 4));
    CK(hipMalloc(&Xs, R * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(fill_rows, dim3((n + 255) / 256), dim3(256), 0, s, X3, X4, n);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned gb = (unsigned)((R + 255) / 256);
    std::printf("n %zu  R %zu\n", n, R);
    auto time = [&](const char* name, auto launch) {
        std::vector<float> t;
        for (int it = 0; it < 9; ++it) {
            CK(hipEventRecord(e0, s));
            launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        std::printf("%-40s median %.3f ms  min %.3f\n", name, t[t.size() / 2], t[0]);
        std::fflush(stdout);
    };
    const size_t Bs[] = {0, n / 8, n / 64, 1u << 20, 1u << 18, 1u << 16, 1u << 12};
    for (size_t B : Bs) {
        hipLaunchKernelGGL(fill_ids, dim3(gb), dim3(256), 0, s, ids, n, R, B, 12345ull);
        char nm[96];
        std::snprintf(nm, sizeof nm, "12-B rows, window %zu rows", B ? B : n);
        time(nm, [&] { hipLaunchKernelGGL(g12, dim3(gb), dim3(256), 0, s, X3, R, ids, Xs); });
        std::snprintf(nm, sizeof nm, "16-B rows+id, window %zu rows", B ? B : n);
        time(nm, [&] { hipLaunchKernelGGL(g16, dim3(gb), dim3(256), 0, s, X4, R, ids, Xs, idout); });
    }
    std::printf("done\n");
    return 0;
}
