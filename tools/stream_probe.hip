// Streaming-read probe: which load shape reaches the HBM roofline on this
// MI355X?  Sums a 1.2 GB float buffer (the C2 coordinate array) with
//   A  float4 per lane, grid-stride, U loads in flight per lane
//   B  the same with nontemporal loads
//   C  the KD passes' shape: 4 points (3 float4) per lane at a 48-byte lane
//      stride
// and reports GB/s (HIP events, mean of 20 launches).
//   hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o /tmp/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void sum_a(const float4* __restrict__ p, size_t n4, float* out) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) {
                if (NT) {
                    typedef float f4 __attribute__((ext_vector_type(4)));
                    const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + i);
                    v[u] = make_float4(t.x, t.y, t.z, t.w);
                } else
                    v[u] = p[i];
            } else {
                v[u] = make_float4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.f) out[0] = acc;
}

template <int K>
__global__ __launch_bounds__(256) void sum_c(const float4* __restrict__ p, size_t nch, float* out) {
    float acc = 0.f;
    for (size_t t = blockIdx.x; t * 256 * K < nch; t += gridDim.x) {
        float4 v[K][3];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const size_t ch = t * 256 * K + (size_t)k * 256 + threadIdx.x;
            if (ch < nch) {
#pragma unroll
                for (int j = 0; j < 3; ++j) v[k][j] = p[ch * 3 + j];
            } else {
#pragma unroll
                for (int j = 0; j < 3; ++j) v[k][j] = make_float4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) acc += v[k][j].x + v[k][j].y + v[k][j].z + v[k][j].w;
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    const size_t nf = 300000000ull;   // 1.2 GB
    float* d = nullptr;
    float* o = nullptr;
    CK(hipMalloc(&d, nf * 4));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(d, 0, nf * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto run = [&](const char* name, auto launch) -> int {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 20;
        printf("%-28s %8.3f ms %8.1f GB/s\n", name, ms, nf * 4 / (ms * 1e6));
        return 0;
    };
    const size_t n4 = nf / 4;
    for (int mult : {4, 8, 16, 32}) {
        const unsigned g = cus * mult;
        char nm[64];
        snprintf(nm, 64, "A U4 grid=%dxCU", mult);
        run(nm, [&] { hipLaunchKernelGGL((sum_a<4, false>), dim3(g), dim3(256), 0, 0, (const float4*)d, n4, o); });
        snprintf(nm, 64, "A U8 grid=%dxCU", mult);
        run(nm, [&] { hipLaunchKernelGGL((sum_a<8, false>), dim3(g), dim3(256), 0, 0, (const float4*)d, n4, o); });
        snprintf(nm, 64, "B U4 nt grid=%dxCU", mult);
        run(nm, [&] { hipLaunchKernelGGL((sum_a<4, true>), dim3(g), dim3(256), 0, 0, (const float4*)d, n4, o); });
        snprintf(nm, 64, "B U8 nt grid=%dxCU", mult);
        run(nm, [&] { hipLaunchKernelGGL((sum_a<8, true>), dim3(g), dim3(256), 0, 0, (const float4*)d, n4, o); });
        snprintf(nm, 64, "C K2 (48B stride) grid=%dxCU", mult);
        run(nm, [&] { hipLaunchKernelGGL((sum_c<2>), dim3(g), dim3(256), 0, 0, (const float4*)d, n4 / 3, o); });
    }
    const unsigned full = (unsigned)((n4 + 255) / 256);
    run("A U1 one pass (no loop)", [&] { hipLaunchKernelGGL((sum_a<1, false>), dim3(full), dim3(256), 0, 0, (const float4*)d, n4, o); });
    return 0;
}
