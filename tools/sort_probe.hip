// Onesweep configuration probe (measurement only, not part of the library):
// rocPRIM radix_sort_pairs of N random (32-bit key, 32-bit id) pairs — the
// shape of the train's (cell key, point id) sort on C2 — under several
// onesweep configurations (sort block size x items per thread, radix rank
// algorithm), median of 7 timed sorts each after 2 warm-ups.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_probe.hip -o tools/sort_probe
//   tools/sort_probe [n=101084014] [key_bits=32]
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void fill_kernel(uint32_t* k, uint32_t* v, size_t n, uint32_t mask, uint64_t seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    k[i] = (uint32_t)x & mask;
    v[i] = (uint32_t)i;
}

__global__ void check_kernel(const uint32_t* k, size_t n, uint32_t* bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 < n && k[i] > k[i + 1]) atomicAdd(bad, 1u);
}

template <class Cfg>
float run(const char* name, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t* k2,
          uint32_t* v2, size_t n, unsigned bits, uint32_t* bad, hipStream_t s) {
    size_t tb = 0;
    {
        rocprim::double_buffer<uint32_t> kb(k1, k2), vb(v1, v2);
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kb, vb, n, 0u, bits, s));
    }
    void* tmp = nullptr;
    CK(hipMalloc(&tmp, tb));
    std::vector<float> t;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t* out = nullptr;
    for (int it = 0; it < 9; ++it) {
        CK(hipMemcpyAsync(k1, k0, n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(v1, v0, n * 4, hipMemcpyDeviceToDevice, s));
        rocprim::double_buffer<uint32_t> kb(k1, k2), vb(v1, v2);
        CK(hipEventRecord(e0, s));
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kb, vb, n, 0u, bits, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) t.push_back(ms);
        out = kb.current();
    }
    CK(hipMemsetAsync(bad, 0, 4, s));
    check_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(out, n, bad);
    uint32_t hb = 0;
    CK(hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    std::printf("%-44s %8.3f ms  %6.2f GB/s per pass-byte  %s\n", name, med,
                (double)n * 16.0 * ((bits + 7) / 8) / (med * 1e-3) / 1e9, hb ? "UNSORTED" : "ok");
    CK(hipFree(tmp));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return med;
}

using rocprim::block_radix_rank_algorithm;
template <unsigned B, unsigned I, unsigned R, block_radix_rank_algorithm A>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<B, I>,
                                        R, A>>;

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 101084014ull;
    const unsigned bits = argc > 2 ? (unsigned)std::atoi(argv[2]) : 32u;
    const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
    uint32_t *k0, *v0, *k1, *v1, *k2, *v2, *bad;
    CK(hipMalloc(&k0, n * 4));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&k1, n * 4));
    CK(hipMalloc(&v1, n * 4));
    CK(hipMalloc(&k2, n * 4));
    CK(hipMalloc(&v2, n * 4));
    CK(hipMalloc(&bad, 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    fill_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(k0, v0, n, mask, 12345);
    CK(hipStreamSynchronize(s));
    std::printf("n = %zu, key bits = %u\n", n, bits);
    run<rocprim::default_config>("default", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    using A = block_radix_rank_algorithm;
    run<OS<1024, 16, 8, A::match>>("1024x16 r8 match (gfx950 default)", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<512, 16, 8, A::match>>("512x16 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<512, 24, 8, A::match>>("512x24 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<256, 16, 8, A::match>>("256x16 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<256, 32, 8, A::match>>("256x32 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<1024, 8, 8, A::match>>("1024x8 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<1024, 24, 8, A::match>>("1024x24 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<256, 16, 8, A::basic_memoize>>("256x16 r8 memoize", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<512, 16, 7, A::match>>("512x16 r7 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    run<OS<1024, 16, 6, A::match>>("1024x16 r6 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    return 0;
}
