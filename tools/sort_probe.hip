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

#include "../pypardis_amd/csrc/rsort.hpp"

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

// The library's own onesweep (pypardis_amd/csrc/rsort.hpp) with I items per
// thread, checked pair for pair against rocPRIM's stable result.
template <int I, int NT = 256>
int run_rs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t* k2, uint32_t* v2,
           const uint32_t* rk, const uint32_t* rv, size_t n, unsigned bits, hipStream_t s) {
    pd::rsort::State st;
    st.look_tiles = (n + (uint64_t)NT * I - 1) / ((uint64_t)NT * I);
    CK(hipMalloc(&st.look, sizeof(uint64_t) * 256 * st.look_tiles));
    CK(hipMemset(st.look, 0, sizeof(uint64_t) * 256 * st.look_tiles));
    CK(hipMalloc(&st.hist, sizeof(uint32_t) * 8 * 256));
    CK(hipMalloc(&st.ticket, sizeof(unsigned long long)));
    std::vector<float> t;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint32_t *ok_k = nullptr, *ok_v = nullptr;
    for (int it = 0; it < 9; ++it) {
        CK(hipMemcpyAsync(k1, k0, n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(v1, v0, n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipEventRecord(e0, s));
        try {
            pd::rsort::sort_pairs<uint32_t, I, NT>(st, k1, v1, k2, v2, n, (int)bits, s, &ok_k, &ok_v);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "rsort: %s\n", e.what());
            return 1;
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) t.push_back(ms);
    }
    std::vector<uint32_t> a(n), b(n), c(n), d(n);
    CK(hipMemcpy(a.data(), ok_k, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), ok_v, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), rk, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d.data(), rv, n * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < n; ++i) diff += (a[i] != c[i] || b[i] != d[i]) ? 1 : 0;
    std::sort(t.begin(), t.end());
    char name[64];
    std::snprintf(name, sizeof(name), "pd::rsort onesweep, %d threads x %d items", NT, I);
    std::printf("%-44s %8.3f ms  %6.2f GB/s per pass-byte  %s (%zu pairs differ from rocPRIM)\n", name,
                t[t.size() / 2], (double)n * 16.0 * ((bits + 7) / 8) / (t[t.size() / 2] * 1e-3) / 1e9,
                diff ? "MISMATCH" : "identical", diff);
    CK(hipFree(st.look));
    CK(hipFree(st.hist));
    CK(hipFree(st.ticket));
    return 0;
}


__global__ void fill64_kernel(uint64_t* k, uint32_t* v, size_t n, uint64_t mask, uint64_t seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    k[i] = x & mask;
    v[i] = (uint32_t)i;
}

// 64-bit keys of `bits` bits (C4: 37): rocPRIM vs the library's sort.
template <int I, int NT = 256>
int run64(size_t n, unsigned bits, hipStream_t s) {
    uint64_t *k0, *k1, *k2;
    uint32_t *v0, *v1, *v2;
    CK(hipMalloc(&k0, n * 8));
    CK(hipMalloc(&k1, n * 8));
    CK(hipMalloc(&k2, n * 8));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&v1, n * 4));
    CK(hipMalloc(&v2, n * 4));
    fill64_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(k0, v0, n, (1ull << bits) - 1ull, 777);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // rocPRIM
    size_t tb = 0;
    {
        rocprim::double_buffer<uint64_t> kb(k1, k2);
        rocprim::double_buffer<uint32_t> vb(v1, v2);
        CK(rocprim::radix_sort_pairs(nullptr, tb, kb, vb, n, 0u, bits, s));
    }
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    std::vector<float> tr, tl;
    std::vector<uint64_t> ka(n), kb2(n);
    std::vector<uint32_t> va(n), vb2(n);
    for (int it = 0; it < 7; ++it) {
        CK(hipMemcpyAsync(k1, k0, n * 8, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(v1, v0, n * 4, hipMemcpyDeviceToDevice, s));
        rocprim::double_buffer<uint64_t> kb(k1, k2);
        rocprim::double_buffer<uint32_t> vb(v1, v2);
        CK(hipEventRecord(e0, s));
        CK(rocprim::radix_sort_pairs(tmp, tb, kb, vb, n, 0u, bits, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) tr.push_back(ms);
        if (it == 6) {
            CK(hipMemcpy(ka.data(), kb.current(), n * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(va.data(), vb.current(), n * 4, hipMemcpyDeviceToHost));
        }
    }
    pd::rsort::State st;
    st.look_tiles = (n + (uint64_t)NT * I - 1) / ((uint64_t)NT * I);
    CK(hipMalloc(&st.look, sizeof(uint64_t) * 256 * st.look_tiles));
    CK(hipMemset(st.look, 0, sizeof(uint64_t) * 256 * st.look_tiles));
    CK(hipMalloc(&st.hist, sizeof(uint32_t) * 8 * 256));
    CK(hipMalloc(&st.ticket, sizeof(unsigned long long)));
    for (int it = 0; it < 7; ++it) {
        CK(hipMemcpyAsync(k1, k0, n * 8, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(v1, v0, n * 4, hipMemcpyDeviceToDevice, s));
        uint64_t* ok;
        uint32_t* ov;
        CK(hipEventRecord(e0, s));
        pd::rsort::sort_pairs<uint64_t, I, NT>(st, k1, v1, k2, v2, n, (int)bits, s, &ok, &ov);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) tl.push_back(ms);
        if (it == 6) {
            CK(hipMemcpy(kb2.data(), ok, n * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(vb2.data(), ov, n * 4, hipMemcpyDeviceToHost));
        }
    }
    size_t diff = 0;
    for (size_t i = 0; i < n; ++i) diff += (ka[i] != kb2[i] || va[i] != vb2[i]) ? 1 : 0;
    std::sort(tr.begin(), tr.end());
    std::sort(tl.begin(), tl.end());
    std::printf("u64 keys, %u bits, n = %zu: rocPRIM %.3f ms, pd::rsort (%d threads x %d items) %.3f ms, %s (%zu differ)\n",
                bits, n, tr[tr.size() / 2], NT, I, tl[tl.size() / 2], diff ? "MISMATCH" : "identical", diff);
    CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(k2));
    CK(hipFree(v0)); CK(hipFree(v1)); CK(hipFree(v2));
    CK(hipFree(tmp)); CK(hipFree(st.look)); CK(hipFree(st.hist)); CK(hipFree(st.ticket));
    return 0;
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
    run<OS<1024, 8, 8, A::match>>("1024x8 r8 match", k0, v0, k1, v1, k2, v2, n, bits, bad, s);
    uint32_t *rk, *rv;
    CK(hipMalloc(&rk, n * 4));
    CK(hipMalloc(&rv, n * 4));
    {   // rocPRIM's stable result, the reference for the library's sort
        size_t tb = 0;
        CK(hipMemcpy(k1, k0, n * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(v1, v0, n * 4, hipMemcpyDeviceToDevice));
        rocprim::double_buffer<uint32_t> kb(k1, k2), vb(v1, v2);
        CK(rocprim::radix_sort_pairs(nullptr, tb, kb, vb, n, 0u, bits, s));
        void* tmp;
        CK(hipMalloc(&tmp, tb));
        CK(rocprim::radix_sort_pairs(tmp, tb, kb, vb, n, 0u, bits, s));
        CK(hipMemcpyAsync(rk, kb.current(), n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(rv, vb.current(), n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipStreamSynchronize(s));
        CK(hipFree(tmp));
    }
    run_rs<32>(k0, v0, k1, v1, k2, v2, rk, rv, n, bits, s);
    run_rs<16, 512>(k0, v0, k1, v1, k2, v2, rk, rv, n, bits, s);
    run_rs<8, 1024>(k0, v0, k1, v1, k2, v2, rk, rv, n, bits, s);
    run_rs<12, 1024>(k0, v0, k1, v1, k2, v2, rk, rv, n, bits, s);
    run_rs<12, 512>(k0, v0, k1, v1, k2, v2, rk, rv, n, bits, s);
    CK(hipFree(k0)); CK(hipFree(v0)); CK(hipFree(k1)); CK(hipFree(v1)); CK(hipFree(k2)); CK(hipFree(v2));
    CK(hipFree(rk)); CK(hipFree(rv));
    // C4's shape: 1.0e9 records would need 16 GB here; 2e8 keeps the box light
    run64<24>(200000000, 37, s);
    run64<12, 512>(200000000, 37, s);
    run64<8, 1024>(200000000, 37, s);
    return 0;
}
