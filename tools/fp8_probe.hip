// Probe: operand lane map of v_mfma_f32_32x32x16_fp8_fp8 on gfx950 and the
// OCP e4m3 conversion.  A[32][16], B[16][32] small integers (exact in e4m3);
// assumed map (as bf16 32x32x16): lane l holds A[l & 31][8 (l >> 5) + j] and
// B[8 (l >> 5) + j][l & 31] in byte j; C/D: col = l & 31, row = (r & 3) +
// 8 (r >> 2) + 4 (l >> 5).  Prints the number of mismatching outputs.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float* A, const float* B, float* C) {
    const int l = threadIdx.x;
    long a = 0, b = 0;
    for (int j = 0; j < 8; j += 2) {
        const int k = 8 * (l >> 5) + j;
        int pa = __builtin_amdgcn_cvt_pk_fp8_f32(A[(l & 31) * 16 + k], A[(l & 31) * 16 + k + 1], 0, false);
        int pb = __builtin_amdgcn_cvt_pk_fp8_f32(B[k * 32 + (l & 31)], B[(k + 1) * 32 + (l & 31)], 0, false);
        a |= (long)(pa & 0xFFFF) << (8 * j);
        b |= (long)(pb & 0xFFFF) << (8 * j);
    }
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
        C[row * 32 + col] = c[r];
    }
}

int main() {
    float hA[32 * 16], hB[16 * 32], hC[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 16; ++k) hA[i * 16 + k] = (float)((i * 3 + k * 5) % 7 - 3);
    for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 32; ++j) hB[k * 32 + j] = (float)((k * 2 + j * 7) % 5 - 2) * (j < 16 ? 1.0f : 0.5f);
    float *dA, *dB, *dC;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            float s = 0;
            for (int k = 0; k < 16; ++k) s += hA[i * 16 + k] * hB[k * 32 + j];
            if (s != hC[i * 32 + j]) { if (bad < 5) printf("C[%d][%d] = %g want %g\n", i, j, hC[i * 32 + j], s); ++bad; }
        }
    printf("fp8 32x32x16 lane map: %d mismatches of 1024\n", bad);
    return bad ? 1 : 0;
}
