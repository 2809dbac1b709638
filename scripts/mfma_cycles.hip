// mfma_cycles.hip -- issue cost of the bf16 MFMA shapes on one SIMD (study tool, not product):
// one wave runs N back-to-back MFMAs on four independent accumulators and stamps s_memtime
// around the loop.  Prints cycles per MFMA for v_mfma_f32_32x32x16_bf16 and the K = 8 form
// v_mfma_f32_32x32x8bf16_1k (the fused filter's augmented k-step needs only 3 of 16 columns).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_cycles scripts/mfma_cycles.hip && ./mfma_cycles
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(64) void k_loop(float* out, long long* cyc, int n) {
    floatx16 a0 = floatx16{}, a1 = floatx16{}, a2 = floatx16{}, a3 = floatx16{};
    const float x = (float)threadIdx.x * 0.001f;
    bf16x8 A, B;
    shortx4 A4, B4;
    for (int i = 0; i < 8; i++) { A[i] = (__bf16)(x + i); B[i] = (__bf16)(x - i); }
    for (int i = 0; i < 4; i++) { A4[i] = (short)(threadIdx.x + i); B4[i] = (short)(threadIdx.x * 3 + i); }
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        if constexpr (SHAPE == 16) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, a3, 0, 0, 0);
        } else {
            a0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(A4, B4, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(A4, B4, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(A4, B4, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(A4, B4, a3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
    for (int r = 0; r < 16; r++) s += a0[r] + a1[r] + a2[r] + a3[r];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(float));
    hipMalloc(&cyc, sizeof(long long));
    const int n = 4096;
    for (int shape : {16, 8, 16, 8}) {
        if (shape == 16) hipLaunchKernelGGL(k_loop<16>, dim3(1), dim3(64), 0, 0, out, cyc, n);
        else hipLaunchKernelGGL(k_loop<8>, dim3(1), dim3(64), 0, 0, out, cyc, n);
        long long c = 0;
        hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        printf("32x32x%d bf16: %.2f cycles per MFMA (s_memtime)\n", shape, (double)c / (4.0 * n));
    }
    hipFree(out);
    hipFree(cyc);
    return 0;
}
