// lds_bcast.hip -- LDS read throughput of ds_read_b128 (study tool, not product): 8 waves of one
// block each issue N reads and sum them; three address patterns:
//   distinct   lane l reads 16 B at 16 l (conflict-free, 1 KiB per wave-instruction)
//   broadcast  the 32 lanes of a half read the same 16 B (two addresses per instruction: the
//              fused filter's C-init read of the train norms)
//   rows       lane l reads row (l & 31) of a padded image (the filter's A-fragment read)
// Prints LDS cycles per wave-instruction per CU (s_memtime over the block).
//   hipcc --offload-arch=gfx950 -O3 -o lds_bcast scripts/lds_bcast.hip && ./lds_bcast
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(512) void k_lds(float* out, long long* cyc, int n) {
    __shared__ __attribute__((aligned(16))) float lds[16384];
    for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = (float)i;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int base;
    if (MODE == 0) base = lane * 4;
    else if (MODE == 1) base = (lane >> 5) * 4;
    else base = (lane & 31) * 76 + (lane >> 5) * 4;  // 304-B rows, 16 B per lane half
    base += wave * 16;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        const int o = (i & 7) * 1024;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float4 v = *reinterpret_cast<const float4*>(&lds[(base + o + u * 2432) & 16383 & ~3]);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    const int nb = 256, n = 2048;
    if (hipMalloc(&out, nb * 512 * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&cyc, nb * sizeof(long long)) != hipSuccess) return 1;
    const char* names[3] = {"distinct", "broadcast", "rows"};
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 3; m++) {
            if (m == 0) hipLaunchKernelGGL(k_lds<0>, dim3(nb), dim3(512), 0, 0, out, cyc, n);
            if (m == 1) hipLaunchKernelGGL(k_lds<1>, dim3(nb), dim3(512), 0, 0, out, cyc, n);
            if (m == 2) hipLaunchKernelGGL(k_lds<2>, dim3(nb), dim3(512), 0, 0, out, cyc, n);
            long long c[nb];
            if (hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 1;
            double s = 0;
            for (int b = 0; b < nb; b++) s += (double)c[b];
            // 8 waves x n x 4 reads per block
            printf("%-9s: %.2f cycles per ds_read_b128 wave-instruction per CU\n", names[m], s / nb / (8.0 * n * 4));
        }
    return 0;
}
