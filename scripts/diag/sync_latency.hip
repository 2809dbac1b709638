// Build: /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o scripts/diag/sync_latency scripts/diag/sync_latency.hip
// Round-trip cost of one tiny launch + host wait, by wait form (diagnostic for DESIGN.md's
// config-L notes): hipStreamSynchronize, hipEventSynchronize, and a host spin on a pinned
// word the kernel writes last (system-scope release by a vector store).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_tiny(int* dev, int v) {
    if (threadIdx.x == 0) dev[0] = v;
}
__global__ void k_flag(volatile int* host_flag, int v) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        host_flag[0] = v;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int* dev;
    CK(hipMalloc(&dev, 64));
    int* hflag;
    CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    int* dflag;
    CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
    hipEvent_t ev, e0, e1;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int N = 5000;
    auto run = [&](const char* name, auto&& body) {
        for (int i = 0; i < 200; i++) body(i);
        auto t = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) body(i + 1000);
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
        printf("%-44s %7.2f us\n", name, us);
    };
    run("launch + hipStreamSynchronize", [&](int i) {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, dev, i);
        (void)hipStreamSynchronize(st);
    });
    run("2 launches + hipStreamSynchronize", [&](int i) {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, dev, i);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, dev, i);
        (void)hipStreamSynchronize(st);
    });
    run("launch + event record + hipEventSynchronize", [&](int i) {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, dev, i);
        (void)hipEventRecord(ev, st);
        (void)hipEventSynchronize(ev);
    });
    run("timed events around launch + sync + elapsed", [&](int i) {
        (void)hipEventRecord(e0, st);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, dev, i);
        (void)hipEventRecord(e1, st);
        (void)hipStreamSynchronize(st);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
    });
    run("launch writing a pinned flag + host spin", [&](int i) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, dflag, i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != i) {
        }
    });
    (void)hipStreamSynchronize(st);
    run("spin, then hipStreamSynchronize", [&](int i) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, dflag, i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != i) {
        }
        (void)hipStreamSynchronize(st);
    });
    return 0;
}
