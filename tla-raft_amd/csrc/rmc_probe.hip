// rmc_probe.hip -- random-access probe peak of the seen-set layout ("BW_rand =
// measured random-gather throughput on the box").  Measurement support, not on the BFS path:
// it times one-slot probes of a table laid out like the seen set (16-B slots {fp.lo, fp.hi},
// open addressing, power-of-two slots) at uniformly random slot indices, so bench.py can put
// the seen-set probe rate of a run next to the rate the HBM sustains for that access pattern.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rmc.h"

namespace {

__device__ __forceinline__ uint64_t pmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill(ulonglong2 *T, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        T[i] = make_ulonglong2(pmix(i) | 1ull, pmix(~i));
}

// Each lane issues PER independent probes (8 in flight at a time), like a wave of successors
// checking their fingerprints against the seen set.
template <int PER>
__global__ __launch_bounds__(256) void k_probe(const ulonglong2 *__restrict__ T, uint64_t mask, uint64_t seed,
                                               unsigned long long *sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t acc = 0;
#pragma unroll
    for (int b = 0; b < PER; b += 8) {
        ulonglong2 e[8];
#pragma unroll
        for (int k = 0; k < 8; k++) e[k] = T[pmix(seed ^ (tid * PER + b + k)) & mask];
#pragma unroll
        for (int k = 0; k < 8; k++) acc ^= e[k].x + e[k].y;
    }
    if (acc == 0x9e3779b97f4a7c15ull) atomicAdd(sink, 1ull);  // keeps the loads live
}

}  // namespace

extern "C" int rmc_probe_peak(int device, uint32_t table_log2, uint64_t probes, double *probes_per_s,
                              double *seconds) {
    if (table_log2 < 10 || table_log2 > 34 || !probes_per_s) return RMC_E_ARG;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return RMC_E_DEVICE;
    const uint64_t n = 1ull << table_log2;
    ulonglong2 *T = nullptr;
    unsigned long long *sink = nullptr;
    if (hipMalloc((void **)&T, n * 16) != hipSuccess) return RMC_E_MEMORY;
    if (hipMalloc((void **)&sink, 8) != hipSuccess) { (void)hipFree(T); return RMC_E_MEMORY; }
    constexpr int PER = 32;
    const uint64_t threads = (probes + PER - 1) / PER;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, T, n);
    hipLaunchKernelGGL((k_probe<PER>), dim3(blocks), dim3(256), 0, 0, T, n - 1, 12345ull, sink);  // warm
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL((k_probe<PER>), dim3(blocks), dim3(256), 0, 0, T, n - 1, 777ull + r, sink);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const hipError_t e = hipGetLastError();
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(sink);
    (void)hipFree(T);
    if (e != hipSuccess) return RMC_E_DEVICE;
    const double done = (double)blocks * 256.0 * PER;
    *probes_per_s = done / (best * 1e-3);
    if (seconds) *seconds = best * 1e-3;
    return RMC_OK;
}
