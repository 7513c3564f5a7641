// Microbenchmark (profiling aid): random no-return 32-bit atomicMin into a table, the MinMax
// insert's alternative to bucketed minima.  8 regions of `cells` u32 each; workgroup b updates
// region b % 8 only (an XCD's L2 then holds its region: gfx950 deals workgroups round-robin to the
// 8 XCDs) or any region (mode 1).  Reports G atomics/s for region sizes 1, 2, 4, 8 MiB per XCD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ __launch_bounds__(256) void k_amin(uint32_t* __restrict__ tab, int64_t cells, int64_t per_wg, int mode,
                                               uint64_t seed) {
    const int region = mode == 0 ? (int)(blockIdx.x & 7) : 0;
    const int64_t span = mode == 0 ? cells : cells * 8;
    uint32_t* t = tab + (int64_t)region * (mode == 0 ? cells : 0);
    for (int64_t i = threadIdx.x; i < per_wg; i += 256) {
        const uint64_t k = seed + (uint64_t)blockIdx.x * (uint64_t)per_wg + (uint64_t)i;
        const uint32_t h = mix(k);
        const uint32_t c = (uint32_t)(((uint64_t)h * (uint64_t)span) >> 32);
        __hip_atomic_fetch_min(t + c, mix(k ^ 0x9E3779B97F4A7C15ULL) >> 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    const int64_t pairs = 53687091;  // C3: 2 rows x 26.8 M keys
    uint32_t* tab;
    hipMalloc(&tab, (size_t)8 * (8 << 20));
    for (int mode = 0; mode < 2; mode++)
        for (int64_t mib = 1; mib <= 8; mib *= 2) {
            const int64_t cells = mib * (1 << 20) / 4;
            for (int wgs = 2048; wgs <= 8192; wgs *= 2) {
                const int64_t per = (pairs + wgs - 1) / wgs;
                hipMemset(tab, 0xFF, (size_t)8 * cells * 4);
                hipLaunchKernelGGL(k_amin, dim3(wgs), dim3(256), 0, 0, tab, cells, per, mode, 1ull);
                hipEvent_t a, b;
                hipEventCreate(&a);
                hipEventCreate(&b);
                hipEventRecord(a);
                const int reps = 5;
                for (int r = 0; r < reps; r++)
                    hipLaunchKernelGGL(k_amin, dim3(wgs), dim3(256), 0, 0, tab, cells, per, mode, (uint64_t)(r + 2) << 40);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                ms /= reps;
                printf("mode %s  region %lld MiB/XCD  wgs %5d  %8.1f us  %6.1f G atomics/s\n",
                       mode == 0 ? "xcd-affine" : "any-region", (long long)mib, wgs, ms * 1e3,
                       (double)per * wgs / (ms * 1e-3) / 1e9);
            }
        }
    return 0;
}
