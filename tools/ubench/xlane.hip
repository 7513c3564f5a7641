// Microbenchmark: throughput of cross-lane primitives vs plain VALU on gfx950 (profiling aid).
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 256
template <int KIND>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned seed) {
    unsigned v[16];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = seed * (threadIdx.x + 1) * (i + 7);
    const unsigned sel = (lane & 1) ? 0xFFFFFFFFu : 0u;
    for (int it = 0; it < N_ITER; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            unsigned a = v[i];
            if constexpr (KIND == 0) {  // plain VALU min (1 op)
                v[i] = min(a, v[(i + 1) & 15]);
            } else if constexpr (KIND == 1) {  // dpp mov (1 op)
                v[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0xB1, 0xF, 0xF, true) + 1u;
            } else if constexpr (KIND == 2) {  // dpp mov + med3 (2 ops)
                unsigned p = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0xB1, 0xF, 0xF, true);
                v[i] = min(max(a, p), max(min(a, p), sel));
            } else if constexpr (KIND == 3) {  // row_half_mirror dpp mov
                v[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0x141, 0xF, 0xF, true) + 1u;
            } else if constexpr (KIND == 4) {  // ds_swizzle xor 4
                v[i] = (unsigned)__builtin_amdgcn_ds_swizzle((int)a, (4 << 10) | 0x1F) + 1u;
            } else if constexpr (KIND == 5) {  // ds_bpermute
                v[i] = (unsigned)__builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, (int)a) + 1u;
            } else if constexpr (KIND == 6) {  // med3 only
                v[i] = min(max(a, v[(i + 3) & 15]), max(min(a, v[(i + 3) & 15]), sel));
            } else if constexpr (KIND == 7) {  // dpp min fused (v_min_u32_dpp)
                unsigned p = (unsigned)__builtin_amdgcn_mov_dpp((int)v[(i + 1) & 15], 0xB1, 0xF, 0xF, true);
                v[i] = min(a, p);
            }
        }
    }
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= v[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int K>
float run(unsigned* d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 16;  // 16 waves... 4 waves per block -> 64 waves per CU
    unsigned* d;
    hipMalloc(&d, sizeof(unsigned) * 256 * blocks);
    const double winstr = (double)blocks * 4 * N_ITER * 16;  // wave-instructions of the main op
    const char* names[] = {"v_min", "dpp_mov quad_perm", "dpp_mov+med3", "dpp row_half_mirror", "ds_swizzle", "ds_bpermute", "med3", "dpp mov + min"};
    float t[8] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks),
                  run<4>(d, blocks), run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks)};
    for (int k = 0; k < 8; k++)
        printf("%-22s %8.3f ms  %6.3f ns per 16-elem-op  -> %.1f G op-groups/s per CU\n", names[k], t[k],
               t[k] * 1e6 / (winstr / 256), winstr / 256 / (t[k] * 1e-3) / 1e9);
    return 0;
}
