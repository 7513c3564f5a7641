// Microbenchmark (profiling aid): issue cost of the compare-exchange building blocks on gfx950.
// Each kernel runs 16 independent chains per lane; reported: ns per wave-op-group per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 256
template <int KIND>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned seed) {
    unsigned v[16];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = seed * (threadIdx.x + 1) * (i + 7);
    const unsigned sel = (lane & 4) ? 0xFFFFFFFFu : 0u;
    const int bpa = (lane ^ 4) << 2;
    for (int it = 0; it < N_ITER; it++) {
        if constexpr (KIND == 9 || KIND == 10) {
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
#if __has_builtin(__builtin_amdgcn_permlane32_swap)
                auto r = KIND == 9 ? __builtin_amdgcn_permlane32_swap(v[i], v[i + 1], false, false)
                                   : __builtin_amdgcn_permlane16_swap(v[i], v[i + 1], false, false);
                unsigned a = r[0], b = r[1];
                v[i] = min(a, b);
                v[i + 1] = max(a, b);
#endif
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            unsigned a = v[i];
            if constexpr (KIND == 0) {  // v_min (1 op)
                v[i] = min(a, v[(i + 1) & 15]);
            } else if constexpr (KIND == 1) {  // med3 (1 VOP3 op)
                v[i] = min(max(a, v[(i + 3) & 15]), max(min(a, v[(i + 3) & 15]), sel));
            } else if constexpr (KIND == 2) {  // dpp mov + med3
                unsigned p = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0xB1, 0xF, 0xF, true);
                v[i] = min(max(a, p), max(min(a, p), sel));
            } else if constexpr (KIND == 3) {  // ds_swizzle xor4 + med3
                unsigned p = (unsigned)__builtin_amdgcn_ds_swizzle((int)a, (4 << 10) | 0x1F);
                v[i] = min(max(a, p), max(min(a, p), sel));
            } else if constexpr (KIND == 4) {  // ds_bpermute + med3
                unsigned p = (unsigned)__builtin_amdgcn_ds_bpermute(bpa, (int)a);
                v[i] = min(max(a, p), max(min(a, p), sel));
            } else if constexpr (KIND == 5) {  // min+max pair on two regs (in-register CE / 2 elems)
                if (i & 1) continue;
                unsigned b = v[i + 1];
                v[i] = min(a, b);
                v[i + 1] = max(a, b);
            } else if constexpr (KIND == 6) {  // ds_swizzle alone
                v[i] = (unsigned)__builtin_amdgcn_ds_swizzle((int)a, (4 << 10) | 0x1F);
            } else if constexpr (KIND == 7) {  // ds_bpermute alone
                v[i] = (unsigned)__builtin_amdgcn_ds_bpermute(bpa, (int)a);
            } else if constexpr (KIND == 8) {  // dpp-fused min (v_min_u32_dpp) 
                unsigned p = (unsigned)__builtin_amdgcn_mov_dpp((int)v[(i + 1) & 15], 0xB1, 0xF, 0xF, true);
                v[i] = min(a, p);
            } else if constexpr (KIND == 11) {  // cndmask select
                v[i] = (lane & 2) ? a : v[(i + 5) & 15];
            } else if constexpr (KIND == 12) {  // min3
                v[i] = min(min(a, v[(i + 1) & 15]), v[(i + 2) & 15]);
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
    const int blocks = 256 * 16;
    unsigned* d;
    hipMalloc(&d, sizeof(unsigned) * 256 * blocks);
    const double groups = (double)blocks * 4 * N_ITER * 16 / 256;  // per-CU wave element-slots
    const char* names[] = {"v_min", "med3", "dpp_mov+med3", "swizzle+med3", "bpermute+med3",
                           "min+max pair (per elem)", "swizzle alone", "bpermute alone",
                           "dpp-fused min", "permlane32_swap+min/max", "permlane16_swap+min/max",
                           "cndmask", "min3"};
    float t[13] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks),
                   run<4>(d, blocks), run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks),
                   run<8>(d, blocks), run<9>(d, blocks), run<10>(d, blocks), run<11>(d, blocks),
                   run<12>(d, blocks)};
    for (int k = 0; k < 13; k++)
        printf("%-26s %8.3f ms  %6.3f ns per wave-element-slot per CU (%.2f clk @2.4GHz)\n", names[k], t[k],
               t[k] * 1e6 / groups, t[k] * 1e6 / groups * 2.4);
    return 0;
}
