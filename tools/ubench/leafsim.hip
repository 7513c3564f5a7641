// Microbenchmark (what-if, results deliberately wrong): the leaf's level-0 chunk sort (k_leaf2's
// sort_regs_oddeven<32> + sort_lanes_upto128 + merge_group_compact) as it runs today, against
// the same instruction mix with its 6 cross-lane stages (DPP move + med3 per element) replaced by
// in-register stages (one op per element) plus 5 LDS transposes of the 32 registers.  If the
// second is markedly faster, an LDS-transposing leaf is worth building.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I sketchml_amd/csrc -o tools/ubench/leafsim tools/ubench/leafsim.hip
#include "../../sketchml_amd/csrc/skml_sketch.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

using namespace skml;

// one in-register stage standing in for a cross-lane one: 16 compare-exchanges
template <int D>
__device__ __forceinline__ void reg_stage(float (&v)[32]) {
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const int j = i ^ D;
        if (j > i) ce(v[i], v[j]);
    }
}

// a register transpose through LDS: 32 b32 writes, 32 b32 reads (lane-rotated pattern)
__device__ __forceinline__ void lds_transpose(float (&v)[32], float* buf, int lane, int rot) {
#pragma unroll
    for (int r = 0; r < 32; r++) buf[r * 64 + lane] = v[r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 32; r++) v[r] = buf[((r + rot) & 31) * 64 + ((lane + r) & 63)];
    __builtin_amdgcn_wave_barrier();
}

// the same with 16-byte LDS accesses (8 writes, 8 reads)
__device__ __forceinline__ void lds_transpose4(float (&v)[32], float* buf, int lane, int rot) {
    float4* b4 = reinterpret_cast<float4*>(buf);
#pragma unroll
    for (int q = 0; q < 8; q++) b4[q * 64 + lane] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const float4 t = b4[((q + rot) & 7) * 64 + ((lane + 8 * q + rot) & 63)];
        v[4 * q] = t.x, v[4 * q + 1] = t.y, v[4 * q + 2] = t.z, v[4 * q + 3] = t.w;
    }
    __builtin_amdgcn_wave_barrier();
}

template <int MODE>
__global__ __launch_bounds__(256, 4) void k_sim(const float* __restrict__ x, int64_t chunks, float* out) {
    __shared__ float buf[4][32 * 64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + wave;
    const int64_t c_tile = tile * 64;
    if (c_tile >= chunks) return;
    uint32_t acc = 0;
#pragma unroll 1
    for (int round = 0; round < 8; round++) {
        set_prio_by_progress(round, 8);
        const int64_t chunk = c_tile + round * 8 + (lane >> 3);
        const float4* src = reinterpret_cast<const float4*>(x + chunk * kChunk);
        float4 f[8];
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = src[j * 8 + (lane & 7)];
        float v[32];
        uint64_t zmask = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                zmask |= __ballot(is_class(e4[e], 0x63));
                v[j * 4 + e] = e4[e];
            }
        }
        acc ^= (uint32_t)zmask;
        float w1[16];
        sort_regs_oddeven<32>(v);
        if constexpr (MODE == 0) {
            sort_lanes_upto128<32, 64>(v, lane);
            merge_group_compact<32>(v, w1, lane, (round & 1) != 0);
        } else if constexpr (MODE == 2) {
            float* b = buf[wave];
            lds_transpose4(v, b, lane, 1);
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            lds_transpose4(v, b, lane, 2);
            reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v);
            lds_transpose4(v, b, lane, 3);
            reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v);
            lds_transpose4(v, b, lane, 5);
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            lds_transpose4(v, b, lane, 7);
            halfclean_regs_compact<32>(v, w1, (round & 1) != 0);
        } else if constexpr (MODE == 3) {  // in-register stages only (no data movement): the VALU floor
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v);
            reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v);
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            halfclean_regs_compact<32>(v, w1, (round & 1) != 0);
        } else {
            float* b = buf[wave];
            // k = 6: 6 stages, k = 7: 7, k = 8: 8 (the last fused with the compaction)
            lds_transpose(v, b, lane, 1);
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            lds_transpose(v, b, lane, 2);
            reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v);
            lds_transpose(v, b, lane, 3);
            reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v); reg_stage<16>(v); reg_stage<8>(v);
            lds_transpose(v, b, lane, 5);
            reg_stage<16>(v); reg_stage<8>(v); reg_stage<4>(v); reg_stage<2>(v); reg_stage<1>(v);
            lds_transpose(v, b, lane, 7);
            halfclean_regs_compact<32>(v, w1, (round & 1) != 0);
        }
#pragma unroll
        for (int r = 0; r < 16; r++) acc ^= __float_as_uint(w1[r]);
    }
    out[tile * 64 + lane] = __uint_as_float(acc);
}

template <int MODE>
float run(const char* name, const float* x, int64_t chunks, float* out) {
    const unsigned grid = (unsigned)(chunks / 64 / 4);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 11; r++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_sim<MODE>, dim3(grid), dim3(256), 0, 0, x, chunks, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r) best = ms < best ? ms : best;
    }
    printf("%-48s %8.1f us\n", name, best * 1e3);
    return best;
}

__global__ void k_fill(float* x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        x[i] = (float)(int32_t)h * 1e-9f;
    }
}

int main() {
    const int64_t n = (int64_t)1 << 26, chunks = n / kChunk;
    float *x, *out;
    CK(hipMalloc(&x, 4 * n));
    CK(hipMalloc(&out, 4 * (chunks + 64)));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, n);
    CK(hipDeviceSynchronize());
    run<0>("level 0 as today (DPP + med3 cross-lane stages)", x, chunks, out);
    run<1>("level 0 with LDS transposes b32 (what-if)", x, chunks, out);
    run<2>("level 0 with LDS transposes b128 (what-if)", x, chunks, out);
    run<3>("level 0 all in-register, no moves (floor)", x, chunks, out);
    return 0;
}
