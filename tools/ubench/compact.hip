// Microbenchmark (profiling aid): variants of the toSparse stream compaction (k_compact in
// skml_sparse.hip) over a 2^28-float, 10 %-dense input, to separate the costs of the ordered
// ticket, the tile size and the look-back from the streaming read itself.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench/compact tools/ubench/compact.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr uint64_t kStAgg = 1ULL << 62, kStPre = 2ULL << 62, kStMask = (1ULL << 62) - 1;
constexpr uint32_t kEpsBelowBits = 0x322BCC77u;
constexpr int kSlabs = 16;  // float4 slabs per thread

__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// MODE 0: full compaction; 1: count only (per-tile count written, no look-back, no output);
// 2: look-back without output writes
template <int THREADS, bool TICKET, int MODE, int LB = 1>
__global__ __launch_bounds__(THREADS) void k_compact_v(const float* __restrict__ x, int64_t dim,
                                                       int32_t* __restrict__ keys, float* __restrict__ vals,
                                                       uint64_t* status, unsigned* ticket, int64_t ntiles,
                                                       int64_t* nnz_out) {
    constexpr int kWaves = THREADS / 64, kTile = THREADS * 4 * kSlabs;
    __shared__ uint32_t wtot[kWaves][kSlabs];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_excl;
    constexpr int kStage = MODE == 3 ? 4096 : 1;  // staged output elements (32 KB)
    __shared__ int32_t sk[kStage];
    __shared__ float sv[kStage];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int64_t tile;
    if (TICKET) {
        if (t == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
        __syncthreads();
        tile = s_tile;
    } else {
        tile = blockIdx.x;
    }
    const int64_t base = tile * kTile;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 f[kSlabs];
    const f32x4* src = reinterpret_cast<const f32x4*>(x + base);
#pragma unroll
    for (int j = 0; j < kSlabs; j++) f[j] = __builtin_nontemporal_load(src + j * THREADS + t);
    uint64_t keep = 0;
#pragma unroll
    for (int j = 0; j < kSlabs; j++) {
        const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t a = __float_as_uint(e4[e]) & 0x7FFFFFFFu;
            keep |= (a > kEpsBelowBits && a <= 0x7F800000u) ? (1ull << (4 * j + e)) : 0ull;
        }
    }
    if (MODE == 1) {
        uint32_t c = __popcll(keep);
        for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
        if (lane == 0) wtot[w][0] = c;
        __syncthreads();
        if (t == 0) {
            uint64_t s = 0;
            for (int u = 0; u < kWaves; u++) s += wtot[u][0];
            status[tile] = s;
        }
        return;
    }
    uint64_t P[kSlabs / 4];
#pragma unroll
    for (int k = 0; k < kSlabs / 4; k++) {
        uint64_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) v |= (uint64_t)__popcll((keep >> (16 * k + 4 * q)) & 15ull) << (16 * q);
        P[k] = v;
    }
    uint64_t own[kSlabs / 4];
#pragma unroll
    for (int k = 0; k < kSlabs / 4; k++) own[k] = P[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int k = 0; k < kSlabs / 4; k++) {
            const uint64_t y = __shfl_up(P[k], off, 64);
            if (lane >= off) P[k] += y;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int j = 0; j < kSlabs; j++) wtot[w][j] = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
    }
    __syncthreads();
    uint32_t slab_pre[kSlabs];
    uint32_t tile_total = 0;
#pragma unroll
    for (int j = 0; j < kSlabs; j++) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int u = 0; u < kWaves; u++) {
            const uint32_t c = wtot[u][j];
            before += u < w ? c : 0u;
            tot += c;
        }
        slab_pre[j] = tile_total + before;
        tile_total += tot;
    }
    if (t < 64) {
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) st_status(&status[0], kStPre | tile_total);
        } else {
            if (lane == 0) st_status(&status[tile], kStAgg | tile_total);
            int64_t p = tile - 1;
            while (true) {  // LB loads per lane: a window of 64 * LB predecessors per step
                uint64_t sv[LB];
#pragma unroll
                for (int k = 0; k < LB; k++) {
                    const int64_t idx = p - (k * 64 + lane);
                    sv[k] = idx >= 0 ? ld_status(&status[idx]) : kStPre;
                }
                while (true) {
                    bool unk = false;
#pragma unroll
                    for (int k = 0; k < LB; k++) unk |= (sv[k] & ~kStMask) == 0;
                    if (!__ballot(unk)) break;
                    __builtin_amdgcn_s_sleep(1);
#pragma unroll
                    for (int k = 0; k < LB; k++)
                        if ((sv[k] & ~kStMask) == 0) sv[k] = ld_status(&status[p - (k * 64 + lane)]);
                }
                int stop = 64 * LB - 1;
                bool found = false;
#pragma unroll
                for (int k = 0; k < LB; k++) {
                    const uint64_t pre = __ballot((sv[k] & ~kStMask) == kStPre);
                    if (!found && pre) {
                        stop = k * 64 + __ffsll((unsigned long long)pre) - 1;
                        found = true;
                    }
                }
                uint64_t contrib = 0;
#pragma unroll
                for (int k = 0; k < LB; k++) contrib += (k * 64 + lane) <= stop ? (sv[k] & kStMask) : 0;
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) contrib += __shfl_xor(contrib, off, 64);
                excl += contrib;
                if (found) break;
                p -= 64 * LB;
            }
            if (lane == 0) st_status(&status[tile], kStPre | (excl + tile_total));
        }
        if (lane == 0) {
            s_excl = excl;
            if (tile == ntiles - 1) *nnz_out = (int64_t)(excl + tile_total);
        }
    }
    __syncthreads();
    if (MODE == 2) return;  // look-back without the output writes
    const int64_t out0 = (int64_t)s_excl;
    if (MODE == 3 && tile_total <= kStage) {  // stage the tile's output in LDS, then coalesced stores
#pragma unroll
        for (int j = 0; j < kSlabs; j++) {
            const uint32_t incl = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
            const uint32_t mine = (uint32_t)(own[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
            uint32_t pos = slab_pre[j] + incl - mine;
            const int32_t e0 = (int32_t)(base + 4 * ((int64_t)j * THREADS + t));
            const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
            for (int e = 0; e < 4; e++)
                if ((keep >> (4 * j + e)) & 1ull) {
                    sk[pos] = e0 + e;
                    sv[pos] = e4[e];
                    pos++;
                }
        }
        __syncthreads();
        for (uint32_t q = t; q < tile_total; q += THREADS) {
            keys[out0 + q] = sk[q];
            vals[out0 + q] = sv[q];
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < kSlabs; j++) {
        const uint64_t incl = (P[j >> 2] >> (16 * (j & 3))) & 0xFFFFull;
        const uint64_t mine = (own[j >> 2] >> (16 * (j & 3))) & 0xFFFFull;
        int64_t pos = out0 + slab_pre[j] + (int64_t)(incl - mine);
        const int32_t e0 = (int32_t)(base + 4 * ((int64_t)j * THREADS + t));
        const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
        for (int e = 0; e < 4; e++)
            if ((keep >> (4 * j + e)) & 1ull) {
                keys[pos] = e0 + e;
                vals[pos] = e4[e];
                pos++;
            }
    }
}

template <int THREADS, bool TICKET, int MODE, int LB = 1>
float run(const char* name, const float* x, int64_t dim, int32_t* keys, float* vals, uint64_t* status,
          int64_t* nnz, int reps) {
    constexpr int64_t kTile = THREADS * 4 * kSlabs;
    const int64_t tiles = dim / kTile;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps + 1; r++) {
        CK(hipMemset(status, 0, sizeof(uint64_t) * (tiles + 8)));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_compact_v<THREADS, TICKET, MODE, LB>), dim3((unsigned)tiles), dim3(THREADS), 0, 0, x, dim,
                           keys, vals, status, reinterpret_cast<unsigned*>(status + tiles), tiles, nnz);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r) {
            best = ms < best ? ms : best;
            sum += ms;
        }
    }
    int64_t h = -1;
    CK(hipMemcpy(&h, nnz, sizeof(h), hipMemcpyDeviceToHost));
    printf("%-34s best %8.1f us  avg %8.1f us  %7.1f GB/s (dense read)  nnz %lld\n", name, best * 1e3, sum / reps * 1e3,
           4.0 * dim / (best * 1e-3) / 1e9, (long long)h);
    return best;
}

__global__ void k_fill(float* x, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        x[i] = (h % 10u == 0u) ? (float)(h >> 8) * 1e-6f + 0.5f : 0.0f;
    }
}

int main(int argc, char** argv) {
    const int64_t dim = (int64_t)1 << 28;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    float *x, *vals;
    int32_t* keys;
    uint64_t* status;
    int64_t* nnz;
    CK(hipMalloc(&x, 4 * dim));
    CK(hipMalloc(&keys, 4 * dim / 8));
    CK(hipMalloc(&vals, 4 * dim / 8));
    CK(hipMalloc(&status, sizeof(uint64_t) * (dim / 4096 + 64)));
    CK(hipMalloc(&nnz, 64));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, dim, 12345u);
    CK(hipDeviceSynchronize());
    run<256, true, 0>("ticket  256 thr 16K tile", x, dim, keys, vals, status, nnz, reps);
    run<256, false, 0>("blockid 256 thr 16K tile", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 0, 2>("ticket  256 thr 16K tile LB128", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 0, 4>("ticket  256 thr 16K tile LB256", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 0, 8>("ticket  256 thr 16K tile LB512", x, dim, keys, vals, status, nnz, reps);
    run<512, true, 0>("ticket  512 thr 32K tile", x, dim, keys, vals, status, nnz, reps);
    run<512, true, 0, 4>("ticket  512 thr 32K tile LB256", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 3>("ticket 256 LDS-staged output", x, dim, keys, vals, status, nnz, reps);
    run<256, false, 3>("blockid 256 LDS-staged output", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 2>("ticket 256 no writes", x, dim, keys, vals, status, nnz, reps);
    run<256, true, 2, 4>("ticket 256 no writes LB256", x, dim, keys, vals, status, nnz, reps);
    run<256, false, 1>("count only 256 thr (read bound)", x, dim, keys, vals, status, nnz, reps);
    run<1024, false, 1>("count only 1024 thr (read bound)", x, dim, keys, vals, status, nnz, reps);
    return 0;
}
