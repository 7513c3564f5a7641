// Microbenchmark (profiling aid): the bucketed MinMaxSketch insert's scatter (k_mm_scatter in
// skml_sparse.hip) at the C3 shape (26.8 M keys, 2 rows, colRatio 0.3), against variants that
// drop one cost at a time: coalesced instead of scattered pair stores, and no input loads.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I sketchml_amd/csrc -o tools/ubench/scatter tools/ubench/scatter.hip
#include "../../sketchml_amd/csrc/skml_sparse.hip"

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

// VARIANT 1: pair stores coalesced (pairs[r * n + i]); 2: cells from a hash of i, no loads
template <int VARIANT>
__global__ __launch_bounds__(kMmThreads) void k_scatter_v(const int32_t* __restrict__ gkeys,
                                                          const int32_t* __restrict__ gbins, int64_t n,
                                                          const uint64_t* __restrict__ bucket_base, int nbuckets,
                                                          uint64_t* __restrict__ pairs,
                                                          const int32_t* __restrict__ cells_in,
                                                          const uint32_t* __restrict__ tile_off, int rows, int zero,
                                                          int64_t ncells) {
    extern __shared__ uint64_t dyn64[];
    uint64_t* dstb = dyn64;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(dyn64 + nbuckets);
    for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) cnt[j] = 0;
    const uint32_t* row = tile_off + (int64_t)blockIdx.x * nbuckets;
    for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) dstb[j] = bucket_base[j] + row[j];
    __syncthreads();
    const int64_t c0 = (int64_t)blockIdx.x * kMmChunk, c1 = std::min<int64_t>(n, c0 + kMmChunk);
    for (int64_t base = c0; base < c1; base += kMmBatch * kMmThreads) {
        int32_t key[kMmBatch], bin[kMmBatch];
        int64_t idx[kMmBatch];
#pragma unroll
        for (int u = 0; u < kMmBatch; u++) {
            const int64_t i = base + u * kMmThreads + threadIdx.x;
            idx[u] = i < c1 ? i : c1 - 1;
            if (VARIANT == 2) {
                key[u] = (int32_t)idx[u];
                bin[u] = (int32_t)(idx[u] & 255);
            } else {
                key[u] = gkeys[idx[u]];
                bin[u] = gbins[idx[u]];
            }
        }
        for (int r = 0; r < rows; r++) {
            int32_t cell[kMmBatch];
#pragma unroll
            for (int u = 0; u < kMmBatch; u++)
                cell[u] = VARIANT == 2 ? (int32_t)(((uint32_t)(idx[u] * 2654435761u + r * 40503u)) % (uint32_t)ncells)
                                       : cells_in[(int64_t)r * n + idx[u]];
#pragma unroll
            for (int u = 0; u < kMmBatch; u++) {
                if (base + u * kMmThreads + threadIdx.x >= c1) continue;
                const int b = cell[u] >> kMmBucketBits;
                const uint64_t dst = dstb[b] + atomicAdd(&cnt[b], 1u);
                const uint64_t v = mm_pair(key[u], bin[u], zero, cell[u]);
                if (VARIANT == 1) pairs[(int64_t)r * n + idx[u]] = v + dst;  // dst kept live
                else pairs[dst] = v;
            }
        }
    }
}

int main() {
    const int64_t n = 26844167;
    const int rows = 2;
    const double ratio = 0.3;
    std::vector<int32_t> hk(n), hb(n);
    uint64_t s = 88172645463325252ull;
    int32_t k = 0;
    for (int64_t i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        k += 1 + (int32_t)(s % 19);
        hk[i] = k;
        hb[i] = (int32_t)((s >> 20) % 129);
    }
    SpGroups g{};
    const int G = 8;
    const int hid[8][2] = {{3, 5}, {0, 6}, {1, 7}, {2, 4}, {5, 3}, {6, 0}, {7, 1}, {4, 2}};
    g.G = G;
    g.rows = rows;
    g.zero = 64;
    g.bin_num = 129;
    int64_t ncell_tot = 0;
    for (int q = 0; q <= G; q++) g.gstart[q] = n * q / G;
    for (int q = 0; q < G; q++) {
        const int64_t m = g.gstart[q + 1] - g.gstart[q];
        g.cols[q] = (int32_t)std::ceil(m * ratio);
        g.inv_cols[q] = 1.0 / g.cols[q];
        g.tab_off[q] = ncell_tot;
        ncell_tot += (int64_t)rows * g.cols[q];
        g.hash_ids[q][0] = hid[q][0];
        g.hash_ids[q][1] = hid[q][1];
    }
    g.ncells = ncell_tot;
    const int nbuckets = (int)((g.ncells + kMmCellsPerBucket - 1) / kMmCellsPerBucket);
    const int64_t tiles = sp_tiles(n, kMmChunkElems);
    int32_t *gk, *gb, *cells;
    uint8_t* need;
    uint32_t *small, *tile_off;
    uint64_t *bucket, *pairs;
    SpGroups* gd;
    const size_t npairs = (size_t)rows * n + (size_t)15 * tiles * nbuckets;
    CK(hipMalloc(&gk, 4 * n));
    CK(hipMalloc(&gb, 4 * n));
    CK(hipMalloc(&cells, 4 * n * rows));
    CK(hipMalloc(&need, n));
    CK(hipMalloc(&small, 4 * (kMaxGroups * kDeltaHist + 64)));
    CK(hipMalloc(&tile_off, 4 * tiles * nbuckets));
    CK(hipMalloc(&bucket, 8 * (2 * nbuckets + 2)));
    CK(hipMalloc(&pairs, 8 * npairs));
    CK(hipMalloc(&gd, sizeof(SpGroups)));
    CK(hipMemcpy(gk, hk.data(), 4 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(gb, hb.data(), 4 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(gd, &g, sizeof(g), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto fn) {
        float best = 1e30f;
        for (int r = 0; r < 6; r++) {
            CK(hipEventRecord(a));
            fn();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r) best = ms < best ? ms : best;
        }
        printf("%-40s %8.1f us\n", name, best * 1e3);
    };
    auto prep = [&]() {
        CK(hipMemset(small, 0, 4 * (kMaxGroups * kDeltaHist + 64)));
        CK(hipMemset(bucket, 0, 8 * (2 * nbuckets + 2)));
        CK(launch_group_prep(0, gk, n, gd, need, small, small + kMaxGroups * kDeltaHist, bucket, nbuckets, cells,
                             tile_off));
        CK(launch_scan_cols(0, bucket, nbuckets, 1));
    };
    timeit("group_prep + bucket scan", prep);
    prep();
    CK(hipDeviceSynchronize());
    timeit("unstaged k_mm_scatter", [&]() {
        hipLaunchKernelGGL(k_mm_scatter, dim3((unsigned)tiles), dim3(kMmThreads), 12 * (size_t)nbuckets, 0, gk, gb, n,
                           gd, bucket, reinterpret_cast<unsigned long long*>(bucket + nbuckets + 1), nbuckets, pairs,
                           cells, tile_off);
    });
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mm_scatter_staged<1024>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mm_scatter_staged<256>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("staged 1024 thr", [&]() {
        hipLaunchKernelGGL(k_mm_scatter_staged<1024>, dim3((unsigned)tiles), dim3(1024),
                           10 * 8 * 1024 + 16 * (size_t)nbuckets + 4, 0, gk, gb, n, gd, bucket, nbuckets, pairs, cells,
                           tile_off);
    });
    timeit("staged 256 thr", [&]() {
        hipLaunchKernelGGL(k_mm_scatter_staged<256>, dim3((unsigned)tiles), dim3(256),
                           10 * 8 * 256 + 16 * (size_t)nbuckets + 4, 0, gk, gb, n, gd, bucket, nbuckets, pairs, cells,
                           tile_off);
    });
    timeit("k_mm_scatter (product: staged 512)", [&]() {
        CK(launch_mm_scatter(0, gk, gb, n, gd, bucket, bucket + nbuckets + 1, nbuckets, pairs, cells, tile_off));
    });
    const size_t lds = 12 * (size_t)nbuckets;
    timeit("coalesced pair stores", [&]() {
        hipLaunchKernelGGL(k_scatter_v<1>, dim3((unsigned)tiles), dim3(kMmThreads), lds, 0, gk, gb, n, bucket,
                           nbuckets, pairs, cells, tile_off, rows, 64, g.ncells);
    });
    timeit("no input loads (cells hashed from i)", [&]() {
        hipLaunchKernelGGL(k_scatter_v<2>, dim3((unsigned)tiles), dim3(kMmThreads), lds, 0, gk, gb, n, bucket,
                           nbuckets, pairs, cells, tile_off, rows, 64, g.ncells);
    });
    timeit("k_mm_bucket", [&]() { CK(launch_mm_bucket(0, pairs, bucket, nbuckets, gd, cells)); });
    printf("n %lld rows %d nbuckets %d tiles %lld\n", (long long)n, rows, nbuckets, (long long)tiles);
    return 0;
}
