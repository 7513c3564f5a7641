// Microbenchmark (profiling aid): streaming ceilings on gfx950 for the quantize shape
// (read 4 B, write 1 B per element) against read-only and copy.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(256) void kern(const float* __restrict__ x, int64_t n, uint8_t* __restrict__ out,
                                            float* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4, wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t tiles = n / 1024;
    float acc = 0.f;
    for (int64_t t = wid; t < tiles; t += nw) {
        const f32x4* src = reinterpret_cast<const f32x4*>(x + t * 1024);
        f32x4 f[4];
#pragma unroll
        for (int j = 0; j < 4; j++) f[j] = KIND & 1 ? __builtin_nontemporal_load(src + j * 64 + lane) : src[j * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (KIND & 2) {
                const uint32_t w = (uint32_t)(f[j].x > 0.f) | ((uint32_t)(f[j].y > 0.f) << 8) |
                                   ((uint32_t)(f[j].z > 0.f) << 16) | ((uint32_t)(f[j].w > 0.f) << 24);
                uint32_t* d = reinterpret_cast<uint32_t*>(out + t * 1024 + j * 256 + lane * 4);
                if (KIND & 4) __builtin_nontemporal_store(w, d);
                else *d = w;
            } else {
                acc += f[j].x + f[j].y + f[j].z + f[j].w;
            }
        }
    }
    if (acc == 12345.f) sink[0] = acc;
}

template <int K>
float run(const float* x, int64_t n, uint8_t* o, float* s, int grid) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern<K>, dim3(grid), dim3(256), 0, 0, x, n, o, s);
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(kern<K>, dim3(grid), dim3(256), 0, 0, x + (r % 4) * n, n, o, s);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 10 * 1000.f;
}

int main() {
    const int64_t n = 1ll << 26;
    float* x;
    uint8_t* o;
    float* s;
    (void)hipMalloc(&x, 4 * n * 4);
    (void)hipMalloc(&o, n);
    (void)hipMalloc(&s, 64);
    (void)hipMemset(x, 0, 4 * n * 4);
    const int grids[] = {1024, 2048, 4096, 16384};
    for (int g : grids) {
        printf("grid %5d: read %6.1f us  read-nt %6.1f  rd+wr1B %6.1f  rd-nt+wr1B %6.1f  rd-nt+wr1B-nt %6.1f\n", g,
               run<0>(x, n, o, s, g), run<1>(x, n, o, s, g), run<2>(x, n, o, s, g), run<3>(x, n, o, s, g),
               run<7>(x, n, o, s, g));
    }
    return 0;
}
