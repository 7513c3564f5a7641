// Probe (gfx950): do the 3-input v_min3_f32 / v_med3_f32 / v_max3_f32 order -0.0 before +0.0 as
// v_min_f32 / v_max_f32 do (Arrays.sort's total order, tools/ubench/zero_minmax.hip), for every
// operand order?  And the 3-input 4-sorter the leaf's network base uses (8 ops instead of 5
// comparators = 10): p = min(a,b), q = max(a,b); o0 = min3(p,c,d), o3 = max3(q,c,d),
// o1 = min(med3(p,c,d), q), o2 = max(med3(q,c,d), p) -- checked on every 4-tuple over
// {-inf, -2, -1, -0, +0, 1, 2, +inf} against the total-order sort.  Also v_minimum3_f32 with |.|
// operands (the leaf's zero / NaN detector): the result is 0 iff a zero is present, NaN iff a
// NaN is present.  Prints one line per check and "ALL OK" at the end.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__device__ __forceinline__ float mn(float a, float b) {
    float r;
    asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float mx(float a, float b) {
    float r;
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float mn3(float a, float b, float c) {
    float r;
    asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float mx3(float a, float b, float c) {
    float r;
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float md3(float a, float b, float c) {
    float r;
    asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float minimum3_abs(float a, float b, float c) {
    float r;
    asm volatile("v_minimum3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

constexpr int kV = 8;
__global__ void k_sort4(const float* vals, unsigned* out) {  // one thread per 4-tuple
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= kV * kV * kV * kV) return;
    const float a = vals[t % kV], b = vals[(t / kV) % kV], c = vals[(t / kV / kV) % kV], d = vals[t / kV / kV / kV];
    const float p = mn(a, b), q = mx(a, b);
    out[4 * t + 0] = __float_as_uint(mn3(p, c, d));
    out[4 * t + 1] = __float_as_uint(mn(md3(p, c, d), q));
    out[4 * t + 2] = __float_as_uint(mx(md3(q, c, d), p));
    out[4 * t + 3] = __float_as_uint(mx3(q, c, d));
}

__global__ void k_three(const float* vals, unsigned* out) {  // min3 / med3 / max3 of every 3-tuple
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= kV * kV * kV) return;
    const float a = vals[t % kV], b = vals[(t / kV) % kV], c = vals[t / kV / kV];
    out[3 * t + 0] = __float_as_uint(mn3(a, b, c));
    out[3 * t + 1] = __float_as_uint(md3(a, b, c));
    out[3 * t + 2] = __float_as_uint(mx3(a, b, c));
}

__global__ void k_detect(const float* x, int n, unsigned* out) {  // minimum3 over |x| in pairs
    float acc = __builtin_inff();
    for (int i = 0; i + 1 < n; i += 2) acc = minimum3_abs(x[i], x[i + 1], acc);
    out[0] = __float_as_uint(acc);
}

static unsigned key(float f) {  // total-order key: -0.0 < +0.0
    unsigned b;
    std::memcpy(&b, &f, 4);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
static float fl(unsigned u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

int main() {
    const float h[kV] = {-__builtin_inff(), -2.0f, -1.0f, -0.0f, 0.0f, 1.0f, 2.0f, __builtin_inff()};
    float* dv;
    unsigned* dout;
    hipMalloc(&dv, sizeof(h));
    hipMalloc(&dout, sizeof(unsigned) * 4 * kV * kV * kV * kV);
    hipMemcpy(dv, h, sizeof(h), hipMemcpyHostToDevice);
    int bad = 0;
    {
        const int T = kV * kV * kV;
        hipLaunchKernelGGL(k_three, dim3((T + 63) / 64), dim3(64), 0, 0, dv, dout);
        unsigned o[3 * kV * kV * kV];
        hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
        int b3 = 0;
        for (int t = 0; t < T; t++) {
            float v[3] = {h[t % kV], h[(t / kV) % kV], h[t / kV / kV]};
            for (int i = 0; i < 3; i++)
                for (int j = i + 1; j < 3; j++)
                    if (key(v[j]) < key(v[i])) std::swap(v[i], v[j]);
            for (int r = 0; r < 3; r++)
                if (o[3 * t + r] != *reinterpret_cast<unsigned*>(&v[r])) b3++;
        }
        printf("min3/med3/max3 over %d 3-tuples with signed zeros: %d mismatches against the total order\n", T, b3);
        bad += b3;
    }
    {
        const int T = kV * kV * kV * kV;
        hipLaunchKernelGGL(k_sort4, dim3((T + 63) / 64), dim3(64), 0, 0, dv, dout);
        static unsigned o[4 * kV * kV * kV * kV];
        hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
        int b4 = 0;
        for (int t = 0; t < T; t++) {
            float v[4] = {h[t % kV], h[(t / kV) % kV], h[(t / kV / kV) % kV], h[t / kV / kV / kV]};
            for (int i = 0; i < 4; i++)
                for (int j = i + 1; j < 4; j++)
                    if (key(v[j]) < key(v[i])) std::swap(v[i], v[j]);
            for (int r = 0; r < 4; r++)
                if (o[4 * t + r] != *reinterpret_cast<unsigned*>(&v[r])) b4++;
        }
        printf("3-input 4-sorter over %d 4-tuples: %d mismatches against the total-order sort\n", T, b4);
        bad += b4;
    }
    {
        const float nan = __builtin_nanf("");
        const float cases[4][6] = {{1.0f, -2.0f, 3.0f, 0.5f, -7.0f, 4.0f},
                                   {1.0f, -2.0f, -0.0f, 0.5f, -7.0f, 4.0f},
                                   {1.0f, 0.0f, 3.0f, 0.5f, -7.0f, 4.0f},
                                   {1.0f, -2.0f, 3.0f, nan, -7.0f, 4.0f}};
        const char* what[4] = {"no zero, no NaN", "a -0.0", "a +0.0", "a NaN"};
        float* dx;
        hipMalloc(&dx, sizeof(cases[0]));
        for (int c = 0; c < 4; c++) {
            hipMemcpy(dx, cases[c], sizeof(cases[c]), hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k_detect, dim3(1), dim3(1), 0, 0, dx, 6, dout);
            unsigned r;
            hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost);
            const float f = fl(r);
            const bool flagged = !(f > 0.0f);  // zero or NaN
            const bool want = c != 0;
            printf("minimum3(|x|) detector, %-15s: result 0x%08x, flagged %d (want %d)\n", what[c], r, flagged, want);
            bad += flagged != want;
        }
        hipFree(dx);
    }
    printf(bad ? "MISMATCHES: %d\n" : "ALL OK\n", bad);
    return bad ? 1 : 0;
}
