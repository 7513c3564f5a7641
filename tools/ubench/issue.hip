// Microbenchmark (profiling aid): VALU issue cost on gfx950 of the building blocks a sorting
// network uses, at 1 / 2 / 4 / 8 waves per SIMD.  Each lane runs 32 independent chains of one
// instruction pattern; reported: SIMD cycles per wave-instruction (in-kernel clock from
// s_memtime / s_memrealtime) and the kernel's wall time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#define N_ITER 4096
#define NV 32

struct Stamp {
    unsigned long long t0, t1, r0, r1;
};

template <int KIND>
__global__ __launch_bounds__(256) void kern(float* out, Stamp* st, float seed) {
    extern __shared__ float pad[];
    float v[NV];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = seed * (float)(threadIdx.x + 1) * (float)(i + 7) - 3.0f;
    const float sel = (lane & 1) ? __builtin_inff() : -__builtin_inff();
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < N_ITER; it++) {
#pragma unroll
        for (int i = 0; i < NV; i++) {
            float a = v[i], b = v[(i + 1) & (NV - 1)], r = a;
            if constexpr (KIND == 0) { asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 1) { asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 2) { asm volatile("v_min_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 3) { asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 4) { asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 5) { asm volatile("v_min_i32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 6) { asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 7) { asm volatile("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 8) { asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 9) { asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 10) { asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 11) { asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 12) { asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(b)); }
            else if constexpr (KIND == 13) { asm volatile("v_min_u32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 14) { asm volatile("v_add_u32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 15) { asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 16) { asm volatile("v_pk_max_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 17) { asm volatile("v_min_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 18) { asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 19) { asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 20) { asm volatile("v_max_f32_e64 %0, -%1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 21) { asm volatile("v_cmp_lt_u32_e64 s[40:41], %1, %2" : "=v"(r) : "v"(a), "v"(b) : "s40", "s41"); }
            else if constexpr (KIND == 22) { asm volatile("v_cndmask_b32_e64 %0, %1, %2, s[40:41]" : "=v"(r) : "v"(a), "v"(b) : "s40", "s41"); }
            else if constexpr (KIND == 23) { asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 24) { asm volatile("v_sad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 25) { asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(sel)); }
            else if constexpr (KIND == 26) { asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a) : "v"(b)); r = a; }
            else if constexpr (KIND == 27) { asm volatile("v_max_f32_dpp %0, -%1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(b), "v"(a)); }
            else if constexpr (KIND == 28) { asm volatile("v_max_f32_dpp %0, -%1, %2 row_mirror row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(b), "v"(a)); }
            else if constexpr (KIND == 30) { asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 31) { asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2" : "=v"(r) : "v"(a), "v"(b) : "vcc"); }
            else if constexpr (KIND == 32) { asm volatile("v_cndmask_b32_e32 %0, %1, %2, vcc" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 33) { asm volatile("v_min_i16_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 34) { asm volatile("v_max_u16_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 35) { asm volatile("v_sub_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 36) { asm volatile("v_mov_b32_e32 %0, %1" : "=v"(r) : "v"(b)); }
            else if constexpr (KIND == 37) { asm volatile("v_min_f32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD" : "=v"(r) : "v"(a), "v"(b)); }
            else if constexpr (KIND == 38) {  // compare-exchange as v_cmp_e32 + 2 x v_cndmask_e32 (3 instructions per 2 values)
                if (i & 1) { r = a; }
                else {
                    float lo, hi;
                    asm volatile("v_cmp_lt_f32_e32 vcc, %2, %3\n\tv_cndmask_b32_e32 %0, %3, %2, vcc\n\tv_cndmask_b32_e32 %1, %2, %3, vcc"
                                 : "=&v"(lo), "=&v"(hi) : "v"(a), "v"(b) : "vcc");
                    r = lo;
                    v[(i + 1) & (NV - 1)] = hi;
                }
            }
            else if constexpr (KIND == 39) {  // compare-exchange as v_min_f32 + v_max_f32 (2 instructions per 2 values)
                if (i & 1) { r = a; }
                else {
                    float lo, hi;
                    asm volatile("v_min_f32 %0, %2, %3\n\tv_max_f32 %1, %2, %3" : "=&v"(lo), "=&v"(hi) : "v"(a), "v"(b));
                    r = lo;
                    v[(i + 1) & (NV - 1)] = hi;
                }
            }
            else if constexpr (KIND == 40) { asm volatile("v_cmp_gt_u32_e32 vcc, %1, %2" : "=v"(r) : "v"(a), "v"(b) : "vcc"); }
            else if constexpr (KIND == 29) {  // two values per instruction: count as 2 per pair
                typedef float f2v __attribute__((ext_vector_type(2)));
                f2v p = {a, b}, q = {sel, sel};
                if (i & 1) { asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(p) : "v"(p), "v"(q)); r = p.x + 0.f; }
                else { asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); }
            }
            v[i] = r;
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) acc += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (lane == 0) st[blockIdx.x * 4 + (threadIdx.x >> 6)] = Stamp{t0, t1, r0, r1};
    if (acc == 12345.f) pad[threadIdx.x] = acc;
}

static const char* g_filter = nullptr;
template <int K>
void run(const char* name, float* d, Stamp* st, Stamp* hst, int cus) {
    if (g_filter && !strstr(name, g_filter)) return;
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;
        const size_t lds = (160 * 1024) / wps - 1024;
        hipFuncSetAttribute((const void*)kern<K>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), lds, 0, d, st, 1.0001f);
        hipEventRecord(a);
        const int reps = 5;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), lds, 0, d, st, 1.0001f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        hipMemcpy(hst, st, sizeof(Stamp) * blocks * 4, hipMemcpyDeviceToHost);
        double cyc = 0, real = 0;
        for (int i = 0; i < blocks * 4; i++) {
            cyc += (double)(hst[i].t1 - hst[i].t0);
            real += (double)(hst[i].r1 - hst[i].r0);
        }
        cyc /= blocks * 4;
        real /= blocks * 4;
        const double ghz = cyc / real * 0.1;  // s_memrealtime runs at 100 MHz
        // per wave (the compare-exchange kinds: instructions per 2 values x NV / 2 per iteration)
        const double instr = (double)N_ITER * (K == 38 ? NV / 2 * 3 : K == 39 ? NV : NV);
        // per SIMD: wps waves, each `instr` instructions, over `cyc` cycles
        printf("%-28s waves/SIMD %d  %6.2f cyc/instr/SIMD (in-wave)  %6.2f (wall)  clk %.2f GHz  %.3f ms\n", name,
               wps, cyc / (instr * wps), ms * 1e-3 * ghz * 1e9 / (instr * wps), ghz, ms);
    }
}

int main(int argc, char** argv) {
    int dev = 0;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    float* d;
    Stamp *st, *hst;
    hipMalloc(&d, sizeof(float) * 256 * cus * 8);
    hipMalloc(&st, sizeof(Stamp) * cus * 8 * 4);
    hst = (Stamp*)malloc(sizeof(Stamp) * cus * 8 * 4);
    if (argc > 1) g_filter = argv[1];
    printf("CUs %d\n", cus);
    run<0>("v_min_f32", d, st, hst, cus);
    run<30>("v_max_f32", d, st, hst, cus);
    run<1>("v_med3_f32", d, st, hst, cus);
    run<2>("v_min_u32", d, st, hst, cus);
    run<3>("v_med3_u32", d, st, hst, cus);
    run<4>("v_min3_u32", d, st, hst, cus);
    run<5>("v_min_i32", d, st, hst, cus);
    run<6>("v_add_u32", d, st, hst, cus);
    run<7>("v_sub_u32", d, st, hst, cus);
    run<8>("v_and_b32", d, st, hst, cus);
    run<9>("v_xor_b32", d, st, hst, cus);
    run<10>("v_bfi_b32", d, st, hst, cus);
    run<11>("v_perm_b32", d, st, hst, cus);
    run<12>("v_mov_b32_dpp", d, st, hst, cus);
    run<13>("v_min_u32_dpp", d, st, hst, cus);
    run<14>("v_add_u32_dpp", d, st, hst, cus);
    run<15>("v_pk_min_u16", d, st, hst, cus);
    run<16>("v_pk_max_f16", d, st, hst, cus);
    run<17>("v_min_f16", d, st, hst, cus);
    run<18>("v_mul_f32", d, st, hst, cus);
    run<19>("v_fma_f32", d, st, hst, cus);
    run<20>("v_max_f32_e64_neg", d, st, hst, cus);
    run<21>("v_cmp_lt_u32_e64", d, st, hst, cus);
    run<22>("v_cndmask_e64_s", d, st, hst, cus);
    run<23>("v_lshrrev_b32", d, st, hst, cus);
    run<24>("v_sad_u32", d, st, hst, cus);
    run<25>("v_max3_f32", d, st, hst, cus);
    run<26>("v_permlane32_swap", d, st, hst, cus);
    run<27>("v_max_f32_dpp_neg_quad", d, st, hst, cus);
    run<28>("v_max_f32_dpp_neg_mirror", d, st, hst, cus);
    run<29>("v_pk_mul_f32/v_mul_f32 alt", d, st, hst, cus);
    run<31>("v_cmp_lt_f32_e32", d, st, hst, cus);
    run<32>("v_cndmask_b32_e32", d, st, hst, cus);
    run<33>("v_min_i16_e32", d, st, hst, cus);
    run<34>("v_max_u16_e32", d, st, hst, cus);
    run<35>("v_sub_f32_e32", d, st, hst, cus);
    run<36>("v_mov_b32_e32", d, st, hst, cus);
    run<37>("v_min_f32_sdwa", d, st, hst, cus);
    run<38>("CE cmp_e32+2xcndmask_e32", d, st, hst, cus);
    run<39>("CE v_min_f32+v_max_f32", d, st, hst, cus);
    run<40>("v_cmp_gt_u32_e32", d, st, hst, cus);
    return 0;
}
