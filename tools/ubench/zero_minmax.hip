// Probe: how v_min_f32 / v_max_f32 / v_med3_f32 order -0.0 and +0.0 on gfx950 (IEEE mode on).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void k(const float* in, unsigned* out) {
    const float a = in[0], b = in[1], ninf = in[2], pinf = in[3];
    float r[8];
    asm volatile("v_min_f32 %0, %1, %2" : "=v"(r[0]) : "v"(a), "v"(b));
    asm volatile("v_min_f32 %0, %1, %2" : "=v"(r[1]) : "v"(b), "v"(a));
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r[2]) : "v"(a), "v"(b));
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r[3]) : "v"(b), "v"(a));
    r[4] = __builtin_amdgcn_fmed3f(a, b, ninf);
    r[5] = __builtin_amdgcn_fmed3f(b, a, ninf);
    r[6] = __builtin_amdgcn_fmed3f(a, b, pinf);
    r[7] = __builtin_amdgcn_fmed3f(b, a, pinf);
    if (threadIdx.x == 0)
        for (int i = 0; i < 8; i++) out[i] = __float_as_uint(r[i]);
}

int main() {
    float h[4] = {-0.0f, 0.0f, -__builtin_inff(), __builtin_inff()};
    float* d;
    unsigned* o;
    unsigned ho[8];
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, sizeof(ho));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
    const char* names[8] = {"min(-0,+0)", "min(+0,-0)", "max(-0,+0)", "max(+0,-0)",
                            "med3(-0,+0,-inf)", "med3(+0,-0,-inf)", "med3(-0,+0,+inf)", "med3(+0,-0,+inf)"};
    for (int i = 0; i < 8; i++) printf("%-18s = 0x%08x\n", names[i], ho[i]);
    return 0;
}
