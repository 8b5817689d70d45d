// Microbenchmark: issue rate of the fp32 VALU forms a bilinear view sum can use:
// v_fma_f32 (VOP3), v_fmac_f32 (VOP2), v_fmac_f32 with a DPP row broadcast on src0 (row_newbcast), and the packed
// v_pk_fma_f32 (two lanes' worth per lane) -- 8 independent accumulator chains per lane, 256-thread workgroups,
// `occ` workgroups per CU, cycles per instruction per SIMD from s_memtime.  Timing only, no product code.
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate_micro.hip -o tools/valu_rate_micro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 2048
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, unsigned long long *cyc, float s) {
    float a[8], b = s + threadIdx.x * 1e-7f, w = 0.999f;
    f32x2 p[8], pb = {b, b * 0.5f}, pw = {w, w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (float)i * 1e-3f;
        p[i] = (f32x2){a[i], a[i] + 1.0f};
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(w));
            if (MODE == 1) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(w));
            if (MODE == 2)
                asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf"
                             : "+v"(a[i]) : "v"(b), "v"(w));
            if (MODE == 3) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(pb), "v"(pw));
            if (MODE == 4) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *out;
    unsigned long long *cyc, hc[4096];
    hipMalloc(&out, 4096 * 256 * sizeof(float));
    hipMalloc(&cyc, 4096 * sizeof(unsigned long long));
    const char *names[] = {"v_fma_f32", "v_fmac_f32", "v_fmac_f32_dpp row_newbcast", "v_pk_fma_f32 (2 per lane)",
                           "v_mul_f32"};
    void (*ks[])(float *, unsigned long long *, float) = {k<0>, k<1>, k<2>, k<3>, k<4>};
    for (int occ : {1, 2, 4, 8}) {
        const int nb = 256 * occ;  // occ workgroups (occ waves per SIMD) on each of 256 CUs
        for (int m = 0; m < 5; ++m) {
            hipLaunchKernelGGL(ks[m], dim3(nb), dim3(256), 0, 0, out, cyc, 1.0f);
            hipDeviceSynchronize();
            hipMemcpy(hc, cyc, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            double mean = 0;
            for (int i = 0; i < nb; ++i) mean += (double)hc[i];
            mean /= nb;
            // occ waves share a SIMD: cycles per instruction per SIMD = wave cycles / (instructions per wave * occ)
            printf("occ %d  %-30s  %6.2f cycles per wave-instruction per SIMD\n", occ, names[m],
                   mean / (ITER * 8.0 * occ));
        }
    }
    return (int)hipGetLastError();
}
