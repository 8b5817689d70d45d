// Microbenchmark: write bandwidth of the fused warp's output pattern (2 frames x 64 channel planes x 480 x 1440 fp32
// = 354 MB, NCHW) by BEV tile shape, tile -> XCD order and store cache policy.  Each
// workgroup (256 threads, one cell per lane) stores its tile's 64 planes with buffer_store_dword, one plane per
// instruction, exactly as k_warp_fuse_v2's store_chunk; TH x (256 / TH) tiles.  Timing only, no product code.
// build: hipcc --offload-arch=gfx950 -O3 tools/store_pattern_micro.hip -o tools/store_pattern_micro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int TH, int AUX, int REMAP>
__global__ __launch_bounds__(256) void k_store(float *__restrict__ out, int Hb, int Wb) {
    constexpr int TW = 256 / TH;
    const int ntx = Wb / TW, nt = ntx * (Hb / TH);
    int tile = blockIdx.x;
    if (REMAP == 1) {  // k_warp_fuse_v2: contiguous eighths of the tiles per XCD (block % 8 = XCD)
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rpw = TH / 4;  // rows per wave
    const int i = ty * TH + wave * rpw + lane / (64 / rpw), j = tx * TW + lane % (64 / rpw);
    const size_t plane = (size_t)Hb * Wb;
    float *chunk = out + (size_t)blockIdx.y * 64 * plane;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)(uint32_t)(plane * 64 * sizeof(float)), 0x00020000);
    const int voff = (i * Wb + j) * 4;
    const float a = (float)(i + j);
#pragma unroll
    for (int q = 0; q < 64; ++q)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, a + (float)q), rs, voff,
                                              (int)(uint32_t)(q * plane * sizeof(float)), AUX);
}

// reference: the same bytes as a plain float4 fill (every wave writes 1 KiB contiguous per instruction)
__global__ __launch_bounds__(256) void k_fill4(float4 *__restrict__ out, size_t n4) {
    for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256)
        out[k] = make_float4(1.f, 2.f, 3.f, (float)k);
}

int main() {
    const int B = 2, Hb = 480, Wb = 1440;
    float *out;
    const size_t n = (size_t)B * 64 * Hb * Wb;
    hipMalloc(&out, n * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Case {
        const char *name;
        void (*k)(float *, int, int);
        int th;
    } cases[] = {
        {"16x16 raster   nt(2)", k_store<16, 2, 0>, 16},   {"16x16 xcd-8ths nt(2)", k_store<16, 2, 1>, 16},
        {"16x16 raster   aux0", k_store<16, 0, 0>, 16},    {"16x16 xcd-8ths aux0", k_store<16, 0, 1>, 16},
        {"16x16 xcd-8ths aux1", k_store<16, 1, 1>, 16},    {"16x16 xcd-8ths aux3", k_store<16, 3, 1>, 16},
        {"8x32  raster   nt(2)", k_store<8, 2, 0>, 8},     {"8x32  xcd-8ths nt(2)", k_store<8, 2, 1>, 8},
        {"8x32  xcd-8ths aux0", k_store<8, 0, 1>, 8},      {"4x64  raster   nt(2)", k_store<4, 2, 0>, 4},
        {"4x64  xcd-8ths nt(2)", k_store<4, 2, 1>, 4},     {"4x64  xcd-8ths aux0", k_store<4, 0, 1>, 4},
    };
    for (int rnd = 0; rnd < 3; ++rnd) {
        for (auto &c : cases) {
            const int nt = (Hb / c.th) * (Wb / (256 / c.th));
            for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(c.k, dim3(nt, B), dim3(256), 0, 0, out, Hb, Wb);
            hipEventRecord(e0);
            const int it = 20;
            for (int k = 0; k < it; ++k) hipLaunchKernelGGL(c.k, dim3(nt, B), dim3(256), 0, 0, out, Hb, Wb);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms / it * 1e3;
            printf("round %d  %-24s %8.1f us  %6.2f TB/s\n", rnd, c.name, us, n * 4.0 / us * 1e-6);
        }
        hipLaunchKernelGGL(k_fill4, dim3(256 * 16), dim3(256), 0, 0, (float4 *)out, n / 4);
        hipEventRecord(e0);
        for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(k_fill4, dim3(256 * 16), dim3(256), 0, 0, (float4 *)out, n / 4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        printf("round %d  %-24s %8.1f us  %6.2f TB/s\n", rnd, "float4 fill (reference)", ms / 20 * 1e3,
               n * 4.0 / (ms / 20 * 1e3) * 1e-6);
    }
    return (int)hipGetLastError();
}
