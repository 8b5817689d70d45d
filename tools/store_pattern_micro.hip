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

// NHWC ([B][Hb][Wb][64], channels-last): the 16 x 16 tile's 64 cells per wave = 4 rows of 16 cells, each row 4 KiB
// contiguous.  LANE: lane = cell (k_warp_fuse_v2's cell mapping), its 256-B run as 16 float4 stores (per instruction
// 64 x 16 B at a 256-B stride, merged in L2); COAL: instruction k writes row k / 4's bytes (k % 4) KiB .. + 1 KiB,
// 16 B per lane, 1 KiB contiguous per instruction (the data would come through LDS).
template <int AUX, bool COAL>
__global__ __launch_bounds__(256) void k_store_nhwc(float *__restrict__ out, int Hb, int Wb) {
    constexpr int TH = 16, TW = 16;
    const int ntx = Wb / TW, nt = ntx * (Hb / TH);
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float *frame = out + (size_t)blockIdx.y * Hb * Wb * 64;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(frame, 0, (int)(uint32_t)((size_t)Hb * Wb * 64 * sizeof(float)), 0x00020000);
    const float a = (float)(lane + tile);
    if (COAL) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int row = ty * TH + wave * 4 + k / 4;
            const int voff = ((row * Wb + tx * TW) * 64) * 4 + ((k % 4) * 64 + lane) * 16;
            const float4 v = make_float4(a, a + 1.f, a + 2.f, (float)k);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int __attribute__((ext_vector_type(4))), v), rs,
                                                   voff, 0, AUX);
        }
    } else {
        const int i = ty * TH + wave * 4 + lane / 16, j = tx * TW + lane % 16;
        const int voff = (i * Wb + j) * 256;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const float4 v = make_float4(a, a + 1.f, a + 2.f, (float)q);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int __attribute__((ext_vector_type(4))), v), rs,
                                                   voff, q * 16, AUX);
        }
    }
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
        {"NHWC 16x16 lane aux0", k_store_nhwc<0, false>, 16}, {"NHWC 16x16 lane nt(2)", k_store_nhwc<2, false>, 16},
        {"NHWC 16x16 coal aux0", k_store_nhwc<0, true>, 16},  {"NHWC 16x16 coal nt(2)", k_store_nhwc<2, true>, 16},
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
