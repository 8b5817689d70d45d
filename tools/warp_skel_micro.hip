// Microbenchmark: the fixed costs of the fused warp's launch structure, without its work.
// Same grid as k_warp_fuse_v2 at the bench geometry (16 x 16 BEV tiles of 480 x 1440, 2 frames, 256 threads), with:
//   bit 1: the per-workgroup prologue loads (per-view footprint boxes, the tile's xs / ys) and readlanes of them,
//   bit 2: one barrier per live view (5 per tile),
//   bit 4: the output stores (64 channel planes per lane, buffer_store_dword nt, the kernel's NCHW pattern: 354 MB),
//   bit 8: the stores as one 16-B store per 4 cells (a lane owns 4 cells x 16 channels; same bytes),
// and a dynamic LDS allocation of 0 or 53 KiB (k_warp_fuse_v2's pool: 3 workgroups per CU).
// Timing only, no product code.  build: hipcc --offload-arch=gfx950 -O3 tools/warp_skel_micro.hip -o tools/warp_skel_micro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int v4i_t __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256, 3) void k_skel(const uint2 *__restrict__ boxes, const float *__restrict__ xs,
                                                 const float *__restrict__ ys, float *__restrict__ out, int Hb, int Wb,
                                                 int V) {
    extern __shared__ unsigned char smem[];
    const int ntx = Wb / 16, nt = ntx * (Hb / 16);
    const int tile = blockIdx.x, b = blockIdx.y;
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = ty * 16 + wave * 4 + (lane >> 4), j = tx * 16 + (lane & 15);
    float acc = 0.0f;
    unsigned lb = 0;
    if (MODE & 1) {
        const uint2 bx = lane < V ? boxes[((int64_t)b * nt + tile) * V + lane] : make_uint2(0u, 0u);
        lb = bx.x ^ bx.y;
        acc = xs[j] + ys[i];
    }
    if (threadIdx.x < 16) smem[threadIdx.x] = 0;
    for (int v = 0; v < V; ++v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)lb, v);
        if ((a & 3u) == 1u) acc += 1.0f;  // about a quarter of the views: skipped (as dead views are)
        else if (MODE & 2) __syncthreads();
    }
    const size_t plane = (size_t)Hb * Wb;
    if (MODE & 4) {
        float *chunk = out + (size_t)b * 64 * plane;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)(uint32_t)(plane * 64 * sizeof(float)), 0x00020000);
        const int voff = (i * Wb + j) * 4;
#pragma unroll
        for (int q = 0; q < 64; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc + (float)q), rs, voff,
                                                  (int)(uint32_t)(q * plane * sizeof(float)), 2);
    }
    if (MODE & 8) {  // lane: row (lane >> 4) of its wave's 4 rows... as k_warp_fuse_v3: 4 channels x 16 cells
        const int l16 = lane & 15;
        float *ob = out + ((size_t)b * 64 + 4 * l16) * plane + (size_t)i * Wb + tx * 16;
#pragma unroll
        for (int uu = 0; uu < 4; ++uu)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                float4 o = make_float4(acc + uu, acc + m, acc, acc);
                *reinterpret_cast<float4 *>(ob + uu * plane + 4 * m) = o;
            }
    }
}

int main() {
    const int B = 2, V = 7, Hb = 480, Wb = 1440, nt = (Hb / 16) * (Wb / 16);
    uint2 *boxes;
    float *xs, *ys, *out;
    hipMalloc(&boxes, (size_t)B * nt * V * sizeof(uint2));
    hipMalloc(&xs, Wb * sizeof(float));
    hipMalloc(&ys, Hb * sizeof(float));
    hipMalloc(&out, (size_t)B * 64 * Hb * Wb * sizeof(float));
    hipMemset(boxes, 0x5a, (size_t)B * nt * V * sizeof(uint2));
    hipMemset(xs, 0, Wb * sizeof(float));
    hipMemset(ys, 0, Hb * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Case {
        const char *name;
        void (*k)(const uint2 *, const float *, const float *, float *, int, int, int);
        int lds;
    } cases[] = {
        {"empty, LDS 0", k_skel<0>, 0},
        {"empty, LDS 53K", k_skel<0>, 53 * 1024},
        {"prologue loads, LDS 53K", k_skel<1>, 53 * 1024},
        {"prologue + barriers, LDS 53K", k_skel<3>, 53 * 1024},
        {"stores (4 B/lane x 64 planes), LDS 53K", k_skel<4>, 53 * 1024},
        {"stores (4 B/lane x 64 planes), LDS 0", k_skel<4>, 0},
        {"stores (16 B/lane, 4 ch x 16 cells), LDS 53K", k_skel<8>, 53 * 1024},
        {"stores (16 B/lane, 4 ch x 16 cells), LDS 0", k_skel<8>, 0},
        {"prologue + barriers + stores, LDS 53K", k_skel<7>, 53 * 1024},
        {"prologue + barriers + stores, LDS 0", k_skel<7>, 0},
    };
    for (int rnd = 0; rnd < 3; ++rnd)
        for (auto &c : cases) {
            for (int w = 0; w < 3; ++w)
                hipLaunchKernelGGL(c.k, dim3(nt, B), dim3(256), c.lds, 0, boxes, xs, ys, out, Hb, Wb, V);
            hipEventRecord(e0);
            const int n = 20;
            for (int it = 0; it < n; ++it)
                hipLaunchKernelGGL(c.k, dim3(nt, B), dim3(256), c.lds, 0, boxes, xs, ys, out, Hb, Wb, V);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            printf("round %d  %-48s %8.1f us per launch\n", rnd, c.name, ms / n * 1e3f);
        }
    return (int)hipGetLastError();
}
