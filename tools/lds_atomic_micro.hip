// Microbenchmark: LDS float atomics (ds_add_f32, no return) vs plain LDS stores on gfx950, by address pattern:
// distinct consecutive dwords, 2 / 4 / 16 lanes per address, and the same dword for the whole wave.
// Design input for the warp backward.  Timing only.
// build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_micro.hip -o tools/lds_atomic_micro
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITER 2048

template <int OP>
__global__ __launch_bounds__(256) void k(float *out, int share) {
    __shared__ float lds[8192];
    const int t = threadIdx.x, lane = t & 63;
    for (int i = t; i < 8192; i += 256) lds[i] = 0.0f;
    __syncthreads();
    // lanes sharing an address: lane / share; waves of the block use separate 2-KiB regions
    const int slot = (t >> 6) * 512 + (lane / share);
    float v = (float)lane * 1e-3f;
    for (int it = 0; it < ITER; ++it) {
        float *p = lds + slot + ((it & 7) << 6);
        if (OP == 0) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (OP == 1) atomicAdd(reinterpret_cast<unsigned *>(p), 1u);
        else *p = v;
        v += 1e-7f;
    }
    __syncthreads();
    if (lds[t] == 12345.0f) out[t] = 1.0f;
}

int main() {
    float *o;
    hipMalloc(&o, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *nm[3] = {"ds_add_f32", "ds_add_u32", "ds_write_b32"};
    for (int op = 0; op < 3; ++op)
        for (int share : {1, 2, 4, 16, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (op == 0) hipLaunchKernelGGL(k<0>, dim3(1024), dim3(256), 0, 0, o, share);
                else if (op == 1) hipLaunchKernelGGL(k<1>, dim3(1024), dim3(256), 0, 0, o, share);
                else hipLaunchKernelGGL(k<2>, dim3(1024), dim3(256), 0, 0, o, share);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep == 1)
                    printf("%-13s lanes/address %2d: %8.1f us, %.2f ns per wave instruction per CU\n", nm[op], share,
                           ms * 1e3, ms * 1e6 / (1024.0 / 256 * 4 * ITER));
            }
        }
    return 0;
}
