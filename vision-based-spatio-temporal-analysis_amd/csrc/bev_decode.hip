// bev_decode.hip -- BEVDetector.decode on the device.
//
// Replaces detector.py:64-125: `_nms2d` (3x3 max-pool peak test), the confidence threshold,
// torch.where compaction, the box arithmetic and the Python O(K^2) greedy centre-distance NMS
// with one `.item()` per pair.  Two kernels, no host synchronisation in between:
//
//   k_decode_peaks  one thread per BEV cell: value v of the heatmap is a peak when it equals the
//                   max of its 3x3 window (F.max_pool2d pads with -inf); the reference's score is
//                   then v * (float)(v == peak) and a cell is a candidate when that exceeds the
//                   threshold.  Candidates are compacted with one atomic per frame counter.
//   k_decode_nms    one workgroup per frame: candidates sorted by (score desc, cell index asc) --
//                   torch.argsort(descending) order, ties broken like a stable sort -- with a
//                   bitonic sort in LDS, boxes computed with the reference's fp32 op sequence, then
//                   the greedy NMS: candidate i is kept when every kept centre is at distance
//                   >= nms_dist (torch.norm of the fp32 difference); the kept set is checked by all
//                   threads in parallel, one workgroup barrier per candidate.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"

namespace {

constexpr int NMS_THREADS = 256;
constexpr int NMS_MAX = 8192;  // candidates a frame's sort / NMS holds in LDS

__global__ void k_decode_peaks(const float *__restrict__ heat, int H, int W, float thresh, int cap,
                               int32_t *__restrict__ cand_idx, float *__restrict__ cand_score,
                               int32_t *__restrict__ count) {
    const int b = blockIdx.y;
    const int64_t hw = (int64_t)H * W;
    const float *hb = heat + (size_t)b * hw;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < hw; c += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(c / W), x = (int)(c - (int64_t)y * W);
        const float v = hb[c];
        float m = -__builtin_inff();
        for (int dy = -1; dy <= 1; ++dy) {
            const int yy = y + dy;
            if (yy < 0 || yy >= H) continue;
            for (int dx = -1; dx <= 1; ++dx) {
                const int xx = x + dx;
                if (xx < 0 || xx >= W) continue;
                const float u = hb[(int64_t)yy * W + xx];
                m = (u > m || u != u) ? u : m;  // max_pool2d: NaN propagates
            }
        }
        const float score = v * ((v == m) ? 1.0f : 0.0f);  // detector.py:69 x * (x == maxpool).float()
        if (score > thresh) {
            const int k = atomicAdd(&count[b], 1);
            if (k < cap) {
                cand_idx[(size_t)b * cap + k] = (int32_t)c;
                cand_score[(size_t)b * cap + k] = score;
            }
        }
    }
}

// ascending 64-bit key = descending score, then ascending cell index
__device__ __forceinline__ uint64_t sort_key(float s, int32_t idx) {
    uint32_t u = __float_as_uint(s);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // monotone float -> uint
    return ((uint64_t)(~u) << 32) | (uint32_t)idx;
}

__global__ __launch_bounds__(NMS_THREADS) void k_decode_nms(
    const int32_t *__restrict__ cand_idx, const float *__restrict__ cand_score, const int32_t *__restrict__ count,
    int cap, const float *__restrict__ offset, const float *__restrict__ size, int H, int W, float x_min, float y_min,
    float res_x, float res_y, float nms_dist, float *__restrict__ boxes, float *__restrict__ scores,
    int32_t *__restrict__ nkept) {
    __shared__ uint64_t keys[NMS_MAX];
    __shared__ float kcx[NMS_MAX], kcy[NMS_MAX];
    __shared__ int nk, too_close;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int K = count[b];
    if (K > cap || K > NMS_MAX) {  // the caller reports the overflow
        if (tid == 0) nkept[b] = -1;
        return;
    }
    int P = 1;
    while (P < K) P <<= 1;
    for (int i = tid; i < P; i += NMS_THREADS)
        keys[i] = (i < K) ? sort_key(cand_score[(size_t)b * cap + i], cand_idx[(size_t)b * cap + i]) : ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)  // bitonic sort, ascending
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += NMS_THREADS) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t a = keys[i], c = keys[l];
                    if (((i & k) == 0) ? (a > c) : (a < c)) {
                        keys[i] = c;
                        keys[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    if (tid == 0) nk = 0;
    __syncthreads();
    const size_t plane = (size_t)H * W;
    const float *ob = offset + (size_t)b * 2 * plane, *sb = size + (size_t)b * 2 * plane;
    float *bo = boxes + (size_t)b * cap * 4;
    float *so = scores + (size_t)b * cap;
    for (int i = 0; i < K; ++i) {
        const int32_t c = (int32_t)(keys[i] & 0xffffffffu);
        const int y = c / W, x = c - y * W;
        // detector.py:103-108, fp32 op by op: x_min + (xs.float() + off_x) * res_x, ...
        const float cx = x_min + ((float)x + ob[c]) * res_x;
        const float cy = y_min + ((float)y + ob[plane + c]) * res_y;
        const int n = nk;
        if (tid == 0) too_close = 0;
        __syncthreads();
        int close = 0;
        for (int j = tid; j < n; j += NMS_THREADS) {
            const float dx = kcx[j] - cx, dy = kcy[j] - cy;
            close |= __builtin_sqrtf(dx * dx + dy * dy) < nms_dist;
        }
        if (close) too_close = 1;
        __syncthreads();
        if (!too_close && tid == 0) {
            kcx[n] = cx;
            kcy[n] = cy;
            bo[4 * n] = cx;
            bo[4 * n + 1] = cy;
            bo[4 * n + 2] = sb[c] * res_x;
            bo[4 * n + 3] = sb[plane + c] * res_y;
            // score = hm[mask]: the candidate's peak value (the key's score bits)
            uint32_t u = ~(uint32_t)(keys[i] >> 32);
            u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
            so[n] = __uint_as_float(u);
            nk = n + 1;
        }
        __syncthreads();
    }
    if (tid == 0) nkept[b] = nk;
}

// ---- frames with more than NMS_MAX candidates (bev_decode_nms_large_f32) ----------------------------
// Keys in global memory, bitonic network over P (a power of two): stages k <= SORT_CHUNK inside
// LDS chunks, larger stages as one global compare-exchange launch per j >= SORT_CHUNK followed by the
// j < SORT_CHUNK steps of that stage inside LDS.  The direction of a pair is decided by the GLOBAL
// index (i & k), so the chunked network is the plain bitonic sort of the whole array.
constexpr int SORT_CHUNK = 8192;   // keys per LDS chunk (64 KiB)
constexpr int SORT_THREADS = 1024;
constexpr int KEPT_LDS = 8192;     // kept centres cached in LDS by the large NMS (64 KiB); the rest from global
constexpr int NMS_L_THREADS = 1024;

__global__ void k_large_keys(const int32_t *__restrict__ cand_idx, const float *__restrict__ cand_score,
                             const int32_t *__restrict__ count, int cap, int P, uint64_t *__restrict__ keys) {
    const int b = blockIdx.y;
    const int K = count[b];
    if (K <= NMS_MAX || K > cap) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < P)
        keys[(size_t)b * P + i] =
            (i < K) ? sort_key(cand_score[(size_t)b * cap + i], cand_idx[(size_t)b * cap + i]) : ~0ull;
}

// stages k = 2 .. SORT_CHUNK (first = 1) or, for one stage k > SORT_CHUNK, its steps j < SORT_CHUNK
__global__ __launch_bounds__(SORT_THREADS) void k_large_sort_chunk(uint64_t *__restrict__ keys,
                                                                   const int32_t *__restrict__ count, int cap, int P,
                                                                   int first, int kstage) {
    __shared__ uint64_t sk[SORT_CHUNK];
    const int b = blockIdx.y;
    const int K = count[b];
    if (K <= NMS_MAX || K > cap) return;
    uint64_t *kb = keys + (size_t)b * P + (size_t)blockIdx.x * SORT_CHUNK;
    const int g0 = blockIdx.x * SORT_CHUNK;
    for (int i = threadIdx.x; i < SORT_CHUNK; i += SORT_THREADS) sk[i] = kb[i];
    __syncthreads();
    const int k_lo = first ? 2 : kstage, k_hi = first ? SORT_CHUNK : kstage;
    for (int k = k_lo; k <= k_hi; k <<= 1)
        for (int j = (first ? k : SORT_CHUNK) >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < SORT_CHUNK; i += SORT_THREADS) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t a = sk[i], c = sk[l];
                    if ((((g0 + i) & k) == 0) ? (a > c) : (a < c)) {
                        sk[i] = c;
                        sk[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < SORT_CHUNK; i += SORT_THREADS) kb[i] = sk[i];
}

__global__ void k_large_sort_step(uint64_t *__restrict__ keys, const int32_t *__restrict__ count, int cap, int P,
                                  int k, int j) {
    const int b = blockIdx.y;
    const int K = count[b];
    if (K <= NMS_MAX || K > cap) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = i ^ j;
    if (i >= P || l <= i) return;
    uint64_t *kb = keys + (size_t)b * P;
    const uint64_t a = kb[i], c = kb[l];
    if (((i & k) == 0) ? (a > c) : (a < c)) {
        kb[i] = c;
        kb[l] = a;
    }
}

// Greedy NMS over the sorted keys, 64 candidates per round: every wave tests the round's candidates
// against its share of the centres kept so far (LDS cache + global beyond it), then wave 0 resolves
// the survivors in order (a survivor is kept, and suppresses the later survivors closer than
// nms_dist) and appends the kept boxes.  Exactly the sequential greedy loop of detector.py:110-121.
__global__ __launch_bounds__(NMS_L_THREADS) void k_large_nms(
    const uint64_t *__restrict__ keys, const int32_t *__restrict__ count, int cap, int P,
    const float *__restrict__ offset, const float *__restrict__ size, int H, int W, float x_min, float y_min,
    float res_x, float res_y, float nms_dist, float *__restrict__ boxes, float *__restrict__ scores,
    int32_t *__restrict__ nkept) {
    __shared__ float kcx[KEPT_LDS], kcy[KEPT_LDS];
    __shared__ int sup[64];
    __shared__ int nk_s;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int K = count[b];
    if (K <= NMS_MAX || K > cap) return;
    const int lane = tid & 63, wave = tid >> 6, nwaves = NMS_L_THREADS / 64;
    const size_t plane = (size_t)H * W;
    const float *ob = offset + (size_t)b * 2 * plane, *sb = size + (size_t)b * 2 * plane;
    const uint64_t *kb = keys + (size_t)b * P;
    float *bo = boxes + (size_t)b * cap * 4;
    float *so = scores + (size_t)b * cap;
    if (tid == 0) nk_s = 0;
    for (int base = 0; base < K; base += 64) {
        if (tid < 64) sup[tid] = 0;
        const int i = base + lane;
        uint64_t key = ~0ull;
        float cx = 0.f, cy = 0.f;
        int32_t c = 0;
        if (i < K) {
            key = kb[i];
            c = (int32_t)(key & 0xffffffffu);
            const int y = c / W, x = c - y * W;
            cx = x_min + ((float)x + ob[c]) * res_x;
            cy = y_min + ((float)y + ob[plane + c]) * res_y;
        }
        __syncthreads();  // sup cleared, nk_s of the previous round visible
        const int n = nk_s;
        int close = 0;
        if (i < K) {
            for (int j = wave; j < n; j += nwaves) {
                float kx, ky;
                if (j < KEPT_LDS) {
                    kx = kcx[j];
                    ky = kcy[j];
                } else {
                    kx = bo[4 * j];
                    ky = bo[4 * j + 1];
                }
                const float dx = kx - cx, dy = ky - cy;
                if (__builtin_sqrtf(dx * dx + dy * dy) < nms_dist) {
                    close = 1;
                    break;
                }
            }
        }
        if (close) sup[lane] = 1;
        __syncthreads();
        if (wave == 0) {
            bool alive = (i < K) && !sup[lane];
            uint64_t live = __ballot(alive);
            uint64_t kept = 0;
            while (live) {
                const int t = __builtin_ctzll(live);  // next survivor in order: kept
                kept |= 1ull << t;
                const float tx = __shfl(cx, t), ty = __shfl(cy, t);
                if (alive && lane > t) {
                    const float dx = tx - cx, dy = ty - cy;
                    if (__builtin_sqrtf(dx * dx + dy * dy) < nms_dist) alive = false;
                }
                live = __ballot(alive) & ~((2ull << t) - 1);
            }
            if ((kept >> lane) & 1) {
                const int slot = n + __builtin_popcountll(kept & ((1ull << lane) - 1));
                if (slot < KEPT_LDS) {
                    kcx[slot] = cx;
                    kcy[slot] = cy;
                }
                bo[4 * slot] = cx;
                bo[4 * slot + 1] = cy;
                bo[4 * slot + 2] = sb[c] * res_x;
                bo[4 * slot + 3] = sb[plane + c] * res_y;
                uint32_t u = ~(uint32_t)(key >> 32);
                u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
                so[slot] = __uint_as_float(u);
            }
            if (lane == 0) nk_s = n + __builtin_popcountll(kept);
        }
        __syncthreads();  // kept centres (LDS and global) and nk_s visible to every wave
    }
    if (tid == 0) nkept[b] = nk_s;
}

}  // namespace

extern "C" {

int bev_decode_peaks_f32(const float *heat, int B, int H, int W, float thresh, int cap, int32_t *cand_idx,
                         float *cand_score, int32_t *count, void *stream) {
    if (B < 0 || H <= 0 || W <= 0 || cap < 0 || B > 65535 || (B > 0 && (!heat || !count))) return BEV_ERR_ARGS;
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(count, 0, sizeof(int32_t) * (size_t)B, st);
    if (e != hipSuccess) return (int)e;
    const int64_t hw = (int64_t)H * W;
    int64_t blocks = (hw + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_decode_peaks, dim3((unsigned)blocks, B), dim3(256), 0, st, heat, H, W, thresh, cap, cand_idx,
                       cand_score, count);
    return (int)hipGetLastError();
}

int bev_decode_nms_f32(const int32_t *cand_idx, const float *cand_score, const int32_t *count, int B, int cap,
                       const float *offset, const float *size, int H, int W, float x_min, float y_min, float res_x,
                       float res_y, float nms_dist, float *boxes, float *scores, int32_t *nkept, void *stream) {
    if (B < 0 || H <= 0 || W <= 0 || cap < 0 || B > 65535 || (int64_t)H * W > 0x7fffffff) return BEV_ERR_ARGS;
    if (B == 0) return 0;
    hipLaunchKernelGGL(k_decode_nms, dim3(B), dim3(NMS_THREADS), 0, (hipStream_t)stream, cand_idx, cand_score, count,
                       cap, offset, size, H, W, x_min, y_min, res_x, res_y, nms_dist, boxes, scores, nkept);
    return (int)hipGetLastError();
}

int bev_decode_max_candidates(void) { return NMS_MAX; }

int bev_decode_nms_large_f32(const int32_t *cand_idx, const float *cand_score, const int32_t *count, int B, int cap,
                             int P, const float *offset, const float *size, int H, int W, float x_min, float y_min,
                             float res_x, float res_y, float nms_dist, uint64_t *keys, float *boxes, float *scores,
                             int32_t *nkept, void *stream) {
    if (B < 0 || H <= 0 || W <= 0 || cap < 0 || B > 65535 || (int64_t)H * W > 0x7fffffff) return BEV_ERR_ARGS;
    if (P < 2 * SORT_CHUNK || (P & (P - 1)) != 0 || P / 256 > 0x7fffffff) return BEV_ERR_ARGS;
    if (B == 0) return 0;
    if (!cand_idx || !cand_score || !count || !offset || !size || !keys || !boxes || !scores || !nkept)
        return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_large_keys, dim3(P / 256, B), dim3(256), 0, st, cand_idx, cand_score, count, cap, P, keys);
    hipLaunchKernelGGL(k_large_sort_chunk, dim3(P / SORT_CHUNK, B), dim3(SORT_THREADS), 0, st, keys, count, cap, P, 1,
                       0);
    for (int k = 2 * SORT_CHUNK; k <= P; k <<= 1) {
        for (int j = k >> 1; j >= SORT_CHUNK; j >>= 1)
            hipLaunchKernelGGL(k_large_sort_step, dim3(P / 256, B), dim3(256), 0, st, keys, count, cap, P, k, j);
        hipLaunchKernelGGL(k_large_sort_chunk, dim3(P / SORT_CHUNK, B), dim3(SORT_THREADS), 0, st, keys, count, cap, P,
                           0, k);
    }
    hipLaunchKernelGGL(k_large_nms, dim3(B), dim3(NMS_L_THREADS), 0, st, keys, count, cap, P, offset, size, H, W,
                       x_min, y_min, res_x, res_y, nms_dist, boxes, scores, nkept);
    return (int)hipGetLastError();
}

}  // extern "C"
