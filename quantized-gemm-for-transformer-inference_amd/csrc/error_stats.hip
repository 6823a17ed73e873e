// error_stats.hip -- the reference's quantization-error metric, on the device.
//
// The reference prints "Mean Quantization error" = mean(C - qC) (timing_quantize.cu:67-70):
// op_subtract(C, qC, E) (op_elemwise.cuh:531-542, one fl(c - q) per element) then E.toHost().mean()
// (tensor.cuh:201-211): a SIGNED sum accumulated sequentially in fp32 on the host, divided by
// (float)(h*w).  At C4 sizes (M = 65536) the host round trip and the sequential sum dominate, so:
//   stats[0]  the reference's number, same order and roundings (one wave walks the elements in order:
//             exact, but latency-bound -- opt-in via reference_order)
//   stats[1]  signed mean, fp64 accumulation (deterministic fixed-shape tree)
//   stats[2]  mean |C - qC|   stats[3]  max |C - qC|   stats[4]  mean |C|  (relative = [2] / [4])
// The differences d = fl(C - qC) are the reference's fp32 E elements in every statistic.
#include "qgemm_internal.h"

namespace qgemm {

namespace {

constexpr int kStatBlocks = 1024, kStatThreads = 256;

struct Acc4 {
    double sum, sum_abs, max_abs, sum_ref;
};

__device__ __forceinline__ Acc4 combine(Acc4 a, const Acc4 &b) {
    a.sum += b.sum;
    a.sum_abs += b.sum_abs;
    a.max_abs = fmax(a.max_abs, b.max_abs);
    a.sum_ref += b.sum_ref;
    return a;
}

__device__ __forceinline__ Acc4 shfl_xor(const Acc4 &a, int off) {
    return Acc4{__shfl_xor(a.sum, off, 64), __shfl_xor(a.sum_abs, off, 64), __shfl_xor(a.max_abs, off, 64),
                __shfl_xor(a.sum_ref, off, 64)};
}

// fixed tree: 64-lane butterfly, then the block's 4 waves in order
__device__ Acc4 block_reduce(Acc4 v, Acc4 *red) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = combine(v, shfl_xor(v, off));
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red[wv] = v;
    __syncthreads();
    Acc4 r = red[0];
    for (int w = 1; w < kStatThreads / 64; ++w) r = combine(r, red[w]);
    return r;
}

__global__ __launch_bounds__(kStatThreads) void error_partials_kernel(const float *__restrict__ C,
                                                                      const float *__restrict__ O, int64_t n,
                                                                      Acc4 *__restrict__ partials) {
    __shared__ Acc4 red[kStatThreads / 64];
    Acc4 v{0.0, 0.0, 0.0, 0.0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float c = C[i];
        const double d = (double)__fsub_rn(c, O[i]);  // the reference's E element, fl(C - qC)
        v.sum += d;
        v.sum_abs += fabs(d);
        v.max_abs = fmax(v.max_abs, fabs(d));
        v.sum_ref += fabs((double)c);
    }
    const Acc4 r = block_reduce(v, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

__global__ __launch_bounds__(kStatThreads) void error_final_kernel(const Acc4 *__restrict__ partials, int nparts,
                                                                   int64_t n, int reference_order,
                                                                   double *__restrict__ stats) {
    __shared__ Acc4 red[kStatThreads / 64];
    Acc4 v{0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < nparts; i += kStatThreads) v = combine(v, partials[i]);
    const Acc4 r = block_reduce(v, red);
    if (threadIdx.x == 0) {
        stats[1] = r.sum / (double)n;
        stats[2] = r.sum_abs / (double)n;
        stats[3] = r.max_abs;
        stats[4] = r.sum_ref / (double)n;
        if (!reference_order) stats[0] = __builtin_nan("");  // not computed
    }
}

// tensor.cuh:201-211 on the host: float sum = 0; for each element sum += e; return sum / (h*w).
// One wave: chunk c+1 (1024 differences, coalesced) is loaded while chunk c, staged in LDS, is added
// in element order -- the sum itself stays one sequential fp32 chain, as in the reference.
constexpr int kRefChunk = 1024;
__global__ __launch_bounds__(64) void error_reference_mean_kernel(const float *__restrict__ C,
                                                                  const float *__restrict__ O, int64_t n,
                                                                  double *__restrict__ stats) {
    __shared__ float stage[2][kRefChunk];
    const int lane = threadIdx.x;
    auto fetch = [&](int64_t base, float (&d)[kRefChunk / 64]) {
#pragma unroll
        for (int j = 0; j < kRefChunk / 64; ++j) {
            const int64_t i = base + j * 64 + lane;
            d[j] = i < n ? __fsub_rn(C[i], O[i]) : 0.0f;
        }
    };
    float d[kRefChunk / 64];
    fetch(0, d);
    float sum = 0.0f;
    int buf = 0;
    for (int64_t base = 0; base < n; base += kRefChunk, buf ^= 1) {
#pragma unroll
        for (int j = 0; j < kRefChunk / 64; ++j) stage[buf][j * 64 + lane] = d[j];
        __syncthreads();
        if (base + kRefChunk < n) fetch(base + kRefChunk, d);  // in flight during the adds
        const int cnt = n - base < kRefChunk ? (int)(n - base) : kRefChunk;
        const float *sb = stage[buf];
        int e = 0;
        for (; e + 4 <= cnt; e += 4) {
            const float4 q = *reinterpret_cast<const float4 *>(sb + e);  // same address in every lane
            sum = __fadd_rn(sum, q.x);
            sum = __fadd_rn(sum, q.y);
            sum = __fadd_rn(sum, q.z);
            sum = __fadd_rn(sum, q.w);
        }
        for (; e < cnt; ++e) sum = __fadd_rn(sum, sb[e]);
    }
    if (lane == 0) stats[0] = (double)__fdiv_rn(sum, (float)(int)n);  // h*w is an int in the reference
}

}  // namespace

size_t error_stats_scratch_bytes() { return sizeof(Acc4) * kStatBlocks; }

hipError_t launch_error_stats(const float *C, const float *O, int64_t n, bool reference_order, double *stats,
                              void *scratch, hipStream_t stream) {
    Acc4 *partials = static_cast<Acc4 *>(scratch);
    int64_t want = (n + kStatThreads - 1) / kStatThreads;
    const int blocks = (int)(want < kStatBlocks ? (want > 0 ? want : 1) : kStatBlocks);
    error_partials_kernel<<<blocks, kStatThreads, 0, stream>>>(C, O, n, partials);
    error_final_kernel<<<1, kStatThreads, 0, stream>>>(partials, blocks, n, reference_order ? 1 : 0, stats);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (reference_order) {
        error_reference_mean_kernel<<<1, 64, 0, stream>>>(C, O, n, stats);
        e = hipGetLastError();
    }
    return e;
}

}  // namespace qgemm
