// outlier.hip -- LLM.int8() mixed-precision decomposition: the feature columns of X
// that hold an outlier are multiplied in fp32, the rest through the int8 absmax path, so the outliers
// no longer set the row scales Cx.  The reference carries only the building blocks, unused:
// op_outlier_extractor / AbsCompareLTEConstFunc (op_elemwise.cuh:293-306, 698-708) and op_round_int8
// (:167-176, 685-695).  Definition (DESIGN.md "Outlier decomposition"; the oracle restates it):
//   outlier column k  : some X[i,k] is not (|x| <= t)  -- AbsCompareLTEConstFunc returns 1 (NaN: 1)
//   O8  = op_quantized_mm(X', W'), X' = X with the outlier columns zeroed, W' = W with those rows zeroed
//   Co  = fmaf chain from +0 over the outlier columns in ascending k: X[i,k] * W[k,j]
//   O   = fl(O8 + Co)            (no outlier columns: O = O8, the plain path)
#include <algorithm>

#include "qgemm_internal.h"

namespace qgemm {

namespace {

// AbsCompareLTEConstFunc (op_elemwise.cuh:296-304): 0 when a in [-b, b], else 1 (NaN -> 1)
__device__ __forceinline__ bool is_outlier(float a, float b) {
    return !(((a >= 0) & (a <= b)) | ((a <= 0) & (-a <= b)));
}

// flags[c] |= outlier over a chunk of rows; thread per column (coalesced along the row)
__global__ __launch_bounds__(256) void outlier_cols_kernel(const float *__restrict__ X, int64_t xsh, int m, int k,
                                                           float t, int rows_per_block,
                                                           unsigned *__restrict__ flags) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= k) return;
    const int r0 = blockIdx.y * rows_per_block, r1 = min(m, r0 + rows_per_block);
    bool any = false;
    for (int r = r0; r < r1; ++r) any |= is_outlier(X[(int64_t)r * xsh + c], t);
    if (any) atomicOr(flags + c, 1u);
}

// ascending indices of the flagged columns (one block, chunked prefix sum); count at idx[-1] slot
__global__ __launch_bounds__(1024) void outlier_index_kernel(const unsigned *__restrict__ flags, int k,
                                                             int *__restrict__ idx, int *__restrict__ count) {
    __shared__ int scan[1024];
    __shared__ int base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < k; c0 += 1024) {
        const int c = c0 + threadIdx.x;
        const int f = (c < k && flags[c]) ? 1 : 0;
        scan[threadIdx.x] = f;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
            const int v = threadIdx.x >= off ? scan[threadIdx.x - off] : 0;
            __syncthreads();
            scan[threadIdx.x] += v;
            __syncthreads();
        }
        if (f) idx[base + scan[threadIdx.x] - 1] = c;
        __syncthreads();
        if (threadIdx.x == 1023) base += scan[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = base;
}

// X' (outlier columns zeroed) and W' (outlier rows zeroed), contiguous outputs
__global__ __launch_bounds__(256) void outlier_mask_kernel(const float *__restrict__ X, int64_t xsh, int m, int k,
                                                           const float *__restrict__ W, int64_t wsh, int n,
                                                           const unsigned *__restrict__ flags,
                                                           float *__restrict__ Xm, float *__restrict__ Wm) {
    const int64_t nx = (int64_t)m * k, total = nx + (int64_t)k * n;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        if (e < nx) {
            const int64_t r = e / k, c = e - r * k;
            Xm[e] = flags[c] ? 0.0f : X[r * xsh + c];
        } else {
            const int64_t f = e - nx, r = f / n, c = f - r * n;
            Wm[f] = flags[r] ? 0.0f : W[r * wsh + c];
        }
    }
}

// O[i,j] = fl(O[i,j] + fmaf-chain over the outlier columns), one thread per output (j fastest)
__global__ __launch_bounds__(256) void outlier_mm_kernel(const float *__restrict__ X, int64_t xsh,
                                                         const float *__restrict__ W, int64_t wsh,
                                                         const int *__restrict__ idx,
                                                         const int *__restrict__ count, float *__restrict__ O,
                                                         int64_t osh, int m, int n) {
    const int cnt = *count;
    if (cnt == 0) return;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)m * n) return;
    const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
    float acc = 0.0f;
    for (int t = 0; t < cnt; ++t) {
        const int c = idx[t];
        acc = __fmaf_rn(X[(int64_t)i * xsh + c], W[(int64_t)c * wsh + j], acc);
    }
    O[(int64_t)i * osh + j] = __fadd_rn(O[(int64_t)i * osh + j], acc);
}

}  // namespace

size_t outlier_scratch_bytes(int m, int n, int k) {
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return a256(sizeof(unsigned) * k) + a256(sizeof(int) * (k + 1)) + a256(sizeof(float) * (size_t)m * k) +
           a256(sizeof(float) * (size_t)k * n);
}

// Phase 1: flags, indices, X', W' into scratch; the caller then runs the int8 chain on (X', W') and
// phase 2 (outlier_finish) adds the fp32 outlier products.
hipError_t outlier_prepare(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, float t,
                           void *scratch, float **Xm, float **Wm, hipStream_t s) {
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char *p = static_cast<char *>(scratch);
    unsigned *flags = reinterpret_cast<unsigned *>(p);
    int *idx = reinterpret_cast<int *>(p + a256(sizeof(unsigned) * k));
    *Xm = reinterpret_cast<float *>(p + a256(sizeof(unsigned) * k) + a256(sizeof(int) * (k + 1)));
    *Wm = *Xm + a256(sizeof(float) * (size_t)m * k) / sizeof(float);
    hipError_t e = hipMemsetAsync(flags, 0, sizeof(unsigned) * k, s);
    if (e != hipSuccess) return e;
    const int rpb = 256;
    outlier_cols_kernel<<<dim3((unsigned)((k + 255) / 256), (unsigned)((m + rpb - 1) / rpb)), 256, 0, s>>>(X, xsh, m, k,
                                                                                                       t, rpb, flags);
    outlier_index_kernel<<<1, 1024, 0, s>>>(flags, k, idx + 1, idx);
    const int64_t total = (int64_t)m * k + (int64_t)k * n;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 16384);
    outlier_mask_kernel<<<blocks, 256, 0, s>>>(X, xsh, m, k, W, wsh, n, flags, *Xm, *Wm);
    return hipGetLastError();
}

hipError_t outlier_finish(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, void *scratch,
                          float *O, int64_t osh, hipStream_t s) {
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const int *idx = reinterpret_cast<const int *>(static_cast<char *>(scratch) + a256(sizeof(unsigned) * k));
    outlier_mm_kernel<<<(unsigned)(((int64_t)m * n + 255) / 256), 256, 0, s>>>(X, xsh, W, wsh, idx + 1, idx, O, osh, m,
                                                                              n);
    return hipGetLastError();
}

int outlier_count_slot(int k, const void *scratch, int *count_host) {
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const int *idx = reinterpret_cast<const int *>(static_cast<const char *>(scratch) + a256(sizeof(unsigned) * k));
    return (int)hipMemcpy(count_host, idx, sizeof(int), hipMemcpyDeviceToHost);
}

}  // namespace qgemm
