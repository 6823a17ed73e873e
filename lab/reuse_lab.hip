// reuse_lab.hip -- LAB: does a streamed read stay in the 256-MB Infinity Cache for a second pass right behind it?
// (The FFN-down pack reads W -- 256 MiB -- twice: column maxima, then quantize + transpose.)  For a buffer of S MiB:
//   cold  : the second pass after a 1-GiB sweep of another buffer
//   fwd   : the second pass right behind the first, same order
//   rev   : the second pass right behind the first, reverse order (the most recent lines first)
// and, with a write stream of S/4 beside the second pass (the pack's packed output), each again.
//   build/reuse_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// block b reads chunk (rev ? nchunk - 1 - b : b) of 64 KiB (256 threads x 16 float4, 4 KiB per wave instruction
// row), optionally writes a quarter of it
template <bool kWrite>
__global__ __launch_bounds__(256) void sweep(const float4 *__restrict__ src, float4 *__restrict__ dst, int64_t nchunk,
                                             int rev, int *sink) {
    for (int64_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        const int64_t ch = rev ? nchunk - 1 - c : c;
        const float4 *p = src + ch * 4096;
        float4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = p[j * 256 + threadIdx.x];
        int x = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) x ^= __float_as_int(v[j].x) ^ __float_as_int(v[j].w);
        if constexpr (kWrite) {
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[ch * 1024 + j * 256 + threadIdx.x] = v[j];
        }
        if (x == 0x12345678) sink[0] = x;
    }
}

int main() {
    const size_t big = (size_t)1 << 30;
    float4 *a, *flush, *dst; int *sink;
    CK(hipMalloc(&a, (size_t)320 << 20)); CK(hipMalloc(&flush, big)); CK(hipMalloc(&dst, (size_t)96 << 20));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, (size_t)320 << 20)); CK(hipMemset(flush, 2, big));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = 256 * 8;
    auto run = [&](const float4 *src, size_t bytes, int rev, bool wr) {
        const int64_t nch = (int64_t)(bytes >> 16);
        if (wr) sweep<true><<<grid, 256>>>(src, dst, nch, rev, sink);
        else sweep<false><<<grid, 256>>>(src, dst, nch, rev, sink);
    };
    for (int i = 0; i < 50; ++i) run(flush, big, 0, false);  // clocks up
    const size_t sizes[] = {(size_t)64 << 20, (size_t)128 << 20, (size_t)192 << 20, (size_t)256 << 20, (size_t)320 << 20};
    for (int wr = 0; wr < 2; ++wr)
        for (size_t S : sizes) {
            float t[3][7];
            for (int r = 0; r < 7; ++r)
                for (int mode = 0; mode < 3; ++mode) {
                    run(flush, big, 0, false);                    // evict
                    if (mode > 0) run(a, S, 0, false);            // first pass (forward)
                    CK(hipEventRecord(e0));
                    run(a, S, mode == 2, wr != 0);                // the timed second pass
                    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&t[mode][r], e0, e1));
                }
            printf("S %3zu MiB%s:", S >> 20, wr ? " + S/4 written" : "              ");
            const char *nm[3] = {"cold", "fwd", "rev"};
            for (int mode = 0; mode < 3; ++mode) {
                std::sort(t[mode], t[mode] + 7);
                const double us = t[mode][3] * 1000;
                printf("  %s %7.1f us (%.2f TB/s)", nm[mode], us, (double)S / (us * 1e-6) / 1e12);
            }
            printf("\n");
        }
    return 0;
}
