// mall_lab.hip -- LAB: streaming read rate of a buffer that stays resident in the 256-MB Infinity Cache
// (back-to-back launches over the same 128 MiB, the pack's input footprint at 4096^3) vs one that does not
// (1 GiB), with and without a 32-MiB write stream beside it.  Tells whether the pack (28.5 us for 128 MiB in +
// 32 MiB out when warm) is bound by the memory side or by its own access shape.
//   build/mall_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// each thread reads kPer float4 spaced a grid apart (fully coalesced 1-KiB wave instructions), XORs them,
// optionally writes one float4 per 4 read (the pack's 4:1 byte ratio)
template <int kPer, bool kWrite>
__global__ __launch_bounds__(512) void stream_kernel(const float4 *__restrict__ src, float4 *__restrict__ dst, int64_t n4,
                                                     int *sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n4; i += stride * kPer) {
        float4 v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) v[j] = i + j * stride < n4 ? src[i + j * stride] : make_float4(0, 0, 0, 0);
        int x = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) x ^= __float_as_int(v[j].x) ^ __float_as_int(v[j].y) ^ __float_as_int(v[j].z) ^ __float_as_int(v[j].w);
        if constexpr (kWrite) {
#pragma unroll
            for (int j = 0; j < kPer; j += 4)
                if (i + j * stride < n4) dst[(i + j * stride) / 4] = v[j];
        }
        if (x == 0x12345678) sink[0] = x;
    }
}

int main() {
    const size_t big = (size_t)1 << 30, hot = (size_t)128 << 20;
    float4 *src, *dst; int *sink;
    CK(hipMalloc(&src, big)); CK(hipMalloc(&dst, big / 4)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, big));
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    struct C { const char *name; size_t bytes; bool write; int grid; };
    std::vector<C> cs = {{"hot128MiB_read", hot, false, 256 * 8}, {"hot128MiB_read+w32", hot, true, 256 * 8},
                         {"hot128MiB_read_g4", hot, false, 256 * 4}, {"cold1GiB_read", big, false, 256 * 8},
                         {"cold1GiB_read+w", big, true, 256 * 8}};
    for (auto &c : cs) {
        const int64_t n4 = c.bytes / 16;
        auto launch = [&]() {
            if (c.write) stream_kernel<16, true><<<c.grid, 512>>>(src, dst, n4, sink);
            else stream_kernel<16, false><<<c.grid, 512>>>(src, dst, n4, sink);
        };
        for (int w = 0; w < 5; ++w) launch();
        std::vector<float> t;
        for (int r = 0; r < 20; ++r) {
            CK(hipEventRecord(a)); launch(); CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
            float ms; CK(hipEventElapsedTime(&ms, a, z)); t.push_back(ms * 1000);
        }
        std::sort(t.begin(), t.end());
        const double by = (double)c.bytes * (c.write ? 1.25 : 1.0);
        printf("%-22s median %8.2f us  min %8.2f us  %.2f TB/s (read%s)\n", c.name, t[t.size() / 2], t[0],
               by / (t[t.size() / 2] * 1e-6) / 1e12, c.write ? " + write" : "");
    }
    return 0;
}
