// strip_lab.hip -- development microbenchmark (not part of the library): HBM read rate of the pack's
// W-strip access (each 1024-thread block reads a 16-column x K-row strip of a row-major [K x N] fp32
// matrix, 64-B row segments, 16 float4 per thread in flight) under two block -> strip orders:
//   xcd : each XCD a contiguous range of strips (the pack kernels' order)
//   rr  : consecutive strips on consecutive XCDs (chip-wide sweep)
//   scat: strips spread by a large odd stride (no two concurrent strips adjacent)
// The cache is flushed by reading a 1-GiB buffer between launches.  Build: make -C .. striplab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int kOrder>
__global__ __launch_bounds__(1024) void strip_read(const float *__restrict__ w, int n, int k, float *out) {
    const int nstrips = n / 16, bid = blockIdx.x;
    int strip;
    if (kOrder == 0) {
        const int xcd = bid & 7, q8 = nstrips >> 3;
        strip = xcd * q8 + (bid >> 3);
    } else if (kOrder == 1) {
        strip = bid;
    } else {
        strip = (int)(((long long)bid * 97) % nstrips);
    }
    const int t = threadIdx.x, c4 = t & 3, rq = t >> 2;  // 4 lanes per row (64 B), 256 rows per pass
    const float *base = w + (int64_t)strip * 16 + 4 * c4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const float4 *>(base + (int64_t)(rq + 256 * i) * n);
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w; }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = acc.x;
}

__global__ void sweep(const float4 *p, int64_t n, float *out) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = p[i]; a.x += v.x; a.y += v.y;
    }
    if (a.x + a.y == 12345.f) out[1] = a.x;
}

int main() {
    const int k = 4096;
    float *w, *out, *fl;
    const int nmax = 16384;
    CK(hipMalloc(&w, (size_t)k * nmax * 4)); CK(hipMalloc(&out, 64));
    CK(hipMemset(w, 0, (size_t)k * nmax * 4));
    const size_t fb = (size_t)1 << 30; CK(hipMalloc(&fl, fb)); CK(hipMemset(fl, 0, fb));
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    for (int n : {4096, 8192, 16384})
        for (int order = 0; order < 3; ++order) {
            std::vector<float> ts;
            for (int r = 0; r < 7; ++r) {
                sweep<<<4096, 256>>>(reinterpret_cast<const float4 *>(fl), fb / 16, out);  // evict W (read-only)
                CK(hipEventRecord(a));
                if (order == 0) strip_read<0><<<n / 16, 1024>>>(w, n, k, out);
                if (order == 1) strip_read<1><<<n / 16, 1024>>>(w, n, k, out);
                if (order == 2) strip_read<2><<<n / 16, 1024>>>(w, n, k, out);
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
                float ms; CK(hipEventElapsedTime(&ms, a, z)); ts.push_back(ms * 1000);
            }
            std::sort(ts.begin(), ts.end());
            const char *nm[3] = {"xcd", "rr", "scat"};
            printf("n %5d order %-4s %8.2f us  %.2f TB/s\n", n, nm[order], ts[3], 4.0 * k * n / (ts[3] * 1e-6) / 1e12);
        }
    return 0;
}
