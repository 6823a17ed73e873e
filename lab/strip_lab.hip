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

template <int kOrder, int kCols = 16>
__global__ __launch_bounds__(1024) void strip_read(const float *__restrict__ w, int n, int k, float *out) {
    const int nstrips = n / kCols, bid = blockIdx.x, nb = gridDim.x;
    int L;
    if (kOrder == 0) L = (bid & 7) * (nb >> 3) + (bid >> 3);  // XCD-contiguous ranges of the logical order
    else if (kOrder == 1) L = bid;
    else L = (int)(((long long)bid * 97) % nb);
    const int strip = L % nstrips, rowblk = L / nstrips;
    constexpr int kLanes = kCols / 4, kRowsPerPass = 1024 / kLanes;
    const int t = threadIdx.x, c4 = t % kLanes, rq = t / kLanes;
    const float *base = w + (int64_t)rowblk * (16 * kRowsPerPass) * n + (int64_t)strip * kCols + 4 * c4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const float4 *>(base + (int64_t)(rq + kRowsPerPass * i) * n);
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
    for (int n : {4096, 16384})
        for (int v = 0; v < 4; ++v) {
            std::vector<float> ts;
            const int cols = v == 0 ? 16 : v == 1 ? 32 : v == 2 ? 64 : 256;
            const int rows = 16 * 1024 / (cols / 4);  // rows one block reads (16 float4 per thread)
            const int nb = (n / cols) * (k / rows);   // blocks to cover all of W once (K split when rows < k)
            for (int r = 0; r < 7; ++r) {
                sweep<<<4096, 256>>>(reinterpret_cast<const float4 *>(fl), fb / 16, out);
                CK(hipEventRecord(a));
                // K-split blocks: block b reads strip b % nstrips, row block b / nstrips (order: XCD-contiguous
                // within the strip index, as in the pack)
                if (v == 0) strip_read<0, 16><<<nb, 1024>>>(w, n, k, out);
                if (v == 1) strip_read<0, 32><<<nb, 1024>>>(w, n, k, out);
                if (v == 2) strip_read<0, 64><<<nb, 1024>>>(w, n, k, out);
                if (v == 3) strip_read<0, 256><<<nb, 1024>>>(w, n, k, out);
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
                float ms; CK(hipEventElapsedTime(&ms, a, z)); ts.push_back(ms * 1000);
            }
            std::sort(ts.begin(), ts.end());
            printf("n %5d strip %3d cols (%4d-B segments, %4d rows per block) %8.2f us  %.2f TB/s\n", n, cols, cols * 4,
                   rows, ts[3], 4.0 * k * n / (ts[3] * 1e-6) / 1e12);
        }
    return 0;
}
