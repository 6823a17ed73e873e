// segread_lab.hip -- development microbenchmark (not part of the library): HBM read rate of a row-major
// [K x N] fp32 matrix read in column blocks of Wc floats (row segments of 4*Wc bytes at a stride of 4*N
// bytes), 256 threads per block, each block a Wc-column x R-row panel -- the access shape of the
// column pack's pass 2 (Wc = 64) against wider panels.   Build: make -C .. segreadlab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int WC, int R>
__global__ __launch_bounds__(256) void panel_read(const float *__restrict__ src, int n, int k, float *out) {
    constexpr int kLanesPerRow = WC / 4;           // float4 per row segment
    constexpr int kRowsPerPass = 256 / kLanesPerRow;
    const int t = threadIdx.x, c4 = t % kLanesPerRow, r0 = t / kLanesPerRow;
    const int64_t col = (int64_t)blockIdx.x * WC + 4 * c4;
    const int64_t row0 = (int64_t)blockIdx.y * R;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int r = r0; r < R; r += kRowsPerPass) {
        const float4 v = *reinterpret_cast<const float4 *>(src + (row0 + r) * n + col);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = acc.x;
}

int main(int argc, char **argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 16384, n = argc > 2 ? atoi(argv[2]) : 4096;
    float *w, *out;
    CK(hipMalloc(&w, (size_t)k * n * 4)); CK(hipMalloc(&out, 64));
    CK(hipMemset(w, 0, (size_t)k * n * 4));
    void *flush; const size_t fb = (size_t)1 << 30; CK(hipMalloc(&flush, fb));
    struct V { const char *name; void (*launch)(const float *, int, int, float *); };
#define VAR(WC, R) {#WC "x" #R, [](const float *s, int n_, int k_, float *o) { \
        panel_read<WC, R><<<dim3(n_ / WC, k_ / R), 256>>>(s, n_, k_, o); }}
    std::vector<V> vs = {VAR(64, 1024), VAR(128, 1024), VAR(256, 1024), VAR(64, 4096), VAR(256, 256), VAR(1024, 256),
                         VAR(128, 512), VAR(256, 512)};
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    for (auto &v : vs) {
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
            CK(hipMemsetAsync(flush, r, fb));  // evict W from the Infinity Cache
            CK(hipEventRecord(a)); v.launch(w, n, k, out); CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
            float ms; CK(hipEventElapsedTime(&ms, a, z)); ts.push_back(ms * 1000);
        }
        std::sort(ts.begin(), ts.end());
        printf("panel %-10s %8.2f us  %.2f TB/s (cold)\n", v.name, ts[4], 4.0 * k * n / (ts[4] * 1e-6) / 1e12);
    }
    return 0;
}
