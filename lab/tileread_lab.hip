// tileread_lab.hip -- development harness (not part of the library): read rates of the W access shapes
// a column-absmax pack can use, on a row-major K x N fp32 matrix, each block reducing what it loaded to
// one max (no stores): 1-KiB row segments of 128/256-row tiles (the tile pack), 64-B / 32-B strip
// segments (the strip packs), and whole rows (contiguous).  Warm (back to back) and cold (after a 1-GiB
// sweep).  Build: make -C .. tilereadlab   Run: build/tileread_lab [K N]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include <hip/hip_runtime.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef int v4i_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

__device__ __forceinline__ float fold(v4i_t x, float p) {
    return fmaxf(fmaxf(p, fabsf(__int_as_float(x[0]))), fmaxf(fmaxf(fabsf(__int_as_float(x[1])), fabsf(__int_as_float(x[2]))),
                                                             fabsf(__int_as_float(x[3]))));
}

// tile: ROWS x 256 columns per block of T threads; thread t: columns 4*(t&63), rows (t>>6)*4 + e + (T/16)*i
template <int T, int ROWS>
__global__ __launch_bounds__(T) void read_tiles(const float *w, int K, int N, float *out) {
    constexpr int W = T / 64;
    constexpr int PER = ROWS / (4 * W);  // i iterations
    const int ncb = N / 256;
    const int cb = blockIdx.x % ncb, kt = blockIdx.x / ncb;
    const auto rs = rsrc(w, 0x7fffffff);
    const int t = threadIdx.x, wv = t >> 6;
    const uint32_t vo = (uint32_t)(cb * 256 + 4 * (t & 63)) * 4u;
    float p = 0.f;
    v4i_t x[PER][4];
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = kt * ROWS + 4 * wv + e + 4 * W * i;
            x[i][e] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)__builtin_amdgcn_readfirstlane(r * N * 4), 0);
        }
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) p = fold(x[i][e], p);
    if (p == 12345.f) out[blockIdx.x] = p;
}

// strip: C columns x all K rows per block of T threads (C = 8: 32-B segments, 16: 64-B), 16 float4 per thread
template <int T, int C>
__global__ __launch_bounds__(T) void read_strips(const float *w, int K, int N, float *out) {
    const int t = threadIdx.x;
    constexpr int LPR = C / 4;               // lanes per row
    constexpr int RPI = T / LPR;             // rows per "i" pass
    const auto rs = rsrc(w + blockIdx.x * C, 0x7fffffff);
    const uint32_t vo = (uint32_t)(((t / LPR) * N + 4 * (t % LPR)) * 4);
    float p = 0.f;
    v4i_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)(j * RPI * N * 4), 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) p = fold(x[j], p);
    if (p == 12345.f) out[blockIdx.x] = p;
}

// rows: one wave per 16-KiB run of a row, T threads, 16 float4 per lane
template <int T>
__global__ __launch_bounds__(T) void read_rows(const float *w, int K, int N, float *out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t run = (int64_t)blockIdx.x * (T / 64) + wv;  // 4096-float run index
    const auto rs = rsrc(w + run * 4096, 16384);
    float p = 0.f;
    v4i_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)lane * 16u, (uint32_t)(j * 1024), 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) p = fold(x[j], p);
    if (p == 12345.f) out[blockIdx.x] = p;
}

__global__ void sweep(const float4 *p, int64_t n, float *out) {
    float s = 0.f;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += p[i].x;
    if (s == 12345.f) out[0] = s;
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 16384;
    float *w, *out, *big;
    CK(hipMalloc(&w, (size_t)K * N * 4)); CK(hipMalloc(&out, 1 << 20)); CK(hipMalloc(&big, 1ull << 30));
    CK(hipMemset(w, 0x3c, (size_t)K * N * 4)); CK(hipMemset(big, 0, 1ull << 30));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    struct V { const char *name; void (*launch)(const float *, int, int, float *); };
    std::vector<V> vs = {
        {"tile 256x256, 1024 thr (1 KiB segs)", [](const float *w, int K, int N, float *o) { read_tiles<1024, 256><<<(K / 256) * (N / 256), 1024>>>(w, K, N, o); }},
        {"tile 128x256, 512 thr  (1 KiB segs)", [](const float *w, int K, int N, float *o) { read_tiles<512, 128><<<(K / 128) * (N / 256), 512>>>(w, K, N, o); }},
        {"tile 64x256, 256 thr   (1 KiB segs)", [](const float *w, int K, int N, float *o) { read_tiles<256, 64><<<(K / 64) * (N / 256), 256>>>(w, K, N, o); }},
        {"strip 16 cols, 1024 thr (64-B segs)", [](const float *w, int K, int N, float *o) { read_strips<1024, 16><<<N / 16, 1024>>>(w, K, N, o); }},
        {"strip 8 cols, 512 thr  (32-B segs)", [](const float *w, int K, int N, float *o) { read_strips<512, 8><<<N / 8, 512>>>(w, K, N, o); }},
        {"rows, 1024 thr (16-KiB runs)", [](const float *w, int K, int N, float *o) { read_rows<1024><<<(int)((int64_t)K * N / 4096 / 16), 1024>>>(w, K, N, o); }},
        {"rows, 256 thr (16-KiB runs)", [](const float *w, int K, int N, float *o) { read_rows<256><<<(int)((int64_t)K * N / 4096 / 4), 256>>>(w, K, N, o); }},
    };
    const double bytes = (double)K * N * 4;
    for (int cold = 0; cold < 2; ++cold)
        for (auto &v : vs) {
            std::vector<float> t;
            for (int r = 0; r < 15; ++r) {
                if (cold) sweep<<<4096, 256>>>((const float4 *)big, (1ll << 30) / 16, out);
                else v.launch(w, K, N, out);
                CK(hipEventRecord(a));
                v.launch(w, K, N, out);
                CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
                float ms; CK(hipEventElapsedTime(&ms, a, b));
                t.push_back(ms * 1000);
            }
            std::sort(t.begin(), t.end());
            printf("%s %-40s %8.2f us  %6.2f TB/s\n", cold ? "cold" : "warm", v.name, t[7], bytes / t[7] * 1e-6);
        }
    return 0;
}
