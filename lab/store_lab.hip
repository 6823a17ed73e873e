// store_lab.hip -- development harness (not part of the library): how fast can 256 blocks x 256 KiB of fp32
// (the GEMM's 4096^3 output, one 256 x 256 tile per CU) be written?  The GEMM's store tail is ~10.4 us per
// block in-kernel; this times the bare store pattern of its epilogue (one 1-KiB row per wave instruction,
// 16 B per lane) and variants, back to back, one process.
// Build: make -C .. storelab   Run: build/store_lab [rounds]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int N = 4096;
typedef float v4f __attribute__((ext_vector_type(4)));

// mode 0: tile rows as the GEMM epilogue writes them (block = 256 x 256 tile, wave instruction = one row)
// mode 1: the same with nontemporal stores
// mode 2: the block's 256 KiB as one contiguous range (not the GEMM's layout: the best case)
template <int kMode>
__global__ __launch_bounds__(512) void store_tile(float *C, float v) {
    const int tid = threadIdx.x;
    const int tm = blockIdx.x / 16, tn = blockIdx.x % 16;
    const v4f x = {v, v + 1, v + 2, v + 3};
    if constexpr (kMode == 2) {
        v4f *p = reinterpret_cast<v4f *>(C + (size_t)blockIdx.x * 65536);
#pragma unroll 8
        for (int i = tid; i < 16384; i += 512) p[i] = x;
    } else {
        const int c4 = (tid & 63) * 4;
#pragma unroll 8
        for (int rr = tid >> 6; rr < 256; rr += 8) {
            v4f *p = reinterpret_cast<v4f *>(C + (size_t)(tm * 256 + rr) * N + tn * 256 + c4);
            if constexpr (kMode == 1) __builtin_nontemporal_store(x, p);
            else *p = x;
        }
    }
}

__global__ __launch_bounds__(512) void read_tile(const float *C, float *out) {
    const int tid = threadIdx.x;
    const int tm = blockIdx.x / 16, tn = blockIdx.x % 16;
    const int c4 = (tid & 63) * 4;
    v4f acc = {0, 0, 0, 0};
#pragma unroll 8
    for (int rr = tid >> 6; rr < 256; rr += 8)
        acc += *reinterpret_cast<const v4f *>(C + (size_t)(tm * 256 + rr) * N + tn * 256 + c4);
    if (acc[0] == 12345.f) out[tid] = acc[1];
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, reps = 50;
    float *C, *out;
    CK(hipMalloc(&C, (size_t)N * N * 4));
    CK(hipMalloc(&out, 4096));
    struct V { const char *name; void (*f)(float *, float *); };
    std::vector<V> vs = {
        {"store_rows", [](float *c, float *) { store_tile<0><<<256, 512>>>(c, 1.f); }},
        {"store_rows_nt", [](float *c, float *) { store_tile<1><<<256, 512>>>(c, 1.f); }},
        {"store_contig", [](float *c, float *) { store_tile<2><<<256, 512>>>(c, 1.f); }},
        {"read_rows", [](float *c, float *o) { read_tile<<<256, 512>>>(c, o); }},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            for (int w = 0; w < 5; ++w) vs[i].f(C, out);
            CK(hipEventRecord(e0));
            for (int j = 0; j < reps; ++j) vs[i].f(C, out);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-14s median %7.2f us  min %7.2f us  %.2f TB/s (64 MiB)\n", vs[i].name, v[v.size() / 2], v[0],
               64.0 * 1048576 / (v[v.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
