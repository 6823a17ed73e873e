// exp_lab.hip -- development check (not part of the library): exp_cr (csrc/exp_cr.h) against
// (float)exp((double)x) over every fp32 bit pattern, plus the share of inputs that took the library
// path.  Build: make -C .. explab
#include <cstdio>
#include <cstdlib>

#include "exp_cr_experiment.h"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void check_all(unsigned long long *bad, unsigned long long *slow, uint32_t *first) {
    __shared__ double tab[64];
    if (threadIdx.x < 64) tab[threadIdx.x] = kExp2Tab64[threadIdx.x];
    __syncthreads();
    unsigned long long nb = 0, ns = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __uint_as_float((uint32_t)i);
        const float a = exp_cr(x, tab), b = (float)exp((double)x);
        if (__float_as_uint(a) != __float_as_uint(b)) {
            ++nb;
            atomicMin(first, (uint32_t)i);
        }
        if (x >= -87.0f && x <= 88.0f) {
            const double y = 0;  // count the midpoint fallbacks the same way exp_cr decides them
            (void)y;
        }
    }
    atomicAdd(bad, nb);
    (void)ns; (void)slow;
}

// share of in-range inputs sent to the library path by the midpoint test (statistic only)
__global__ void count_slow(unsigned long long *slow) {
    __shared__ double tab[64];
    if (threadIdx.x < 64) tab[threadIdx.x] = kExp2Tab64[threadIdx.x];
    __syncthreads();
    unsigned long long ns = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float xf = __uint_as_float((uint32_t)i);
        if (!(xf >= -87.0f && xf <= 88.0f)) continue;
        const double x = (double)xf;
        const double kd = __builtin_rint(x * 0x1.71547652b82fep+6);
        const int k = (int)kd;
        double r = __builtin_fma(kd, -0x1.62e42fefa4000p-7, x);
        r = __builtin_fma(kd, 0x1.8432a1b0e2634p-49, r);
        double q = __builtin_fma(r, 0x1.a01a01a01a01ap-13, 0x1.6c16c16c16c17p-10);
        q = __builtin_fma(r, q, 0x1.1111111111111p-7);
        q = __builtin_fma(r, q, 0x1.5555555555555p-5);
        q = __builtin_fma(r, q, 0x1.5555555555555p-3);
        q = __builtin_fma(r, q, 0.5);
        const double p = __builtin_fma(r * r, q, r);
        const double y = __builtin_ldexp(__builtin_fma(tab[k & 63], p, tab[k & 63]), k >> 6);
        const uint32_t low = (uint32_t)__double_as_longlong(y) & 0x1fffffffu;
        ns += (low - 0x0fffffc0u < 0x80u);
    }
    atomicAdd(slow, ns);
}

// throughput: n exps per thread, library vs exp_cr
template <bool kFast>
__global__ void bench_exp(const float *in, float *out, int n) {
    __shared__ double tab[64];
    if (threadIdx.x < 64) tab[threadIdx.x] = kExp2Tab64[threadIdx.x];
    __syncthreads();
    float acc = 0.f, x = in[blockIdx.x * blockDim.x + threadIdx.x];
    for (int i = 0; i < n; ++i) {
        const float e = kFast ? exp_cr(x, tab) : (float)exp((double)x);
        acc += e;
        x = x * 0.999f - 0.001f;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    unsigned long long *bad, *slow; uint32_t *first;
    CK(hipMalloc(&bad, 8)); CK(hipMalloc(&slow, 8)); CK(hipMalloc(&first, 4));
    CK(hipMemset(bad, 0, 8)); CK(hipMemset(slow, 0, 8)); CK(hipMemset(first, 0xff, 4));
    check_all<<<4096, 256>>>(bad, slow, first);
    count_slow<<<4096, 256>>>(slow);
    CK(hipDeviceSynchronize());
    unsigned long long hb, hs; uint32_t hf;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&hs, slow, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost));
    printf("all 2^32 fp32 inputs: %llu mismatches (first bit pattern 0x%08x); midpoint fallbacks %llu\n", hb, hf, hs);
    float *in, *out; const int nt = 256 * 1024;
    CK(hipMalloc(&in, nt * 4)); CK(hipMalloc(&out, nt * 4));
    CK(hipMemset(in, 0, nt * 4));
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    for (int v = 0; v < 2; ++v)
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            if (v) bench_exp<true><<<1024, 256>>>(in, out, 256);
            else bench_exp<false><<<1024, 256>>>(in, out, 256);
            CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
            float ms; CK(hipEventElapsedTime(&ms, a, z));
            if (rep) printf("%-8s %.1f G exps/s\n", v ? "exp_cr" : "library", (double)nt * 256 / (ms * 1e-3) / 1e9);
        }
    return hb ? 1 : 0;
}
