// chain_lab.hip -- development microbenchmark (not part of the library): cycles per dependent fp32 add
// in a sequential chain, with all 64 lanes active vs one lane, and with two interleaved chains.
// Build: make -C .. chainlab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int kMode>
__global__ void chain(const float *in, float *out, long long *cyc, int n) {
    const int lane = threadIdx.x;
    float a = in[lane], b = in[lane + 64], s = 0.0f, s2 = 0.0f;
    const long long t0 = __builtin_readcyclecounter();
    if (kMode == 0 || lane == 0) {
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                s = __fadd_rn(s, a);
                if (kMode == 2) s2 = __fadd_rn(s2, b);
            }
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    out[lane] = s + s2;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *in, *out; long long *cyc;
    CK(hipMalloc(&in, 4096)); CK(hipMalloc(&out, 4096)); CK(hipMalloc(&cyc, 8 * 1024));
    CK(hipMemset(in, 0, 4096));
    const int n = 1000;
    const char *names[3] = {"64 lanes, one chain", "1 lane, one chain", "1 lane, two chains"};
    for (int m = 0; m < 3; ++m) {
        for (int it = 0; it < 3; ++it) {
            if (m == 0) chain<0><<<1, 64>>>(in, out, cyc, n);
            if (m == 1) chain<1><<<1, 64>>>(in, out, cyc, n);
            if (m == 2) chain<2><<<1, 64>>>(in, out, cyc, n);
        }
        CK(hipDeviceSynchronize());
        long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
        printf("%-22s %.2f cycles per add step\n", names[m], (double)c / (32.0 * n));
    }
    return 0;
}
