// pp_lab.hip -- development harness for the ping-pong GEMM (gemm_i8_pp) against the round-1 product
// kernel (gemm_i8_v3), and the bare int8-MFMA peak probe.  Not part of the library.
//   build/pp_lab m n k rounds [names]      A/B, interleaved rounds in one process, bit-checked vs v3
//   build/pp_lab 0 0 0 0 peak              bare MFMA issue: 16x16x64 and 32x32x32, 2 s each
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#define QGEMM_LAB 1
#include "gemm_legacy.h"

using namespace qgemm;
using namespace qgemm::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_i8(int8_t *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (int8_t)((int)(mix64(seed + i) >> 56) - 128);
}
__global__ void fill_f(float *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 0.5f + (float)(mix64(seed + i) >> 40) * (1.0f / 16777216.0f);
}

typedef int v16i_t __attribute__((ext_vector_type(16)));

// Bare MFMA issue: the product kernel's wave tile (128 x 64 outputs, 32 independent 16x16 accumulators
// or 8 32x32 ones), two operand sets of random bits in registers (each MFMA reads a different (a, b)
// pair, so the operands change from one MFMA to the next as in the GEMM), 512-thread blocks = 2 waves
// per SIMD, one block per CU.  No VALU, no memory in the loop.  In-kernel clock from stamps.
template <bool k32>
__global__ __launch_bounds__(512, 1) void mfma_peak(int iters, uint64_t seed, int *out, unsigned long long *stamp) {
    const int tid = threadIdx.x;
    if (tid == 0) { stamp[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime(); stamp[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime(); }
    uint64_t z = mix64(seed + blockIdx.x * 512 + tid);
    int x = 0;
    if constexpr (!k32) {
        v4i a[2][8], b[2][4], acc[8][4];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int i = 0; i < 8; ++i) { z = mix64(z); a[s][i] = v4i{(int)z, (int)(z >> 32), (int)(z * 3), (int)(z >> 17)}; }
#pragma unroll
            for (int i = 0; i < 4; ++i) { z = mix64(z); b[s][i] = v4i{(int)z, (int)(z >> 32), (int)(z * 5), (int)(z >> 13)}; }
        }
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[s][mi], b[s][ni], acc[mi][ni], 0, 0, 0);
        }
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
    } else {
        v4i a[4][4], b[4][2];
        v16i_t acc[4][2];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { z = mix64(z); a[s][i] = v4i{(int)z, (int)(z >> 32), (int)(z * 3), (int)(z >> 17)}; }
#pragma unroll
            for (int i = 0; i < 2; ++i) { z = mix64(z); b[s][i] = v4i{(int)z, (int)(z >> 32), (int)(z * 5), (int)(z >> 13)}; }
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = v16i_t{};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s][mi], b[s][ni], acc[mi][ni], 0, 0, 0);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int r = 0; r < 16; ++r) x ^= acc[mi][ni][r];
    }
    out[blockIdx.x * 512 + tid] = x;
    if (tid == 0) { stamp[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime(); stamp[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime(); }
}

template <bool k32>
static void run_peak(double seconds) {
    int *out; unsigned long long *st;
    const int nb = 256, iters = 2048;  // 2048 x 64 16x16x64 MFMAs per wave (= 32 x 32x32x32 x 64)
    CK(hipMalloc(&out, nb * 512 * 4)); CK(hipMalloc(&st, nb * 4 * 8));
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    int launches = 0; float ms = 0;
    CK(hipEventRecord(a));
    while (ms < seconds * 1000) {
        for (int i = 0; i < 20; ++i) mfma_peak<k32><<<nb, 512>>>(iters, 7 + launches + i, out, st);
        launches += 20;
        CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
    }
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)nb * 4);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int i = 0; i < nb; ++i) clk.push_back((double)(h[i * 4 + 2] - h[i * 4]) / (double)(h[i * 4 + 3] - h[i * 4 + 1]) * 0.1);
    std::sort(clk.begin(), clk.end());
    // per wave per iteration: 64 MFMAs 16x16x64 (32768 ops each) or 32 MFMAs 32x32x32 (65536 ops each)
    const double ops = 64.0 * 32768 * (double)iters * 8 * nb;
    const double us = ms * 1000 / launches;
    printf("mfma_peak %s: %.1f us per launch, %.1f TOPS (%.1f%% of 5033), in-kernel clock median %.3f GHz "
           "(min %.3f max %.3f); pipe peak at that clock %.1f TOPS -> %.1f%% of it\n",
           k32 ? "32x32x32" : "16x16x64", us, ops / us * 1e-6, ops / us * 1e-6 / 50.332, clk[nb / 2], clk[0], clk[nb - 1],
           256.0 * 4 * 2048 * clk[nb / 2] * 1e-3, 100.0 * (ops / us * 1e-6) / (256.0 * 4 * 2048 * clk[nb / 2] * 1e-3));
    CK(hipFree(out)); CK(hipFree(st));
}

typedef void (*KernelFn)(GemmArgs);
struct Variant { const char *name; KernelFn fn; };

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 20;
    const char *only = argc > 5 ? argv[5] : nullptr;
    if (only && std::string(only) == "peak") {
        run_peak<false>(2.0); run_peak<true>(2.0); run_peak<false>(2.0); run_peak<true>(2.0);
        return 0;
    }
    const bool clock_mode = only && std::string(only) == "clock";
    int64_t mp = round_up(m, 256), np_ = round_up(n, 256), kp = round_up(k, 128);
    int8_t *A, *B; float *Cx, *Cw, *C, *Cref;
    CK(hipMalloc(&A, mp * kp)); CK(hipMalloc(&B, np_ * kp));
    CK(hipMalloc(&Cx, mp * 4)); CK(hipMalloc(&Cw, np_ * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    fill_i8<<<4096, 256>>>(A, mp * kp, 1); fill_i8<<<4096, 256>>>(B, np_ * kp, 2);
    fill_f<<<64, 256>>>(Cx, mp, 3); fill_f<<<64, 256>>>(Cw, np_, 4);
    CK(hipDeviceSynchronize());
    GemmArgs p{A, B, Cx, Cw, C, n, 1, m, n, kp, (int)(mp / BM), (int)(np_ / BN), 1.0f / (127.0f * 127.0f)};
    std::vector<Variant> vs = {
        {"v3p", gemm_i8_v3<kStoreLds, true, kPrio>},
        {"pp0", gemm_i8_pp<0>},
        {"pp1", gemm_i8_pp<1>},
        {"pp1_nostore", gemm_i8_pp<1, kEpiNone, kPPNoStore>},
        {"pp1_nodma_ns", gemm_i8_pp<1, kEpiNone, kPPNoStore | kPPNoDma>},
        {"pp2", gemm_i8_pp<2>},
        {"pp2_nostore", gemm_i8_pp<2, kEpiNone, kPPNoStore>},
    };
    if (clock_mode) {
        // per variant: 2 s of back-to-back launches, then one stamped launch; per block the main-loop and
        // epilogue durations and in-kernel clocks (median over blocks)
        struct SV { const char *name; KernelFn fn; };
        std::vector<SV> sv = {
            {"pp1", gemm_i8_pp<1, kEpiNone, kPPStamp>},
            {"pp1_nostore", gemm_i8_pp<1, kEpiNone, kPPStamp | kPPNoStore>},
            {"pp1_nodma_ns", gemm_i8_pp<1, kEpiNone, kPPStamp | kPPNoStore | kPPNoDma>},
            {"pp2", gemm_i8_pp<2, kEpiNone, kPPStamp>},
        };
        dim3 g(p.tiles_m * p.tiles_n), b(kThreads);
        const int nb = p.tiles_m * p.tiles_n;
        for (auto &v : sv) {
            hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
            int launches = 0; float ms = 0;
            CK(hipEventRecord(a));
            while (ms < 2000) {
                for (int i = 0; i < 200; ++i) v.fn<<<g, b>>>(p);
                launches += 200;
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st((size_t)4096 * 6);
            CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_pp_stamp), st.size() * 8));
            std::vector<double> lc, lu, ec, eu;
            for (int i = 0; i < nb; ++i) {
                const unsigned long long *q = &st[(size_t)i * 6];
                lc.push_back((double)(q[2] - q[0]) / (double)(q[3] - q[1]) * 0.1);
                lu.push_back((double)(q[3] - q[1]) * 0.01);
                ec.push_back((double)(q[4] - q[2]) / std::max(1.0, (double)(q[5] - q[3])) * 0.1);
                eu.push_back((double)(q[5] - q[3]) * 0.01);
            }
            auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
            printf("%-14s avg launch %7.2f us  loop: clock %.3f GHz, %6.2f us/block  epilogue: clock %.3f GHz, %6.2f us/block\n",
                   v.name, ms * 1000 / launches, med(lc), med(lu), med(ec), med(eu));
        }
        return 0;
    }
    if (only) {
        std::vector<Variant> keep;
        const std::string list = std::string(",") + only + ",";
        for (auto &v : vs)
            if (list.find(std::string(",") + v.name + ",") != std::string::npos) keep.push_back(v);
        vs = keep;
    }
    dim3 grid(p.tiles_m * p.tiles_n), block(kThreads);
    GemmArgs pr = p; pr.C = Cref;
    gemm_i8_v3<kStoreLds, true, kPrio><<<grid, block>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<grid, block>>>(p);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-8s rep %d mismatches %zu\n", v.name, rep, bad);
        }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<grid, block>>>(p);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<grid, block>>>(p);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms * 1000 / reps);
        }
    double ops = 2.0 * m * n * (double)k;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto v = t[vi]; std::sort(v.begin(), v.end());
        printf("%-8s median %8.2f us  min %8.2f us  %7.1f TOPS  %5.1f%% of 5033\n", vs[vi].name, v[v.size() / 2], v[0],
               ops / (v[v.size() / 2] * 1e-6) / 1e12, 100 * ops / (v[v.size() / 2] * 1e-6) / 1e12 / 5033.2);
    }
    return 0;
}
