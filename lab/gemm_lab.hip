// gemm_lab.hip -- development harness: A/B the GEMM kernel variants and ablations in ONE process,
// interleaved rounds (cdna_hip_programming.md s5.4 rule 24), on random packed operands.
// Not part of the library.  Build: make -C .. lab   Run: build/gemm_lab [m n k rounds]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#include "gemm_variants.h"

using namespace qgemm;
using namespace qgemm::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_i8(int8_t *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (int8_t)((int)(mix64(seed + i) >> 56) - 128 > 127 ? 127 : (int)(mix64(seed + i) >> 56) - 128);
}
__global__ void fill_f(float *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 0.5f + (float)(mix64(seed + i) >> 40) * (1.0f / 16777216.0f);
}

// row-major [rows][k_pad] -> tiled 1-KiB blocks of 16 rows x 64 bytes
__global__ void to_tiled(const int8_t *src, int8_t *dst, int64_t rows, int64_t kp) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * kp; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / kp, k = i % kp;
        dst[((r >> 4) * (kp / 64) + (k >> 6)) * 1024 + (r & 15) * 64 + (k & 63)] = src[i];
    }
}


// peak mode: bare v_mfma_i32_16x16x64_i8 issue, operands in registers (8 A x 4 B fragments, 32
// independent accumulators = the product kernel's wave tile), 512-thread blocks (2 waves/SIMD), one
// block per CU; every iteration XORs a new pattern into the operands so their bits keep toggling as on
// random data.  Per-block stamps give the in-kernel clock.
__global__ __launch_bounds__(512, 1) void mfma_peak(int iters, uint64_t seed, int *out, unsigned long long *stamp) {
    const int tid = threadIdx.x;
    if (tid == 0) { stamp[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime(); stamp[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime(); }
    v4i a[8], b[4], acc[8][4];
    uint64_t z = mix64(seed + blockIdx.x * 512 + tid);
#pragma unroll
    for (int i = 0; i < 8; ++i) { z = mix64(z); a[i] = v4i{(int)z, (int)(z >> 32), (int)(z * 3), (int)(z >> 17)}; }
#pragma unroll
    for (int i = 0; i < 4; ++i) { z = mix64(z); b[i] = v4i{(int)z, (int)(z >> 32), (int)(z * 5), (int)(z >> 13)}; }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
    unsigned pat = (unsigned)z | 0x01010101u;
    for (int it = 0; it < iters; ++it) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pat = pat * 1664525u + 1013904223u;
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] ^= (int)pat;
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] ^= (int)(pat >> 3);
    }
    int x = 0;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
    out[blockIdx.x * 512 + tid] = x;
    if (tid == 0) { stamp[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime(); stamp[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime(); }
}

typedef void (*KernelFn)(GemmArgs);
struct Variant { const char *name; KernelFn fn; bool check; bool tiled = false; int threads = kThreads; int grid = 0; };

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 20;
    const char *only = argc > 5 ? argv[5] : nullptr;  // run just this variant (for rocprofv3)
    int64_t mp = round_up(m, 256), np_ = round_up(n, 256), kp = round_up(k, 128);
    int8_t *A, *B; float *Cx, *Cw, *C, *Cref;
    CK(hipMalloc(&A, mp * kp)); CK(hipMalloc(&B, np_ * kp));
    CK(hipMalloc(&Cx, mp * 4)); CK(hipMalloc(&Cw, np_ * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    fill_i8<<<4096, 256>>>(A, mp * kp, 1); fill_i8<<<4096, 256>>>(B, np_ * kp, 2);
    fill_f<<<64, 256>>>(Cx, mp, 3); fill_f<<<64, 256>>>(Cw, np_, 4);
    int8_t *At, *Bt;
    CK(hipMalloc(&At, mp * kp)); CK(hipMalloc(&Bt, np_ * kp));
    to_tiled<<<4096, 256>>>(A, At, mp, kp); to_tiled<<<4096, 256>>>(B, Bt, np_, kp);
    CK(hipDeviceSynchronize());
    GemmArgs p{A, B, Cx, Cw, C, n, 1, m, n, kp, (int)(mp / BM), (int)(np_ / BN), 1.0f / (127.0f * 127.0f)};
    GemmArgs pt = p; pt.A = At; pt.B = Bt;
    std::vector<Variant> vs = {
        {"v1_direct", gemm_i8_v1<kStoreDirect, true>, true},
        {"v1_nostore", gemm_i8_v1<kStoreNone, true>, false},
        {"v1_ldsstore", gemm_i8_v1<kStoreLds, true>, true},
        {"v2_direct", gemm_i8_v2<kStoreDirect, true>, true},
        {"v2_nostore", gemm_i8_v2<kStoreNone, true>, false},
        {"v2_ldsstore", gemm_i8_v2<kStoreLds, true>, true},
        {"v2p_direct", gemm_i8_v2<kStoreDirect, true, kPrio>, true},
        {"v2p_nostore", gemm_i8_v2<kStoreNone, true, kPrio>, false},
        {"v2_noglds_ns", gemm_i8_v2<kStoreNone, true, kNoGlds>, false},
        {"v2_nolds_ns", gemm_i8_v2<kStoreNone, true, kNoLdsRead>, false},
        {"v2_nothing_ns", gemm_i8_v2<kStoreNone, true, kNoLdsRead | kNoGlds>, false},
        {"v3_direct", gemm_i8_v3<kStoreDirect, true>, true},
        {"v3_nostore", gemm_i8_v3<kStoreNone, true>, false},
        {"v3p_direct", gemm_i8_v3<kStoreDirect, true, kPrio>, true},
        {"v3p_lds", gemm_i8_v3<kStoreLds, true, kPrio>, true},
        {"v3p_nostore", gemm_i8_v3<kStoreNone, true, kPrio>, false},
        {"v3p_ns_nobar", gemm_i8_v3<kStoreNone, true, kPrio | kNoBarrier>, false},
        {"v3p_ns_novm", gemm_i8_v3<kStoreNone, true, kPrio | kNoVmWait>, false},
        {"v3p_ns_noglds", gemm_i8_v3<kStoreNone, true, kPrio | kNoGlds>, false},
        {"v3p_ns_nothing", gemm_i8_v3<kStoreNone, true, kPrio | kNoGlds | kNoBarrier | kNoVmWait>, false},
        {"v7_lds", gemm_i8_v7<kStoreLds, false>, true},
        {"v7_nostore", gemm_i8_v7<kStoreNone, false>, false},
        {"v7d_lds", gemm_i8_v7<kStoreLds, true>, true},
        {"v7d_nostore", gemm_i8_v7<kStoreNone, true>, false},
        {"v9_lds", gemm_i8_v9<kStoreLds>, true, false, 256},
        {"v9_nostore", gemm_i8_v9<kStoreNone>, false, false, 256},
        {"v9t8_nostore", gemm_i8_v9<kStoreNone, 8>, false, false, 256},
        {"v9t32_nostore", gemm_i8_v9<kStoreNone, 32>, false, false, 256},
        {"v7e_lds", gemm_i8_v7<kStoreLds, false, 8, kV7Early>, true},
        {"v7e_nostore", gemm_i8_v7<kStoreNone, false, 8, kV7Early>, false},
        {"v5_s3", gemm_i8_v5<3>, true},
        {"v6_s4_direct", gemm_i8_v6<4, kStoreDirect>, true},
        {"v6_s4_lds", gemm_i8_v6<4, kStoreLds>, true},
        {"v6_s4_nostore", gemm_i8_v6<4, kStoreNone>, false},
        {"v6_s3_direct", gemm_i8_v6<3, kStoreDirect>, true},
        {"v6_s3_nostore", gemm_i8_v6<3, kStoreNone>, false},
        {"v6t_s4_lds", gemm_i8_v6<4, kStoreLds, true>, true, true},
        {"v6t_s4_nostore", gemm_i8_v6<4, kStoreNone, true>, false, true},
        {"v6t_s3_nostore", gemm_i8_v6<3, kStoreNone, true>, false, true},
    };
    // clock mode: build/gemm_lab m n k 0 clock -- per stamped variant, 2 s of back-to-back launches,
    // then one stamped launch: in-kernel clock = d(memtime)/d(memrealtime) x 100 MHz (median over blocks)
    if (only && std::string(only) == "clock") {
        struct SV { const char *name; KernelFn fn; };
        std::vector<SV> sv = {
            {"v7_lds", gemm_i8_v7<kStoreLds, false, 8, kV7Stamp>},
            {"v7_nostore", gemm_i8_v7<kStoreNone, false, 8, kV7Stamp>},
            {"v7_noglds_ns", gemm_i8_v7<kStoreNone, false, 8, kV7Stamp | kV7NoGlds>},
            {"v7e_lds", gemm_i8_v7<kStoreLds, false, 8, kV7Stamp | kV7Early>},
            {"v7e_nostore", gemm_i8_v7<kStoreNone, false, 8, kV7Stamp | kV7Early>},
        };
        dim3 g(p.tiles_m * p.tiles_n), b(kThreads);
        int nb = p.tiles_m * p.tiles_n;
        for (auto &v : sv) {
            hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
            int launches = 0; float ms = 0;
            CK(hipEventRecord(a));
            while (ms < 2000) {
                for (int i = 0; i < 200; ++i) v.fn<<<g, b>>>(p);
                launches += 200;
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
            }
            v.fn<<<g, b>>>(p);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st((size_t)4096 * 6);
            CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8));
            std::vector<double> loop_clk, epi_clk, loop_us, epi_us;
            for (int i = 0; i < nb; ++i) {
                const unsigned long long *s6 = &st[(size_t)i * 6];
                loop_clk.push_back((double)(s6[2] - s6[0]) / (double)(s6[3] - s6[1]) * 0.1);
                loop_us.push_back((double)(s6[3] - s6[1]) * 0.01);
                epi_clk.push_back((double)(s6[4] - s6[2]) / std::max(1.0, (double)(s6[5] - s6[3])) * 0.1);
                epi_us.push_back((double)(s6[5] - s6[3]) * 0.01);
            }
            auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
            printf("%-14s avg launch %7.2f us  loop: clock %.3f GHz, %6.2f us/block  epilogue: clock %.3f GHz, %6.2f us/block\n",
                   v.name, ms * 1000 / launches, med(loop_clk), med(loop_us), med(epi_clk), med(epi_us));
        }
        return 0;
    }
    // peak mode: build/gemm_lab 256 256 128 0 peak (sizes unused)
    if (only && std::string(only) == "peak") {
        int *out; unsigned long long *st;
        const int nb = 256, iters = 4096;
        CK(hipMalloc(&out, nb * 512 * 4)); CK(hipMalloc(&st, nb * 4 * 8));
        hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
        int launches = 0; float ms = 0;
        CK(hipEventRecord(a));
        while (ms < 2000) {
            for (int i = 0; i < 20; ++i) mfma_peak<<<nb, 512>>>(iters, 7 + launches + i, out, st);
            launches += 20;
            CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
        }
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h((size_t)nb * 4);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> clk;
        for (int i = 0; i < nb; ++i) clk.push_back((double)(h[i * 4 + 2] - h[i * 4]) / (double)(h[i * 4 + 3] - h[i * 4 + 1]) * 0.1);
        std::sort(clk.begin(), clk.end());
        const double ops = 2.0 * 16 * 16 * 64 * 32 * (double)iters * 8 * nb;  // per launch
        const double us = ms * 1000 / launches;
        printf("mfma_peak: %.1f us per launch, %.1f TOPS (%.1f%% of 5033), in-kernel clock median %.3f GHz (min %.3f max %.3f); "
               "at that clock the pipe peak is %.1f TOPS\n", us, ops / us * 1e-6, ops / us * 1e-6 / 50.332, clk[nb / 2], clk[0],
               clk[nb - 1], 256.0 * 4 * 2048 * clk[nb / 2] * 1e-3);
        return 0;
    }
    // small mode: build/gemm_lab m n k rounds small -- the small-tile kernels (128 and 64) at split-K
    // S = 1, 2, 4 on library-style scratch, interleaved rounds
    if (only && std::string(only) == "small") {
        unsigned *tick; int32_t *slabs;
        CK(hipMalloc(&tick, 4096)); CK(hipMemset(tick, 0, 4096));
        const int t64m = (int)(mp / 64), t64n = (int)(np_ / 64);
        CK(hipMalloc(&slabs, (size_t)t64m * t64n * 8 * 64 * 64 * 4 + (size_t)(mp / 128) * (np_ / 128) * 8 * 128 * 128 * 4));
        struct SV { const char *name; KernelFn fn; int TB, S; };
        std::vector<SV> sv = {
            {"t128_S1", gemm_i8_small<128>, 128, 1}, {"t128_S2", gemm_i8_small<128>, 128, 2},
            {"t128_S4", gemm_i8_small<128>, 128, 4}, {"t64_S1", gemm_i8_small<64>, 64, 1},
            {"t64_S2", gemm_i8_small<64>, 64, 2}, {"t64_S4", gemm_i8_small<64>, 64, 4},
            {"t64_S8", gemm_i8_small<64>, 64, 8},
            {"t64d3_S1", gemm_i8_small<64, 0, 3>, 64, 1}, {"t64d3_S2", gemm_i8_small<64, 0, 3>, 64, 2},
            {"t64d4_S1", gemm_i8_small<64, 0, 4>, 64, 1}, {"t64d4_S2", gemm_i8_small<64, 0, 4>, 64, 2},
            {"t64d4_S4", gemm_i8_small<64, 0, 4>, 64, 4}, {"t64d6_S1", gemm_i8_small<64, 0, 6>, 64, 1},
            {"t64d8_S1", gemm_i8_small<64, 0, 8>, 64, 1}, {"t64d8_S2", gemm_i8_small<64, 0, 8>, 64, 2},
            {"t32d2_S1", gemm_i8_small<32>, 32, 1}, {"t32d3_S1", gemm_i8_small<32, 0, 3>, 32, 1},
            {"t32d4_S1", gemm_i8_small<32, 0, 4>, 32, 1},
            // direct-load small tiles (gemm_i8_sd<TB, KW, D>)
            {"sd64k1d4", gemm_i8_sd<64, 1, 4>, 64, 1}, {"sd64k1d8", gemm_i8_sd<64, 1, 8>, 64, 1},
            {"sd64k4d4", gemm_i8_sd<64, 4, 4>, 64, 1}, {"sd64k4d6", gemm_i8_sd<64, 4, 6>, 64, 1},
            {"sd32k1d8", gemm_i8_sd<32, 1, 8>, 32, 1}, {"sd32k4d4", gemm_i8_sd<32, 4, 4>, 32, 1},
            {"sd32k4d8", gemm_i8_sd<32, 4, 8>, 32, 1}, {"sd32k4d12", gemm_i8_sd<32, 4, 12>, 32, 1},
        };
        auto args = [&](const SV &v, float *out) {
            GemmArgs q = p; q.C = out; q.splits = v.S; q.slabs = slabs; q.tickets = tick; q.reset_tickets = 1;
            q.tiles_m = (int)(mp / v.TB); q.tiles_n = (int)(np_ / v.TB);
            return q;
        };
        auto grid_of = [&](const SV &v) { return dim3((unsigned)((mp / v.TB) * (np_ / v.TB) * v.S)); };
        std::vector<float> h1((size_t)m * n), h2((size_t)m * n);
        sv[0].fn<<<grid_of(sv[0]), 256>>>(args(sv[0], Cref));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h1.data(), Cref, h1.size() * 4, hipMemcpyDeviceToHost));
        for (auto &v : sv) {
            if ((int64_t)(k / 128) / v.S < 1) continue;
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<grid_of(v), 256>>>(args(v, C));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h2.data(), C, h2.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < h1.size(); ++i) bad += memcmp(&h1[i], &h2[i], 4) != 0;
            printf("check %-8s mismatches %zu\n", v.name, bad);
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        std::vector<std::vector<float>> t(sv.size());
        for (int r = 0; r < std::max(rounds, 3); ++r)
            for (size_t vi = 0; vi < sv.size(); ++vi) {
                if ((int64_t)(k / 128) / sv[vi].S < 1) continue;  // a slice needs >= 1 k-step
                const GemmArgs q = args(sv[vi], C);
                const dim3 g = grid_of(sv[vi]);
                for (int w = 0; w < 3; ++w) sv[vi].fn<<<g, 256>>>(q);
                CK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i) sv[vi].fn<<<g, 256>>>(q);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[vi].push_back(ms * 1000 / reps);
            }
        for (size_t vi = 0; vi < sv.size(); ++vi) {
            if (t[vi].empty()) continue;
            auto v = t[vi]; std::sort(v.begin(), v.end());
            printf("%-8s median %8.2f us  min %8.2f us  (%u blocks)\n", sv[vi].name, v[v.size() / 2], v[0], grid_of(sv[vi]).x);
        }
        return 0;
    }
    // split mode: build/gemm_lab m n k rounds split -- the product kernel at split-K S = 1, 2, 4 (and the
    // slab-free ablation: tickets only, wrong sums) on library-style scratch (tickets zeroed once,
    // reducers re-zero them), interleaved rounds
    if (only && std::string(only) == "split") {
        const int tiles = p.tiles_m * p.tiles_n;
        unsigned *tick; int32_t *slabs;
        CK(hipMalloc(&tick, 4096)); CK(hipMemset(tick, 0, 4096));
        CK(hipMalloc(&slabs, (size_t)tiles * 8 * BM * BN * 4));
        struct SV { const char *name; KernelFn fn; int S; };
        std::vector<SV> sv = {
            {"S1", gemm_i8_v3<kStoreLds, true, kPrio>, 1},
            {"S2", gemm_i8_v3<kStoreLds, true, kPrio>, 2},
            {"S2_noslab", gemm_i8_v3<kStoreLds, true, kPrio | kNoSlab>, 2},
            {"S4", gemm_i8_v3<kStoreLds, true, kPrio>, 4},
            {"S4_noslab", gemm_i8_v3<kStoreLds, true, kPrio | kNoSlab>, 4},
        };
        auto args = [&](int S, float *out) {
            GemmArgs q = p; q.C = out; q.splits = S; q.slabs = slabs; q.tickets = tick; q.reset_tickets = 1;
            return q;
        };
        std::vector<float> h1((size_t)m * n), h2((size_t)m * n);
        sv[0].fn<<<dim3(tiles), dim3(kThreads)>>>(args(1, Cref));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h1.data(), Cref, h1.size() * 4, hipMemcpyDeviceToHost));
        for (auto &v : sv) {
            if (std::string(v.name).find("noslab") != std::string::npos) continue;
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<dim3(tiles * v.S), dim3(kThreads)>>>(args(v.S, C));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h2.data(), C, h2.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < h1.size(); ++i) bad += memcmp(&h1[i], &h2[i], 4) != 0;
            printf("check %-10s mismatches %zu\n", v.name, bad);
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        std::vector<std::vector<float>> t(sv.size());
        for (int r = 0; r < std::max(rounds, 3); ++r)
            for (size_t vi = 0; vi < sv.size(); ++vi) {
                const GemmArgs q = args(sv[vi].S, C);
                const dim3 g(tiles * sv[vi].S);
                for (int w = 0; w < 3; ++w) sv[vi].fn<<<g, dim3(kThreads)>>>(q);
                CK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i) sv[vi].fn<<<g, dim3(kThreads)>>>(q);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[vi].push_back(ms * 1000 / reps);
            }
        for (size_t vi = 0; vi < sv.size(); ++vi) {
            auto v = t[vi]; std::sort(v.begin(), v.end());
            printf("%-10s median %8.2f us  min %8.2f us\n", sv[vi].name, v[v.size() / 2], v[0]);
        }
        return 0;
    }
    if (only) {
        std::vector<Variant> keep;
        const std::string list = std::string(",") + only + ",";  // comma-separated names
        for (auto &v : vs)
            if (list.find(std::string(",") + v.name + ",") != std::string::npos || std::string(v.name) == "v1_direct")
                keep.push_back(v);
        vs = keep;
    }
    dim3 grid(p.tiles_m * p.tiles_n), block(kThreads);
    // reference output from v1_direct
    GemmArgs pr = p; pr.C = Cref;
    vs[0].fn<<<grid, dim3(vs[0].threads)>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (!v.check) continue;
        CK(hipMemset(C, 0xff, (size_t)m * n * 4));
        v.fn<<<v.grid ? dim3(v.grid) : grid, dim3(v.threads)>>>(v.tiled ? pt : p);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
        printf("check %-14s mismatches %zu\n", v.name, bad);
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            const GemmArgs &pp = vs[vi].tiled ? pt : p;
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<vs[vi].grid ? dim3(vs[vi].grid) : grid, dim3(vs[vi].threads)>>>(pp);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<vs[vi].grid ? dim3(vs[vi].grid) : grid, dim3(vs[vi].threads)>>>(pp);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms * 1000 / reps);
        }
    double ops = 2.0 * m * n * (double)k;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto v = t[vi]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  %7.1f TOPS  %5.1f%% of 5033\n", vs[vi].name, v[v.size() / 2], v[0],
               ops / (v[v.size() / 2] * 1e-6) / 1e12, 100 * ops / (v[v.size() / 2] * 1e-6) / 1e12 / 5033.2);
    }
    return 0;
}
