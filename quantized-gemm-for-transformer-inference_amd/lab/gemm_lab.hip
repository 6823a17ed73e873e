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

typedef void (*KernelFn)(GemmArgs);
struct Variant { const char *name; KernelFn fn; bool check; bool tiled = false; };

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
    if (only) {
        std::vector<Variant> keep;
        for (auto &v : vs)
            if (std::string(v.name) == only || std::string(v.name) == "v1_direct") keep.push_back(v);
        vs = keep;
    }
    dim3 grid(p.tiles_m * p.tiles_n), block(kThreads);
    // reference output from v1_direct
    GemmArgs pr = p; pr.C = Cref;
    vs[0].fn<<<grid, block>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (!v.check) continue;
        CK(hipMemset(C, 0xff, (size_t)m * n * 4));
        v.fn<<<grid, block>>>(v.tiled ? pt : p);
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
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<grid, block>>>(pp);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<grid, block>>>(pp);
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
