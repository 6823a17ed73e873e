// chain2_lab.hip -- development harness (not part of the library): the drop-in call's two launches
// (single-pass pack, then the ping-pong GEMM) back to back as bench.py runs them, each timed by
// hipExtLaunchKernel events, against the GEMM alone; and the kernel-boundary price of dirty L2
// lines: a kernel writing 32 MiB (plain / sc1 write-through / nt 16-B stores) ahead of the GEMM.
// Build: make -C .. chain2lab   Run: build/chain2_lab [reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>
#include <hip/hip_ext.h>

#define QGEMM_LAB 1
#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "gemm_legacy.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int kAux>
__global__ __launch_bounds__(256) void dirty_kernel(float *dst, int64_t n4) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
        __builtin_amdgcn_raw_buffer_store_b128(v4i_t{(int)i, 1, 2, 3}, rs, (uint32_t)(i * 16), 0, kAux);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const int M = 4096, N = 4096, K = 4096;
    float *X, *W, *C, *D;
    CK(hipMalloc(&X, (size_t)M * K * 4)); CK(hipMalloc(&W, (size_t)K * N * 4)); CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMalloc(&D, 64 << 20));
    void *pa, *pb;
    CK(hipMalloc(&pa, packed_bytes(M, K))); CK(hipMalloc(&pb, packed_bytes(N, K)));
    launch_fill_uniform(X, (int64_t)M * K, 1, -1.f, 1.f, 0);
    launch_fill_uniform(W, (int64_t)K * N, 2, -1.f, 1.f, 0);
    const PackedView va = packed_view(pa, M, K), vb = packed_view(pb, N, K);
    GemmArgs p{va.q, vb.q, va.scale, vb.scale, C, N, 1, M, N, va.k_pad, M / BM, N / BN, 1.0f / (127.0f * 127.0f)};
    p.splits = 1;
    const dim3 grid(p.tiles_m * p.tiles_n);
    hipEvent_t e[8];
    for (auto &x : e) CK(hipEventCreate(&x));
    auto gemm = [&](hipEvent_t a, hipEvent_t b) {
        hipExtLaunchKernelGGL((gemm_i8_pp<1, kEpiNone>), grid, dim3(kThreads), 0, 0, a, b, 0, p);
    };
    auto pack = [&](hipEvent_t a, hipEvent_t b) {
        CK(hipEventRecord(a));
        CK(launch_pack_single_pass(X, K, M, K, va, W, N, N, vb, 127.f, 0));
        CK(hipEventRecord(b));
    };
    auto dirty = [&](int mode) {
        const int64_t n4 = (32 << 20) / 16;
        if (mode == 1) dirty_kernel<0><<<2048, 256>>>(D, n4);
        if (mode == 2) dirty_kernel<16><<<2048, 256>>>(D, n4);  // sc1: write-through
        if (mode == 3) dirty_kernel<2><<<2048, 256>>>(D, n4);   // nt
    };
    // warm
    for (int i = 0; i < 20; ++i) { pack(e[0], e[1]); gemm(e[2], e[3]); }
    CK(hipDeviceSynchronize());
    const char *names[] = {"gemm alone", "gemm after dirty plain 32MiB", "gemm after sc1 32MiB", "gemm after nt 32MiB",
                           "pack+gemm (bench chain)"};
    for (int round = 0; round < 3; ++round)
        for (int mode = 0; mode < 5; ++mode) {
            std::vector<float> tg, tp, tw;
            for (int i = 0; i < reps; ++i) {
                CK(hipEventRecord(e[4]));
                if (mode == 4) pack(e[0], e[1]);
                else dirty(mode);
                gemm(e[2], e[3]);
                CK(hipEventRecord(e[5]));
                CK(hipEventSynchronize(e[5]));
                float ms;
                CK(hipEventElapsedTime(&ms, e[2], e[3])); tg.push_back(ms * 1000);
                CK(hipEventElapsedTime(&ms, e[4], e[5])); tw.push_back(ms * 1000);
                if (mode == 4) { CK(hipEventElapsedTime(&ms, e[0], e[1])); tp.push_back(ms * 1000); }
            }
            auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.f : v[v.size() / 2]; };
            printf("%-30s gemm %7.2f us  pack %7.2f us  whole %7.2f us\n", names[mode], med(tg), med(tp), med(tw));
        }
    // back-to-back chain throughput (as bench.py): pack, gemm, pack, gemm ... -- plain vs nt (non-temporal)
    // output stores: does keeping C out of the Infinity Cache leave X and W resident for the next pack?
    for (int round = 0; round < 3; ++round)
        for (int nt = 0; nt < 2; ++nt) {
            CK(hipEventRecord(e[6]));
            for (int i = 0; i < 200; ++i) {
                CK(launch_pack_single_pass(X, K, M, K, va, W, N, N, vb, 127.f, 0));
                if (nt) gemm_i8_pp<1, kEpiNone, kPPNtStore><<<grid, kThreads>>>(p);
                else gemm_i8_pp<1, kEpiNone><<<grid, kThreads>>>(p);
            }
            CK(hipEventRecord(e[7])); CK(hipEventSynchronize(e[7]));
            float ms; CK(hipEventElapsedTime(&ms, e[6], e[7]));
            printf("chain back to back (%s C stores): %.2f us per call\n", nt ? "nt" : "plain", ms * 1000 / 200);
        }
    // per-kernel times inside the chain, nt vs plain
    for (int nt = 0; nt < 2; ++nt) {
        std::vector<float> tg, tp;
        for (int i = 0; i < 40; ++i) {
            pack(e[0], e[1]);
            if (nt) hipExtLaunchKernelGGL((gemm_i8_pp<1, kEpiNone, kPPNtStore>), grid, dim3(kThreads), 0, 0, e[2], e[3], 0, p);
            else gemm(e[2], e[3]);
            CK(hipEventSynchronize(e[3]));
            float ms;
            CK(hipEventElapsedTime(&ms, e[2], e[3])); tg.push_back(ms * 1000);
            CK(hipEventElapsedTime(&ms, e[0], e[1])); tp.push_back(ms * 1000);
        }
        std::sort(tg.begin(), tg.end()); std::sort(tp.begin(), tp.end());
        printf("%s C stores: pack %.2f us, gemm %.2f us (medians)\n", nt ? "nt" : "plain", tp[tp.size() / 2], tg[tg.size() / 2]);
    }
    return 0;
}
