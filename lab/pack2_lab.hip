// pack2_lab.hip -- development harness (not part of the library): the single-pass pack with 16-column
// W strips (1024-thread blocks, one per CU) against 8-column strips (512-thread blocks, two per CU),
// bit-compared.  Experiments measured here and dropped: 1024-thread 8-column blocks forced to 64
// VGPRs (two blocks per CU, X rows two waves each): spills, 36.7 us at 4096^3; a dispatch order that
// sweeps the columns chip-wide instead of XCD-contiguous strip ranges: +13 us at n = 16384; the
// 8-column kernel held to 80 VGPRs for three blocks per CU: 8 VGPRs spilled, 33.4 vs 28.8 us.
// Build: make -C .. pack2lab   Run: build/pack2_lab [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

namespace qgemm {
namespace {

}  // namespace
}  // namespace qgemm

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int reps = argc > 4 ? atoi(argv[4]) : 20, rounds = 7;
    float *X, *W; void *PX, *PW, *PX2, *PW2;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&PX2, packed_bytes(m, k))); CK(hipMalloc(&PW2, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    PackedView vx2 = packed_view(PX2, m, k), vw2 = packed_view(PW2, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    auto single = [&]() { CK(launch_pack_single_pass_kind(X, k, m, k, vx, W, n, n, vw, 127.f, s0, 16)); };
    auto p8h = [&]() { CK(launch_pack_single_pass_kind(X, k, m, k, vx2, W, n, n, vw2, 127.f, s0, 8)); };
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"strips16", single}, {"strips8", p8h}};
    {
    CK(hipMemset(PX2, 0x5a, packed_bytes(m, k))); CK(hipMemset(PW2, 0x5a, packed_bytes(n, k)));
    single(); p8h(); CK(hipStreamSynchronize(s0));
    {
        auto cmp = [&](const void *a, const void *b, size_t bytes) {
            std::vector<char> ha(bytes), hb(bytes);
            CK(hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost));
            return memcmp(ha.data(), hb.data(), bytes) ? "DIFF" : "same";
        };
        printf("parity (8- vs 16-column strips): xq %s  wq %s  cx %s  cw %s\n", cmp(vx.q, vx2.q, vx.rows_pad * vx.k_pad),
               cmp(vw.q, vw2.q, vw.rows_pad * vw.k_pad), cmp(vx.scale, vx2.scale, vx.rows_pad * 4),
               cmp(vw.scale, vw2.scale, vw.rows_pad * 4));
    }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            for (int w = 0; w < 3; ++w) vs[i].f();
            CK(hipEventRecord(e0, s0));
            for (int j = 0; j < reps; ++j) vs[i].f();
            CK(hipEventRecord(e1, s0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    // cold-cache timing: a 1-GiB sweep (memset) between launches evicts the inputs from the 256-MB
    // Infinity Cache; each launch is timed alone with events
    {
        void *flush; const size_t fb = (size_t)1 << 30;
        CK(hipMalloc(&flush, fb));
        hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
        for (size_t i = 0; i < vs.size(); ++i) {
            std::vector<float> v;
            for (int r = 0; r < 15; ++r) {
                CK(hipMemsetAsync(flush, r, fb, s0));
                CK(hipEventRecord(a, s0)); vs[i].f(); CK(hipEventRecord(z, s0)); CK(hipEventSynchronize(z));
                float ms; CK(hipEventElapsedTime(&ms, a, z)); v.push_back(ms * 1000);
            }
            std::sort(v.begin(), v.end());
            printf("%-14s cold median %8.2f us  min %8.2f us\n", vs[i].name, v[v.size() / 2], v[0]);
        }
        CK(hipFree(flush));
    }
    const double bytes = 4.0 * m * k + 4.0 * k * n + (double)m * k + (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  (%.2f TB/s for the full pack bytes)\n", vs[i].name, v[v.size() / 2], v[0],
               bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
