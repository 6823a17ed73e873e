// pack_lab.hip -- development harness for the pack stage (not part of the library): times the
// single-pass pack against W-strip-only + X-rows kernels run sequentially or concurrently on two
// streams (fork/join with events).   Build: make -C .. packlab   Run: build/pack_lab [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#include "../csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int reps = argc > 4 ? atoi(argv[4]) : 20, rounds = 5;
    float *X, *W; void *PX, *PW, *PX2, *PW2;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&PX2, packed_bytes(m, k))); CK(hipMalloc(&PW2, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    PackedView vx2 = packed_view(PX2, m, k), vw2 = packed_view(PW2, n, k);
    PackedView vnone = packed_view(PX2, 0, k);
    hipStream_t s0, s1; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t fork, join; CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    auto single = [&]() { CK(launch_pack_single_pass(X, k, m, k, vx, W, n, n, vw, 127.f, s0)); };
    auto wonly = [&](hipStream_t s) { CK(launch_pack_single_pass(X, k, 0, k, vnone, W, n, n, vw2, 127.f, s)); };
    auto xonly = [&](hipStream_t s) { CK(launch_pack_rows(X, k, 1, m, k, 127.f, vx2, s)); };
    auto seq = [&]() { wonly(s0); xonly(s0); };
    auto conc = [&]() {
        CK(hipEventRecord(fork, s0)); CK(hipStreamWaitEvent(s1, fork, 0));
        xonly(s1); wonly(s0);
        CK(hipEventRecord(join, s1)); CK(hipStreamWaitEvent(s0, join, 0));
    };
    auto conc_xfirst = [&]() {
        CK(hipEventRecord(fork, s0)); CK(hipStreamWaitEvent(s1, fork, 0));
        wonly(s1); xonly(s0);
        CK(hipEventRecord(join, s1)); CK(hipStreamWaitEvent(s0, join, 0));
    };
    auto wo = [&]() { wonly(s0); };
    auto xo = [&]() { xonly(s0); };
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"single_pass", single}, {"w_then_x", seq}, {"concurrent", conc},
                         {"concurrent_b", conc_xfirst}, {"w_only", wo}, {"x_only", xo}};
    // parity: the split paths must give the same bytes as the single pass
    single(); seq(); CK(hipStreamSynchronize(s0));
    {
        size_t bx = packed_bytes(m, k), bw = packed_bytes(n, k);
        std::vector<char> a(bx), b(bx), c(bw), d(bw);
        CK(hipMemcpy(a.data(), vx.q, vx.rows_pad * vx.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), vx2.q, vx.rows_pad * vx.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), vw.q, vw.rows_pad * vw.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(d.data(), vw2.q, vw.rows_pad * vw.k_pad, hipMemcpyDeviceToHost));
        printf("parity x %s  w %s\n", memcmp(a.data(), b.data(), vx.rows_pad * vx.k_pad) ? "DIFF" : "same",
               memcmp(c.data(), d.data(), vw.rows_pad * vw.k_pad) ? "DIFF" : "same");
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
    const double bytes = 4.0 * m * k + 4.0 * k * n + (double)m * k + (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  (%.2f TB/s for the full pack bytes)\n", vs[i].name, v[v.size() / 2], v[0],
               bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
