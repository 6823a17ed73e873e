// pack_lab.hip -- development harness for the pack stage (not part of the library): times the
// single-pass pack against W-strip-only + X-rows kernels run sequentially or concurrently on two
// streams (fork/join with events).   Build: make -C .. packlab   Run: build/pack_lab [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#include <hip/hip_ext.h>

#include "../csrc/pack.hip"

using namespace qgemm;

// ---- W-strip timeline probe: pack_w_strip_body's phases with s_memrealtime stamps (block-median) ----
__device__ unsigned long long g_wst[4096][6];
__global__ __launch_bounds__(1024) void wstrip_probe_kernel(const float *__restrict__ w, int64_t wsh, int k, int n,
                                                            float range, float *__restrict__ scale,
                                                            int8_t *__restrict__ q, int64_t k_pad, int nstrips) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
    const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c4 = t & 3, rq = t >> 2;
    if (t == 0) g_wst[bid][0] = __builtin_amdgcn_s_memrealtime();
    const int64_t n0 = (int64_t)strip * kWsCols;
    float *red = reinterpret_cast<float *>(lds);
    float *s_sh = red + 16 * 16;
    uint8_t *img = lds + 4096;
    const int64_t istride = k_pad + 16;
    float4 v[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            v[i][e] = (r < k) ? *reinterpret_cast<const float4 *>(w + (int64_t)r * wsh + n0 + 4 * c4)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            if (r >= 1 && r < k) {
                p0 = cand_max(p0, v[i][e].x);
                p1 = cand_max(p1, v[i][e].y);
                p2 = cand_max(p2, v[i][e].z);
                p3 = cand_max(p3, v[i][e].w);
            }
        }
    __syncthreads();
    if (t == 0) g_wst[bid][1] = __builtin_amdgcn_s_memrealtime();  // all loads consumed
#pragma unroll
    for (int off = 4; off < 64; off <<= 1) {
        p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
        p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
        p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
        p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
    }
    if (lane < 4) {
        red[wv * 16 + 4 * lane + 0] = p0;
        red[wv * 16 + 4 * lane + 1] = p1;
        red[wv * 16 + 4 * lane + 2] = p2;
        red[wv * 16 + 4 * lane + 3] = p3;
    }
    __syncthreads();
    if (t < kWsCols) {
        float pp = red[t];
#pragma unroll
        for (int ww = 1; ww < 16; ++ww) pp = fmaxf(pp, red[ww * 16 + t]);
        const float cw = absmax_finish(w[n0 + t], pp);
        s_sh[t] = inv_divide(range, cw);
        scale[n0 + t] = cw;
    }
    __syncthreads();
    if (t == 0) g_wst[bid][2] = __builtin_amdgcn_s_memrealtime();  // scales known
    const float s0 = s_sh[4 * c4 + 0], s1 = s_sh[4 * c4 + 1], s2 = s_sh[4 * c4 + 2], s3 = s_sh[4 * c4 + 3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r0 = 4 * rq + 1024 * i;
        if (r0 >= k_pad) continue;
        int qv[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool in = r0 + e < k;
            qv[e][0] = in ? quant_i8(v[i][e].x, s0) : 0;
            qv[e][1] = in ? quant_i8(v[i][e].y, s1) : 0;
            qv[e][2] = in ? quant_i8(v[i][e].z, s2) : 0;
            qv[e][3] = in ? quant_i8(v[i][e].w, s3) : 0;
        }
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
            *reinterpret_cast<uint32_t *>(img + (int64_t)(4 * c4 + cc) * istride + r0) =
                pack4(qv[0][cc], qv[1][cc], qv[2][cc], qv[3][cc]);
    }
    __syncthreads();
    if (t == 0) g_wst[bid][3] = __builtin_amdgcn_s_memrealtime();  // image in LDS
    const int64_t words = (int64_t)kWsCols * k_pad / 16;
    for (int64_t x = t; x < words; x += 1024) {
        const int64_t row = x / (k_pad / 16), col16 = x % (k_pad / 16);
        *reinterpret_cast<uint4 *>(q + (n0 + row) * k_pad + col16 * 16) =
            *reinterpret_cast<const uint4 *>(img + row * istride + col16 * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) g_wst[bid][4] = __builtin_amdgcn_s_memrealtime();  // stores acknowledged
}

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
    // same stream, the second kernel's dispatch packet without the barrier bit (hipExtAnyOrderLaunch):
    // it may start while the first still runs; the next ordinary launch waits for both
    auto x_any = [&](hipStream_t s) {
        hipExtLaunchKernelGGL((pack_rows_vec_kernel<16>), dim3((unsigned)(vx2.rows_pad / 4)), dim3(256), 0, s, nullptr,
                              nullptr, hipExtAnyOrderLaunch, (const float *)X, (int64_t)k, m, k, 127.f, vx2.scale,
                              vx2.q, vx2.rows_pad, vx2.k_pad);
        CK(hipGetLastError());
    };
    auto any_wx = [&]() { wonly(s0); x_any(s0); };
    auto wo = [&]() { wonly(s0); };
    auto xo = [&]() { xonly(s0); };
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"single_pass", single}, {"w_then_x", seq}, {"concurrent", conc},
                         {"concurrent_b", conc_xfirst}, {"anyorder_w_x", any_wx}, {"w_only", wo}, {"x_only", xo}};
    // parity: the split paths must give the same bytes as the single pass
    single(); any_wx(); CK(hipStreamSynchronize(s0));
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
    {   // W-strip phase timeline (block-median, 100 MHz ticks -> us), after the timed rounds
        const int nstrips = n / kWsCols;
        const size_t lds = 4096 + (size_t)kWsCols * (vw2.k_pad + 16);
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(wstrip_probe_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        for (int it = 0; it < 20; ++it)
            wstrip_probe_kernel<<<nstrips, 1024, lds, s0>>>(W, n, k, n, 127.f, vw2.scale, vw2.q, vw2.k_pad, nstrips);
        CK(hipStreamSynchronize(s0));
        std::vector<unsigned long long> st((size_t)4096 * 6);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wst), st.size() * 8));
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nstrips; ++b) t0 = std::min(t0, st[(size_t)b * 6]);
        const char *nm[5] = {"start", "loads consumed", "scales", "LDS image", "stores acked"};
        for (int ph = 0; ph < 5; ++ph) {
            std::vector<double> v;
            for (int b = 0; b < nstrips; ++b) v.push_back((st[(size_t)b * 6 + ph] - t0) * 0.01);
            std::sort(v.begin(), v.end());
            printf("wstrip %-15s  min %6.2f  median %6.2f  max %6.2f us (from first block start)\n", nm[ph], v[0],
                   v[v.size() / 2], v.back());
        }
    }
    const double bytes = 4.0 * m * k + 4.0 * k * n + (double)m * k + (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  (%.2f TB/s for the full pack bytes)\n", vs[i].name, v[v.size() / 2], v[0],
               bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
