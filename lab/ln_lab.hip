// ln_lab.hip -- development check (not part of the library): add+layernorm with and without the fused
// pack must give identical Y; prints mismatch counts.  Build: make -C .. lnlab
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/encoder_ops.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_lab(float *p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)(((uint32_t)i * 2654435761u + seed) % 20011u) / 10000.0f - 1.0f;
}

int main(int argc, char **argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 512, w = argc > 2 ? atoi(argv[2]) : 1024;
    float *A, *B, *Y1, *Y2; void *pk;
    CK(hipMalloc(&A, (size_t)rows * w * 4)); CK(hipMalloc(&B, (size_t)rows * w * 4));
    CK(hipMalloc(&Y1, (size_t)rows * w * 4)); CK(hipMalloc(&Y2, (size_t)rows * w * 4));
    CK(hipMalloc(&pk, packed_bytes(rows, w)));
    fill_lab<<<512, 256>>>(A, (int64_t)rows * w, 1); fill_lab<<<512, 256>>>(B, (int64_t)rows * w, 7);
    CK(launch_add_layernorm_rows(A, B, Y1, rows, w, nullptr));
    CK(launch_add_layernorm_rows_pack(A, B, Y2, rows, w, 127.0f, packed_view(pk, rows, w), nullptr));
    CK(hipDeviceSynchronize());
    std::vector<float> h1((size_t)rows * w), h2((size_t)rows * w);
    CK(hipMemcpy(h1.data(), Y1, h1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), Y2, h2.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0; int first = -1;
    for (size_t i = 0; i < h1.size(); ++i) if (memcmp(&h1[i], &h2[i], 4)) { if (first < 0) first = (int)i; ++bad; }
    printf("rows %d w %d: Y(pack) vs Y(plain) mismatches %zu (first at row %d)\n", rows, w, bad, first < 0 ? -1 : first / w);
    // checksums of everything the fused kernel writes, to compare two builds of the kernel
    PackedView v = packed_view(pk, rows, w);
    std::vector<unsigned char> hq(v.rows_pad * v.k_pad), hs(v.rows_pad * 4);
    CK(hipMemcpy(hq.data(), v.q, hq.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), v.scale, hs.size(), hipMemcpyDeviceToHost));
    auto fnv = [](const unsigned char *p, size_t n) { uint64_t h = 1469598103934665603ull; for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull; return h; };
    printf("hash Y %016llx q %016llx scale %016llx\n", (unsigned long long)fnv((const unsigned char *)h2.data(), h2.size() * 4),
           (unsigned long long)fnv(hq.data(), hq.size()), (unsigned long long)fnv(hs.data(), hs.size()));
    // host restatement of the plain kernel (sequential fp32 sums), then repeated launches bit-compared
    std::vector<float> ha((size_t)rows * w), hb((size_t)rows * w), hy((size_t)rows * w);
    CK(hipMemcpy(ha.data(), A, ha.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), B, hb.size() * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < rows; ++r) {
        const float *a = &ha[(size_t)r * w], *b = &hb[(size_t)r * w];
        volatile float s = 0.f;
        for (int c = 0; c < w; ++c) s = s + (a[c] + b[c]);
        const float mean = s / (float)w;
        volatile float v = 0.f;
        for (int c = 0; c < w; ++c) { volatile float d = (a[c] + b[c]) - mean; volatile float dd = d * d; v = v + dd; }
        const float var = v / (float)w;
        for (int c = 0; c < w; ++c) hy[(size_t)r * w + c] = ((a[c] + b[c]) - mean) / var;
    }
    size_t hbad = 0;
    for (size_t i = 0; i < h1.size(); ++i) hbad += memcmp(&h1[i], &hy[i], 4) != 0;
    printf("host restatement vs plain kernel: %zu mismatches\n", hbad);
    const int reps = argc > 3 ? atoi(argv[3]) : 200;
    size_t badruns = 0, badrows = 0;
    for (int it = 0; it < reps; ++it) {
        CK(launch_add_layernorm_rows_pack(A, B, Y2, rows, w, 127.0f, packed_view(pk, rows, w), nullptr));
        CK(hipMemcpy(h2.data(), Y2, h2.size() * 4, hipMemcpyDeviceToHost));
        size_t br = 0;
        for (int r = 0; r < rows; ++r) br += memcmp(&h2[(size_t)r * w], &hy[(size_t)r * w], (size_t)w * 4) != 0;
        badruns += br > 0; badrows += br;
    }
    // the scalar (general) kernel against the register-resident one the launchers picked
    {
        PackedView v = packed_view(pk, rows, w);
        void *pk2; float *Y3; CK(hipMalloc(&pk2, packed_bytes(rows, w))); CK(hipMalloc(&Y3, (size_t)rows * w * 4));
        PackedView v2 = packed_view(pk2, rows, w);
        CK(launch_add_layernorm_rows_pack(A, B, Y2, rows, w, 127.0f, v, nullptr));
        const size_t lds = sizeof(float) * 4 * ((w + 3) & ~3);
        add_layernorm_rows_kernel<true><<<(unsigned)((v2.rows_pad + 3) / 4), 256, lds>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
        CK(hipDeviceSynchronize());
        auto same = [&](const void *x, const void *z, size_t n) {
            std::vector<char> hx(n), hz(n);
            CK(hipMemcpy(hx.data(), x, n, hipMemcpyDeviceToHost)); CK(hipMemcpy(hz.data(), z, n, hipMemcpyDeviceToHost));
            return memcmp(hx.data(), hz.data(), n) == 0 ? "same" : "DIFF";
        };
        printf("vector vs scalar kernel: Y %s  q %s  scale %s\n", same(Y2, Y3, (size_t)rows * w * 4),
               same(v.q, v2.q, v.rows_pad * v.k_pad), same(v.scale, v2.scale, v.rows_pad * 4));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        if (w <= 1024) {  // the LDS-walking chain in the same register-resident kernel
            add_layernorm_rows_vec_kernel<true, 4, 0, false, false><<<(unsigned)((v2.rows_pad + 3) / 4), 256, sizeof(float) * 4 * w>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
            CK(hipDeviceSynchronize());
            printf("hop chain vs LDS chain: Y %s  q %s  scale %s\n", same(Y2, Y3, (size_t)rows * w * 4),
                   same(v.q, v2.q, v.rows_pad * v.k_pad), same(v.scale, v2.scale, v.rows_pad * 4));
        }
        if (w <= 1024) {  // the round-3..6 interleaved layout (one hop per 4 elements)
            add_layernorm_rows_vec_kernel<true, 4, 0, true, false><<<(unsigned)((v2.rows_pad + 3) / 4), 256, 0>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
            CK(hipDeviceSynchronize());
            printf("block hops vs interleaved hops: Y %s  q %s  scale %s\n", same(Y2, Y3, (size_t)rows * w * 4),
                   same(v.q, v2.q, v.rows_pad * v.k_pad), same(v.scale, v2.scale, v.rows_pad * 4));
        }
        for (int rep = 0; rep < 3; ++rep)
        for (int var = 0; var < 4; ++var) {
            if (var >= 2 && w > 1024) break;
            std::vector<float> ts;
            for (int it = 0; it < 30; ++it) {
                CK(hipEventRecord(e0));
                if (var == 0) CK(launch_add_layernorm_rows_pack(A, B, Y2, rows, w, 127.0f, v, nullptr));
                else if (var == 3) add_layernorm_rows_vec_kernel<true, 4, 0, true, false><<<(unsigned)((v2.rows_pad + 3) / 4), 256, 0>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
                else if (var == 2) add_layernorm_rows_vec_kernel<true, 4, 0, false, false><<<(unsigned)((v2.rows_pad + 3) / 4), 256, sizeof(float) * 4 * w>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
                else add_layernorm_rows_kernel<true><<<(unsigned)((v2.rows_pad + 3) / 4), 256, lds>>>(A, B, Y3, rows, w, v2.q, v2.scale, v2.k_pad, v2.rows_pad, 127.0f);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms * 1000);
            }
            std::sort(ts.begin(), ts.end());
            const char *nm[4] = {"vector (block hops, product)", "scalar", "vector (LDS chain)", "vector (interleaved hops)"};
            printf("%s kernel: median %.2f us\n", nm[var], ts[ts.size() / 2]);
        }
    }
    // phase stamps (s_memrealtime, 100 MHz) of the fused kernel, medians over rows
    {
        PackedView v = packed_view(pk, rows, w);
        const size_t lds = sizeof(float) * 4 * ((w + 3) & ~3);
        for (int it = 0; it < 5; ++it)
            add_layernorm_rows_vec_kernel<true, 4, 1><<<(unsigned)((v.rows_pad + 3) / 4), 256, lds>>>(A, B, Y2, rows, w, v.q, v.scale, v.k_pad, v.rows_pad, 127.0f);
        CK(hipDeviceSynchronize());
        static unsigned long long st[4096][8];
        CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ln_stamp), sizeof(st)));
        const char *names[6] = {"load a+b", "mean chain", "d^2", "var chain", "y loop", "pack"};
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int r = 0; r < rows && r < 4096; ++r) { t0 = std::min(t0, st[r][0]); t1 = std::max(t1, st[r][6]); }
        for (int ph = 0; ph < 6; ++ph) {
            std::vector<double> d;
            for (int r = 0; r < rows && r < 4096; ++r) d.push_back((st[r][ph + 1] - st[r][ph]) * 10.0 / 1000.0);
            std::sort(d.begin(), d.end());
            printf("  %-12s median %6.2f us  max %6.2f us\n", names[ph], d[d.size() / 2], d.back());
        }
        printf("  kernel span (first start to last end) %.2f us\n", (t1 - t0) * 10.0 / 1000.0);
    }
    printf("%d repeated fused launches: %zu runs with wrong rows, %zu wrong rows total\n", reps, badruns, badrows);
    return 0;
}
