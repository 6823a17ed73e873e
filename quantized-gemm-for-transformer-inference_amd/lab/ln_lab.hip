// ln_lab.hip -- development check (not part of the library): add+layernorm with and without the fused
// pack must give identical Y; prints mismatch counts.  Build: make -C .. lnlab
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/encoder_ops.hip"

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
    printf("%d repeated fused launches: %zu runs with wrong rows, %zu wrong rows total\n", reps, badruns, badrows);
    return 0;
}
