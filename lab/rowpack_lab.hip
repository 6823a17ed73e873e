// rowpack_lab.hip -- lab harness (not part of the library): the encoder's activation packs (pack_rows at 512 rows of
// 1 024 / 4 096 floats, BASELINE config 5) -- the staged launch (8 rows per 512-thread block, rows staged in LDS and
// written as whole 128-B lines: 64 blocks at 512 rows) against more, smaller blocks with direct stores, so that more
// CUs pull the rows (adopted in round 6 below 2 048 rows: pack_rows_pair_kernel).  Every variant is compared byte for byte
// with the staged one.
// Build: make -C lab rowpack_lab   Run: lab/build/rowpack_lab [rows len reps]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace qgemm {
namespace {
// 4 rows per 256-thread block (one wave per row, pack_rows_vec_body's 4-row group = the block), dword stores straight
// into the fragment-major q: twice the product's blocks
template <int R, int G>
__global__ __launch_bounds__(64 * G) void rows_direct_kernel(const float *__restrict__ src, int64_t sh, int rows, int len,
                                                             float range, float *__restrict__ scale, int8_t *__restrict__ q,
                                                             int64_t rows_pad, int64_t k_pad) {
    pack_rows_vec_body<R, false, false, false, G>(xcd_contig(blockIdx.x, 0, gridDim.x), src, sh, rows, len, range, scale, q,
                                                  rows_pad, k_pad);
}
}  // namespace
}  // namespace qgemm

__global__ void fill_lab(float *p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)(((uint32_t)i * 2654435761u + seed) % 20011u) / 10000.0f - 1.0f;
}

int main(int argc, char **argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 512, len = argc > 2 ? atoi(argv[2]) : 1024;
    const int reps = argc > 3 ? atoi(argv[3]) : 50;
    float *X; void *p0, *p1;
    CK(hipMalloc(&X, (size_t)rows * len * 4));
    CK(hipMalloc(&p0, packed_bytes(rows, len))); CK(hipMalloc(&p1, packed_bytes(rows, len)));
    fill_lab<<<512, 256>>>(X, (int64_t)rows * len, 3);
    PackedView v0 = packed_view(p0, rows, len), v1 = packed_view(p1, rows, len);
    const int R = rows_regs(len);
    if (R != 4 && R != 16) { printf("len %d: R %d not covered\n", len, R); return 1; }
    // the staged 8-row kernel (the launcher's choice from 2 048 rows; before round 6 at every row count)
    auto product = [&]() {
        if (R == 4) pack_rows_vec_kernel<4><<<(unsigned)(v0.rows_pad / 8), 512>>>(X, len, rows, len, 127.0f, v0.scale, v0.q, v0.rows_pad, v0.k_pad);
        else pack_rows_vec_kernel<16><<<(unsigned)(v0.rows_pad / 8), 512>>>(X, len, rows, len, 127.0f, v0.scale, v0.q, v0.rows_pad, v0.k_pad);
        CK(hipGetLastError());
    };
    auto direct = [&](int g) {
#define RD(Rv, Gv) rows_direct_kernel<Rv, Gv><<<(unsigned)(v1.rows_pad / Gv), 64 * Gv>>>(X, len, rows, len, 127.0f, v1.scale, v1.q, v1.rows_pad, v1.k_pad)
        if (R == 4) { if (g == 4) RD(4, 4); else if (g == 2) RD(4, 2); else RD(4, 1); }
        else { if (g == 4) RD(16, 4); else if (g == 2) RD(16, 2); else RD(16, 1); }
#undef RD
        CK(hipGetLastError());
    };
    auto same = [&](const void *x, const void *z, size_t n) {
        std::vector<char> hx(n), hz(n);
        CK(hipMemcpy(hx.data(), x, n, hipMemcpyDeviceToHost)); CK(hipMemcpy(hz.data(), z, n, hipMemcpyDeviceToHost));
        return memcmp(hx.data(), hz.data(), n) == 0 ? "same" : "DIFF";
    };
    product();
    for (int g : {4, 2, 1}) {
        CK(hipMemset(p1, 0x5a, packed_bytes(rows, len)));
        direct(g); CK(hipDeviceSynchronize());
        printf("rows %d len %d R %d: %d rows / block direct vs staged q %s scale %s\n", rows, len, R, g,
               same(v0.q, v1.q, v0.rows_pad * v0.k_pad), same(v0.scale, v1.scale, v0.rows_pad * 4));
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char *nm[4] = {"8 rows / block, staged lines", "4 rows / block, direct dword stores",
                         "2 rows / block, direct (product < 2048 rows)", "1 row / block, direct dword stores"};
    for (int round = 0; round < 3; ++round)
        for (int var = 0; var < 4; ++var) {
            std::vector<float> ts;
            for (int it = 0; it < reps; ++it) {  // 20 back-to-back launches per sample (the encoder's dependent chain)
                CK(hipEventRecord(e0));
                for (int l = 0; l < 20; ++l) { if (var == 0) product(); else direct(var == 1 ? 4 : var == 2 ? 2 : 1); }
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms * 1000 / 20);
            }
            std::sort(ts.begin(), ts.end());
            printf("  %-40s median %6.2f us  min %6.2f us per launch\n", nm[var], ts[ts.size() / 2], ts[0]);
        }
    return 0;
}
