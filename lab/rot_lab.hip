// rot_lab.hip -- LAB: the order in which gemm_i8_fm's waves store their output rows (GemmArgs::rot_rows), at the
// FFN-up shape (2048 x 16384 x 4096: 64-KiB output rows, where the product rotates) and the C4 shard (16-KiB rows,
// where it does not).  Random packed int8 operands, GEMM back to back, interleaved rounds; every variant's output
// compared with rot_rows 0.
//   rot 1: (7 tn + 3 tm) mod 32 row pairs (product).  Round 4 also ran, through a temporary switch on rot_rows in
//   the kernel, 2: + 8 x wave, 3: + 16 x wm, 4: (13 tn + 5 tm), 5: tn + 8 tm, 6: + 16 x wn -- FFN up 117.0-118.4
//   vs 117.8 us for rot 1 and 122.3 unrotated, the shard 114.4-115.6 for all (profiles/r04_rot_variants_lab.log):
//   nothing better than the product's order, so the switch was removed; this harness now compares 0 and 1.
//   Round 5: gemm_i8_fm stores from registers and the field is GemmArgs::wide_rows (paired nontemporal stores at 0,
//   plain per-tile stores at 1); the rotation is gone (lab/gemm_ds.h), so rot 1 here now means wide-row stores.
//   build/rot_lab [rounds]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_bytes(uint32_t *p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = x;
    }
}
__global__ void fill_scales(float *p, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = 0.5f + (float)(i % 97) / 97.0f;
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, reps = 10;
    struct Shape { int m, n, k; };
    const Shape shapes[2] = {{2048, 16384, 4096}, {8192, 4096, 4096}};
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (const Shape &sh : shapes) {
        const int m = sh.m, n = sh.n, k = sh.k;
        int8_t *A, *B; float *Cx, *Cw, *C;
        CK(hipMalloc(&A, (size_t)m * k)); CK(hipMalloc(&B, (size_t)n * k));
        CK(hipMalloc(&Cx, m * 4)); CK(hipMalloc(&Cw, n * 4)); CK(hipMalloc(&C, (size_t)m * n * 4));
        fill_bytes<<<2048, 256>>>(reinterpret_cast<uint32_t *>(A), (int64_t)m * k / 4, 1u);
        fill_bytes<<<2048, 256>>>(reinterpret_cast<uint32_t *>(B), (int64_t)n * k / 4, 2u);
        fill_scales<<<(m + 255) / 256, 256>>>(Cx, m); fill_scales<<<(n + 255) / 256, 256>>>(Cw, n);
        auto gemm = [&](int rot) {
            GemmArgs p{};
            p.A = A; p.B = B; p.Cx = Cx; p.Cw = Cw; p.C = C; p.csh = n; p.csw = 1; p.m = m; p.n = n; p.k_pad = k;
            p.tiles_m = m / 256; p.tiles_n = n / 256; p.inv_r2 = 1.0f / (127.f * 127.f); p.splits = 1; p.wide_rows = rot;
            gemm_i8_fm<kEpiNone><<<p.tiles_m * p.tiles_n, 256>>>(p);
        };
        std::vector<float> ref((size_t)m * n), got(ref.size());
        gemm(0); CK(hipDeviceSynchronize()); CK(hipGetLastError());
        CK(hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
        for (int r = 1; r <= 1; ++r) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            gemm(r); CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
            if (memcmp(ref.data(), got.data(), ref.size() * 4)) printf("rot %d DIFF\n", r);
        }
        for (int i = 0; i < 200; ++i) gemm(1);  // clocks up
        std::vector<float> t[2];
        for (int rd = 0; rd < rounds; ++rd)
            for (int r = 0; r <= 1; ++r) {
                gemm(r); gemm(r);
                CK(hipEventRecord(e0));
                for (int j = 0; j < reps; ++j) gemm(r);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t[r].push_back(ms * 1000 / reps);
            }
        printf("%d x %d x %d\n", m, n, k);
        for (int r = 0; r <= 1; ++r) {
            std::sort(t[r].begin(), t[r].end());
            printf("  rot %d  median %7.2f us  min %7.2f\n", r, t[r][t[r].size() / 2], t[r][0]);
        }
        CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(Cx)); CK(hipFree(Cw)); CK(hipFree(C));
    }
    return 0;
}
