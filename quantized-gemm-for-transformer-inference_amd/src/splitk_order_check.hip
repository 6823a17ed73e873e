// splitk_order_check.hip -- GPU check of gemm_i8_fm's ticket-first split-K hand-off in BOTH arrival orders
// (the product's kFirst64 = 31 gives slice 0 the shorter K range, so slice 0 nearly always arrives
// first and publishes the slab; the order where slice 1 publishes while slice 0 spins was never exercised).
//
// Instantiates the product kernel with kFirst64 = 8 (slice 0 = 1/8 of K: slice 0 publishes), 31 (the product)
// and 56 (slice 1 = 1/8 of K: slice 1 finishes long before slice 0 and takes the producer role), on random
// int8 operands in the fragment-major packed layout, and requires every output bit of every variant, over
// `reps` calls each on one reused scratch (tickets reset by the waiter), to equal the unsplit kernel's.
// Prints one JSON line; exit 0 = all equal.   build/splitk_order_check [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/gemm_i8_kernels.h"

using namespace qgemm;
using namespace qgemm::gemm;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("{\"error\": \"HIP %s at line %d\"}\n", hipGetErrorString(e_), __LINE__);    \
            return 2;                                                                           \
        }                                                                                       \
    } while (0)

__global__ void fill_i8(int8_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (int8_t)((int)(x % 255u) - 127);
    }
}

__global__ void fill_scale(float *p, int n, uint32_t seed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0.25f + (float)((i * 37u + seed) % 101u) / 64.0f;
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 2048, n = argc > 2 ? atoi(argv[2]) : 4096;
    const int k = argc > 3 ? atoi(argv[3]) : 16384, reps = argc > 4 ? atoi(argv[4]) : 20;
    if (m % 256 || n % 256 || k % 128 || (m / 256) * (n / 256) > 4096) {
        printf("{\"error\": \"shape: whole 256-tiles, k %% 128 == 0\"}\n");
        return 2;
    }
    const int tiles_m = m / 256, tiles_n = n / 256, tiles = tiles_m * tiles_n;
    int8_t *A, *B;
    float *Cx, *Cw, *Cref, *C;
    int32_t *slabs;
    unsigned *tickets;
    CK(hipMalloc(&A, (size_t)m * k)); CK(hipMalloc(&B, (size_t)n * k));
    CK(hipMalloc(&Cx, m * 4)); CK(hipMalloc(&Cw, n * 4));
    CK(hipMalloc(&Cref, (size_t)m * n * 4)); CK(hipMalloc(&C, (size_t)m * n * 4));
    CK(hipMalloc(&slabs, (size_t)tiles * 256 * 256 * 4)); CK(hipMalloc(&tickets, (size_t)tiles * 4));
    CK(hipMemset(tickets, 0, (size_t)tiles * 4));
    fill_i8<<<2048, 256>>>(A, (size_t)m * k, 11u); fill_i8<<<2048, 256>>>(B, (size_t)n * k, 12u);
    fill_scale<<<(m + 255) / 256, 256>>>(Cx, m, 3u); fill_scale<<<(n + 255) / 256, 256>>>(Cw, n, 4u);
    GemmArgs p{};
    p.A = A; p.B = B; p.Cx = Cx; p.Cw = Cw; p.csh = n; p.csw = 1; p.m = m; p.n = n; p.k_pad = k;
    p.tiles_m = tiles_m; p.tiles_n = tiles_n; p.inv_r2 = 1.0f / (127.0f * 127.0f); p.splits = 1;
    p.C = Cref;
    gemm_i8_fm<><<<tiles, kFmThreads>>>(p);  // unsplit reference
    CK(hipDeviceSynchronize());
    std::vector<float> want((size_t)m * n), got(want.size());
    CK(hipMemcpy(want.data(), Cref, want.size() * 4, hipMemcpyDeviceToHost));
    p.C = C; p.splits = 2; p.slabs = slabs; p.tickets = tickets; p.reset_tickets = 1;
    struct V { int first64; void (*fn)(GemmArgs); };
    const V vs[] = {{8, gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 8>},
                    {31, gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 31>},
                    {56, gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 56>}};
    long long bad_total = 0;
    printf("{\"m\": %d, \"n\": %d, \"k\": %d, \"reps\": %d, \"variants\": [", m, n, k, reps);
    for (int vi = 0; vi < 3; ++vi) {
        long long bad = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            vs[vi].fn<<<tiles * 2, kFmThreads>>>(p);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < got.size(); ++i) bad += memcmp(&got[i], &want[i], 4) != 0;
        }
        std::vector<unsigned> tk(tiles);
        CK(hipMemcpy(tk.data(), tickets, tiles * 4, hipMemcpyDeviceToHost));
        long long live = 0;
        for (unsigned t : tk) live += t != 0;
        printf("%s{\"first64\": %d, \"mismatches\": %lld, \"tickets_left_nonzero\": %lld}", vi ? ", " : "", vs[vi].first64,
               bad, live);
        bad_total += bad + live;
    }
    printf("], \"ok\": %s}\n", bad_total == 0 ? "true" : "false");
    return bad_total == 0 ? 0 : 1;
}
