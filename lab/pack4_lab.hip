// pack4_lab.hip -- development harness (not part of the library): the persistent register-tile pack
// (pack_tiles_kernel) against the product packers (single-pass strips / rows+colmax+pass2), bit for bit
// on both packed operands (scales and every q byte, padding included), and timed back to back.
// Needs lab/tile_pack_experiment.patch applied to csrc/pack.hip (the tile pack was dropped: DESIGN.md s5).
// Build: make -C .. pack4lab   Run: build/pack4_lab [reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>

#define QGEMM_LAB 1
#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void poke(float *p, int64_t i, float v) { p[i] = v; }

static hipError_t product_pack(const float *X, const float *W, int m, int n, int k, PackedView va, PackedView vb) {
    hipError_t e = launch_pack_single_pass(X, k, m, k, va, W, n, n, vb, 127.f, 0);
    if (e != hipErrorNotSupported) return e;
    e = launch_pack_rows_and_colmax(X, k, m, k, va, W, n, n, vb, 127.f, 0);
    if (e != hipSuccess) return e;
    return launch_pack_cols_pass2(W, n, k, n, 127.f, vb, 0);
}

// the tile pack with a forced grid (lab: also shapes below the product's 128-tile threshold)
static void tile_pack(const float *X, const float *W, int m, int n, int k, PackedView va, PackedView vb, int cus,
                      bool stamped = false) {
    TilePackArgs a;
    a.x = X; a.xsh = k; a.m = m; a.k = k; a.x_scale = va.scale; a.x_q = va.q; a.x_rows_pad = va.rows_pad;
    a.k_pad = va.k_pad; a.w = W; a.wsh = n; a.n = n; a.w_scale = vb.scale; a.w_q = vb.q; a.w_rows_pad = vb.rows_pad;
    a.colmax = vb.scratch; a.counters = vb.scratch + vb.rows_pad;
    a.ncb = (int)(vb.rows_pad / kTpCols); a.ntk = (k + kTpRows - 1) / kTpRows;
    a.cb_per_round = std::min(kTpWPerCu * cus / a.ntk, a.ncb);
    a.rounds = (a.ncb + a.cb_per_round - 1) / a.cb_per_round;
    a.range = 127.f; a.zero_words = nullptr; a.nzero = 0;
    if (stamped) pack_tiles_kernel<true><<<a.cb_per_round * a.ntk, kTpThreads>>>(a);
    else pack_tiles_kernel<false><<<a.cb_per_round * a.ntk, kTpThreads>>>(a);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct Shape { int m, n, k; bool time; };
    std::vector<Shape> shapes = {{1000, 300, 520, false}, {257, 1028, 1000, false}, {64, 2048, 4100, false},
                                 {300, 512, 16384, false}, {512, 3072, 1024, false}, {4096, 4096, 4096, true},
                                 {2048, 16384, 4096, true}, {2048, 4096, 16384, true}, {8192, 4096, 4096, true}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (const Shape &sh : shapes) {
        const int m = sh.m, n = sh.n, k = sh.k;
        float *X, *W;
        CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
        CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, 0));
        CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, 0));
        if (!sh.time) {  // edge values: quirk seeds, NaN/inf, a column of NaN below a negative seed
            poke<<<1, 1>>>(W, 0, -5.0f);                       // column 0: negative seed larger than the rest
            poke<<<1, 1>>>(W, (int64_t)3 * n + 7, NAN);
            poke<<<1, 1>>>(W, (int64_t)(k - 1) * n + n - 1, INFINITY);
            for (int r = 1; r < k; ++r) poke<<<1, 1>>>(W, (int64_t)r * n + 5, NAN);
            poke<<<1, 1>>>(W, 5, -0.25f);
            poke<<<1, 1>>>(X, 0, -7.0f);
            poke<<<1, 1>>>(X, (int64_t)1 * k + 2, NAN);
        }
        const size_t ba = packed_bytes(m, k), bb = packed_bytes(n, k);
        void *pa1, *pb1, *pa2, *pb2;
        CK(hipMalloc(&pa1, ba)); CK(hipMalloc(&pb1, bb)); CK(hipMalloc(&pa2, ba)); CK(hipMalloc(&pb2, bb));
        CK(hipMemset(pa1, 0x5a, ba)); CK(hipMemset(pb1, 0x5a, bb)); CK(hipMemset(pa2, 0x5a, ba)); CK(hipMemset(pb2, 0x5a, bb));
        const PackedView va1 = packed_view(pa1, m, k), vb1 = packed_view(pb1, n, k);
        const PackedView va2 = packed_view(pa2, m, k), vb2 = packed_view(pb2, n, k);
        CK(hipMemset(vb2.scratch, 0, (vb2.rows_pad + 2 * vb2.rows_pad / kTpCols) * 4));  // tile-pack state: zero once
        CK(product_pack(X, W, m, n, k, va1, vb1));
        for (int it = 0; it < 3; ++it) tile_pack(X, W, m, n, k, va2, vb2, cus);  // repeated: the state must self-clean
        CK(hipDeviceSynchronize());
        auto cmp = [&](const PackedView &v1, const PackedView &v2, const char *what) {
            std::vector<uint8_t> h1(v1.rows_pad * v1.k_pad), h2(h1.size());
            std::vector<float> s1(v1.rows_pad), s2(v1.rows_pad);
            CK(hipMemcpy(h1.data(), v1.q, h1.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), v2.q, h2.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(s1.data(), v1.scale, s1.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(s2.data(), v2.scale, s2.size() * 4, hipMemcpyDeviceToHost));
            size_t bq = 0, bs = 0;
            for (size_t i = 0; i < h1.size(); ++i) bq += h1[i] != h2[i];
            for (size_t i = 0; i < s1.size(); ++i) bs += !(s1[i] == s2[i] || (s1[i] != s1[i] && s2[i] != s2[i]));
            printf("  %s: q mismatches %zu, scale mismatches %zu\n", what, bq, bs);
        };
        printf("%dx%dx%d (ntk %d, ncb %d)\n", m, n, k, (k + kTpRows - 1) / kTpRows, (int)(vb2.rows_pad / 256));
        cmp(va1, va2, "A");
        cmp(vb1, vb2, "B");
        std::vector<uint32_t> st(vb2.rows_pad + 2 * vb2.rows_pad / kTpCols);
        CK(hipMemcpy(st.data(), vb2.scratch, st.size() * 4, hipMemcpyDeviceToHost));
        size_t dirty = 0;
        for (auto w : st) dirty += w != 0;
        printf("  tile-pack state words left nonzero: %zu\n", dirty);
        if (sh.time) {
            std::vector<float> t1, t2;
            for (int r = 0; r < 5; ++r) {
                for (int which = 0; which < 2; ++which) {
                    for (int w = 0; w < 3; ++w) which ? tile_pack(X, W, m, n, k, va2, vb2, cus) : (void)product_pack(X, W, m, n, k, va1, vb1);
                    CK(hipEventRecord(e0));
                    for (int i = 0; i < reps; ++i) which ? tile_pack(X, W, m, n, k, va2, vb2, cus) : (void)product_pack(X, W, m, n, k, va1, vb1);
                    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                    (which ? t2 : t1).push_back(ms * 1000 / reps);
                }
            }
            std::sort(t1.begin(), t1.end()); std::sort(t2.begin(), t2.end());
            const double bytes = 5.0 * m * k + 5.0 * (double)k * n;
            printf("  product pack %.2f us (%.2f TB/s)   tile pack %.2f us (%.2f TB/s)\n", t1[2], bytes / t1[2] * 1e-6,
                   t2[2], bytes / t2[2] * 1e-6);
            {  // phase stamps of one launch after the timed runs (us since the earliest block start)
                tile_pack(X, W, m, n, k, va2, vb2, cus, true);
                CK(hipDeviceSynchronize());
                const int ntk = (k + kTpRows - 1) / kTpRows;
                const int nb = std::min(kTpWPerCu * cus / ntk, (int)(vb2.rows_pad / 256)) * ntk;
                std::vector<unsigned long long> st((size_t)4096 * 8);
                CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_tp_stamp), st.size() * 8));
                unsigned long long t0 = ~0ull;
                for (int b = 0; b < nb; ++b) t0 = std::min(t0, st[b * 8]);
                double ph[5][3];  // median / min / max per stamp over the W-tile blocks (stamp 4: X blocks' end)
                (void)ntk;
                for (int i = 0; i < 5; ++i) {
                    std::vector<double> v;
                    for (int b = 0; b < nb; ++b)
                        v.push_back((st[b * 8 + i] - t0) * 0.01);
                    std::sort(v.begin(), v.end());
                    ph[i][0] = v[v.size() / 2]; ph[i][1] = v[0]; ph[i][2] = v.back();
                }
                printf("  stamps (us, median [min..max]): start %.2f [%.2f..%.2f]  X done %.2f [%.2f..%.2f]  W published %.2f "
                       "[%.2f..%.2f]  wait over %.2f [%.2f..%.2f]  end %.2f [%.2f..%.2f]\n",
                       ph[0][0], ph[0][1], ph[0][2], ph[1][0], ph[1][1], ph[1][2], ph[2][0], ph[2][1], ph[2][2], ph[3][0],
                       ph[3][1], ph[3][2], ph[4][0], ph[4][1], ph[4][2]);
            }
        }
        CK(hipFree(X)); CK(hipFree(W)); CK(hipFree(pa1)); CK(hipFree(pb1)); CK(hipFree(pa2)); CK(hipFree(pb2));
    }
    return 0;
}
