// pack5_lab.hip -- development harness (not part of the library): the column-group pack (X rows launch +
// persistent column-group W launch, W read once in 1-KiB row segments) against the library's current
// pass for the shape (single-pass strips for K <= 4096, the two-pass column pack above), bit-compared
// on poisoned outputs, then timed warm (back to back) and cold (1-GiB sweep between launches).
// Needs lab/pack_w_group_experiment.patch applied to csrc/pack.hip + csrc/qgemm_internal.h (the dropped
// column-group pack: bit-exact, 1.9x slower than the strip pass at FFN up -- DESIGN.md s5).
// Build: make -C .. pack5lab   Run: build/pack5_lab [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#define QGEMM_LAB 1
#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 2048, n = argc > 2 ? atoi(argv[2]) : 16384, k = argc > 3 ? atoi(argv[3]) : 4096;
    int reps = argc > 4 ? atoi(argv[4]) : 10;
    float *X, *W;
    void *PX, *PW, *PX2, *PW2;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&PX2, packed_bytes(m, k))); CK(hipMalloc(&PW2, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    // a few columns whose largest magnitude is the negative seed (the quirk), a NaN and an inf
    {
        std::vector<float> row0(n);
        CK(hipMemcpy(row0.data(), W, n * 4, hipMemcpyDeviceToHost));
        for (int j = 0; j < n; j += 97) row0[j] = -3.0f;
        CK(hipMemcpy(W, row0.data(), n * 4, hipMemcpyHostToDevice));
        float nan = __builtin_nanf(""), inf = __builtin_inff();
        CK(hipMemcpy(W + (size_t)(k / 2) * n + 5, &nan, 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(W + (size_t)(k - 1) * n + 7, &inf, 4, hipMemcpyHostToDevice));
    }
    PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    PackedView vx2 = packed_view(PX2, m, k), vw2 = packed_view(PW2, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    auto lib = [&]() {
        hipError_t e = launch_pack_single_pass(X, k, m, k, vx, W, n, n, vw, 127.f, s0);
        if (e == hipErrorNotSupported) {
            CK(launch_pack_rows_and_colmax(X, k, m, k, vx, W, n, n, vw, 127.f, s0));
            CK(launch_pack_cols_pass2(W, n, k, n, 127.f, vw, s0));
        } else {
            CK(e);
        }
    };
    auto grp = [&]() { CK(launch_pack_groups(X, k, m, k, vx2, W, n, n, vw2, 127.f, s0)); };
    auto cmp = [&](const void *a, const void *b, size_t bytes) {
        std::vector<char> ha(bytes), hb(bytes);
        CK(hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < bytes; ++i) bad += ha[i] != hb[i];
        return bad;
    };
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(PX2, 0x5a, packed_bytes(m, k), s0));
        CK(hipMemsetAsync(PW2, 0x5a, packed_bytes(n, k), s0));
        lib();
        grp();
        CK(hipStreamSynchronize(s0));
        printf("parity rep %d: xq %zu  wq %zu  cx %zu  cw %zu bytes differ\n", rep, cmp(vx.q, vx2.q, vx.rows_pad * vx.k_pad),
               cmp(vw.q, vw2.q, vw.rows_pad * vw.k_pad), cmp(vx.scale, vx2.scale, vx.rows_pad * 4),
               cmp(vw.scale, vw2.scale, vw.rows_pad * 4));
    }
    // W launch alone (scratch zeroed by a memset ahead of it)
    auto grp_w = [&]() {
        const int gsize = (int)(vw2.k_pad / 128), ncb = (int)(vw2.rows_pad / 256);
        const int ngroups = std::max(1, std::min(ncb, 256 / gsize));
        CK(hipMemsetAsync(vw2.scratch, 0, (vw2.rows_pad + ncb) * 4, s0));
        GroupPackArgs ga{W, n, k, n, 127.f, vw2.scale, vw2.q, vw2.k_pad, ncb, gsize, ngroups, vw2.scratch,
                         vw2.scratch + vw2.rows_pad};
        pack_w_group_kernel<<<(unsigned)(ngroups * gsize), kGrpThreads, 0, s0>>>(ga);
    };
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"library", lib}, {"groups", grp}, {"groups_w", grp_w}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 5; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].f(); vs[i].f();
            CK(hipEventRecord(e0, s0));
            for (int j = 0; j < reps; ++j) vs[i].f();
            CK(hipEventRecord(e1, s0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    const double bytes = 5.0 * m * k + 5.0 * (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-10s warm median %8.2f us  min %8.2f  (%.2f TB/s of the algorithmic %.0f MB)\n", vs[i].name, v[v.size() / 2],
               v[0], bytes / (v[v.size() / 2] * 1e-6) / 1e12, bytes * 1e-6);
    }
    // stamps of the last W launch: per step, medians over blocks of the phase boundaries (us)
    {
        CK(hipDeviceSynchronize());
        grp_w();
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> st(256 * 16 * 6);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_grp_stamp), st.size() * 8));
        const int gsize = (int)(vw2.k_pad / 128), ncb = (int)(vw2.rows_pad / 256);
        const int ngroups = std::max(1, std::min(ncb, 256 / gsize));
        const int nb = ngroups * gsize, steps = (ncb + ngroups - 1) / ngroups;
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nb; ++b) t0 = std::min(t0, st[(size_t)b * 96]);
        printf("stamps (us from the first block's start; medians over %d blocks): start, +read, +B1, +poll(ctl), +B2\n", nb);
        for (int s = 0; s < std::min(steps, 16); ++s) {
            std::vector<double> c[5];
            for (int b = 0; b < nb; ++b)
                for (int i = 0; i < 5; ++i) c[i].push_back((double)(st[((size_t)b * 16 + s) * 6 + i] - t0) * 0.01);
            for (auto &x : c) std::sort(x.begin(), x.end());
            printf("  step %2d: start %7.2f  read %7.2f  B1 %7.2f  poll %7.2f  B2 %7.2f   (B2 min %7.2f max %7.2f)\n", s,
                   c[0][nb / 2], c[1][nb / 2], c[2][nb / 2], c[3][nb / 2], c[4][nb / 2], c[4][0], c[4][nb - 1]);
        }
    }
    {
        void *flush; const size_t fb = (size_t)1 << 30;
        CK(hipMalloc(&flush, fb));
        for (size_t i = 0; i < vs.size(); ++i) {
            std::vector<float> v;
            for (int r = 0; r < 9; ++r) {
                CK(hipMemsetAsync(flush, r, fb, s0));
                CK(hipEventRecord(e0, s0)); vs[i].f(); CK(hipEventRecord(e1, s0)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); v.push_back(ms * 1000);
            }
            std::sort(v.begin(), v.end());
            printf("%-10s cold median %8.2f us  min %8.2f\n", vs[i].name, v[v.size() / 2], v[0]);
        }
        CK(hipFree(flush));
    }
    return 0;
}
