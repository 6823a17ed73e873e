// w4_lab.hip -- LAB harness: the 4-wave 128x128-wave-tile GEMM (gemm_w4.h) against the product ping-pong
// kernel, bit-checked and timed in interleaved rounds in one process; `clock` mode: in-kernel loop clocks.
//   build/w4_lab m n k rounds [names|clock]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#define QGEMM_LAB 1
#include "gemm_w4.h"

using namespace qgemm;
using namespace qgemm::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_i8(int8_t *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (int8_t)((int)(mix64(seed + i) >> 56) - 128);
}
__global__ void fill_f(float *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 0.5f + (float)(mix64(seed + i) >> 40) * (1.0f / 16777216.0f);
}

typedef void (*KernelFn)(GemmArgs);
struct Variant { const char *name; KernelFn fn; int threads; bool flayout = false; };

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 20;
    const char *only = argc > 5 ? argv[5] : nullptr;
    int64_t mp = round_up(m, 256), np_ = round_up(n, 256), kp = round_up(k, 128);
    int8_t *A, *B; float *Cx, *Cw, *C, *Cref;
    CK(hipMalloc(&A, mp * kp)); CK(hipMalloc(&B, np_ * kp));
    CK(hipMalloc(&Cx, mp * 4)); CK(hipMalloc(&Cw, np_ * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    fill_i8<<<4096, 256>>>(A, mp * kp, 1); fill_i8<<<4096, 256>>>(B, np_ * kp, 2);
    fill_f<<<64, 256>>>(Cx, mp, 3); fill_f<<<64, 256>>>(Cw, np_, 4);
    CK(hipDeviceSynchronize());
    GemmArgs p{A, B, Cx, Cw, C, n, 1, m, n, kp, (int)(mp / BM), (int)(np_ / BN), 1.0f / (127.0f * 127.0f)};
    int8_t *AF, *BF;
    CK(hipMalloc(&AF, mp * kp)); CK(hipMalloc(&BF, np_ * kp));
    relayout_f_kernel<<<(unsigned)((mp / 16) * (kp / 64) / 4), 256>>>(A, AF, mp, kp);
    relayout_f_kernel<<<(unsigned)((np_ / 16) * (kp / 64) / 4), 256>>>(B, BF, np_, kp);
    CK(hipDeviceSynchronize());
    GemmArgs pf = p; pf.A = AF; pf.B = BF;
    std::vector<Variant> vs = {
        {"pp2", gemm_i8_pp<2>, 512},
        {"pp2_nostore", gemm_i8_pp<2, kEpiNone, kPPNoStore>, 512},
        {"w4", gemm_i8_w4<kW4PadT>, 256},
        {"w4_t256", gemm_i8_w4<0>, 256},
        {"w4_nostore", gemm_i8_w4<kW4PadT | kW4NoStore>, 256},
        {"w4_nodma_ns", gemm_i8_w4<kW4PadT | kW4NoStore | kW4NoDma>, 256},
        {"w4_noread_ns", gemm_i8_w4<kW4PadT | kW4NoStore | kW4NoRead>, 256},
        {"w4_bare_ns", gemm_i8_w4<kW4PadT | kW4NoStore | kW4NoRead | kW4NoDma>, 256},
        {"w4s", gemm_i8_w4s<0>, 256},
        {"w4s_nostore", gemm_i8_w4s<kW4NoStore>, 256},
        {"w4s_nodma_ns", gemm_i8_w4s<kW4NoStore | kW4NoDma>, 256},
        {"f4", gemm_i8_f4<0>, 256, true},
        {"f4_nostore", gemm_i8_f4<kW4NoStore>, 256, true},
        {"f4rm", gemm_i8_f4<kW4RowMajor>, 256, false},
        {"ppF", gemm_i8_pp<2, kEpiNone, kPPLayoutF>, 512, true},
        {"ppF_nostore", gemm_i8_pp<2, kEpiNone, kPPLayoutF | kPPNoStore>, 512, true},
        {"f4_noload_ns", gemm_i8_f4<kW4NoStore | kW4NoRead>, 256, true},
        {"f4_noA_ns", gemm_i8_f4<kW4NoStore | kW4NoA>, 256, true},
        {"f4_noB_ns", gemm_i8_f4<kW4NoStore | kW4NoB>, 256, true},
        {"f4_k1_ns", gemm_i8_f4<kW4NoStore | kW4K1>, 256, true},
        {"f4sync", gemm_i8_f4<kW4Sync>, 256, true},
        {"f4nt", gemm_i8_f4<kW4Nt>, 256, true},
        {"f4noprio", gemm_i8_f4<kW4NoPrio>, 256, true},
        {"f4direct", gemm_i8_f4<kW4Direct>, 256, true},
        {"f4sync_nostore", gemm_i8_f4<kW4Sync | kW4NoStore>, 256, true},
        {"f4_k4_ns", gemm_i8_f4<kW4NoStore | kW4K4>, 256, true},
    };
    dim3 grid(p.tiles_m * p.tiles_n);
    // stride mode: the product-form kernel (nontemporal stores) with the output row stride n vs n + 32 / n + 64
    // floats -- does the epilogue's store pattern pay for a power-of-two row stride?
    if (only && std::string(only) == "stride") {
        float *Cp; CK(hipMalloc(&Cp, (size_t)m * (n + 64) * 4));
        struct SV { const char *name; KernelFn fn; int pad; };
        constexpr int NV = 5;
        const SV sv[NV] = {{"f4nt", gemm_i8_f4<kW4Nt>, 0}, {"f4nt pad32", gemm_i8_f4<kW4Nt>, 32},
                           {"f4nt pad64", gemm_i8_f4<kW4Nt>, 64}, {"f4nt rot", gemm_i8_f4<kW4Nt | kW4Rot>, 0},
                           {"f4nt gscale", gemm_i8_f4<kW4Nt | kW4GScale>, 0}};
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        std::vector<std::vector<float>> t(NV);
        dim3 grid(p.tiles_m * p.tiles_n);
        std::vector<float> h0((size_t)m * n), h1((size_t)m * n);
        for (int v = 0; v < NV; ++v) {  // every variant writes the same C (row stride aside)
            if (sv[v].pad) continue;
            GemmArgs q = pf; q.C = C;
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            sv[v].fn<<<grid, 256>>>(q);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(v ? h1.data() : h0.data(), C, h0.size() * 4, hipMemcpyDeviceToHost));
            if (v) printf("check %-14s %s\n", sv[v].name, memcmp(h0.data(), h1.data(), h0.size() * 4) ? "DIFF" : "same");
        }
        for (int r = 0; r < std::max(rounds, 3); ++r)
            for (int v = 0; v < NV; ++v) {
                GemmArgs q = pf; q.C = sv[v].pad ? Cp : C; q.csh = n + sv[v].pad;
                for (int w = 0; w < 3; ++w) sv[v].fn<<<grid, 256>>>(q);
                CK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i) sv[v].fn<<<grid, 256>>>(q);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[v].push_back(ms * 1000 / reps);
            }
        for (int v = 0; v < NV; ++v) {
            std::sort(t[v].begin(), t[v].end());
            printf("%-14s median %8.2f us  min %8.2f us\n", sv[v].name, t[v][t[v].size() / 2], t[v][0]);
        }
        return 0;
    }
    if (only && std::string(only) == "spread") {
        // round 5: attribute the block-end spread of the product kernel's store tail.  After 2 s of
        // back-to-back launches, one stamped launch: per block its XCD, tile (tm, tn) as gemm_i8_f4 maps it, and the
        // realtime stamps (us from the first start) of its start, loop end and end.  rows `blk,...` for offline analysis
        unsigned long long *w4_sym;
        CK(hipGetSymbolAddress((void **)&w4_sym, HIP_SYMBOL(g_w4_stamp)));
        const int nb = p.tiles_m * p.tiles_n;
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
            float ms = 0;
            CK(hipEventRecord(a));
            while (ms < 2000) {
                for (int i = 0; i < 200; ++i) gemm_i8_f4<kW4Stamp><<<grid, 256>>>(pf);
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st((size_t)4096 * 6);
            CK(hipMemcpy(st.data(), w4_sym, st.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long s0 = ~0ull;
            for (int i = 0; i < nb; ++i) s0 = std::min(s0, st[(size_t)i * 6 + 1]);
            for (int i = 0; i < nb; ++i) {
                const unsigned long long *q = &st[(size_t)i * 6];
                // gemm_i8_f4's map: xcd_remap, then group_tiles (kGroupM 4)
                const int xcd = i & 7, q8 = nb >> 3, r8 = nb & 7;
                const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (i >> 3);
                const int per_group = 4 * p.tiles_n, grp = wid / per_group, first_m = grp * 4;
                const int gsz = std::min(p.tiles_m - first_m, 4), w = wid - grp * per_group;
                const int tm = first_m + w % gsz, tn = w / gsz;
                printf("blk,%d,%d,%d,%d,%d,%.2f,%.2f,%.2f,%.4f\n", rep, i, xcd, tm, tn, (q[1] - s0) * 0.01,
                       (q[3] - s0) * 0.01, (q[5] - s0) * 0.01, (double)(q[4] - q[2]) / std::max(1.0, (double)(q[5] - q[3])) * 0.1);
            }
        }
        return 0;
    }
    if (only && std::string(only) == "clock") {
        struct SV { const char *name; KernelFn fn; int threads; unsigned long long *sym; };
        unsigned long long *pp_sym, *w4_sym;
        CK(hipGetSymbolAddress((void **)&pp_sym, HIP_SYMBOL(g_pp_stamp)));
        CK(hipGetSymbolAddress((void **)&w4_sym, HIP_SYMBOL(g_w4_stamp)));
        std::vector<SV> sv = {
            {"pp2", gemm_i8_pp<2, kEpiNone, kPPStamp>, 512, pp_sym},
            {"w4", gemm_i8_w4<kW4PadT | kW4Stamp>, 256, w4_sym},
            {"w4_nostore", gemm_i8_w4<kW4PadT | kW4Stamp | kW4NoStore>, 256, w4_sym},
            {"w4_bare_ns", gemm_i8_w4<kW4PadT | kW4Stamp | kW4NoStore | kW4NoRead | kW4NoDma>, 256, w4_sym},
            {"w4s", gemm_i8_w4s<kW4Stamp>, 256, w4_sym},
            {"w4s_nostore", gemm_i8_w4s<kW4Stamp | kW4NoStore>, 256, w4_sym},
            {"f4", gemm_i8_f4<kW4Stamp>, 256, w4_sym},
            {"f4_nostore", gemm_i8_f4<kW4Stamp | kW4NoStore>, 256, w4_sym},
            {"f4_noload_ns", gemm_i8_f4<kW4Stamp | kW4NoStore | kW4NoRead>, 256, w4_sym},
            {"f4_noB_ns", gemm_i8_f4<kW4Stamp | kW4NoStore | kW4NoB>, 256, w4_sym},
            {"f4_k1_ns", gemm_i8_f4<kW4Stamp | kW4NoStore | kW4K1>, 256, w4_sym},
            {"f4sync", gemm_i8_f4<kW4Stamp | kW4Sync>, 256, w4_sym},
            {"f4_k4_ns", gemm_i8_f4<kW4Stamp | kW4NoStore | kW4K4>, 256, w4_sym},
            {"ppF", gemm_i8_pp<2, kEpiNone, kPPStamp | kPPLayoutF>, 512, pp_sym},
        };
        const int nb = p.tiles_m * p.tiles_n;
        if (argc > 6) {  // clock mode: optional name filter
            std::vector<SV> keep;
            const std::string list = std::string(",") + argv[6] + ",";
            for (auto &v : sv)
                if (list.find(std::string(",") + v.name + ",") != std::string::npos) keep.push_back(v);
            sv = keep;
        }
        for (auto &v : sv) {
            hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
            int launches = 0; float ms = 0;
            CK(hipEventRecord(a));
            while (ms < 2000) {
                for (int i = 0; i < 200; ++i)
                    v.fn<<<grid, v.threads>>>(strncmp(v.name, "f4", 2) == 0 || strncmp(v.name, "ppF", 3) == 0 ? pf : p);
                launches += 200;
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st((size_t)4096 * 6);
            CK(hipMemcpy(st.data(), v.sym, st.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> lc, lu, ec, eu;
            for (int i = 0; i < nb; ++i) {
                const unsigned long long *q = &st[(size_t)i * 6];
                lc.push_back((double)(q[2] - q[0]) / (double)(q[3] - q[1]) * 0.1);
                lu.push_back((double)(q[3] - q[1]) * 0.01);
                ec.push_back((double)(q[4] - q[2]) / std::max(1.0, (double)(q[5] - q[3])) * 0.1);
                eu.push_back((double)(q[5] - q[3]) * 0.01);
            }
            auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
            printf("%-14s avg launch %7.2f us  loop: clock %.3f GHz, %6.2f us/block  epilogue: clock %.3f GHz, %6.2f us/block\n",
                   v.name, ms * 1000 / launches, med(lc), med(lu), med(ec), med(eu));
            // skew of the LAST launch (realtime stamps, 100 MHz): starts, loop ends, block ends vs the first start
            unsigned long long s0 = ~0ull, s1 = 0, l0 = ~0ull, l1 = 0, e0 = ~0ull, e1 = 0;
            for (int i = 0; i < nb; ++i) {
                const unsigned long long *q = &st[(size_t)i * 6];
                s0 = std::min(s0, q[1]); s1 = std::max(s1, q[1]);
                l0 = std::min(l0, q[3]); l1 = std::max(l1, q[3]);
                e0 = std::min(e0, q[5]); e1 = std::max(e1, q[5]);
            }
            printf("%-14s   skew (us from first start): starts %.2f..%.2f  loop ends %.2f..%.2f  block ends %.2f..%.2f\n",
                   v.name, 0.0, (s1 - s0) * 0.01, (l0 - s0) * 0.01, (l1 - s0) * 0.01, (e0 - s0) * 0.01, (e1 - s0) * 0.01);
        }
        return 0;
    }
    if (only) {
        std::vector<Variant> keep;
        const std::string list = std::string(",") + only + ",";
        for (auto &v : vs)
            if (list.find(std::string(",") + v.name + ",") != std::string::npos) keep.push_back(v);
        vs = keep;
    }
    GemmArgs pr = p; pr.C = Cref;
    gemm_i8_pp<2><<<grid, 512>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (strstr(v.name, "_ns") || strstr(v.name, "nostore")) continue;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<grid, v.threads>>>(v.flayout ? pf : p);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-12s rep %d mismatches %zu\n", v.name, rep, bad);
        }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            const GemmArgs &pv = vs[vi].flayout ? pf : p;
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<grid, vs[vi].threads>>>(pv);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<grid, vs[vi].threads>>>(pv);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms * 1000 / reps);
        }
    double ops = 2.0 * m * n * (double)k;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto v = t[vi]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  %7.1f TOPS  %5.1f%% of 5033\n", vs[vi].name, v[v.size() / 2], v[0],
               ops / (v[v.size() / 2] * 1e-6) / 1e12, 100 * ops / (v[v.size() / 2] * 1e-6) / 1e12 / 5033.2);
    }
    return 0;
}
