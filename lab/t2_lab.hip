// t2_lab.hip -- LAB harness for gemm_t2.h (two teams of 4 waves per 256 x 256 tile) against the product
// gemm_i8_fm, bit-checked, timed in interleaved rounds in one process; `clock` mode: in-kernel stamps per team.
//   build/t2_lab m n k rounds spec[,spec...] [clock]
// spec: fm | fms (fm split-K 2, both slabs) | fmfNN (ticket-first split-K, slice 0 = NN/64 of K) | fk (in-CU split-K) | t2 | t2ns | t2nl | t2np | t2late | t2s:N (team 1 sleeps N x 512 cycles) | t2p:N (team 0 at
//       priority 2 for its first N sub-steps) | t2sp:N:M (both)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#define QGEMM_LAB 1
#include "gemm_t2.h"
#include "gemm_fk.h"

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
struct Variant {
    std::string name;
    KernelFn fn;
    int threads;
    int p0, p1;      // g_t2_param[0..1]
    bool stamped;    // a stamping build exists
    KernelFn sfn;    // the stamping build
    bool nostore;
    int kind = 0;    // 0: 256-tile grid, 1: fm split-K 2 (slabs + tickets), 2: fk (256 x 128 regions)
};

static Variant make(const std::string &spec) {
    Variant v{spec, nullptr, 512, 0, 0, true, nullptr, false};
    int a = 0, b = 0;
    if (spec == "fm") { v.fn = gemm_i8_fm<>; v.threads = 256; v.stamped = false; }
    else if (spec == "fmrot") { v.fn = gemm_i8_fm<>; v.threads = 256; v.stamped = false; v.kind = 3; }
    else if (spec == "fk") { v.fn = gemm_i8_fk<>; v.threads = 256; v.stamped = false; v.kind = 2; }
    else if (spec == "fmf28") { v.fn = gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 28>; v.threads = 256; v.stamped = false; v.kind = 1; }
    else if (spec == "fmf30") { v.fn = gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 30>; v.threads = 256; v.stamped = false; v.kind = 1; }
    else if (spec == "fmf31") { v.fn = gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 31>; v.threads = 256; v.stamped = false; v.kind = 1; }
    else if (spec == "fmf32") { v.fn = gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 32>; v.threads = 256; v.stamped = false; v.kind = 1; }
    else if (spec == "t2") { v.fn = gemm_i8_t2<kT2Nt>; v.sfn = gemm_i8_t2<kT2Nt | kT2Stamp>; }
    else if (spec == "t2plain") { v.fn = gemm_i8_t2<0>; v.sfn = gemm_i8_t2<kT2Stamp>; }
    else if (spec == "t2ns") { v.fn = gemm_i8_t2<kT2NoStore>; v.sfn = gemm_i8_t2<kT2NoStore | kT2Stamp>; v.nostore = true; }
    else if (spec == "t2nl") { v.fn = gemm_i8_t2<kT2NoStore | kT2NoLoad>; v.sfn = gemm_i8_t2<kT2NoStore | kT2NoLoad | kT2Stamp>; v.nostore = true; }
    else if (spec == "t2np") { v.fn = gemm_i8_t2<kT2Nt | kT2NoPrio>; v.sfn = gemm_i8_t2<kT2Nt | kT2NoPrio | kT2Stamp>; }
    else if (spec == "t2late") { v.fn = gemm_i8_t2<kT2Nt | kT2Late>; v.sfn = gemm_i8_t2<kT2Nt | kT2Late | kT2Stamp>; }
    else if (sscanf(spec.c_str(), "t2sp:%d:%d", &a, &b) == 2) {
        v.fn = gemm_i8_t2<kT2Nt | kT2Sleep | kT2Prio>; v.sfn = gemm_i8_t2<kT2Nt | kT2Sleep | kT2Prio | kT2Stamp>; v.p0 = a; v.p1 = b;
    } else if (sscanf(spec.c_str(), "t2s:%d", &a) == 1) {
        v.fn = gemm_i8_t2<kT2Nt | kT2Sleep>; v.sfn = gemm_i8_t2<kT2Nt | kT2Sleep | kT2Stamp>; v.p0 = a;
    } else if (sscanf(spec.c_str(), "t2p:%d", &a) == 1) {
        v.fn = gemm_i8_t2<kT2Nt | kT2Prio>; v.sfn = gemm_i8_t2<kT2Nt | kT2Prio | kT2Stamp>; v.p1 = a;
    } else { printf("unknown variant %s\n", spec.c_str()); exit(2); }
    return v;
}

static void set_params(const Variant &v) {
    int prm[4] = {v.p0, v.p1, 0, 0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_t2_param), prm, sizeof(prm)));
}

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 20;
    std::string specs = argc > 5 ? argv[5] : "fm,t2";
    const bool clock = argc > 6 && std::string(argv[6]) == "clock";
    if (m % 256 || n % 256 || k % 128) { printf("lab shapes are whole 256 x 256 tiles, k %% 128 == 0\n"); return 2; }
    std::vector<Variant> vs;
    for (size_t s = 0; s < specs.size();) {
        size_t e = specs.find(',', s);
        if (e == std::string::npos) e = specs.size();
        vs.push_back(make(specs.substr(s, e - s)));
        s = e + 1;
    }
    int64_t kp = k;
    int8_t *A, *B; float *Cx, *Cw, *C, *Cref;
    CK(hipMalloc(&A, (int64_t)m * kp)); CK(hipMalloc(&B, (int64_t)n * kp));
    CK(hipMalloc(&Cx, m * 4)); CK(hipMalloc(&Cw, n * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    fill_i8<<<4096, 256>>>(A, (int64_t)m * kp, 1); fill_i8<<<4096, 256>>>(B, (int64_t)n * kp, 2);
    fill_f<<<64, 256>>>(Cx, m, 3); fill_f<<<64, 256>>>(Cw, n, 4);
    CK(hipDeviceSynchronize());
    GemmArgs p{};
    p.A = A; p.B = B; p.Cx = Cx; p.Cw = Cw; p.C = C; p.csh = n; p.csw = 1; p.m = m; p.n = n; p.k_pad = kp;
    p.tiles_m = m / BM; p.tiles_n = n / BN; p.inv_r2 = 1.0f / (127.0f * 127.0f); p.splits = 1;
    const int nb = p.tiles_m * p.tiles_n;
    dim3 grid(nb);
    int32_t *slabs; unsigned *tickets;
    CK(hipMalloc(&slabs, (size_t)nb * 2 * 256 * 256 * 4)); CK(hipMalloc(&tickets, 4096 * 4));
    CK(hipMemset(tickets, 0, 4096 * 4));
    auto args = [&](const Variant &v) {
        GemmArgs q = p;
        if (v.kind == 1) { q.splits = 2; q.slabs = slabs; q.tickets = tickets; q.reset_tickets = 1; }
        if (v.kind == 2) q.tiles_n = n / 128;
        if (v.kind == 3) q.wide_rows = 1;
        return q;
    };
    auto grid_of = [&](const Variant &v) { return dim3(v.kind == 1 || v.kind == 2 ? nb * 2 : nb); };

    if (clock) {
        unsigned long long *sym;
        CK(hipGetSymbolAddress((void **)&sym, HIP_SYMBOL(g_t2_stamp)));
        for (auto &v : vs) {
            if (!v.stamped) continue;
            set_params(v);
            hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
            int launches = 0; float ms = 0;
            CK(hipEventRecord(a));
            while (ms < 2000) {
                for (int i = 0; i < 200; ++i) v.sfn<<<grid, v.threads>>>(p);
                launches += 200;
                CK(hipEventRecord(z)); CK(hipEventSynchronize(z)); CK(hipEventElapsedTime(&ms, a, z));
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> st((size_t)nb * 12);
            CK(hipMemcpy(st.data(), sym, st.size() * 8, hipMemcpyDeviceToHost));
            auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
            unsigned long long s0 = ~0ull;
            for (int i = 0; i < nb; ++i) s0 = std::min(s0, std::min(st[(size_t)i * 12 + 1], st[(size_t)i * 12 + 7]));
            printf("%-12s avg launch %7.2f us\n", v.name.c_str(), ms * 1000 / launches);
            for (int t = 0; t < 2; ++t) {
                std::vector<double> lc, lu, eu, st_, le, be;
                for (int i = 0; i < nb; ++i) {
                    const unsigned long long *q = &st[(size_t)i * 12 + t * 6];
                    lc.push_back((double)(q[2] - q[0]) / (double)(q[3] - q[1]) * 0.1);
                    lu.push_back((double)(q[3] - q[1]) * 0.01);
                    eu.push_back((double)(q[5] - q[3]) * 0.01);
                    st_.push_back((double)(q[1] - s0) * 0.01);
                    le.push_back((double)(q[3] - s0) * 0.01);
                    be.push_back((double)(q[5] - s0) * 0.01);
                }
                auto mn = [](const std::vector<double> &x) { return *std::min_element(x.begin(), x.end()); };
                auto mx = [](const std::vector<double> &x) { return *std::max_element(x.begin(), x.end()); };
                printf("  team %d: loop %.3f GHz %6.2f us, epilogue %6.2f us | start %.2f..%.2f  loop end %.2f..%.2f  end %.2f..%.2f\n",
                       t, med(lc), med(lu), med(eu), mn(st_), mx(st_), mn(le), mx(le), mn(be), mx(be));
            }
        }
        return 0;
    }

    GemmArgs pr = p; pr.C = Cref;
    gemm_i8_fm<><<<grid, 256>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (v.nostore) continue;
        set_params(v);
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<grid_of(v), v.threads>>>(args(v));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-12s rep %d mismatches %zu\n", v.name.c_str(), rep, bad);
        }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    // pre-warm the clocks
    for (int i = 0; i < 400; ++i) gemm_i8_fm<><<<grid, 256>>>(p);
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            set_params(vs[vi]);
            const GemmArgs pa = args(vs[vi]);
            const dim3 g = grid_of(vs[vi]);
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<g, vs[vi].threads>>>(pa);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<g, vs[vi].threads>>>(pa);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms * 1000 / reps);
        }
    double ops = 2.0 * m * n * (double)k;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto v = t[vi]; std::sort(v.begin(), v.end());
        printf("%-12s median %8.2f us  min %8.2f us  %7.1f TOPS  %5.1f%% of 5033\n", vs[vi].name.c_str(), v[v.size() / 2],
               v[0], ops / (v[v.size() / 2] * 1e-6) / 1e12, 100 * ops / (v[v.size() / 2] * 1e-6) / 1e12 / 5033.2);
    }
    return 0;
}
