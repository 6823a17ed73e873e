// ds_lab.hip -- LAB harness for gemm_ds.h (swapped MFMA operands, epilogue stored straight from registers) against
// the product gemm_i8_fm: bit-checked, timed in interleaved rounds in one process.
//   build/ds_lab m n k rounds spec[,spec...]
// spec: fm | fmrot (wide_rows) | r4 | r4w (the round-4 kernel, lab/gemm_fm_r4.h) | ds (nt, packed, mi outer) | dsp (plain stores) | dss (scalar dequantize) | dsn (ni outer)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#define QGEMM_LAB 1
#include "gemm_ds.h"
#include "gemm_fm_r4.h"
#include "gemm_fm_var.h"

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
    bool stamped = false;
    bool nostore = false;
    bool rot = false;  // gemm_i8_fm's wide-row stores (the product sets them for >= 64-KiB output rows)
    int outlier = -1;  // >= 0: gemm_i8_fm<kEpiOutlier> with this many outlier columns (not bit-checked against fm)
};

static Variant make(const std::string &spec) {
    if (spec == "fm") return {spec, gemm_i8_fm<>};
    if (spec == "fmrot") return {spec, gemm_i8_fm<>, false, false, true};  // product wide-row (LDS image) stores
    if (spec == "fo0") { Variant v{spec, gemm_i8_fm<kEpiOutlier>, false, true}; v.outlier = 0; return v; }
    if (spec == "fo8") { Variant v{spec, gemm_i8_fm<kEpiOutlier>, false, true}; v.outlier = 8; return v; }
    // lab/gemm_fm_var.h (lab/make_variant_fm.py): k0 = the product, k1 no s_setprio, k2 no sched_barrier, k3 A/B
    // interleaved load order; pN = the row's two loads before MFMA N and N + 4
    if (spec == "k0") return {spec, gemm_i8_fm_var<0>};
    if (spec == "k1") return {spec, gemm_i8_fm_var<1>};
    if (spec == "k2") return {spec, gemm_i8_fm_var<2>};
    if (spec == "k3") return {spec, gemm_i8_fm_var<3>};
    if (spec == "sw") return {spec, gemm_i8_fm_var<6>};   // rows share the first-operand (W) fragment
    if (spec == "g8") return {spec, gemm_i8_fm_var<4>};   // XCD patches of 8 tile-rows
    if (spec == "g2") return {spec, gemm_i8_fm_var<5>};   // XCD patches of 2 tile-rows
    if (spec == "p1") return {spec, gemm_i8_fm_var<11>};
    if (spec == "p2") return {spec, gemm_i8_fm_var<12>};
    if (spec == "p3") return {spec, gemm_i8_fm_var<13>};
    if (spec == "r4") return {spec, gemm_i8_fm_r4<>};
    if (spec == "r4w") return {spec, gemm_i8_fm_r4<>, false, false, true};
    if (spec == "ds") return {spec, gemm_i8_ds<kDsNt | kDsPacked | kDsRowMajorOrder>};
    if (spec == "dsp") return {spec, gemm_i8_ds<kDsPacked | kDsRowMajorOrder>};
    if (spec == "dss") return {spec, gemm_i8_ds<kDsNt | kDsRowMajorOrder>};
    if (spec == "dsn") return {spec, gemm_i8_ds<kDsNt | kDsPacked>};
    if (spec == "dsP") return {spec, gemm_i8_ds<kDsPacked | kDsPair | kDsRowMajorOrder>};
    if (spec == "dsPn") return {spec, gemm_i8_ds<kDsNt | kDsPacked | kDsPair | kDsRowMajorOrder>};
    if (spec == "dsPnc") return {spec, gemm_i8_ds<kDsNt | kDsPacked | kDsPair>};  // column bands first
    if (spec == "dsPT") return {spec, gemm_i8_ds<kDsPacked | kDsPair | kDsRowMajorOrder | kDsStamp>, true};
    if (spec == "dsPnT") return {spec, gemm_i8_ds<kDsNt | kDsPacked | kDsPair | kDsRowMajorOrder | kDsStamp>, true};
    if (spec == "dspT") return {spec, gemm_i8_ds<kDsPacked | kDsRowMajorOrder | kDsStamp>, true};
    if (spec == "dsT") return {spec, gemm_i8_ds<kDsNt | kDsPacked | kDsRowMajorOrder | kDsStamp>, true};
    if (spec == "dsX") return {spec, gemm_i8_ds<kDsPacked | kDsNoStore>, false, true};
    if (spec == "dsXT") return {spec, gemm_i8_ds<kDsPacked | kDsNoStore | kDsStamp>, true, true};
    printf("unknown variant %s\n", spec.c_str());
    exit(2);
}

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 20;
    std::string specs = argc > 5 ? argv[5] : "fm,ds";
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

    // outlier operands: X (m x k) and W (k x n) fp32, 8 ascending columns, the count per variant
    float *Xo, *Wo; int *ocols, *ocnt;
    CK(hipMalloc(&Xo, (size_t)m * k * 4)); CK(hipMalloc(&Wo, (size_t)k * n * 4));
    CK(hipMalloc(&ocols, 64)); CK(hipMalloc(&ocnt, 4 * 16));
    fill_f<<<4096, 256>>>(Xo, (int64_t)m * k, 5); fill_f<<<4096, 256>>>(Wo, (int64_t)k * n, 6);
    {
        int hc[8] = {5, 100, 1000, 2000, 2500, 3000, 3500, k - 1};
        int hn[16] = {0, 8};
        CK(hipMemcpy(ocols, hc, sizeof(hc), hipMemcpyHostToDevice));
        CK(hipMemcpy(ocnt, hn, sizeof(hn), hipMemcpyHostToDevice));
    }
    auto vargs = [&](const Variant &v) {
        GemmArgs q = p;
        q.wide_rows = v.rot;
        if (v.outlier >= 0) {
            q.xo = Xo; q.xo_ld = k; q.wo = Wo; q.wo_ld = n; q.ocols = ocols; q.ocount = ocnt + (v.outlier ? 1 : 0);
        }
        return q;
    };
    GemmArgs pr = p; pr.C = Cref;
    gemm_i8_fm<><<<grid, 256>>>(pr);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (v.nostore) continue;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            GemmArgs q = p; q.wide_rows = v.rot;
            v.fn<<<grid, 256>>>(q);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-6s rep %d mismatches %zu\n", v.name.c_str(), rep, bad);
        }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int i = 0; i < 400; ++i) gemm_i8_fm<><<<grid, 256>>>(p);  // pre-warm the clocks
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            GemmArgs q = vargs(vs[vi]);
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<grid, 256>>>(q);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<grid, 256>>>(q);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms * 1000 / reps);
        }
    double ops = 2.0 * m * n * (double)k;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto v = t[vi]; std::sort(v.begin(), v.end());
        printf("%-6s median %8.2f us  min %8.2f us  %7.1f TOPS  %5.1f%% of 5033\n", vs[vi].name.c_str(), v[v.size() / 2],
               v[0], ops / (v[v.size() / 2] * 1e-6) / 1e12, 100 * ops / (v[v.size() / 2] * 1e-6) / 1e12 / 5033.2);
    }
    // stamped variants: 2 s back to back, then the last launch's per-block stamps (100 MHz s_memrealtime)
    unsigned long long *sym;
    CK(hipGetSymbolAddress((void **)&sym, HIP_SYMBOL(g_ds_stamp)));
    for (auto &v : vs) {
        if (!v.stamped) continue;
        float ms = 0;
        CK(hipEventRecord(e0));
        while (ms < 2000) {
            for (int i = 0; i < 200; ++i) v.fn<<<grid, 256>>>(vargs(v));
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        }
        std::vector<unsigned long long> st((size_t)nb * 4);
        CK(hipMemcpy(st.data(), sym, st.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long s0 = ~0ull;
        for (int i = 0; i < nb; ++i) s0 = std::min(s0, st[(size_t)i * 4]);
        std::vector<double> le, be, tail;
        for (int i = 0; i < nb; ++i) {
            le.push_back((st[(size_t)i * 4 + 1] - s0) * 0.01);
            be.push_back((st[(size_t)i * 4 + 2] - s0) * 0.01);
            tail.push_back(be.back() - le.back());
        }
        auto mn = [](const std::vector<double> &x) { return *std::min_element(x.begin(), x.end()); };
        auto mx = [](const std::vector<double> &x) { return *std::max_element(x.begin(), x.end()); };
        double tm = 0; for (double x : tail) tm += x; tm /= tail.size();
        printf("%-6s stamps: loop end %.2f..%.2f  block end %.2f..%.2f  tail %.2f..%.2f (mean %.2f) us\n", v.name.c_str(),
               mn(le), mx(le), mn(be), mx(be), mn(tail), mx(tail), tm);
    }
    return 0;
}
