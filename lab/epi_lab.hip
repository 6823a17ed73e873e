// epi_lab.hip -- LAB harness for lab/gemm_fm_epi.h (make_epi_fm.py): the product gemm_i8_fm's epilogue store shapes,
// cache policies and tile maps, on packed operands made by the product's own single-pass pack from fp32 inputs.
// Every variant's output is compared bit for bit with the product kernel's (wide_rows set as the library sets it);
// then interleaved rounds time (a) the GEMM alone and (b) the whole drop-in call = product pack + variant GEMM, so a
// store policy that leaves the output in the caches pays for it in the next call's pack, as in bench.py.
//   build/epi_lab m n k rounds spec[,spec...]
// spec = name of a row of the table in make() below (ldsb*: lab/gemm_fm_ldsb.h, the B-through-LDS experiment)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "gemm_fm_epi.h"
#include "gemm_fm_ldsb.h"
#include "gemm_fm_tile.h"

using namespace qgemm;
using namespace qgemm::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_u(float *p, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)(mix64(seed * 0x9E3779B97F4A7C15ULL + i) >> 40) * (2.0f / 16777216.0f) - 1.0f;
}

typedef void (*KernelFn)(GemmArgs);
struct Variant {
    std::string name;
    KernelFn fn;
    int wide;  // GemmArgs.wide_rows
    int tmsz = 256, tnsz = 256;  // workgroup tile (lab/gemm_fm_tile.h: kTM x kTN)
};

static Variant make(const std::string &s, int lib_wide) {
    // product kernel, as the library launches it, and with the other wide_rows setting
    if (s == "prod") return {s, gemm_i8_fm<>, lib_wide};
    if (s == "img") return {s, gemm_i8_fm<>, 1};
    if (s == "pairs") return {s, gemm_i8_fm<>, 0};
    // generated copies: e<map><store><aux>
    if (s == "img_m1") return {s, gemm_i8_fm_epi<1, 0, -1>, 1};
    if (s == "img_m2") return {s, gemm_i8_fm_epi<2, 0, -1>, 1};
    if (s == "img_m3") return {s, gemm_i8_fm_epi<3, 0, -1>, 1};
    if (s == "pairs_m1") return {s, gemm_i8_fm_epi<1, 0, -1>, 0};
    if (s == "pairs_m2") return {s, gemm_i8_fm_epi<2, 0, -1>, 0};
    if (s == "img_m4") return {s, gemm_i8_fm_epi<4, 0, -1>, 1};
    if (s == "img_m5") return {s, gemm_i8_fm_epi<5, 0, -1>, 1};
    if (s == "pairs_m4") return {s, gemm_i8_fm_epi<4, 0, -1>, 0};
    if (s == "pairs_m5") return {s, gemm_i8_fm_epi<5, 0, -1>, 0};
    if (s == "oct_m1") return {s, gemm_i8_fm_epi<1, 4, -1>, 0};
    if (s == "oct_m4") return {s, gemm_i8_fm_epi<4, 4, -1>, 0};
    if (s == "oct_m5") return {s, gemm_i8_fm_epi<5, 4, -1>, 0};
    if (s == "quad_m1") return {s, gemm_i8_fm_epi<1, 3, -1>, 0};
    if (s == "quad_m4") return {s, gemm_i8_fm_epi<4, 3, -1>, 0};
    // lab/gemm_fm_ldsb.h (make_ldsb_fm.py): B through an LDS-DMA ring
    if (s == "ldsb0") return {s, gemm_i8_fm_ldsb<0>, 0};
    if (s == "ldsb1") return {s, gemm_i8_fm_ldsb<1>, 0};
    if (s == "ldsb2") return {s, gemm_i8_fm_ldsb<2>, 0};
    // the product's map and image stores with other row-rotation formulas (make_epi_fm.py, kAux 100..104)
    if (s == "rot0") return {s, gemm_i8_fm_epi<1, 0, 100>, 1};
    if (s == "rot1") return {s, gemm_i8_fm_epi<1, 0, 101>, 1};
    if (s == "rot2") return {s, gemm_i8_fm_epi<1, 0, 102>, 1};
    if (s == "rot3") return {s, gemm_i8_fm_epi<1, 0, 103>, 1};
    if (s == "rot4") return {s, gemm_i8_fm_epi<1, 0, 104>, 1};
    if (s == "row1k") return {s, gemm_i8_fm_epi<0, 5, -1>, 1};
    if (s == "row1k_m1") return {s, gemm_i8_fm_epi<1, 5, -1>, 1};
    if (s == "nostore") return {s, gemm_i8_fm_epi<0, 2, -1>, 0};
    if (s == "nostore_m2") return {s, gemm_i8_fm_epi<2, 2, -1>, 0};
    if (s == "pairs_plain") return {s, gemm_i8_fm_epi<0, 1, 0>, 0};
    if (s == "pairs_nt") return {s, gemm_i8_fm_epi<0, 1, 2>, 0};
    if (s == "pairs_sc1") return {s, gemm_i8_fm_epi<0, 1, 16>, 0};
    if (s == "pairs_sc0sc1") return {s, gemm_i8_fm_epi<0, 1, 17>, 0};
    if (s == "pairs_ntsc1") return {s, gemm_i8_fm_epi<0, 1, 18>, 0};
    if (s == "pairs_ntsc0sc1") return {s, gemm_i8_fm_epi<0, 1, 19>, 0};
    if (s == "quad") return {s, gemm_i8_fm_epi<0, 3, -1>, 0};
    if (s == "quad_m2") return {s, gemm_i8_fm_epi<2, 3, -1>, 0};
    if (s == "oct") return {s, gemm_i8_fm_epi<0, 4, -1>, 0};
    if (s == "oct_m2") return {s, gemm_i8_fm_epi<2, 4, -1>, 0};
    // lab/gemm_fm_tile.h (make_tile_fm.py): workgroup tile kTM x kTN, XCD patches of kGM tile-rows; _img / _pairs = the
    // wide-row LDS-image stores / the paired register stores
    if (s == "t256_g8_img") return {s, gemm_i8_fm_tile<256, 256, 8>, 1, 256, 256};
    if (s == "t256_g4_pairs") return {s, gemm_i8_fm_tile<256, 256, 4>, 0, 256, 256};
    if (s == "t128x512_g4_img") return {s, gemm_i8_fm_tile<128, 512, 4>, 1, 128, 512};
    if (s == "t128x512_g8_img") return {s, gemm_i8_fm_tile<128, 512, 8>, 1, 128, 512};
    if (s == "t128x512_g16_img") return {s, gemm_i8_fm_tile<128, 512, 16>, 1, 128, 512};
    if (s == "t128x512_g4_pairs") return {s, gemm_i8_fm_tile<128, 512, 4>, 0, 128, 512};
    if (s == "t128x512_g8_pairs") return {s, gemm_i8_fm_tile<128, 512, 8>, 0, 128, 512};
    if (s == "t128x512_g16_pairs") return {s, gemm_i8_fm_tile<128, 512, 16>, 0, 128, 512};
    if (s == "t512x128_g2_pairs") return {s, gemm_i8_fm_tile<512, 128, 2>, 0, 512, 128};
    if (s == "t512x128_g4_pairs") return {s, gemm_i8_fm_tile<512, 128, 4>, 0, 512, 128};
    printf("unknown variant %s\n", s.c_str());
    exit(2);
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 2048, n = argc > 2 ? atoi(argv[2]) : 16384, k = argc > 3 ? atoi(argv[3]) : 4096;
    const int rounds = argc > 4 ? atoi(argv[4]) : 5, reps = 10;
    const std::string specs = argc > 5 ? argv[5] : "prod,pairs";
    if (m % 256 || n % 256 || k % 128 || k > 4096) { printf("lab shapes: whole 256 x 256 tiles, k %% 128 == 0, k <= 4096\n"); return 2; }
    const int lib_wide = n >= 16384 ? 1 : 0;  // gemm_i8.hip: wide_rows = csh >= 16384
    std::vector<Variant> vs;
    for (size_t s = 0; s < specs.size();) {
        size_t e = specs.find(',', s);
        if (e == std::string::npos) e = specs.size();
        vs.push_back(make(specs.substr(s, e - s), lib_wide));
        s = e + 1;
    }
    float *X, *W, *C, *Cref;
    void *pa, *pb;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    CK(hipMalloc(&pa, packed_bytes(m, k))); CK(hipMalloc(&pb, packed_bytes(n, k)));
    fill_u<<<4096, 256>>>(X, (int64_t)m * k, 1);
    fill_u<<<4096, 256>>>(W, (int64_t)k * n, 2);
    const PackedView va = packed_view(pa, m, k), vb = packed_view(pb, n, k);
    auto pack = [&]() { CK(launch_pack_single_pass(X, k, m, k, va, W, n, n, vb, 127.0f, nullptr)); };
    pack();
    CK(hipDeviceSynchronize());
    GemmArgs p{};
    p.A = va.q; p.B = vb.q; p.Cx = va.scale; p.Cw = vb.scale; p.C = Cref; p.csh = n; p.csw = 1; p.m = m; p.n = n;
    p.k_pad = va.k_pad; p.tiles_m = m / BM; p.tiles_n = n / BN; p.inv_r2 = 1.0f / (127.0f * 127.0f); p.splits = 1;
    p.wide_rows = lib_wide;
    const dim3 grid(p.tiles_m * p.tiles_n);
    gemm_i8_fm<><<<grid, 256>>>(p);
    CK(hipDeviceSynchronize());
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    auto args = [&](const Variant &v) {
        GemmArgs q = p;
        q.C = C;
        q.wide_rows = v.wide;
        q.tiles_m = m / v.tmsz;
        q.tiles_n = n / v.tnsz;
        return q;
    };
    auto vgrid = [&](const Variant &v) { return dim3((m / v.tmsz) * (n / v.tnsz)); };
    for (auto &v : vs)
        if (m % v.tmsz || n % v.tnsz) { printf("%s: %d x %d is not a whole number of %d x %d tiles\n", v.name.c_str(), m, n, v.tmsz, v.tnsz); return 2; }
    for (auto &v : vs) {
        if (v.name.rfind("nostore", 0) == 0) continue;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(C, 0xff, (size_t)m * n * 4));
            v.fn<<<vgrid(v), 256>>>(args(v));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-14s rep %d mismatches %zu\n", v.name.c_str(), rep, bad);
        }
    }
    fflush(stdout);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> tg(vs.size()), tc(vs.size());
    for (int i = 0; i < 200; ++i) { pack(); gemm_i8_fm<><<<grid, 256>>>(p); }  // pre-warm the clocks
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            const GemmArgs q = args(vs[vi]);
            const dim3 g = vgrid(vs[vi]);
            for (int w = 0; w < 3; ++w) vs[vi].fn<<<g, 256>>>(q);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) vs[vi].fn<<<g, 256>>>(q);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            tg[vi].push_back(ms * 1000 / reps);
            for (int w = 0; w < 2; ++w) { pack(); vs[vi].fn<<<g, 256>>>(q); }
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) { pack(); vs[vi].fn<<<g, 256>>>(q); }
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            tc[vi].push_back(ms * 1000 / reps);
        }
    const double ops = 2.0 * m * n * (double)k;
    printf("# %d x %d x %d, %d rounds x %d launches; gemm = the GEMM alone, call = product pack + GEMM\n", m, n, k, rounds, reps);
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto g = tg[vi], c = tc[vi];
        std::sort(g.begin(), g.end());
        std::sort(c.begin(), c.end());
        const double gm = g[g.size() / 2], cm = c[c.size() / 2];
        printf("%-14s gemm median %8.2f us min %8.2f (%5.1f%% of 5033)   call median %8.2f us min %8.2f  -> %7.1f calls/s\n",
               vs[vi].name.c_str(), gm, g[0], 100 * ops / (gm * 1e-6) / 1e12 / 5033.2, cm, c[0], 1e6 / cm);
    }
    return 0;
}
