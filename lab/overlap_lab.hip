// overlap_lab.hip -- development harness (not part of the library): can the HBM-bound pack overlap the
// MFMA-bound GEMM inside one op_mm_quantize call?  Existing kernels only, chunked over M (and N) and
// launched on several streams with event dependencies, against the serial two-launch call.  Every
// plan is bit-compared with the serial output.
// Build: make -C .. overlaplab   Run: build/overlap_lab [m n k rounds]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>
#include <string>
#include <hip/hip_ext.h>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "gemm_legacy.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static PackedView sub_view(PackedView v, int64_t r0, int64_t rows) {
    PackedView s = v;
    s.scale = v.scale + r0;
    s.q = v.q + r0 * v.k_pad;
    s.rows_pad = rows;
    return s;
}

struct Ctx {
    int m, n, k;
    float *X, *W, *C;
    PackedView vx, vw;
};

// pack X rows [x0, x1) and W columns [w0, w1) in one single-pass launch
static void pack_wx(const Ctx &c, int x0, int x1, int w0, int w1, hipStream_t s) {
    CK(launch_pack_single_pass_kind(c.X + (int64_t)x0 * c.k, c.k, x1 - x0, c.k, sub_view(c.vx, x0, x1 - x0),
                                    c.W + w0, c.n, w1 - w0, sub_view(c.vw, w0, w1 - w0), 127.f, s, 0));
}

static void run_gemm(const Ctx &c, int r0, int r1, int c0, int c1, hipStream_t s) {
    const int64_t kp = c.vx.k_pad;
    GemmArgs p{c.vx.q + r0 * kp, c.vw.q + c0 * kp, c.vx.scale + r0, c.vw.scale + c0, c.C + (int64_t)r0 * c.n + c0,
               c.n, 1, r1 - r0, c1 - c0, kp, (r1 - r0 + 255) / 256, (c1 - c0 + 255) / 256, 1.0f / (127.0f * 127.0f),
               1, nullptr, nullptr, nullptr, 0};
    gemm_i8_pp<1><<<p.tiles_m * p.tiles_n, kThreads, 0, s>>>(p);
    CK(hipGetLastError());
}

// One launch, two independent roles: blocks [0, ngemm) run GEMM tiles of a pre-packed problem, the
// rest pack another problem (8-column W strips, then 8-row X groups).  Measures how much of the pack
// hides under the GEMM when both share the chip inside ONE launch (no stream sync involved).
struct PackItems {
    const float *x; int64_t xsh; int m, k; PackedView vx;
    const float *w; int64_t wsh; int n; PackedView vw;
    int nstrips;
};
__global__ __launch_bounds__(512, 2) void probe_kernel(GemmArgs g, int ngemm, PackItems pk) {
    __shared__ __attribute__((aligned(16))) int8_t lds[pp_lds_bytes<kEpiNone>()];
    const int b = blockIdx.x;
    if (b < ngemm) {
        pp_tile_body<1>(g, lds, xcd_remap(b, ngemm), 0, 1);
        return;
    }
    const int i = b - ngemm;
    if (i < pk.nstrips) {
        const int xcd = i & 7, q8 = pk.nstrips >> 3, r8 = pk.nstrips & 7;
        const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (i >> 3);
        pack_w_strip8_body(strip, pk.w, pk.wsh, pk.k, 127.f, pk.vw.scale, pk.vw.q, pk.vw.k_pad,
                           reinterpret_cast<float *>(lds));
    } else {
        pack_rows_vec_body<16>((int64_t)(i - pk.nstrips) * 2, pk.x, pk.xsh, pk.m, pk.k, 127.f, pk.vx.scale, pk.vx.q,
                               pk.vx.rows_pad, pk.vx.k_pad);
    }
}

int main(int argc, char **argv) {
    Ctx c;
    c.m = argc > 1 ? atoi(argv[1]) : 4096;
    c.n = argc > 2 ? atoi(argv[2]) : 4096;
    c.k = argc > 3 ? atoi(argv[3]) : 4096;
    const int rounds = argc > 4 ? atoi(argv[4]) : 7, reps = 20;
    const int m = c.m, n = c.n, k = c.k;
    void *PX, *PW;
    float *Cref;
    CK(hipMalloc(&c.X, (size_t)m * k * 4)); CK(hipMalloc(&c.W, (size_t)k * n * 4));
    CK(hipMalloc(&c.C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(launch_fill_uniform(c.X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(c.W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    c.vx = packed_view(PX, m, k);
    c.vw = packed_view(PW, n, k);
    // a second, independent problem for the concurrency probes
    Ctx d = c;
    void *PX2, *PW2;
    CK(hipMalloc(&d.C, (size_t)m * n * 4));
    CK(hipMalloc(&PX2, packed_bytes(m, k))); CK(hipMalloc(&PW2, packed_bytes(n, k)));
    d.vx = packed_view(PX2, m, k);
    d.vw = packed_view(PW2, n, k);

    hipStream_t s[4];
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    // CU-masked streams: mask A = bits of the first half of the mask words, mask B = the rest
    // (QG_MASK=1: even/odd bits instead)
    int ncu = 0;
    {
        hipDeviceProp_t prop;
        CK(hipGetDeviceProperties(&prop, 0));
        ncu = prop.multiProcessorCount;
    }
    hipStream_t ms[2];
    {
        const char *mm = getenv("QG_MASK");
        const int mode = mm ? atoi(mm) : 0;
        std::vector<uint32_t> ma((ncu + 31) / 32, 0), mb((ncu + 31) / 32, 0);
        for (int i = 0; i < ncu; ++i) {
            const bool a = mode == 0 ? i < ncu / 2 : (i & 1) == 0;
            (a ? ma : mb)[i / 32] |= 1u << (i % 32);
        }
        CK(hipExtStreamCreateWithCUMask(&ms[0], (uint32_t)ma.size(), ma.data()));
        CK(hipExtStreamCreateWithCUMask(&ms[1], (uint32_t)mb.size(), mb.data()));
        printf("CUs %d, mask mode %d\n", ncu, mode);
    }
    const int nev = 64;
    std::vector<hipEvent_t> ev(nev);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int evi = 0;
    auto rec = [&](hipStream_t st) { hipEvent_t e = ev[evi++ % nev]; CK(hipEventRecord(e, st)); return e; };
    auto dep = [&](hipStream_t st, hipEvent_t e) { CK(hipStreamWaitEvent(st, e, 0)); };
    // every plan starts on s[0] and ends on s[0]
    auto fork = [&](int nstreams) { hipEvent_t e = rec(s[0]); for (int i = 1; i < nstreams; ++i) dep(s[i], e); };
    auto join = [&](int nstreams) { for (int i = 1; i < nstreams; ++i) dep(s[0], rec(s[i])); };
    const int hm = m / 2, hn = n / 2;

    auto probe = [&](const Ctx &gd, int ngemm, bool with_pack) {
        const int64_t kp = gd.vx.k_pad;
        GemmArgs g{gd.vx.q, gd.vw.q, gd.vx.scale, gd.vw.scale, gd.C, gd.n, 1, gd.m, gd.n, kp, gd.m / 256, gd.n / 256,
                   1.0f / (127.0f * 127.0f), 1, nullptr, nullptr, nullptr, 0};
        PackItems pk{c.X, c.k, c.m, c.k, c.vx, c.W, c.n, c.n, c.vw, c.n / 8};
        const int npack = with_pack ? c.n / 8 + c.m / 8 : 0;
        probe_kernel<<<ngemm + npack, 512, 0, s[0]>>>(g, ngemm, pk);
        CK(hipGetLastError());
    };
    struct Plan { std::string name; std::function<void()> f; bool checks; };
    std::vector<Plan> plans = {
        {"serial", [&] { pack_wx(c, 0, m, 0, n, s[0]); run_gemm(c, 0, m, 0, n, s[0]); }, true},
        {"halvesM", [&] {
             fork(2);
             pack_wx(c, 0, hm, 0, n, s[0]);
             dep(s[1], rec(s[0]));
             run_gemm(c, 0, hm, 0, n, s[0]);
             pack_wx(c, hm, m, 0, 0, s[1]);
             run_gemm(c, hm, m, 0, n, s[1]);
             join(2);
         }, true},
        {"quad", [&] {
             fork(3);
             pack_wx(c, 0, hm, 0, hn, s[0]);
             dep(s[1], rec(s[0]));
             run_gemm(c, 0, hm, 0, hn, s[0]);
             pack_wx(c, 0, 0, hn, n, s[1]);
             dep(s[2], rec(s[1]));
             run_gemm(c, 0, hm, hn, n, s[1]);
             pack_wx(c, hm, m, 0, 0, s[2]);
             run_gemm(c, hm, m, 0, n, s[2]);
             join(3);
         }, true},
        {"quad2", [&] {
             fork(3);
             pack_wx(c, 0, hm, 0, hn, s[0]);
             dep(s[1], rec(s[0]));
             run_gemm(c, 0, hm, 0, hn, s[0]);
             pack_wx(c, hm, m, hn, n, s[1]);
             dep(s[2], rec(s[1]));
             run_gemm(c, hm, m, 0, n, s[1]);
             run_gemm(c, 0, hm, hn, n, s[2]);
             join(3);
         }, true},
        {"quarterM", [&] {
             // W + X0 first, then X1..X3 packs back to back on s[0]; GEMM chunks on s[1..3]
             const int q = m / 4;
             fork(4);
             pack_wx(c, 0, q, 0, n, s[0]);
             dep(s[1], rec(s[0]));
             run_gemm(c, 0, q, 0, n, s[1]);
             for (int i = 1; i < 4; ++i) {
                 pack_wx(c, i * q, (i + 1) * q, 0, 0, s[0]);
                 hipStream_t g = s[1 + i % 3];
                 dep(g, rec(s[0]));
                 run_gemm(c, i * q, (i + 1) * q, 0, n, g);
             }
             join(4);
         }, true},
        // concurrency probes on an independent problem d (no dependency at all)
        {"G128", [&] { run_gemm(d, 0, hm, 0, n, s[0]); }, false},
        {"G64", [&] { run_gemm(d, 0, hm, 0, hn, s[0]); }, false},
        {"PXhalf", [&] { pack_wx(c, hm, m, 0, 0, s[0]); }, false},
        {"PWhalf", [&] { pack_wx(c, 0, 0, hn, n, s[0]); }, false},
        {"PXW", [&] { pack_wx(c, 0, m, 0, n, s[0]); }, false},
        {"G128||PXhalf", [&] {
             fork(2);
             run_gemm(d, 0, hm, 0, n, s[0]);
             pack_wx(c, hm, m, 0, 0, s[1]);
             join(2);
         }, false},
        {"G128||G128", [&] {
             fork(2);
             run_gemm(d, 0, hm, 0, n, s[0]);
             run_gemm(c, hm, m, 0, n, s[1]);
             join(2);
         }, false},
        {"PXh||PXh", [&] {
             fork(2);
             pack_wx(c, hm, m, 0, 0, s[0]);
             pack_wx(d, 0, hm, 0, 0, s[1]);
             join(2);
         }, false},
        {"mG128||mPXW", [&] {
             // CU-masked streams: GEMM on mask A, pack on mask B
             hipEvent_t e = rec(s[0]);
             dep(ms[0], e); dep(ms[1], e);
             run_gemm(d, 0, hm, 0, n, ms[0]);
             pack_wx(c, 0, m, 0, n, ms[1]);
             dep(s[0], rec(ms[0])); dep(s[0], rec(ms[1]));
         }, false},
        {"mG128", [&] {
             hipEvent_t e = rec(s[0]);
             dep(ms[0], e);
             run_gemm(d, 0, hm, 0, n, ms[0]);
             dep(s[0], rec(ms[0]));
         }, false},
        {"mPXW", [&] {
             hipEvent_t e = rec(s[0]);
             dep(ms[1], e);
             pack_wx(c, 0, m, 0, n, ms[1]);
             dep(s[0], rec(ms[1]));
         }, false},
        {"prG128", [&] { probe(d, 128, false); }, false},
        {"prG256", [&] { probe(d, 256, false); }, false},
        {"prPXW", [&] { probe(d, 0, true); }, false},
        {"prG128+PXW", [&] { probe(d, 128, true); }, false},
        {"prG256+PXW", [&] { probe(d, 256, true); }, false},
        {"G256", [&] { run_gemm(d, 0, m, 0, n, s[0]); }, false},
        {"G128||PXW", [&] {
             fork(2);
             run_gemm(d, 0, hm, 0, n, s[0]);
             pack_wx(c, 0, m, 0, n, s[1]);
             join(2);
         }, false},
    };
    // one serial call into Cref, then every checked plan bit-compared
    pack_wx(c, 0, m, 0, n, s[0]);
    {
        GemmArgs dummy{};
        (void)dummy;
    }
    run_gemm(c, 0, m, 0, n, s[0]);
    CK(hipStreamSynchronize(s[0]));
    CK(hipMemcpy(Cref, c.C, (size_t)m * n * 4, hipMemcpyDeviceToDevice));
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    // d: packed operands of its own (the probes only run its GEMM)
    pack_wx(d, 0, m, 0, n, s[0]);
    CK(hipStreamSynchronize(s[0]));
    for (auto &p : plans) {
        if (!p.checks) continue;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(c.C, 0xff, (size_t)m * n * 4, s[0]));
            CK(hipMemsetAsync(PX, 0x5a, packed_bytes(m, k), s[0]));
            CK(hipMemsetAsync(PW, 0x5a, packed_bytes(n, k), s[0]));
            p.f();
            CK(hipStreamSynchronize(s[0]));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hgot.data(), c.C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check %-10s rep %d mismatches %zu\n", p.name.c_str(), rep, bad);
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(plans.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < plans.size(); ++i) {
            for (int w = 0; w < 3; ++w) plans[i].f();
            CK(hipEventRecord(e0, s[0]));
            for (int j = 0; j < reps; ++j) plans[i].f();
            CK(hipEventRecord(e1, s[0]));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    CK(hipDeviceSynchronize());
    for (size_t i = 0; i < plans.size(); ++i) {
        auto v = t[i];
        std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us\n", plans[i].name.c_str(), v[v.size() / 2], v[0]);
    }
    return 0;
}
