// c4_lab.hip -- LAB: the 8-column single-pass call (pack_single_pass8_kernel<5> + gemm_i8_fm; C2 4096^3 and the C4
// shard 8192 x 4096 x 4096) with W's and / or X's fp32 loads non-temporal.  Per call the C4 shard moves X 128 MiB +
// W 64 MiB in, 48 MiB packed, 128 MiB of C: more than the 256-MB Infinity Cache holds, so the inputs are not found
// again by the next call anyway and default loads may only push the packed operands out before the GEMM reads them
// (lab/c3g_lab.hip: the FFN-down GEMM ran 11 % slower with its operands evicted).  At C2 (224 MiB per call) the
// inputs do stay resident between calls, so non-temporal loads should cost there (measured: they do, and the
// GEMM does not move; profiles/r04_c4_lab_*.log, with a staggered-first-wave GEMM that did not pay either).  Now
// also the packed outputs' store policy: non-temporal or write-through stores leave fewer dirty L2 lines to write
// back at the pack's end.  Steady-state calls, events around each kernel, interleaved rounds; every variant's
// output compared with the default's.
//   build/c4_lab [m n k rounds]
// Needs the rejected knobs: `git apply lab/cache_policy_knobs_experiment.patch` (csrc/pack.hip, gemm_i8_kernels.h)
// before building, `git apply -R` after.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 8192, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    const int rounds = argc > 4 ? atoi(argv[4]) : 7, reps = 10;
    if (n % 256 || m % 256 || k > 4096 || k % 128 || n > 8192) { printf("lab shape: 8-column pass, 256-tiles\n"); return 2; }
    float *X, *W, *C; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4)); CK(hipMalloc(&C, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    const int nstrips = n / kWs8Cols, npad = (int)((vw.rows_pad - n) / kWs8Cols), nx = (int)(vx.rows_pad / 8);
    const int g = nstrips + npad + nx;
#define QG_P8(WA, XA, WS, XS)                                                                                      \
    pack_single_pass8_kernel<5, false, WA, XA, WS, XS><<<g, 512, 0, s0>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, \
                                                                 W, n, n, vw.scale, vw.q, vw.rows_pad, nstrips,    \
                                                                 127.f, nullptr, 0)
    // variants: 0 default; 1-3 non-temporal loads (X / W / both, round 4: rejected); 4 packed W stored nt, 5 packed
    // X stored nt, 6 both nt, 7 packed W stored sc1 (write-through): fewer dirty L2 lines at the pack's end
    auto pack = [&](int v) {
        if (v == 0) QG_P8(0, 0, 0, false);
        if (v == 1) QG_P8(0, 2, 0, false);
        if (v == 2) QG_P8(2, 0, 0, false);
        if (v == 3) QG_P8(2, 2, 0, false);
        if (v == 4) QG_P8(0, 0, 2, false);
        if (v == 5) QG_P8(0, 0, 0, true);
        if (v == 6) QG_P8(0, 0, 2, true);
        if (v == 7) QG_P8(0, 0, 16, false);
    };
    const int tiles_m = m / 256, tiles_n = n / 256;
    auto gemm = [&](int stagger = 0) {
        gemm::GemmArgs p{};
        p.A = vx.q; p.B = vw.q; p.Cx = vx.scale; p.Cw = vw.scale; p.C = C; p.csh = n; p.csw = 1; p.m = m; p.n = n;
        p.k_pad = vx.k_pad; p.tiles_m = tiles_m; p.tiles_n = tiles_n; p.inv_r2 = 1.0f / (127.f * 127.f); p.splits = 1;
        using namespace gemm;
        if (stagger == 0) gemm_i8_fm<kEpiNone><<<tiles_m * tiles_n, 256, 0, s0>>>(p);
        if (stagger == 1) gemm_i8_fm<kEpiNone, false, kSplitNone, true, 30, false, 1><<<tiles_m * tiles_n, 256, 0, s0>>>(p);
        if (stagger == 2) gemm_i8_fm<kEpiNone, false, kSplitNone, true, 30, false, 2><<<tiles_m * tiles_n, 256, 0, s0>>>(p);
        if (stagger == 3) gemm_i8_fm<kEpiNone, false, kSplitNone, true, 30, false, 3><<<tiles_m * tiles_n, 256, 0, s0>>>(p);
    };
    // modes: pack variant v (0..7) + GEMM; 8: GEMM back to back
    constexpr int kModes = 9;
    const char *names[kModes] = {"default", "nt_x", "nt_w", "nt_w_x", "st_nt_w", "st_nt_x", "st_nt_wx", "st_sc1_w",
                                 "gemm_b2b"};
    std::vector<float> ref((size_t)m * n), got(ref.size());
    pack(0); gemm(); CK(hipStreamSynchronize(s0)); CK(hipGetLastError());
    CK(hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
    for (int v = 1; v < 8; ++v) {
        CK(hipMemsetAsync(PW, 0x5a, packed_bytes(n, k), s0)); CK(hipMemsetAsync(PX, 0x5a, packed_bytes(m, k), s0));
        CK(hipMemsetAsync(C, 0xff, (size_t)m * n * 4, s0));
        pack(v); gemm(); CK(hipStreamSynchronize(s0)); CK(hipGetLastError());
        CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
        printf("check %-8s %s\n", names[v], memcmp(ref.data(), got.data(), ref.size() * 4) ? "DIFF" : "same");
    }
    hipEvent_t ev[3];
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < 200; ++i) { pack(0); gemm(); }  // clocks up
    std::vector<float> tp[kModes], tg[kModes];
    for (int r = 0; r < rounds; ++r)
        for (int md = 0; md < kModes; ++md) {
            float ap = 0, ag = 0;
            for (int j = 0; j < reps + 3; ++j) {
                CK(hipEventRecord(ev[0], s0));
                if (md < 8) pack(md);
                CK(hipEventRecord(ev[1], s0)); gemm();
                CK(hipEventRecord(ev[2], s0)); CK(hipEventSynchronize(ev[2]));
                float x;
                if (j < 3) continue;
                CK(hipEventElapsedTime(&x, ev[0], ev[1])); ap += x;
                CK(hipEventElapsedTime(&x, ev[1], ev[2])); ag += x;
            }
            tp[md].push_back(ap * 1000 / reps); tg[md].push_back(ag * 1000 / reps);
        }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("%d x %d x %d\n", m, n, k);
    for (int md = 0; md < kModes; ++md)
        printf("%-9s pack %7.2f us  gemm %7.2f us  call %7.2f us\n", names[md], med(tp[md]), med(tg[md]),
               med(tp[md]) + med(tg[md]));
    return 0;
}
