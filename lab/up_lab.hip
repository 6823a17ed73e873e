// up_lab.hip -- LAB: the FFN-up single pass (pack_single_pass32_kernel<204>: 512 W strips of 32 columns x 4096
// rows = 512 KiB each, then 128 X blocks of 16 rows = 256 KiB each, one 1024-thread block per CU).  640 blocks on
// 256 CUs run in 2.5 strip-times while the work is 2.25: does the last half-round of X blocks leave half the chip
// idle?  Variants (every output byte compared with the product's):
//   prod     : the product launch
//   wonly    : the 512 strips alone            xonly16 : the 128 X blocks alone
//   x8       : strips, then 256 X blocks of 8 rows (waves 8..15 of an X block idle)
//   x8first  : the 256 X8 blocks first, then the strips
//   x16first : the 128 X16 blocks first, then the strips
// Measured (profiles/r04_up_lab.log): prod 87.45, wonly 85.90, x8 87.40 us -- no tail to recover.  The harness now
// times the whole FFN-up call (pack + gemm_i8_fm with row rotation), the pack's W loads default vs non-temporal:
// does the GEMM run faster when W's fp32 lines have not displaced the packed operands from the Infinity Cache?
//   build/up_lab [m n k rounds]
// Needs the rejected knobs: `git apply lab/cache_policy_knobs_experiment.patch` (csrc/pack.hip, gemm_i8_kernels.h)
// before building, `git apply -R` after.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace qgemm {
// kXRows 8 or 16; kXFirst: the X blocks take the first block indices
template <int kXRows, bool kXFirst>
__global__ __launch_bounds__(1024) void lab_pass32_kernel(
    const float *__restrict__ x, int64_t xsh, int m, int k, float *__restrict__ x_scale, int8_t *__restrict__ x_q,
    int64_t x_rows_pad, int64_t k_pad, const float *__restrict__ w, int64_t wsh, int n, float *__restrict__ w_scale,
    int8_t *__restrict__ w_q, int64_t w_rows_pad, int nstrips, int nx, float range) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_w[kW32LdsBytes];
    __shared__ float red[16 * 32 + 32];
    const int npad = (int)((w_rows_pad - n) / kW32Cols);
    int bid = blockIdx.x;
    bool xrole;
    if constexpr (kXFirst) {
        xrole = bid < nx;
        bid = xrole ? bid + nstrips + npad : bid - nx;
    } else {
        xrole = bid >= nstrips + npad;
    }
    if (!xrole && bid < nstrips) {
        int strip = bid;
        if (nstrips % 8 == 0) {  // the product's order (kMap 204: groups of 2 adjacent strips, 4 phases)
            const int per = nstrips / 4, g = bid % 2, j = (bid % per) / 2, ph = bid / per;
            strip = (j * 4 + ph) * 2 + g;
        }
        pack_w_strip32_body(strip, w, wsh, k, range, w_scale, w_q, k_pad, lds_w, red);
    } else if (!xrole) {
        const int64_t n0 = n + (int64_t)(bid - nstrips) * kW32Cols;
        zero_packed_rows(w_q, n0, kW32Cols, k_pad, threadIdx.x, 1024);
        if (threadIdx.x < kW32Cols) w_scale[n0 + threadIdx.x] = 0.0f;
    } else {
        const int64_t xb = bid - nstrips - npad;
        const int rsw = (int)(k_pad >> 2) + 16, wv = threadIdx.x >> 6;
        uint32_t *xstage = reinterpret_cast<uint32_t *>(lds_w);
        if (wv < kXRows)
            pack_rows_vec_body<16, false, false, true>(xb * (kXRows / 4), x, xsh, m, k, range, x_scale, x_q, x_rows_pad,
                                                       k_pad, nullptr, xstage + wv * rsw);
        __syncthreads();
        if (wv < kXRows) write_staged_rows<kXRows>(xstage, rsw, x_q, xb * kXRows, k_pad);
    }
}
}  // namespace qgemm

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 2048, n = argc > 2 ? atoi(argv[2]) : 16384, k = argc > 3 ? atoi(argv[3]) : 4096;
    const int rounds = argc > 4 ? atoi(argv[4]) : 7, reps = 10;
    if (n % 256 || m % 256 || k > 4096 || k % 128) { printf("lab shape: n, m %% 256, k <= 4096\n"); return 2; }
    float *X, *W, *C; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4)); CK(hipMalloc(&C, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    const int nstrips = n / kW32Cols, npad = (int)((vw.rows_pad - n) / kW32Cols), nx16 = (int)(vx.rows_pad / 16);
    auto pack = [&](int aux) {
        if (aux == 2)
            pack_single_pass32_kernel<204, 2><<<nstrips + npad + nx16, 1024, 0, s0>>>(
                X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, n, vw.scale, vw.q, vw.rows_pad, nstrips, 127.f,
                nullptr, 0);
        else
            pack_single_pass32_kernel<204, 0><<<nstrips + npad + nx16, 1024, 0, s0>>>(
                X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, n, vw.scale, vw.q, vw.rows_pad, nstrips, 127.f,
                nullptr, 0);
    };
    const int tiles_m = m / 256, tiles_n = n / 256;
    auto gemm = [&]() {
        gemm::GemmArgs p{};
        p.A = vx.q; p.B = vw.q; p.Cx = vx.scale; p.Cw = vw.scale; p.C = C; p.csh = n; p.csw = 1; p.m = m; p.n = n;
        p.k_pad = vx.k_pad; p.tiles_m = tiles_m; p.tiles_n = tiles_n; p.inv_r2 = 1.0f / (127.f * 127.f); p.splits = 1;
        p.wide_rows = n >= 16384 ? 1 : 0;
        gemm::gemm_i8_fm<gemm::kEpiNone><<<tiles_m * tiles_n, 256, 0, s0>>>(p);
    };
    // outputs: the nt pack writes the same bytes
    std::vector<float> ref((size_t)m * n), got(ref.size());
    pack(0); gemm(); CK(hipStreamSynchronize(s0)); CK(hipGetLastError());
    CK(hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemsetAsync(PW, 0x5a, packed_bytes(n, k), s0)); CK(hipMemsetAsync(C, 0xff, (size_t)m * n * 4, s0));
    pack(2); gemm(); CK(hipStreamSynchronize(s0)); CK(hipGetLastError());
    CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
    printf("check nt pack: %s\n", memcmp(ref.data(), got.data(), ref.size() * 4) ? "DIFF" : "same");
    hipEvent_t ev[3];
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < 200; ++i) { pack(0); gemm(); }  // clocks up
    // mode 0: pack default + GEMM; 1: pack nt + GEMM; 2: GEMM back to back
    const char *names[3] = {"call_default", "call_nt_w", "gemm_b2b"};
    std::vector<float> tp[3], tg[3];
    for (int r = 0; r < rounds; ++r)
        for (int md = 0; md < 3; ++md) {
            float ap = 0, ag = 0;
            for (int j = 0; j < reps + 2; ++j) {
                CK(hipEventRecord(ev[0], s0));
                if (md < 2) pack(md == 1 ? 2 : 0);
                CK(hipEventRecord(ev[1], s0)); gemm();
                CK(hipEventRecord(ev[2], s0)); CK(hipEventSynchronize(ev[2]));
                float x;
                if (j < 2) continue;
                CK(hipEventElapsedTime(&x, ev[0], ev[1])); ap += x;
                CK(hipEventElapsedTime(&x, ev[1], ev[2])); ag += x;
            }
            tp[md].push_back(ap * 1000 / reps); tg[md].push_back(ag * 1000 / reps);
        }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    for (int md = 0; md < 3; ++md)
        printf("%-13s pack %7.2f us  gemm %7.2f us  call %7.2f us\n", names[md], med(tp[md]), med(tg[md]),
               med(tp[md]) + med(tg[md]));
    return 0;
}
