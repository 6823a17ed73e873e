// maskpack_lab.hip -- LAB: where the LLM.int8() masked single-pass pack (pack_single_pass8_kernel<4, true>) spends the
// time it adds over the plain pass (<5, false>): 33.1 vs 28.3 us in the round-4 c2_outlier trace.  Every variant runs
// right after the product's flags launch (outlier_flags_kernel with the fused index), so all see the same cache
// state (flags just read X); `alone` variants run back to back without it.  Variants:
//   plain    <5, false>                         (no mask at all)
//   mask     <4, true>, 8 outlier columns       (the product)
//   mask5    <5, true>, 8 outlier columns       (the round-2 register budget)
//   mask0    <4, true>, no outlier column       (the mask machinery alone: count 0)
// Interleaved rounds, events around each launch; the outputs of mask / mask5 compared bit for bit.
//   build/maskpack_lab [m n k rounds]
// NOTE (round 6): written against the round-5 outlier.hip (per-stream accumulator slots, flags_acc); it does not build
// against the current tree, whose fast path keeps no state between calls (git show bd71824:quantized-gemm-for-transformer-inference_amd/csrc/outlier.hip).
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>
#include <string>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "../quantized-gemm-for-transformer-inference_amd/csrc/outlier.hip"
#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void sweep_kernel(const float *X, int64_t n4, uint32_t *sink) {
    float a = 0.f;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 x = reinterpret_cast<const float4 *>(X)[i];
        a += x.x + x.y + x.z + x.w;
    }
    if (a == 12345.f) sink[0] = 1u;  // keeps the loads
}

// the product flags launch's streaming part alone (same grid, loads, LDS combine, atomics into a scratch word array;
// no arrival counters, no last-workgroup index build): flags - flags_notail = the tail
__global__ __launch_bounds__(1024) void flags_notail_kernel(const float *__restrict__ X, int64_t xsh, int m, int k,
                                                            float t, uint32_t *__restrict__ acc, int nwords) {
    __shared__ uint32_t nibs[3][256];
    const int tid = threadIdx.x, ct = tid & 255, g = tid >> 8;
    const int c = blockIdx.x * 1024 + 4 * ct;
    const int r0 = blockIdx.y * 64 + g * 16, r1 = min(m, r0 + 16);
    uint32_t nib = 0;
    if (c < k) {
        const float *p = X + (int64_t)r0 * xsh + c;
#pragma unroll 16
        for (int r = r0; r < r1; ++r, p += xsh) {
            const float4 x = *reinterpret_cast<const float4 *>(p);
            nib |= (is_outlier(x.x, t) ? 1u : 0u) | (is_outlier(x.y, t) ? 2u : 0u) | (is_outlier(x.z, t) ? 4u : 0u) |
                   (is_outlier(x.w, t) ? 8u : 0u);
        }
    }
    if (g > 0) nibs[g - 1][ct] = nib;
    __syncthreads();
    if (g == 0) {
        for (int j = 0; j < 3; ++j) nib |= nibs[j][ct];
        uint32_t word = nib << (4 * (ct & 7));
        word |= __shfl_xor(word, 1, 64);
        word |= __shfl_xor(word, 2, 64);
        word |= __shfl_xor(word, 4, 64);
        const int w = blockIdx.x * 32 + (ct >> 3);
        if ((ct & 7) == 0 && w < nwords && word) __hip_atomic_fetch_or(acc + w, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void put_outliers(float *X, int m, int k, int every, int ncols) {
    // ncols columns spread over k (bench.py outlier_columns), every `every`-th row |x| = 30
    const int c = blockIdx.x, i = threadIdx.x + blockIdx.y * 256;
    if (c >= ncols || i * every >= m) return;
    const int col = (k / ncols) * c + 7 * c + 3;
    X[(int64_t)i * every * k + col] = (i & 1) ? 30.0f : -30.0f;
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    const int rounds = argc > 4 ? atoi(argv[4]) : 9, reps = 10;
    float *X, *W; void *PX, *PW, *scr;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&scr, outlier_scratch_bytes(m, n, k)));
    void *scr2;  // a second scratch: flags runs on it while the pack reads the first one's (unchanged) mask
    CK(hipMalloc(&scr2, outlier_scratch_bytes(m, n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    put_outliers<<<dim3(8, (m / 50 + 255) / 256 + 1), 256>>>(X, m, k, 50, 8);
    CK(hipDeviceSynchronize());
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    const OutlierScratch v = scratch_view(scr, m, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    const int nstrips = n / kWs8Cols, npad = (int)((vw.rows_pad - n) / kWs8Cols), nx = (int)(vx.rows_pad / 8);
    const int g = nstrips + npad + nx;
    const int64_t wo_ld = round_up(n, 256);
    const float range = 127.f;
    const OutlierScratch v2 = scratch_view(scr2, m, k);
    // mode 0: flags into the pack's scratch; 1: flags into scratch2 (the pack's mask words were written long ago);
    // 2: a plain read sweep of X instead of flags; 3: the flags launch's streaming part alone (flags_notail_kernel)
    auto flags = [&](float t, int mode = 0) {
        if (mode == 0) CK(outlier_scan(X, k, m, k, t, v, s0, /*index=*/false));  // the fast path's flags launch
        else if (mode == 1) CK(outlier_scan(X, k, m, k, t, v2, s0));
        else if (mode == 2) sweep_kernel<<<1024, 256, 0, s0>>>(X, (int64_t)m * k / 4, v2.partial);
        else flags_notail_kernel<<<dim3((k + 1023) / 1024, (m + 63) / 64), 1024, 0, s0>>>(X, k, m, k, t, v2.partial,
                                                                                         (k + 31) / 32);
    };
    // the stream's accumulator: the product's GEMM zeroes it after the pack; here (no GEMM) a variant's repeated
    // flags launches OR the same words again, and each variant starts from a zeroed accumulator
    uint32_t *acc = flags_acc(outlier_ticket_slot(s0));
    const OutlierMask om{acc, v.nwords, v.idx};
    auto pack = [&](int var) {
        if (var == 0)
            pack_single_pass8_kernel<5><<<g, 512, 0, s0>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, n,
                                                           vw.scale, vw.q, vw.rows_pad, nstrips, range, nullptr, 0);
        else if (var == 2)
            pack_single_pass8_kernel<5, true><<<g, 512, 0, s0>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n,
                                                                 n, vw.scale, vw.q, vw.rows_pad, nstrips, range, nullptr,
                                                                 0, om);
        else
            pack_single_pass8_kernel<4, true><<<g, 512, 0, s0>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n,
                                                                 n, vw.scale, vw.q, vw.rows_pad, nstrips, range, nullptr,
                                                                 0, om);
    };
    struct V { std::string name; int pack; float t; bool with_flags; int fmode; };
    std::vector<V> vs = {{"plain", 0, 6.f, true, 0}, {"mask", 1, 6.f, true, 0}, {"mask5", 2, 6.f, true, 0},
                         {"mask0", 1, 1e30f, true, 0}, {"plain_alone", 0, 6.f, false, 0}, {"mask_alone", 1, 6.f, false, 0},
                         {"mask_sweep", 1, 6.f, true, 2}, {"plain_sweep", 0, 6.f, true, 2},
                         {"mask_notail", 1, 6.f, true, 3}};
    // bit check: mask vs mask5
    std::vector<int8_t> a(vx.rows_pad * vx.k_pad), b(a.size());
    CK(hipMemsetAsync(acc, 0, 4 * v.nwords, s0));
    flags(6.f); pack(1); CK(hipStreamSynchronize(s0));
    int cnt = 0; CK(hipMemcpy(&cnt, v.idx, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(a.data(), vx.q, a.size(), hipMemcpyDeviceToHost));
    CK(hipMemsetAsync(vx.q, 0x5a, a.size(), s0));
    flags(6.f); pack(2); CK(hipStreamSynchronize(s0));
    CK(hipMemcpy(b.data(), vx.q, b.size(), hipMemcpyDeviceToHost));
    printf("outlier columns %d; mask5 vs mask X packed: %s\n", cnt, memcmp(a.data(), b.data(), a.size()) ? "DIFF" : "same");
    hipEvent_t ev[3];
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < 300; ++i) { flags(6.f); pack(1); }  // clocks up
    std::vector<std::vector<float>> tf(vs.size()), tp(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            const V &x = vs[i];
            CK(hipMemsetAsync(acc, 0, 4 * v.nwords, s0));
            flags(x.t, 0);  // the pack's own mask current for this variant's threshold (alone / flags2 / sweep reuse it)
            for (int w = 0; w < 3; ++w) { if (x.with_flags) flags(x.t, x.fmode); pack(x.pack); }
            float af = 0, ap = 0;
            for (int j = 0; j < reps; ++j) {
                CK(hipEventRecord(ev[0], s0));
                if (x.with_flags) flags(x.t, x.fmode);
                CK(hipEventRecord(ev[1], s0));
                pack(x.pack);
                CK(hipEventRecord(ev[2], s0));
                CK(hipEventSynchronize(ev[2]));
                float y;
                CK(hipEventElapsedTime(&y, ev[0], ev[1])); af += y;
                CK(hipEventElapsedTime(&y, ev[1], ev[2])); ap += y;
            }
            tf[i].push_back(af * 1000 / reps); tp[i].push_back(ap * 1000 / reps);
        }
    auto med = [](std::vector<float> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
    for (size_t i = 0; i < vs.size(); ++i)
        printf("%-12s flags %7.2f us  pack %7.2f us\n", vs[i].name.c_str(), med(tf[i]), med(tp[i]));
    return 0;
}
