// pack_lab.hip -- development harness for the pack stage (not part of the library): times the
// single-pass pack against W-strip-only + X-rows kernels run sequentially or concurrently on two
// streams (fork/join with events).   Build: make -C .. packlab   Run: build/pack_lab [m n k reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <cstring>

#include <hip/hip_ext.h>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

namespace qgemm {
namespace {
// ------------------------------------------------------------------------------------------------
// EXPERIMENT (lab only, slower than the single pass: 37.8 vs 30.5 us at 4096^3, 147 vs 96 us at
// 2048x4096x16384 -- 32-B W row segments and 128 KiB in flight per CU): pack engine (row-major X and W, K <= 4096, n % 8 == 0): ONE persistent launch, one 1024-thread
// block per CU, two 512-thread groups in ping-pong over work items of 128 KiB of fp32 each:
//   W item = 8 columns x all K rows of W (a "half strip"): 64 floats per thread in registers
//   X item = 8 rows of X, one wave per row (16 float4 per lane)
// Phase p: group (p & 1) ISSUES the loads of its next item; the other group waits for the loads it
// issued in phase p-1 and reduces / quantizes / stores that item.  Phases are separated by raw
// s_barrier (no fence, so the loads stay in flight across it): at every moment one group per CU has
// 128 KiB of reads in flight while the other computes, and HBM does not idle behind the compute
// phases as it did with one item per block (single-pass kernel: load, then compute, then store).
// Block b's items are b, b+G, b+2G, ... (G = grid); group g takes every other one.  W items come
// first; items idx, idx+8, idx+16, idx+24 (one XCD, same phase) get adjacent half strips, so the
// four 32-B segments of each 128-B line of W are fetched into that XCD's L2 together.
constexpr int kEngCols = 8;       // columns per W item
constexpr int kEngMaxK = 4096;    // 16 rows per thread x 256 row groups
constexpr int kEngThreads = 1024; // two groups of 512

struct EngineArgs {
    const float *x;
    int64_t xsh;
    int m, k;
    float *x_scale;
    int8_t *x_q;
    int64_t x_rows_pad, k_pad;
    const float *w;
    int64_t wsh;
    int n;
    float *w_scale;
    int8_t *w_q;
    int64_t w_rows_pad;
    int n_w_items, n_items;
    float range;
};

__device__ __forceinline__ void engine_sync_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int engine_strip(int idx, int nstrips) {
    const int xcd = idx & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (idx >> 3);
}

__global__ __launch_bounds__(kEngThreads) void pack_engine_kernel(EngineArgs a) {
    __shared__ float red[2][8][kEngCols];  // [group][wave][column] candidate maxima
    __shared__ float seed_sh[2][kEngCols];
    __shared__ float scale_sh[2][kEngCols];
    const int g = threadIdx.x >> 9, gt = threadIdx.x & 511, lane = threadIdx.x & 63, wg = gt >> 6;
    const int G = gridDim.x, b = blockIdx.x;
    const int n_mine = b < a.n_items ? (a.n_items - b + G - 1) / G : 0;
    // W item thread map: c4 = gt & 1 (columns 4c4..4c4+3 of the item), rq = gt >> 1: rows 16rq + e
    const int c4 = gt & 1, rq = gt >> 1;
    float4 v[16];
    for (int p = 0; p <= n_mine; ++p) {
        const bool load = (p & 1) == g && p < n_mine;
        const bool comp = (p & 1) != g && p >= 1;
        const int item = b + (load ? p : p - 1) * G;
        const bool is_w = item < a.n_w_items;
        if (load) {
            if (is_w) {
                const int64_t n0 = (int64_t)engine_strip(item, a.n_w_items) * kEngCols;
                // one running address (opaque to LICM: 16 hoisted 64-bit row addresses would spill)
                const float *pw = a.w + n0 + 4 * c4 + (int64_t)(16 * rq) * a.wsh;
                if (a.k >= kEngMaxK) {  // every row exists: branch-free loads
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        v[e] = *reinterpret_cast<const float4 *>(pw);
                        pw += a.wsh;
                        asm volatile("" : "+v"(pw));
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        v[e] = 16 * rq + e < a.k ? *reinterpret_cast<const float4 *>(pw)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                        pw += a.wsh;
                        asm volatile("" : "+v"(pw));
                    }
                }
            } else {
                const int64_t row = (int64_t)(item - a.n_w_items) * 8 + wg;
                const int nfull = a.k >> 2;
                const float4 *s4 = reinterpret_cast<const float4 *>(a.x + row * a.xsh);
                if (row < a.m && nfull >= 1024) {  // whole row in 16 chunks per lane
#pragma unroll
                    for (int j = 0; j < 16; ++j) v[j] = s4[lane + j * 64];
                } else {
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const int c = lane + j * 64;
                        v[j] = (row < a.m && c < nfull) ? s4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
        }
        // ---- part A: candidates (W: to LDS; X: the whole row) ----
        int64_t n0 = 0;
        if (comp && is_w) {
            n0 = (int64_t)engine_strip(item, a.n_w_items) * kEngCols;
            float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int r = 16 * rq + e;
                if (r >= 1 && r < a.k) {
                    p0 = cand_max(p0, v[e].x);
                    p1 = cand_max(p1, v[e].y);
                    p2 = cand_max(p2, v[e].z);
                    p3 = cand_max(p3, v[e].w);
                }
            }
#pragma unroll
            for (int off = 2; off < 64; off <<= 1) {  // lanes with the same c4
                p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
                p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
                p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
                p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
            }
            if (lane < 2) {
                red[g][wg][4 * lane + 0] = p0;
                red[g][wg][4 * lane + 1] = p1;
                red[g][wg][4 * lane + 2] = p2;
                red[g][wg][4 * lane + 3] = p3;
            }
            if (rq == 0) {  // row 0 = the seeds (op_reduction.cuh:105)
                seed_sh[g][4 * c4 + 0] = v[0].x;
                seed_sh[g][4 * c4 + 1] = v[0].y;
                seed_sh[g][4 * c4 + 2] = v[0].z;
                seed_sh[g][4 * c4 + 3] = v[0].w;
            }
        } else if (comp) {
            const int64_t row = (int64_t)(item - a.n_w_items) * 8 + wg;
            uint32_t *qrow = reinterpret_cast<uint32_t *>(a.x_q + row * a.k_pad);
            const int64_t nq = a.k_pad >> 2;
            if (row >= a.m) {  // padding row
                for (int64_t c = lane; c < nq; c += 64) qrow[c] = 0u;
                if (lane == 0) a.x_scale[row] = 0.0f;
            } else {
                const float *srow = a.x + row * a.xsh;
                const int len = a.k, nfull = len >> 2;
                float pm = -INFINITY;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int c = lane + j * 64;
                    if (c < nfull) {
                        pm = (c == 0) ? pm : cand_max(pm, v[j].x);  // element 0 is the seed
                        pm = cand_max(pm, v[j].y);
                        pm = cand_max(pm, v[j].z);
                        pm = cand_max(pm, v[j].w);
                    }
                }
                const int tail0 = nfull << 2;
                if (tail0 + lane < len && tail0 + lane > 0) pm = cand_max(pm, srow[tail0 + lane]);
                pm = wave_max(pm);
                const float seed = nfull > 0 ? __shfl(v[0].x, 0, 64) : srow[0];
                const float cx = absmax_finish(seed, pm);
                const float sc = inv_divide(a.range, cx);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int c = lane + j * 64;
                    if (c < nfull)
                        qrow[c] = pack4(quant_i8(v[j].x, sc), quant_i8(v[j].y, sc), quant_i8(v[j].z, sc),
                                        quant_i8(v[j].w, sc));
                }
                const int64_t first_zero = nfull + ((len & 3) ? 1 : 0);
                if ((len & 3) && lane == 0) {
                    int bb[4] = {0, 0, 0, 0};
                    for (int e = 0; e < (len & 3); ++e) bb[e] = quant_i8(srow[tail0 + e], sc);
                    qrow[nfull] = pack4(bb[0], bb[1], bb[2], bb[3]);
                }
                for (int64_t c = first_zero + lane; c < nq; c += 64) qrow[c] = 0u;
                if (lane == 0) a.x_scale[row] = cx;
            }
        }
        engine_sync_lds();
        // ---- part B: W scales ----
        if (comp && is_w && gt < kEngCols) {
            float pm = red[g][0][gt];
#pragma unroll
            for (int ww = 1; ww < 8; ++ww) pm = fmaxf(pm, red[g][ww][gt]);  // -inf or >= +0: exact
            const float cw = absmax_finish(seed_sh[g][gt], pm);
            scale_sh[g][gt] = inv_divide(a.range, cw);
            a.w_scale[n0 + gt] = cw;
        }
        engine_sync_lds();
        // ---- part C: W quantize + store: 16 consecutive k bytes of one column = one 16-B store ----
        if (comp && is_w && 16 * rq < a.k_pad) {
            const int kin = a.k - 16 * rq;  // rows of this run that exist (>= 16: all)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {  // one column at a time: 16 quantized bytes -> one 16-B store
                const float sc = scale_sh[g][4 * c4 + cc];
                int qv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float xv = cc == 0 ? v[e].x : cc == 1 ? v[e].y : cc == 2 ? v[e].z : v[e].w;
                    qv[e] = e < kin ? quant_i8(xv, sc) : 0;
                }
                uint4 o;
                o.x = pack4(qv[0], qv[1], qv[2], qv[3]);
                o.y = pack4(qv[4], qv[5], qv[6], qv[7]);
                o.z = pack4(qv[8], qv[9], qv[10], qv[11]);
                o.w = pack4(qv[12], qv[13], qv[14], qv[15]);
                *reinterpret_cast<uint4 *>(a.w_q + (n0 + 4 * c4 + cc) * a.k_pad + 16 * rq) = o;
            }
        }
        // part C's LDS reads (scale_sh) finish before the next phase's part B rewrites them
        engine_sync_lds();
    }
    // zero padding rows of packed W (and their scales), grid-stride
    const int64_t pad_rows = a.w_rows_pad - a.n;
    const int64_t pad_words = pad_rows * a.k_pad / 16;
    uint4 *wq_pad = reinterpret_cast<uint4 *>(a.w_q + (int64_t)a.n * a.k_pad);
    for (int64_t i = (int64_t)b * kEngThreads + threadIdx.x; i < pad_words; i += (int64_t)G * kEngThreads)
        wq_pad[i] = make_uint4(0, 0, 0, 0);
    for (int64_t i = (int64_t)b * kEngThreads + threadIdx.x; i < pad_rows; i += (int64_t)G * kEngThreads)
        a.w_scale[a.n + i] = 0.0f;
}

}  // namespace
static hipError_t launch_pack_engine(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w, int64_t wsh,
                              int n, PackedView outw, float range, hipStream_t stream) {
    if (k < 1 || k > kEngMaxK || n % kEngCols != 0 || !rows_vec_ok(x, xsh, 1, m) || !cols_vec_ok(w, wsh, n))
        return hipErrorNotSupported;
    static int cus[64] = {0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (!cus[dev]) {
        int c = 0;
        if ((e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        cus[dev] = c > 0 ? c : 256;
    }
    EngineArgs a{x, xsh, m, k, outx.scale, outx.q, outx.rows_pad, outx.k_pad, w, wsh, n, outw.scale, outw.q,
                 outw.rows_pad, n / kEngCols, n / kEngCols + (int)(outx.rows_pad / 8), range};
    const int grid = a.n_items < cus[dev] ? (a.n_items > 0 ? a.n_items : 1) : cus[dev];
    pack_engine_kernel<<<grid, kEngThreads, 0, stream>>>(a);
    return hipGetLastError();
}

}  // namespace qgemm

using namespace qgemm;

// ---- W-strip timeline probe: pack_w_strip_body's phases with s_memrealtime stamps (block-median) ----
__device__ unsigned long long g_wst[4096][6];
template <bool kDirect>
__global__ __launch_bounds__(1024) void wstrip_probe_kernel(const float *__restrict__ w, int64_t wsh, int k, int n,
                                                            float range, float *__restrict__ scale,
                                                            int8_t *__restrict__ q, int64_t k_pad, int nstrips) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
    const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c4 = t & 3, rq = t >> 2;
    if (t == 0) g_wst[bid][0] = __builtin_amdgcn_s_memrealtime();
    const int64_t n0 = (int64_t)strip * kWsCols;
    float *red = reinterpret_cast<float *>(lds);
    float *s_sh = red + 16 * 16;
    uint8_t *img = lds + 4096;
    const int64_t istride = k_pad + 16;
    float4 v[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            v[i][e] = (r < k) ? *reinterpret_cast<const float4 *>(w + (int64_t)r * wsh + n0 + 4 * c4)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            if (r >= 1 && r < k) {
                p0 = cand_max(p0, v[i][e].x);
                p1 = cand_max(p1, v[i][e].y);
                p2 = cand_max(p2, v[i][e].z);
                p3 = cand_max(p3, v[i][e].w);
            }
        }
    __syncthreads();
    if (t == 0) g_wst[bid][1] = __builtin_amdgcn_s_memrealtime();  // all loads consumed
#pragma unroll
    for (int off = 4; off < 64; off <<= 1) {
        p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
        p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
        p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
        p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
    }
    if (lane < 4) {
        red[wv * 16 + 4 * lane + 0] = p0;
        red[wv * 16 + 4 * lane + 1] = p1;
        red[wv * 16 + 4 * lane + 2] = p2;
        red[wv * 16 + 4 * lane + 3] = p3;
    }
    __syncthreads();
    if (t < kWsCols) {
        float pp = red[t];
#pragma unroll
        for (int ww = 1; ww < 16; ++ww) pp = fmaxf(pp, red[ww * 16 + t]);
        const float cw = absmax_finish(w[n0 + t], pp);
        s_sh[t] = inv_divide(range, cw);
        scale[n0 + t] = cw;
    }
    __syncthreads();
    if (t == 0) g_wst[bid][2] = __builtin_amdgcn_s_memrealtime();  // scales known
    const float s0 = s_sh[4 * c4 + 0], s1 = s_sh[4 * c4 + 1], s2 = s_sh[4 * c4 + 2], s3 = s_sh[4 * c4 + 3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r0 = 4 * rq + 1024 * i;
        if (r0 >= k_pad) continue;
        int qv[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool in = r0 + e < k;
            qv[e][0] = in ? quant_i8(v[i][e].x, s0) : 0;
            qv[e][1] = in ? quant_i8(v[i][e].y, s1) : 0;
            qv[e][2] = in ? quant_i8(v[i][e].z, s2) : 0;
            qv[e][3] = in ? quant_i8(v[i][e].w, s3) : 0;
        }
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const uint32_t d = pack4(qv[0][cc], qv[1][cc], qv[2][cc], qv[3][cc]);
            if constexpr (kDirect)  // straight to packed row n0+4c4+cc: 64-B runs per column per wave
                *reinterpret_cast<uint32_t *>(q + (n0 + 4 * c4 + cc) * k_pad + r0) = d;
            else
                *reinterpret_cast<uint32_t *>(img + (int64_t)(4 * c4 + cc) * istride + r0) = d;
        }
    }
    if constexpr (kDirect) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) g_wst[bid][3] = __builtin_amdgcn_s_memrealtime();
        if (t == 0) g_wst[bid][4] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    __syncthreads();
    if (t == 0) g_wst[bid][3] = __builtin_amdgcn_s_memrealtime();  // image in LDS
    const int64_t words = (int64_t)kWsCols * k_pad / 16;
    for (int64_t x = t; x < words; x += 1024) {
        const int64_t row = x / (k_pad / 16), col16 = x % (k_pad / 16);
        *reinterpret_cast<uint4 *>(q + (n0 + row) * k_pad + col16 * 16) =
            *reinterpret_cast<const uint4 *>(img + row * istride + col16 * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) g_wst[bid][4] = __builtin_amdgcn_s_memrealtime();  // stores acknowledged
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 4096;
    int reps = argc > 4 ? atoi(argv[4]) : 20, rounds = 5;
    float *X, *W; void *PX, *PW, *PX2, *PW2;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&PX2, packed_bytes(m, k))); CK(hipMalloc(&PW2, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    PackedView vx2 = packed_view(PX2, m, k), vw2 = packed_view(PW2, n, k);
    PackedView vnone = packed_view(PX2, 0, k);
    hipStream_t s0, s1; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t fork, join; CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    auto single = [&]() { CK(launch_pack_single_pass(X, k, m, k, vx, W, n, n, vw, 127.f, s0)); };
    auto wonly = [&](hipStream_t s) { CK(launch_pack_single_pass(X, k, 0, k, vnone, W, n, n, vw2, 127.f, s)); };
    auto xonly = [&](hipStream_t s) { CK(launch_pack_rows(X, k, 1, m, k, 127.f, vx2, s)); };
    auto seq = [&]() { wonly(s0); xonly(s0); };
    auto conc = [&]() {
        CK(hipEventRecord(fork, s0)); CK(hipStreamWaitEvent(s1, fork, 0));
        xonly(s1); wonly(s0);
        CK(hipEventRecord(join, s1)); CK(hipStreamWaitEvent(s0, join, 0));
    };
    auto conc_xfirst = [&]() {
        CK(hipEventRecord(fork, s0)); CK(hipStreamWaitEvent(s1, fork, 0));
        wonly(s1); xonly(s0);
        CK(hipEventRecord(join, s1)); CK(hipStreamWaitEvent(s0, join, 0));
    };
    // same stream, the second kernel's dispatch packet without the barrier bit (hipExtAnyOrderLaunch):
    // it may start while the first still runs; the next ordinary launch waits for both
    auto x_any = [&](hipStream_t s) {
        hipExtLaunchKernelGGL((pack_rows_vec_kernel<16>), dim3((unsigned)(vx2.rows_pad / 4)), dim3(256), 0, s, nullptr,
                              nullptr, hipExtAnyOrderLaunch, (const float *)X, (int64_t)k, m, k, 127.f, vx2.scale,
                              vx2.q, vx2.rows_pad, vx2.k_pad);
        CK(hipGetLastError());
    };
    auto any_wx = [&]() { wonly(s0); x_any(s0); };
    auto engine = [&]() { CK(launch_pack_engine(X, k, m, k, vx2, W, n, n, vw2, 127.f, s0)); };
    auto wo = [&]() { wonly(s0); };
    auto xo = [&]() { xonly(s0); };
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"single_pass", single}, {"w_then_x", seq}, {"concurrent", conc},
                         {"concurrent_b", conc_xfirst}, {"anyorder_w_x", any_wx}, {"engine", engine}, {"w_only", wo}, {"x_only", xo}};
    // parity: the split paths must give the same bytes as the single pass
    CK(hipMemset(PX2, 0x5a, packed_bytes(m, k))); CK(hipMemset(PW2, 0x5a, packed_bytes(n, k)));
    single(); engine(); CK(hipStreamSynchronize(s0));
    {
        size_t bx = packed_bytes(m, k), bw = packed_bytes(n, k);
        std::vector<char> a(bx), b(bx), c(bw), d(bw);
        CK(hipMemcpy(a.data(), vx.q, vx.rows_pad * vx.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), vx2.q, vx.rows_pad * vx.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), vw.q, vw.rows_pad * vw.k_pad, hipMemcpyDeviceToHost));
        CK(hipMemcpy(d.data(), vw2.q, vw.rows_pad * vw.k_pad, hipMemcpyDeviceToHost));
        std::vector<float> sa(vx.rows_pad), sb(vx.rows_pad), sc(vw.rows_pad), sd(vw.rows_pad);
        CK(hipMemcpy(sa.data(), vx.scale, sa.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sb.data(), vx2.scale, sb.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sc.data(), vw.scale, sc.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sd.data(), vw2.scale, sd.size() * 4, hipMemcpyDeviceToHost));
        printf("parity (engine vs single pass) x %s  w %s  cx %s  cw %s\n",
               memcmp(a.data(), b.data(), vx.rows_pad * vx.k_pad) ? "DIFF" : "same",
               memcmp(c.data(), d.data(), vw.rows_pad * vw.k_pad) ? "DIFF" : "same",
               memcmp(sa.data(), sb.data(), sa.size() * 4) ? "DIFF" : "same",
               memcmp(sc.data(), sd.data(), sc.size() * 4) ? "DIFF" : "same");
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            for (int w = 0; w < 3; ++w) vs[i].f();
            CK(hipEventRecord(e0, s0));
            for (int j = 0; j < reps; ++j) vs[i].f();
            CK(hipEventRecord(e1, s0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    for (int direct = 0; direct < 2; ++direct) {   // W-strip phase timeline (block-median, 100 MHz ticks -> us)
        const int nstrips = n / kWsCols;
        const size_t lds = 4096 + (size_t)kWsCols * (vw2.k_pad + 16);
        auto kern = direct ? wstrip_probe_kernel<true> : wstrip_probe_kernel<false>;
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
        for (int it = 0; it < 20; ++it) kern<<<nstrips, 1024, lds, s0>>>(W, n, k, n, 127.f, vw2.scale, vw2.q, vw2.k_pad, nstrips);
        CK(hipEventRecord(a, s0));
        for (int it = 0; it < 50; ++it) kern<<<nstrips, 1024, lds, s0>>>(W, n, k, n, 127.f, vw2.scale, vw2.q, vw2.k_pad, nstrips);
        CK(hipEventRecord(z, s0)); CK(hipEventSynchronize(z));
        float ms; CK(hipEventElapsedTime(&ms, a, z));
        if (direct) {  // parity of the direct-store image against the single pass
            std::vector<char> c(vw.rows_pad * vw.k_pad), d(vw.rows_pad * vw.k_pad);
            single(); CK(hipStreamSynchronize(s0));
            CK(hipMemcpy(c.data(), vw.q, c.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(d.data(), vw2.q, d.size(), hipMemcpyDeviceToHost));
            printf("direct-store W image %s\n", memcmp(c.data(), d.data(), (size_t)n * vw.k_pad) ? "DIFF" : "same");
        }
        printf("wstrip probe (%s): %.2f us per launch\n", direct ? "direct global stores" : "LDS transpose", ms * 1000 / 50);
        std::vector<unsigned long long> st((size_t)4096 * 6);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wst), st.size() * 8));
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nstrips; ++b) t0 = std::min(t0, st[(size_t)b * 6]);
        const char *nm[5] = {"start", "loads consumed", "scales", "LDS image", "stores acked"};
        for (int ph = 0; ph < 5; ++ph) {
            std::vector<double> v;
            for (int b = 0; b < nstrips; ++b) v.push_back((st[(size_t)b * 6 + ph] - t0) * 0.01);
            std::sort(v.begin(), v.end());
            printf("  %-15s  min %6.2f  median %6.2f  max %6.2f us (from first block start)\n", nm[ph], v[0],
                   v[v.size() / 2], v.back());
        }
    }
    const double bytes = 4.0 * m * k + 4.0 * k * n + (double)m * k + (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us  (%.2f TB/s for the full pack bytes)\n", vs[i].name, v[v.size() / 2], v[0],
               bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
