// encoder_ops.hip -- the row operations of the encoder counterpart that sit
// between its quantized linears: the reference's op_multiply + op_softmax (attention.cuh:65-68,
// op_softmax.cuh:6-29) and op_add + op_layernorm (transformer.cu:58-59, op_layernorm.cuh:6-33).
//
// The reference runs one THREAD per row with sequential fp32 sums.  Here one WAVE per row: the
// elementwise parts run across the lanes, and each sum stays ONE sequential fp32 chain in element
// order (the row is staged in LDS and every lane walks it), so the results keep the reference's
// rounding sequence.  Decisions where the reference is not defined precisely (encoder):
//   exp    : correctly rounded fp32 exp, fl32(exp((double)x)) (CUDA's expf is within 2 ulp, host
//            expf differs again; the oracle uses the same definition)
//   pow(d,2): fl32(d * d) (CUDA's float pow(float, int) overload)
//   grids  : every row is processed (the reference's launch covers ceil(w/256)*256 rows, which is
//            all of them whenever w >= h, as in every shape it runs)
#include "qgemm_internal.h"

namespace qgemm {

namespace {

constexpr int kRowWaves = 4;       // rows per 256-thread block
constexpr int kMaxRowLen = 4096;   // LDS staging per wave: 16 KiB

// sequential fp32 sum of row[0..w) in element order (every lane computes the same chain; the reads
// are LDS broadcasts).  The chain is latency-bound: groups of G elements are read with G/4 b128 loads
// issued together, so each group waits out the LDS latency once (G = 64: 4x fewer exposed latencies
// than groups of 16), then the 16-element and scalar tails.
template <int G>
__device__ __forceinline__ void seq_sum_groups(const float *row, int w, int &e, float &sum) {
    for (; e + G <= w; e += G) {
        float4 q[G / 4];
#pragma unroll
        for (int j = 0; j < G / 4; ++j) q[j] = *reinterpret_cast<const float4 *>(row + e + 4 * j);
#pragma unroll
        for (int j = 0; j < G / 4; ++j) {
            sum = __fadd_rn(sum, q[j].x);
            sum = __fadd_rn(sum, q[j].y);
            sum = __fadd_rn(sum, q[j].z);
            sum = __fadd_rn(sum, q[j].w);
        }
    }
}
__device__ __forceinline__ float seq_sum(const float *row, int w) {
    float sum = 0.0f;
    int e = 0;
    seq_sum_groups<64>(row, w, e, sum);
    seq_sum_groups<16>(row, w, e, sum);
    for (; e < w; ++e) sum = __fadd_rn(sum, row[e]);
    return sum;
}

// The same sequential fp32 sum over a row held in registers: element 4(l + 64 i) + c is x[i].c of lane l
// (the layout of add_layernorm_rows_vec_kernel), w4 = w / 4 float4 columns.  The running sum hops from
// lane to lane: every step is one v_add_f32 whose first operand is the LEFT neighbour's sum (DPP
// wave_ror:1: lane l reads lane l - 1, lane 0 reads lane 63), then three in-lane adds.  Every lane runs
// every step, so after step t of group i lane t - 1 holds the chain through its own four elements
// (induction: each step extends the chain that had reached the left neighbour one step earlier), and lane 63
// hands a full group on to lane 0 of the next.  Per element one dependent add and no LDS round trip: the
// LDS-walking chain (seq_sum) spends ~7-8 cycles per element waiting on its ds_read groups.  The result is
// the sum in lane (w4 - 1) mod 64, broadcast.
__device__ __forceinline__ float hop_step(float s, const float4 &v) {
    s = __fadd_rn(hop_left(s), v.x);
    s = __fadd_rn(s, v.y);
    s = __fadd_rn(s, v.z);
    return __fadd_rn(s, v.w);
}
template <int kV>
__device__ __forceinline__ float lane_chain_sum(const float4 (&x)[kV], int w4) {
    float s = 0.0f;
    int last = 63;
#pragma unroll
    for (int i = 0; i < kV; ++i) {
        const int n = w4 - 64 * i < 64 ? w4 - 64 * i : 64;
        if (n <= 0) break;
        int t = 0;
        for (; t + 8 <= n; t += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) s = hop_step(s, x[i]);
        }
        for (; t < n; ++t) s = hop_step(s, x[i]);
        last = n - 1;
    }
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), last));
}

// The same chain over the block layout: lane l holds the kV consecutive float4 columns kV l .. kV l + kV - 1
// (elements 4 kV l .. 4 kV (l + 1) - 1), so the running sum hops once per 4 kV elements instead of once per 4:
// step t is one v_add_f32 on the left neighbour's sum, then 4 kV - 1 in-lane adds, and after step t lane t - 1
// holds the chain through its own block (the induction of lane_chain_sum).  nl = the lanes that hold elements
// (<= 64); elements past the row must be -0.0f (x + -0 == x for every x, -0 and NaN included), so the last
// lane's adds stay uniform.  Each hop costs the DPP read's wait states on top of its add: 16-element blocks
// spend ~4.5 cycles per element against ~6 for lane_chain_sum's 4.
template <int kV>
__device__ __forceinline__ float block_step(float s, const float4 (&x)[kV]) {
    s = __fadd_rn(hop_left(s), x[0].x);
    s = __fadd_rn(s, x[0].y);
    s = __fadd_rn(s, x[0].z);
    s = __fadd_rn(s, x[0].w);
#pragma unroll
    for (int i = 1; i < kV; ++i) {
        s = __fadd_rn(s, x[i].x);
        s = __fadd_rn(s, x[i].y);
        s = __fadd_rn(s, x[i].z);
        s = __fadd_rn(s, x[i].w);
    }
    return s;
}
template <int kV>
__device__ __forceinline__ float lane_block_sum(const float4 (&x)[kV], int nl) {
    float s = 0.0f;
    int t = 0;
    for (; t + 4 <= nl; t += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s = block_step<kV>(s, x);
    }
    for (; t < nl; ++t) s = block_step<kV>(s, x);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), nl - 1));
}

// fl((x - mean)^2): pow(x - mean, 2) as fp32 d*d (CUDA's float pow(float, int) overload)
__device__ __forceinline__ float sq_dev(float x, float mean) {
    const float d = __fsub_rn(x, mean);
    return __fmul_rn(d, d);
}

__global__ __launch_bounds__(64 * kRowWaves) void softmax_rows_kernel(const float *S, float *P, int64_t rows, int w,
                                                                      float scale) {  // P may be S (in place)
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * kRowWaves + wv;
    if (row >= rows) return;
    const float *s = S + row * w;
    float *p = P + row * w;
    float *st = stage + wv * ((w + 3) & ~3);  // 16-B aligned row stage
    // max: seed = first element, then "if (x > max) max = x" (op_softmax.cuh:13-18) -- NaN never wins
    const float seed = __fmul_rn(s[0], scale);
    float cand = -INFINITY;
    for (int c = lane + 1; c < w; c += 64) {
        const float x = __fmul_rn(s[c], scale);  // op_multiply(QK_T, scale_factor) (attention.cuh:65)
        cand = (x > cand) ? x : cand;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_xor(cand, off, 64);
        cand = (o > cand) ? o : cand;
    }
    const float mx = (cand > seed) ? cand : seed;
    for (int c = lane; c < w; c += 64) {
        const float d = __fsub_rn(__fmul_rn(s[c], scale), mx);
        st[c] = (float)exp((double)d);  // correctly rounded fp32 exp
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done (one wave per row)
    __builtin_amdgcn_wave_barrier();
    const float sum = seq_sum(st, w);   // op_softmax.cuh:20-24, in column order
    for (int c = lane; c < w; c += 64) p[c] = __fdiv_rn(st[c], sum);
}

// kPack: also quantize the output row for the next quantized linear (the pack_rows step of
// linear(), fused): absmax with the signed seed y[0] over |y[c]|, c >= 1 (maxnum: NaN never wins),
// s = fl(range / Cx), q = sat_i8(trunc(fl(y * s))) -- the same operations as pack_rows_vec_body, so
// the packed row is bit-identical to packing Y afterwards.  Rows [rows, rows_pad) of the packed view
// get zero bytes and a zero scale; columns [w, k_pad) zero bytes.
// kStamp (lab only; 0 in the library): s_memrealtime stamps at the phase boundaries (g_ln_stamp)
__device__ unsigned long long g_ln_stamp[4096][8];
template <bool kPack, int kStamp = 0>
__global__ __launch_bounds__(64 * kRowWaves) void add_layernorm_rows_kernel(const float *__restrict__ A,
                                                                            const float *__restrict__ B,
                                                                            float *__restrict__ Y, int64_t rows,
                                                                            int w, int8_t *__restrict__ q,
                                                                            float *__restrict__ qscale,
                                                                            int64_t k_pad, int64_t rows_pad,
                                                                            float range) {
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * kRowWaves + wv;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kStamp != 0)
            if (lane == 0 && row < 4096) g_ln_stamp[row][i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    if (kPack && row >= rows && row < rows_pad) {  // padding row of the packed view
        auto qrow = [&](int64_t c) __attribute__((always_inline)) -> uint32_t & { return *qword(q, row, 4 * c, k_pad); };  // fragment-major q
        for (int64_t c = lane; c < k_pad / 4; c += 64) qrow(c) = 0u;
        if (lane == 0) qscale[row] = 0.0f;
        return;
    }
    if (row >= rows) return;
    const float *a = A + row * w, *b = B + row * w;
    float *y = Y + row * w;
    float *st = stage + wv * ((w + 3) & ~3);
    for (int c = lane; c < w; c += 64) st[c] = __fadd_rn(a[c], b[c]);  // op_add (transformer.cu:58)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    stamp(1);
    const float fw = (float)w;                                 // "mean/w": int -> float
    const float mean = __fdiv_rn(seq_sum(st, w), fw);          // op_layernorm.cuh:15-19
    stamp(2);
    __builtin_amdgcn_wave_barrier();
    // the squared deviations replace the row in LDS (each lane rewrites the columns it owns)
    for (int c = lane; c < w; c += 64) {
        st[c] = sq_dev(st[c], mean);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    stamp(3);
    const float var = __fdiv_rn(seq_sum(st, w), fw);           // :21-25
    stamp(4);
    float cand = -INFINITY;
    __builtin_amdgcn_wave_barrier();
    for (int c = lane; c < w; c += 64) {                       // (x - mean) / var (:28), as written
        const float v = __fdiv_rn(__fsub_rn(__fadd_rn(a[c], b[c]), mean), var);
        y[c] = v;
        if constexpr (kPack) {
            st[c] = v;  // each lane overwrites only the columns it owns
            if (c > 0) cand = fmaxf(cand, absmax_candidate(v));
        }
    }
    stamp(5);
    if constexpr (kPack) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) cand = fmaxf(cand, __shfl_xor(cand, off, 64));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const float cx = absmax_finish(st[0], cand);
        const float sc = inv_divide(range, cx);
        auto qrow = [&](int64_t c) __attribute__((always_inline)) -> uint32_t & { return *qword(q, row, 4 * c, k_pad); };  // fragment-major q
        for (int c4 = lane; c4 < (int)(k_pad / 4); c4 += 64) {
            int qb[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) qb[e] = 4 * c4 + e < w ? quant_i8(st[4 * c4 + e], sc) : 0;
            qrow(c4) = (uint32_t)(qb[0] & 0xff) | ((uint32_t)(qb[1] & 0xff) << 8) | ((uint32_t)(qb[2] & 0xff) << 16) |
                       ((uint32_t)(qb[3] & 0xff) << 24);
        }
        if (lane == 0) qscale[row] = cx;
    }
    stamp(6);
}

// The same add + layernorm (+ pack) for rows of w % 4 == 0 floats, 16-B aligned: each lane holds kV float4
// columns (columns 4j..4j+3 of float4 column j, layout below) in registers from the first load to the last
// use, so neither the normalisation nor the pack re-reads A, B or LDS; each packed dword is one lane's four
// columns.
// kHop (the product): both sums hop lane to lane over the registers; false: staged in LDS and walked by
// seq_sum (lab comparison).  kBlk (the product): lane l holds the float4 columns j = kV l + i (a block of 4 kV
// consecutive elements, lane_block_sum: one hop per block, and each lane's packed dwords of a 16-element
// block are one 16-B piece of the fragment-major row); false: j = lane + 64 i (lane_chain_sum, one hop per 4
// elements; the round-3 to round-6 product, kept for the lab comparison)
template <bool kPack, int kV, int kStamp = 0, bool kHop = true, bool kBlk = true>
__global__ __launch_bounds__(64 * kRowWaves) void add_layernorm_rows_vec_kernel(
    const float *__restrict__ A, const float *__restrict__ B, float *__restrict__ Y, int64_t rows, int w,
    int8_t *__restrict__ q, float *__restrict__ qscale, int64_t k_pad, int64_t rows_pad, float range) {
    static_assert(!kBlk || kHop, "the block layout has no LDS-walking form");
    static_assert(!kBlk || kV % 4 == 0, "the block layout stores whole 16-B pieces of the packed row");
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * kRowWaves + wv;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kStamp != 0)
            if (lane == 0 && row < 4096) g_ln_stamp[row][i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    if (kPack && row >= rows && row < rows_pad) {  // padding row of the packed view
        auto qrow = [&](int64_t c) __attribute__((always_inline)) -> uint32_t & { return *qword(q, row, 4 * c, k_pad); };  // fragment-major q
        for (int64_t c = lane; c < k_pad / 4; c += 64) qrow(c) = 0u;
        if (lane == 0) qscale[row] = 0.0f;
        return;
    }
    if (row >= rows) return;
    const int w4 = w >> 2;
    const float4 *a = reinterpret_cast<const float4 *>(A + row * w), *b = reinterpret_cast<const float4 *>(B + row * w);
    float4 *y = reinterpret_cast<float4 *>(Y + row * w);
    float *st = stage + wv * w;
    auto col = [&](int i) __attribute__((always_inline)) { return kBlk ? kV * lane + i : lane + 64 * i; };
    const int nl = (w4 + kV - 1) / kV;  // kBlk: the lanes that hold elements
    float4 x[kV];
#pragma unroll
    for (int i = 0; i < kV; ++i) {
        const int j = col(i);
        x[i] = kBlk ? make_float4(-0.0f, -0.0f, -0.0f, -0.0f) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (j < w4) {
            const float4 av = a[j], bv = b[j];
            x[i] = make_float4(__fadd_rn(av.x, bv.x), __fadd_rn(av.y, bv.y), __fadd_rn(av.z, bv.z),
                               __fadd_rn(av.w, bv.w));  // op_add (transformer.cu:58)
            if constexpr (!kHop) reinterpret_cast<float4 *>(st)[j] = x[i];
        }
    }
    if constexpr (!kHop) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    stamp(1);
    const float fw = (float)w;
    const float sum_x = kBlk ? lane_block_sum<kV>(x, nl) : kHop ? lane_chain_sum<kV>(x, w4) : seq_sum(st, w);
    const float mean = __fdiv_rn(sum_x, fw);  // op_layernorm.cuh:15-19
    stamp(2);
    // the squared deviations, formed from the registers (a chain that formed them itself would carry the
    // sub -> mul latency on every add: measured 2x slower)
    float var;
    if constexpr (kHop) {
        float4 d[kV];
#pragma unroll
        for (int i = 0; i < kV; ++i) {
            d[i] = make_float4(sq_dev(x[i].x, mean), sq_dev(x[i].y, mean), sq_dev(x[i].z, mean), sq_dev(x[i].w, mean));
            if (kBlk && col(i) >= w4) d[i] = make_float4(-0.0f, -0.0f, -0.0f, -0.0f);  // past the row: the identity
        }
        stamp(3);
        var = __fdiv_rn(kBlk ? lane_block_sum<kV>(d, nl) : lane_chain_sum<kV>(d, w4), fw);  // :21-25
    } else {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kV; ++i) {
            const int j = lane + 64 * i;
            if (j < w4)
                reinterpret_cast<float4 *>(st)[j] =
                    make_float4(sq_dev(x[i].x, mean), sq_dev(x[i].y, mean), sq_dev(x[i].z, mean), sq_dev(x[i].w, mean));
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        stamp(3);
        var = __fdiv_rn(seq_sum(st, w), fw);                       // :21-25
    }
    stamp(4);
    float cand = -INFINITY;
#pragma unroll
    for (int i = 0; i < kV; ++i) {
        const int j = col(i);
        if (j < w4) {
            float4 v;                                                // (x - mean) / var (:28), as written
            v.x = __fdiv_rn(__fsub_rn(x[i].x, mean), var);
            v.y = __fdiv_rn(__fsub_rn(x[i].y, mean), var);
            v.z = __fdiv_rn(__fsub_rn(x[i].z, mean), var);
            v.w = __fdiv_rn(__fsub_rn(x[i].w, mean), var);
            y[j] = v;
            x[i] = v;
            if constexpr (kPack) {
                if (j > 0) cand = fmaxf(cand, absmax_candidate(v.x));
                cand = fmaxf(cand, absmax_candidate(v.y));
                cand = fmaxf(cand, absmax_candidate(v.z));
                cand = fmaxf(cand, absmax_candidate(v.w));
            }
        }
    }
    stamp(5);
    if constexpr (kPack) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) cand = fmaxf(cand, __shfl_xor(cand, off, 64));
        const float seed = __shfl(x[0].x, 0, 64);  // column 0: lane 0, i = 0
        const float cx = absmax_finish(seed, cand);
        const float sc = inv_divide(range, cx);
        auto qrow = [&](int64_t c) __attribute__((always_inline)) -> uint32_t & { return *qword(q, row, 4 * c, k_pad); };  // fragment-major q
        uint32_t pk[kV];
#pragma unroll
        for (int i = 0; i < kV; ++i)
            pk[i] = (uint32_t)(quant_i8(x[i].x, sc) & 0xff) | ((uint32_t)(quant_i8(x[i].y, sc) & 0xff) << 8) |
                    ((uint32_t)(quant_i8(x[i].z, sc) & 0xff) << 16) | ((uint32_t)(quant_i8(x[i].w, sc) & 0xff) << 24);
        if constexpr (kBlk) {
            // dwords kV l + 4g .. + 3 = k 16 (kV l / 4 + g) .. + 15: one aligned 16-B piece of the row
#pragma unroll
            for (int g = 0; g < kV / 4; ++g) {
                const int j0 = col(4 * g);
                if (j0 + 3 < w4) {
                    *reinterpret_cast<uint4 *>(qword(q, row, 4 * j0, k_pad)) =
                        make_uint4(pk[4 * g], pk[4 * g + 1], pk[4 * g + 2], pk[4 * g + 3]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j0 + e < w4) qrow(j0 + e) = pk[4 * g + e];
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < kV; ++i)
                if (col(i) < w4) qrow(col(i)) = pk[i];
        }
        for (int64_t c4 = w4 + lane; c4 < k_pad / 4; c4 += 64) qrow(c4) = 0u;  // padding columns
        if (lane == 0) qscale[row] = cx;
    }
    stamp(6);
}

// register-resident path: w % 4 == 0, w <= 256 * kV (kV = 4, 8 or 16), 16-B aligned rows
template <bool kPack>
hipError_t launch_ln_vec(const float *A, const float *B, float *Y, int64_t rows, int w, int8_t *q, float *qscale,
                         int64_t k_pad, int64_t rows_pad, float range, int64_t grid_rows, hipStream_t stream) {
    const size_t lds = 0;  // the sums run in registers (kHop)
    const unsigned grid = (unsigned)((grid_rows + kRowWaves - 1) / kRowWaves);
    if (w <= 1024)
        add_layernorm_rows_vec_kernel<kPack, 4><<<grid, 64 * kRowWaves, lds, stream>>>(A, B, Y, rows, w, q, qscale, k_pad,
                                                                                      rows_pad, range);
    else if (w <= 2048)
        add_layernorm_rows_vec_kernel<kPack, 8><<<grid, 64 * kRowWaves, lds, stream>>>(A, B, Y, rows, w, q, qscale, k_pad,
                                                                                      rows_pad, range);
    else
        add_layernorm_rows_vec_kernel<kPack, 16><<<grid, 64 * kRowWaves, lds, stream>>>(A, B, Y, rows, w, q, qscale,
                                                                                       k_pad, rows_pad, range);
    return hipGetLastError();
}

bool ln_vec_ok(const float *A, const float *B, const float *Y, int w) {
    const uintptr_t al = reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(Y);
    return w % 4 == 0 && w <= kMaxRowLen && (al & 15) == 0;
}

}  // namespace

hipError_t launch_softmax_rows(const float *S, float *P, int64_t rows, int w, float scale, hipStream_t stream) {
    if (w < 1 || w > kMaxRowLen || rows < 0) return hipErrorInvalidValue;
    if (rows == 0) return hipSuccess;
    const size_t lds = sizeof(float) * kRowWaves * ((w + 3) & ~3);
    softmax_rows_kernel<<<(unsigned)((rows + kRowWaves - 1) / kRowWaves), 64 * kRowWaves, lds, stream>>>(S, P, rows, w,
                                                                                                      scale);
    return hipGetLastError();
}

hipError_t launch_add_layernorm_rows(const float *A, const float *B, float *Y, int64_t rows, int w,
                                     hipStream_t stream) {
    if (w < 1 || w > kMaxRowLen || rows < 0) return hipErrorInvalidValue;
    if (rows == 0) return hipSuccess;
    if (ln_vec_ok(A, B, Y, w)) return launch_ln_vec<false>(A, B, Y, rows, w, nullptr, nullptr, 0, 0, 0.0f, rows, stream);
    const size_t lds = sizeof(float) * kRowWaves * ((w + 3) & ~3);
    add_layernorm_rows_kernel<false><<<(unsigned)((rows + kRowWaves - 1) / kRowWaves), 64 * kRowWaves, lds, stream>>>(
        A, B, Y, rows, w, nullptr, nullptr, 0, 0, 0.0f);
    return hipGetLastError();
}

hipError_t launch_add_layernorm_rows_pack(const float *A, const float *B, float *Y, int64_t rows, int w, float range,
                                          PackedView out, hipStream_t stream) {
    if (w < 1 || w > kMaxRowLen || rows < 1 || out.k_pad < w || out.rows_pad < rows) return hipErrorInvalidValue;
    if (ln_vec_ok(A, B, Y, w))
        return launch_ln_vec<true>(A, B, Y, rows, w, out.q, out.scale, out.k_pad, out.rows_pad, range, out.rows_pad, stream);
    const size_t lds = sizeof(float) * kRowWaves * ((w + 3) & ~3);
    add_layernorm_rows_kernel<true><<<(unsigned)((out.rows_pad + kRowWaves - 1) / kRowWaves), 64 * kRowWaves, lds,
                                      stream>>>(A, B, Y, rows, w, out.q, out.scale, out.k_pad, out.rows_pad, range);
    return hipGetLastError();
}

}  // namespace qgemm
