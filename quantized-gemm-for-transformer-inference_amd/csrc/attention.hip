// attention.hip -- the encoder's fp32 attention core (attention.cuh:58-69) in ONE launch per block of
// the encoder: for every (head, 32-query tile) a workgroup computes
//   S = Q_h K_h^T                  op_mm<float> on the transposed view    (attention.cuh:58-60)
//   P = softmax(S * 1/sqrt(d_k))   op_multiply + op_softmax               (attention.cuh:65-68)
//   heads[:, h*d_k..] = P V_h      op_mm<float>                           (attention.cuh:69)
// with S and P kept in LDS (the three-launch form writes and re-reads the H x seq x seq score tensor
// through HBM twice).  Every step keeps the arithmetic of the separate kernels bit for bit:
//   * both products are v_mfma_f32_16x16x4_f32 chains from +0 over k ascending, zero-padded to a
//     multiple of 4, then fl(res + 0) when k % 32 != 0 -- the reference's op_matmul_kernel chain
//     (op_mm.cuh:37-39) with its zero-padded last 32-wide tile, exactly as gemm_f32.hip;
//   * softmax as softmax_rows_kernel: products fl(s * scale), max seeded by the first element with a
//     strict >, correctly rounded fp32 exp of fl(x - max), ONE sequential fp32 sum in column order,
//     then fl(e / sum).
// Envelope: d_k <= 64, seq <= 512 (S tile 32 x 512 fp32 = 64 KiB of LDS, Q tile and K / V staged
// through LDS in 256-key chunks: 155 KiB in all); outside it the encoder runs the three kernels.
#include "qgemm_internal.h"

#include <type_traits>

namespace qgemm {

namespace {

constexpr int kAttnMaxSeq = 512;
constexpr int kAttnMaxDk = 64;
constexpr int kSStride = kAttnMaxSeq + 4;  // S row stride (floats): consecutive rows 4 banks apart
constexpr int kKStride = 68;               // K chunk [key][d_k]: B-fragment reads (16 keys x 4 k) conflict-free
constexpr int kVStride = 80;               // V chunk [key][d_k]: B-fragment reads (4 keys x 16 cols) conflict-free
constexpr int kQStride = 68;               // Q tile [query][d_k]: A-fragment reads conflict-free

// Tile configurations.  kTQ query rows per workgroup, kChunk keys per K / V chunk, one 16-column QK tile
// per wave (kChunk = 16 x waves), two softmax rows per wave (kTQ = 2 x waves).
//   <32, 256, 1024>: 153 KiB of LDS, one workgroup per CU (the library's choice);
//   <16, 128, 512> : 77 KiB, two workgroups per CU whose phases could overlap -- measured slower
//                    (36.5 vs 30.6 us at config 5: twice the K / V staging, one QK chain per wave).
template <int kTQ, int kChunk, int kThreads>
struct AttnTile {
    static constexpr int kWaves = kThreads / 64;
    static_assert(kChunk == 16 * kWaves && kTQ == 2 * kWaves, "one QK column tile and two softmax rows per wave");
    static constexpr int kRowFrags = kTQ / 16;
    static constexpr int kKVFloats = kChunk * kVStride;
    static constexpr int kWavesPerEu = 4;  // 4 waves per SIMD either way: <= 128 VGPRs
};

typedef float v4f __attribute__((ext_vector_type(4)));

// kSkip (lab ablation only; 0 in the library): 1 = no QK^T MFMAs, 2 = no softmax, 4 = no PV MFMAs,
// 8 = no sequential sums, 16 = s_memrealtime stamps at the phase boundaries (g_attn_stamp)
__device__ unsigned long long g_attn_stamp[4096][8];
template <int kTQ, int kChunk, int kThreads, int kSkip = 0>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void attention_fused_kernel(
    const float *__restrict__ qkv, int d, int dk, int seq, float scale, float *__restrict__ heads) {
    using T = AttnTile<kTQ, kChunk, kThreads>;
    constexpr int kAttnThreads = kThreads, kRF = T::kRowFrags;
    __shared__ __attribute__((aligned(16))) float S[kTQ * kSStride];
    __shared__ __attribute__((aligned(16))) float KV[T::kKVFloats];
    __shared__ __attribute__((aligned(16))) float Qs[kTQ * kQStride];
    // XCD-aware: blocks b, b+8, ... share an XCD; each XCD gets a contiguous range of (head, query tile)
    // pairs, so a head's query tiles (and its K / V re-reads) stay in one L2
    const int nwg = gridDim.x * gridDim.y, lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int xq = nwg >> 3, xr = nwg & 7, xc = lin & 7;
    const int logical = (xc < xr ? xc * (xq + 1) : xr * (xq + 1) + (xc - xr) * xq) + (lin >> 3);
    const int h = logical / gridDim.x, q0 = (logical - h * gridDim.x) * kTQ;
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t ld = 3 * (int64_t)d;
    const float *Qb = qkv + (int64_t)h * dk, *Kb = qkv + d + (int64_t)h * dk, *Vb = qkv + 2 * (int64_t)d + (int64_t)h * dk;
    const int lr = lane & 15, lk = lane >> 4;  // MFMA operand lane: row lr of the fragment, k offset lk
    const int rows = seq - q0 < kTQ ? seq - q0 : kTQ;
    const int nchunks = (seq + kChunk - 1) / kChunk;
    const int seq32 = (seq + 31) & ~31;  // the reference's k extent for P V: seq zero-padded to its 32-wide tile
    const int dk4 = (dk + 3) >> 2;  // float4 columns of a K / V row (the last one zero-padded)
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr ((kSkip & 16) != 0)
            if (t == 0) g_attn_stamp[bid & 4095][i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // K / V chunks as float4 pieces, kPer per thread, fetched into registers one chunk ahead -- chunk
    // c+1's global loads are in flight under chunk c's MFMAs, V chunk 0's under the last QK chunk and
    // the softmax -- then written to KV ([key][stride], zero past seq and past d_k)
    constexpr int kPer = kChunk * 16 / kThreads;
    auto fetch = [&](float4 (&r)[kPer], const float *src, int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int f = t + i * kThreads, row = f >> 4, c4 = f & 15, j = c0 + row;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < seq && c4 < dk4) {
                const float *p = src + j * ld + 4 * c4;
                if (4 * c4 + 3 < dk && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
                    v = *reinterpret_cast<const float4 *>(p);
                } else {
                    v.x = p[0];
                    v.y = 4 * c4 + 1 < dk ? p[1] : 0.f;
                    v.z = 4 * c4 + 2 < dk ? p[2] : 0.f;
                    v.w = 4 * c4 + 3 < dk ? p[3] : 0.f;
                }
            }
            r[i] = v;
        }
    };
    auto put = [&](const float4 (&r)[kPer], int stride) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int f = t + i * kThreads;
            *reinterpret_cast<float4 *>(KV + (f >> 4) * stride + 4 * (f & 15)) = r[i];
        }
    };

    // ---- S[32][seq] = Q K^T, one K chunk at a time: wave w computes 16-column tile w of the chunk for
    // both 16-row halves (one B fragment, two A fragments)
    const int ns32 = ((dk + 31) & ~31) >> 2;  // k-steps over d_k zero-padded to 32: 8 or 16
    // the Q tile through LDS (coalesced row loads once per workgroup, not per wave), with K chunk 0
    float4 pf[kPer];
    fetch(pf, Kb, 0);
    for (int f = t; f < kTQ * 16; f += kAttnThreads) {
        const int row = f >> 4, c4 = f & 15, i = q0 + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < seq && c4 < dk4) {
            const float *p = Qb + i * ld + 4 * c4;
            v.x = p[0];
            v.y = 4 * c4 + 1 < dk ? p[1] : 0.f;
            v.z = 4 * c4 + 2 < dk ? p[2] : 0.f;
            v.w = 4 * c4 + 3 < dk ? p[3] : 0.f;
        }
        *reinterpret_cast<float4 *>(Qs + row * kQStride + 4 * c4) = v;
    }
    float qa[kRF][16];
    for (int c = 0; c < nchunks; ++c) {
        if (c) __syncthreads();  // every wave is done with the previous chunk
        put(pf, kKStride);
        __syncthreads();
        if (c + 1 < nchunks) fetch(pf, Kb, (c + 1) * kChunk);
        else fetch(pf, Vb, 0);
        if (c == 0) {
#pragma unroll
            for (int rf = 0; rf < kRF; ++rf)
#pragma unroll
                for (int s = 0; s < 16; ++s) qa[rf][s] = Qs[(rf * 16 + lr) * kQStride + 4 * s + lk];
            stamp(1);
        }
        const int col = c * kChunk + wave * 16 + lr;
        if (c * kChunk + wave * 16 < seq) {
            const float *krow = KV + (wave * 16 + lr) * kKStride + lk;
            v4f acc[kRF];
#pragma unroll
            for (int rf = 0; rf < kRF; ++rf) acc[rf] = v4f{0.f, 0.f, 0.f, 0.f};
            // k-steps over the reference's zero-padded extent (d_k rounded up to 32: Q and K are zero past
            // d_k, so those steps are its padded tile's +0 adds) -- 8 or 16 steps with no per-step
            // condition, the B fragments read together
            auto steps = [&](auto kSteps) __attribute__((always_inline)) {
                constexpr int kS = decltype(kSteps)::value;
                float kb[kS];
#pragma unroll
                for (int s = 0; s < kS; ++s) kb[s] = krow[4 * s];
#pragma unroll
                for (int s = 0; s < kS; ++s)
#pragma unroll
                    for (int rf = 0; rf < kRF; ++rf)
                        acc[rf] = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[rf][s], kb[s], acc[rf], 0, 0, 0);
            };
            if (!(kSkip & 1)) {
                if (ns32 == 16) steps(std::integral_constant<int, 16>());
                else steps(std::integral_constant<int, 8>());
            }
            if (col < seq) {
#pragma unroll
                for (int rf = 0; rf < kRF; ++rf)
#pragma unroll
                    for (int r = 0; r < 4; ++r) S[(rf * 16 + 4 * lk + r) * kSStride + col] = acc[rf][r];
            }
        }
    }
    __syncthreads();
    stamp(2);

    // ---- softmax of rows 2w and 2w+1: max and exp across the lanes, the two sequential sums at once
    // (lanes 0 and 1), the division across the lanes -- all through the LDS row (keeping the scaled
    // scores and exps in registers instead measured 1 us slower per launch)
    for (int rr = 0; rr < 2 && !(kSkip & 2); ++rr) {
        const int rl = wave * 2 + rr;
        if (rl >= rows) break;
        float *srow = S + rl * kSStride;
        const float seed = __fmul_rn(srow[0], scale);
        float cand = -INFINITY;
        for (int c = lane + 1; c < seq; c += 64) {
            const float x = __fmul_rn(srow[c], scale);  // op_multiply(QK_T, scale_factor)
            cand = (x > cand) ? x : cand;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float o = __shfl_xor(cand, off, 64);
            cand = (o > cand) ? o : cand;
        }
        const float mx = (cand > seed) ? cand : seed;
        for (int c = lane; c < seq; c += 64) srow[c] = (float)exp((double)__fsub_rn(__fmul_rn(srow[c], scale), mx));
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's exps are in LDS
    __builtin_amdgcn_wave_barrier();
    stamp(6);
    // the two sums at once, each hopping lane to lane (hop_left): row 2w in lanes 0-31, row 2w+1 in lanes
    // 32-63, lane h of a half holding elements 16h .. 16h+15 of its row in registers; after step t the
    // chain through lane h = t - 1 of each half sits in that lane (lane 32 starts from lane 31's initial
    // zero; both halves run the same instructions).  Elements past seq are -0.0f, which leaves any sum
    // unchanged, so the last lane's 16 adds stay uniform.  Per element one dependent add, no LDS reads
    // inside the chain (the LDS-walking form exposed one read latency per 64 elements).
    float sum_a = 0.0f, sum_b = 0.0f;
    if (!(kSkip & 8)) {
        const int hl = lane & 31, nl = (seq + 15) >> 4;  // lanes per half that hold elements (nl <= 32)
        const float *srow = S + (wave * 2 + (lane >> 5)) * kSStride + 16 * hl;
        float e[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (hl < nl && wave * 2 + (lane >> 5) < rows) v = *reinterpret_cast<const float4 *>(srow + 4 * j);
            e[4 * j] = v.x; e[4 * j + 1] = v.y; e[4 * j + 2] = v.z; e[4 * j + 3] = v.w;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (16 * hl + j >= seq) e[j] = -0.0f;
        float s = 0.0f;
        for (int t = 0; t < nl; ++t) {
            s = __fadd_rn(hop_left(s), e[0]);
#pragma unroll
            for (int j = 1; j < 16; ++j) s = __fadd_rn(s, e[j]);
        }
        sum_a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), nl - 1));
        sum_b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 32 + nl - 1));
    }
    stamp(7);
    for (int rr = 0; rr < 2 && !(kSkip & 2); ++rr) {
        const int rl = wave * 2 + rr;
        const float srr = rr == 0 ? sum_a : sum_b;
        if (rl >= rows) break;
        float *srow = S + rl * kSStride;
        for (int c = lane; c < seq; c += 64) srow[c] = __fdiv_rn(srow[c], srr);
        if (lane < seq32 - seq) srow[seq + lane] = 0.0f;  // P over the zero-padded k range (< 32 columns)
    }

    // ---- heads = P V, one V chunk at a time: waves 0 .. kRF*ceil(d_k/16)-1 own output tile (row
    // fragment w % kRF, column tile w / kRF) and carry its accumulator across the chunks (the k chain
    // stays in order)
    const int nct2 = (dk + 15) >> 4, nks32 = seq32 >> 2;
    const bool pv_wave = wave < kRF * nct2;
    const int rf = wave % kRF, ct = wave / kRF;
    const int col = ct * 16 + lr;
    const float *prow = S + (rf * 16 + lr) * kSStride + lk;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nchunks; ++c) {
        __syncthreads();  // P complete (c = 0) / the previous V chunk consumed
        if (c == 0) stamp(3);
        put(pf, kVStride);
        __syncthreads();
        if (c == 0) stamp(4);
        if (c + 1 < nchunks) fetch(pf, Vb, (c + 1) * kChunk);
        if (pv_wave && !(kSkip & 4)) {
            // k-steps over the reference's zero-padded extent (seq rounded up to 32: P and V are zero
            // past seq, so those steps are its padded tile's +0 adds), in groups of 8 -- a whole number
            // of groups per chunk, no per-step conditions; group g+1's operands are read from LDS while
            // group g's MFMAs run (the accumulation chain itself stays in k order)
            const int s_beg = c * (kChunk / 4), s_end = min(nks32, (c + 1) * (kChunk / 4));
            const float *vcol = KV + (lk - c * kChunk) * kVStride + col;
            auto read = [&](float (&pa)[8], float (&vb)[8], int s0) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    pa[u] = prow[4 * (s0 + u)];
                    vb[u] = vcol[4 * (s0 + u) * kVStride];
                }
            };
            auto mfma8 = [&](const float (&pa)[8], const float (&vb)[8]) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[u], vb[u], acc, 0, 0, 0);
            };
            float pa0[8], vb0[8], pa1[8], vb1[8];
            if (s_beg < s_end) read(pa0, vb0, s_beg);
            for (int s0 = s_beg; s0 < s_end; s0 += 16) {
                const bool two = s0 + 8 < s_end;
                if (two) read(pa1, vb1, s0 + 8);
                mfma8(pa0, vb0);
                if (s0 + 16 < s_end) read(pa0, vb0, s0 + 16);
                if (two) mfma8(pa1, vb1);
            }
        }
    }
    stamp(5);
    if (pv_wave && col < dk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rl = rf * 16 + 4 * lk + r;
            if (rl < rows) heads[(int64_t)(q0 + rl) * d + (int64_t)h * dk + col] = acc[r];
        }
    }
}

}  // namespace

hipError_t launch_attention_fused(const float *qkv, int seq, int d, int n_heads, float scale, float *heads,
                                  hipStream_t stream) {
    if (n_heads < 1 || d % n_heads) return hipErrorInvalidValue;
    const int dk = d / n_heads;
    if (seq < 1 || seq > kAttnMaxSeq || dk > kAttnMaxDk) return hipErrorNotSupported;
    constexpr int kTQ = 32;
    attention_fused_kernel<kTQ, 256, 1024><<<dim3((unsigned)((seq + kTQ - 1) / kTQ), (unsigned)n_heads), 1024, 0, stream>>>(
        qkv, d, dk, seq, scale, heads);
    return hipGetLastError();
}

}  // namespace qgemm
