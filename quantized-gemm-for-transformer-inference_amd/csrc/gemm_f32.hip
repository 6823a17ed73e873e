// gemm_f32.hip -- the reference's UNQUANTIZED path, op_mm<float,float> (op_mm.cuh:49-65 ->
// op_matmul_kernel<float,float> :9-46), used by the harnesses for the error metric and the
// "unquantized GEMM" timing line (timing_quantize.cu:27-35).
//
// Bit-exact with the reference: every output is res = +0 then res = fmaf(a_k, b_k, res) for k
// ascending (nvcc contracts :38), followed by the zero-padded products of the last 32-wide tile,
// which only turn a -0 result into +0 (one fl(res + 0)).  Arbitrary strides (the Index() macro).
// 128x128 or 64x64 tile per 256-thread block, k staged 16 or 64 at a time through LDS (64: a whole
// tile's loads in flight per round trip -- the attention PV GEMM is latency-bound at 128 blocks).
#include "qgemm_internal.h"

namespace qgemm {

namespace {


// Tile TM x TN per 256-thread block, (TM/16) x (TN/16) outputs per thread (rows ty*RM.., cols tx*RN..).
// Operand tiles are staged through LDS as [k][row] / [k][col]; the global->LDS mapping follows the
// operand's contiguous dimension, so row-major, transposed and head-sliced views all load coalesced.
template <int TM, int TN, int TK>
__global__ __launch_bounds__(256) void mm_f32_kernel(const float *__restrict__ A, int64_t ash, int64_t asw,
                                                     const float *__restrict__ B, int64_t bsh, int64_t bsw,
                                                     float *__restrict__ C, int64_t csh, int64_t csw, int m, int n,
                                                     int k, int64_t a_bs, int64_t b_bs, int64_t c_bs) {
    constexpr int RM = TM / 16, RN = TN / 16;  // 16 x 16 threads
    static_assert(RM >= 1 && RN >= 4 && RN % 4 == 0, "B fragment read as float4");
    // batch z (attention heads): operands offset by the batch strides
    A += blockIdx.z * a_bs;
    B += blockIdx.z * b_bs;
    C += blockIdx.z * c_bs;
    __shared__ __attribute__((aligned(16))) float As[TK][TM + 4];
    __shared__ __attribute__((aligned(16))) float Bs[TK][TN + 4];
    const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
    const int64_t i0 = (int64_t)blockIdx.y * TM, j0 = (int64_t)blockIdx.x * TN;
    const bool a_kc = asw == 1;  // A's k is contiguous (row-major A)
    const bool b_nc = bsw == 1;  // B's n is contiguous (row-major B); else k contiguous (B^T view)
    float acc[RM][RN];
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b) acc[a][b] = 0.0f;
    constexpr int NA = TK * TM / 256, NB = TK * TN / 256;  // staged elements per thread
    float ra[NA], rb[NB];
    auto fetch = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < NA; ++x) {
            const int e = x * 256 + t;
            const int kk = a_kc ? (e % TK) : (e / TM), r = a_kc ? (e / TK) : (e % TM);
            const int64_t gi = i0 + r, gk = k0 + kk;
            ra[x] = (gi < m && gk < k) ? A[gi * ash + gk * asw] : 0.0f;
        }
#pragma unroll
        for (int x = 0; x < NB; ++x) {
            const int e = x * 256 + t;
            const int kb = b_nc ? (e / TN) : (e % TK), c = b_nc ? (e % TN) : (e / TK);
            const int64_t gj = j0 + c, gkb = k0 + kb;
            rb[x] = (gj < n && gkb < k) ? B[gkb * bsh + gj * bsw] : 0.0f;
        }
    };
    auto deposit = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < NA; ++x) {
            const int e = x * 256 + t;
            As[a_kc ? (e % TK) : (e / TM)][a_kc ? (e / TK) : (e % TM)] = ra[x];
        }
#pragma unroll
        for (int x = 0; x < NB; ++x) {
            const int e = x * 256 + t;
            Bs[b_nc ? (e / TN) : (e % TK)][b_nc ? (e % TN) : (e / TK)] = rb[x];
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < k; k0 += TK) {
        deposit();
        __syncthreads();
        if (k0 + TK < k) fetch(k0 + TK);  // next tile's loads in flight during this tile's FMAs
        const int kmax = min(TK, k - k0);
        for (int kk = 0; kk < kmax; ++kk) {
            float av[RM], bv[RN];
#pragma unroll
            for (int a = 0; a < RM; ++a) av[a] = As[kk][ty * RM + a];
#pragma unroll
            for (int b = 0; b < RN; b += 4) *reinterpret_cast<float4 *>(bv + b) = *reinterpret_cast<const float4 *>(&Bs[kk][tx * RN + b]);
#pragma unroll
            for (int a = 0; a < RM; ++a)
#pragma unroll
                for (int b = 0; b < RN; ++b) acc[a][b] = __fmaf_rn(av[a], bv[b], acc[a][b]);
        }
        __syncthreads();
    }
    const bool padded = (k % 32) != 0;  // reference: trailing fma(0, 0, res) products of the last tile
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b) {
            const int64_t gi = i0 + ty * RM + a, gj = j0 + tx * RN + b;
            if (gi < m && gj < n) C[gi * csh + gj * csw] = padded ? __fadd_rn(acc[a][b], 0.0f) : acc[a][b];
        }
}

}  // namespace

hipError_t launch_mm_f32(const float *A, int64_t ash, int64_t asw, const float *B, int64_t bsh, int64_t bsw, float *C,
                         int64_t csh, int64_t csw, int m, int n, int k, hipStream_t stream) {
    return launch_mm_f32_batched(A, ash, asw, 0, B, bsh, bsw, 0, C, csh, csw, 0, m, n, k, 1, stream);
}

hipError_t launch_mm_f32_batched(const float *A, int64_t ash, int64_t asw, int64_t a_bs, const float *B, int64_t bsh,
                                 int64_t bsw, int64_t b_bs, float *C, int64_t csh, int64_t csw, int64_t c_bs, int m,
                                 int n, int k, int batch, hipStream_t stream) {
    // 128 x 128 tiles only for >= 1024 such blocks, else 64 x 64 (more waves per SIMD to hide the load
    // latency: attention QK^T 29 -> 19 us); k is never split: every output is one sequential fmaf
    // chain (a 32 x 64 tile measured slower on the attention PV GEMM)
    const int64_t big = (int64_t)((n + 127) / 128) * ((m + 127) / 128) * batch;
    if (big >= 1024) {
        const dim3 grid((unsigned)((n + 127) / 128), (unsigned)((m + 127) / 128), (unsigned)batch);
        mm_f32_kernel<128, 128, 16><<<grid, 256, 0, stream>>>(A, ash, asw, B, bsh, bsw, C, csh, csw, m, n, k, a_bs, b_bs,
                                                          c_bs);
    } else {
        const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((m + 63) / 64), (unsigned)batch);
        if (k >= 256)  // long chains: a whole 64-deep k tile per load round trip (attention PV)
            mm_f32_kernel<64, 64, 64><<<grid, 256, 0, stream>>>(A, ash, asw, B, bsh, bsw, C, csh, csw, m, n, k, a_bs,
                                                                b_bs, c_bs);
        else           // short k (attention QK^T, k = d_k): 16-deep tiles, next one prefetched
            mm_f32_kernel<64, 64, 16><<<grid, 256, 0, stream>>>(A, ash, asw, B, bsh, bsw, C, csh, csw, m, n, k, a_bs,
                                                                b_bs, c_bs);
    }
    return hipGetLastError();
}

}  // namespace qgemm
