// gemm_f32.hip -- the reference's UNQUANTIZED path, op_mm<float,float> (op_mm.cuh:49-65 ->
// op_matmul_kernel<float,float> :9-46), used by the harnesses for the error metric and the
// "unquantized GEMM" timing line (timing_quantize.cu:27-35).
//
// Bit-exact with the reference: every output is res = +0 then res = fmaf(a_k, b_k, res) for k
// ascending (nvcc contracts :38), followed by the zero-padded products of the last 32-wide tile,
// which only turn a -0 result into +0 (one fl(res + 0)).  Arbitrary strides (the Index() macro).
// 64x64 tile per 256-thread block, 4x4 outputs per thread, k staged 16 at a time through LDS.
#include "qgemm_internal.h"

namespace qgemm {

namespace {

constexpr int TM = 64, TN = 64, TK = 16;

__global__ __launch_bounds__(256) void mm_f32_kernel(const float *__restrict__ A, int64_t ash, int64_t asw,
                                                     const float *__restrict__ B, int64_t bsh, int64_t bsw,
                                                     float *__restrict__ C, int64_t csh, int64_t csw, int m, int n,
                                                     int k, int64_t a_bs, int64_t b_bs, int64_t c_bs) {
    // batch z (attention heads): operands offset by the batch strides
    A += blockIdx.z * a_bs;
    B += blockIdx.z * b_bs;
    C += blockIdx.z * c_bs;
    __shared__ float As[TK][TM + 1];
    __shared__ float Bs[TK][TN + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t i0 = (int64_t)blockIdx.y * TM, j0 = (int64_t)blockIdx.x * TN;
    float acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0f;
    for (int k0 = 0; k0 < k; k0 += TK) {
        for (int e = threadIdx.x; e < TK * TM; e += 256) {
            const int kk = e / TM, r = e % TM;  // A tile, stored [k][row]
            const int64_t gi = i0 + r, gk = k0 + kk;
            As[kk][r] = (gi < m && gk < k) ? A[gi * ash + gk * asw] : 0.0f;
            const int kb = e / TN, c = e % TN;  // B tile, stored [k][col]
            const int64_t gj = j0 + c, gkb = k0 + kb;
            Bs[kb][c] = (gj < n && gkb < k) ? B[gkb * bsh + gj * bsw] : 0.0f;
        }
        __syncthreads();
        const int kmax = min(TK, k - k0);
        for (int kk = 0; kk < kmax; ++kk) {
            float av[4], bv[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) av[a] = As[kk][ty * 4 + a];
#pragma unroll
            for (int b = 0; b < 4; ++b) bv[b] = Bs[kk][tx * 4 + b];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = __fmaf_rn(av[a], bv[b], acc[a][b]);
        }
        __syncthreads();
    }
    const bool padded = (k % 32) != 0;  // reference: trailing fma(0, 0, res) products of the last tile
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int64_t gi = i0 + ty * 4 + a, gj = j0 + tx * 4 + b;
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
    const dim3 grid((unsigned)((n + TN - 1) / TN), (unsigned)((m + TM - 1) / TM), (unsigned)batch);
    mm_f32_kernel<<<grid, 256, 0, stream>>>(A, ash, asw, B, bsh, bsw, C, csh, csw, m, n, k, a_bs, b_bs, c_bs);
    return hipGetLastError();
}

}  // namespace qgemm
