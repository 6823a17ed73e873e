// pack.hip -- absmax + quantize kernels (the reference's op_absmax / op_inv_divide / op_multiply
// steps, op_mm.cuh:75-89), fused into two HBM-streaming passes that emit MFMA-ready int8 operands.
//
// A "packed operand" (include/qgemm.h) is [scale: rows_pad f32][q: rows_pad x k_pad int8], where each
// packed row is one reduction vector: a row of X (scale Cx) or a column of W (scale Cw, stored
// transposed so k is contiguous for the MFMA B fragment).  Padding (rows >= rows, k >= len) is zero.
//
//   pack_rows : the reduction vector is contiguous-ish in memory (X row-major, or W column-major).
//               One wave per vector: absmax over the vector (wave shuffle reduction), then quantize.
//               Replaces op_reduction_kernel_colwise (op_reduction.cuh:71-92: one thread per row,
//               lanes 16 KiB apart) + op_elemwise_unary_kernel(InvDivideConstFunc) +
//               op_elemwise_binary_w_bcast_kernel(MultiplyWithTypecastFunc) -- 3 launches, 2 reads.
//   pack_cols : the reduction vector is strided (W row-major: a column).  Pass 1 reduces coalesced
//               1024-column strips of 64 rows and merges strips with an order-free integer atomicMax;
//               pass 2 re-reads W (from the Infinity Cache at the sizes that matter), quantizes and
//               transposes 128x64 tiles through LDS.
//               Replaces op_reduction_kernel_rowwise (op_reduction.cuh:96-117) + 2 elementwise launches.
#include "qgemm_internal.h"

namespace qgemm {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_max(float p) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p = fmaxf(p, __shfl_xor(p, off, kWave));
    return p;
}

__device__ __forceinline__ float cand_max(float p, float x) {
    float a = absmax_candidate(x);
    return (a > p) ? a : p;  // NaN never wins: comparison is false
}

__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
    return (uint32_t)(a & 0xff) | ((uint32_t)(b & 0xff) << 8) | ((uint32_t)(c & 0xff) << 16) |
           ((uint32_t)(d & 0xff) << 24);
}

// ------------------------------------------------------------------------------------------------
// pack_rows, vector path: rows of `len` floats at src + r*sh, unit inner stride, 16-B aligned rows.
// R > 0: each lane keeps R float4 chunks in registers (len <= 256*R), one HBM read.
// R == 0: two streaming passes (second pass mostly L2 hits).
template <int R>
__global__ __launch_bounds__(256) void pack_rows_vec_kernel(const float *__restrict__ src, int64_t sh, int rows,
                                                            int len, float range, float *__restrict__ scale,
                                                            int8_t *__restrict__ q, int64_t rows_pad,
                                                            int64_t k_pad) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows_pad) return;
    uint32_t *qrow = reinterpret_cast<uint32_t *>(q + row * k_pad);
    const int64_t nq = k_pad >> 2;  // uint32 words per packed row
    if (row >= rows) {              // padding row
        for (int64_t c = lane; c < nq; c += kWave) qrow[c] = 0u;
        if (lane == 0) scale[row] = 0.0f;
        return;
    }
    const float *srow = src + row * sh;
    const float4 *s4 = reinterpret_cast<const float4 *>(srow);
    const int nfull = len >> 2;  // complete float4 chunks
    const float seed = srow[0];

    float p = -INFINITY;
    float4 v[R > 0 ? R : 1];
    if constexpr (R > 0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int c = lane + j * kWave;
            v[j] = (c < nfull) ? s4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int c = lane + j * kWave;
            if (c < nfull) {
                p = (c == 0) ? p : cand_max(p, v[j].x);  // element 0 is the seed
                p = cand_max(p, v[j].y);
                p = cand_max(p, v[j].z);
                p = cand_max(p, v[j].w);
            }
        }
    } else {
        for (int c = lane; c < nfull; c += kWave) {
            float4 x = s4[c];
            p = (c == 0) ? p : cand_max(p, x.x);
            p = cand_max(p, x.y);
            p = cand_max(p, x.z);
            p = cand_max(p, x.w);
        }
    }
    const int tail0 = nfull << 2;  // scalar tail elements [tail0, len)
    if (tail0 + lane < len && tail0 + lane > 0) p = cand_max(p, srow[tail0 + lane]);
    p = wave_max(p);
    const float cx = absmax_finish(seed, p);
    const float s = inv_divide(range, cx);

    if constexpr (R > 0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int c = lane + j * kWave;
            if (c < nfull)
                qrow[c] = pack4(quant_i8(v[j].x, s), quant_i8(v[j].y, s), quant_i8(v[j].z, s), quant_i8(v[j].w, s));
        }
    } else {
        for (int c = lane; c < nfull; c += kWave) {
            float4 x = s4[c];
            qrow[c] = pack4(quant_i8(x.x, s), quant_i8(x.y, s), quant_i8(x.z, s), quant_i8(x.w, s));
        }
    }
    // partial tail word, then zero padding words
    const int64_t first_zero = nfull + ((len & 3) ? 1 : 0);
    if ((len & 3) && lane == 0) {
        int b[4] = {0, 0, 0, 0};
        for (int e = 0; e < (len & 3); ++e) b[e] = quant_i8(srow[tail0 + e], s);
        qrow[nfull] = pack4(b[0], b[1], b[2], b[3]);
    }
    for (int64_t c = first_zero + lane; c < nq; c += kWave) qrow[c] = 0u;
    if (lane == 0) scale[row] = cx;
}

// pack_rows, generic strides (any sh, sw): scalar loads, two passes.
__global__ __launch_bounds__(256) void pack_rows_generic_kernel(const float *__restrict__ src, int64_t sh,
                                                                int64_t sw, int rows, int len, float range,
                                                                float *__restrict__ scale, int8_t *__restrict__ q,
                                                                int64_t rows_pad, int64_t k_pad) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows_pad) return;
    int8_t *qrow = q + row * k_pad;
    if (row >= rows) {
        for (int64_t c = lane; c < k_pad; c += kWave) qrow[c] = 0;
        if (lane == 0) scale[row] = 0.0f;
        return;
    }
    const float *srow = src + row * sh;
    const float seed = srow[0];
    float p = -INFINITY;
    for (int64_t c = 1 + lane; c < len; c += kWave) p = cand_max(p, srow[c * sw]);
    p = wave_max(p);
    const float cx = absmax_finish(seed, p);
    const float s = inv_divide(range, cx);
    for (int64_t c = lane; c < k_pad; c += kWave) qrow[c] = (c < len) ? (int8_t)quant_i8(srow[c * sw], s) : 0;
    if (lane == 0) scale[row] = cx;
}

// ------------------------------------------------------------------------------------------------
// pack_cols pass 1: per-column max of |x| over rows 1..len-1 of a [len x cols] row-major matrix
// (row stride sh, unit column stride).  The seed row 0 is combined in pass 2.  Candidates are
// non-negative and NaN-free, so float order == uint order of (bits + 1); 0 encodes "no candidate".
constexpr int kColStrip = 1024;  // columns per block (256 threads x float4)
constexpr int kColRows = 64;     // rows per block

template <bool VEC>
__global__ __launch_bounds__(256) void colmax_kernel(const float *__restrict__ src, int64_t sh, int len, int cols,
                                                     uint32_t *__restrict__ colmax) {
    const int64_t r0 = 1 + (int64_t)blockIdx.y * kColRows;
    const int64_t r1 = min((int64_t)len, r0 + kColRows);
    if constexpr (VEC) {
        const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
        if (c >= cols) return;
        float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
        const float *base = src + c;
#pragma unroll 8
        for (int64_t r = r0; r < r1; ++r) {
            float4 x = *reinterpret_cast<const float4 *>(base + r * sh);
            p0 = cand_max(p0, x.x);
            p1 = cand_max(p1, x.y);
            p2 = cand_max(p2, x.z);
            p3 = cand_max(p3, x.w);
        }
        if (p0 >= 0.f) atomicMax(colmax + c + 0, __float_as_uint(p0) + 1u);
        if (p1 >= 0.f) atomicMax(colmax + c + 1, __float_as_uint(p1) + 1u);
        if (p2 >= 0.f) atomicMax(colmax + c + 2, __float_as_uint(p2) + 1u);
        if (p3 >= 0.f) atomicMax(colmax + c + 3, __float_as_uint(p3) + 1u);
    } else {
        for (int64_t c = (int64_t)blockIdx.x * kColStrip + threadIdx.x; c < min((int64_t)cols, (int64_t)(blockIdx.x + 1) * kColStrip);
             c += 256) {
            float p = -INFINITY;
            for (int64_t r = r0; r < r1; ++r) p = cand_max(p, src[r * sh + c]);
            if (p >= 0.f) atomicMax(colmax + c, __float_as_uint(p) + 1u);
        }
    }
}

// pack_cols pass 2: finish the column scale, quantize, transpose a [128 k][64 col] tile through LDS
// and write 64 packed rows x 128 bytes.  Grid: (rows_pad/64, k_pad/128).
constexpr int kTc = 64;             // output rows (= input columns) per block
constexpr int kTk = 128;            // k per block
constexpr int kTStride = kTk + 16;  // LDS row stride (bytes), keeps 16-B alignment

template <bool VEC>
__global__ __launch_bounds__(256) void pack_cols_kernel(const float *__restrict__ src, int64_t sh, int len, int cols,
                                                        float range, const uint32_t *__restrict__ colmax,
                                                        float *__restrict__ scale, int8_t *__restrict__ q,
                                                        int64_t k_pad) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[kTc * kTStride];
    __shared__ float s_sh[kTc];
    const int t = threadIdx.x;
    const int64_t n0 = (int64_t)blockIdx.x * kTc;
    const int64_t k0 = (int64_t)blockIdx.y * kTk;
    if (t < kTc) {
        const int64_t j = n0 + t;
        float cx = 0.0f, s = 0.0f;
        if (j < cols) {
            const uint32_t e = colmax[j];
            const float p = e ? __uint_as_float(e - 1u) : -INFINITY;
            cx = absmax_finish(src[j], p);  // seed = row 0 (op_reduction.cuh:105)
            s = inv_divide(range, cx);
        }
        s_sh[t] = s;
        if (blockIdx.y == 0) scale[j] = cx;
    }
    __syncthreads();
    const int col4 = t & 15;  // 4 input columns n0 + 4*col4 .. +3
    const int rg = t >> 4;    // rows k0 + 4*rg + 64*h + {0..3}
    const float s0 = s_sh[4 * col4 + 0], s1 = s_sh[4 * col4 + 1], s2 = s_sh[4 * col4 + 2], s3 = s_sh[4 * col4 + 3];
    const int64_t c = n0 + 4 * col4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        int qv[4][4];  // [row i][col e]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t kk = k0 + 4 * rg + 64 * h + i;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (kk < len) {
                const float *rp = src + kk * sh + c;
                if constexpr (VEC) {
                    if (c < cols) x = *reinterpret_cast<const float4 *>(rp);
                } else {
                    if (c + 0 < cols) x.x = rp[0];
                    if (c + 1 < cols) x.y = rp[1];
                    if (c + 2 < cols) x.z = rp[2];
                    if (c + 3 < cols) x.w = rp[3];
                }
            }
            // padding columns have s = 0 -> 0*x = 0 (x finite or zero-filled); force 0 anyway
            qv[i][0] = (kk < len && c + 0 < cols) ? quant_i8(x.x, s0) : 0;
            qv[i][1] = (kk < len && c + 1 < cols) ? quant_i8(x.y, s1) : 0;
            qv[i][2] = (kk < len && c + 2 < cols) ? quant_i8(x.z, s2) : 0;
            qv[i][3] = (kk < len && c + 3 < cols) ? quant_i8(x.w, s3) : 0;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
            *reinterpret_cast<uint32_t *>(tile + (4 * col4 + e) * kTStride + 4 * rg + 64 * h) =
                pack4(qv[0][e], qv[1][e], qv[2][e], qv[3][e]);
    }
    __syncthreads();
    const int n = t >> 2;          // packed row within the tile
    const int kc = (t & 3) * 32;   // byte offset within the 128-byte k slice
    const uint4 *lp = reinterpret_cast<const uint4 *>(tile + n * kTStride + kc);
    uint4 *gp = reinterpret_cast<uint4 *>(q + (n0 + n) * k_pad + k0 + kc);
    gp[0] = lp[0];
    gp[1] = lp[1];
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fill_uniform_kernel(float *__restrict__ dst, int64_t count, uint64_t seed,
                                                           float lo, float hi) {
    const uint64_t key = mix64(seed + 0x9E3779B97F4A7C15ULL);
    const float span = __fsub_rn(hi, lo);
    const float shift = __fdiv_rn(lo, span);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t z = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        const float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
        dst[i] = __fmul_rn(__fadd_rn(u, shift), span);
    }
}

}  // namespace

hipError_t launch_pack_rows(const float *src, int64_t sh, int64_t sw, int rows, int len, float range, PackedView out,
                            hipStream_t stream) {
    const dim3 grid((unsigned)(out.rows_pad / 4)), block(256);
    const bool vec = sw == 1 && (sh % 4 == 0 || rows == 1) && (reinterpret_cast<uintptr_t>(src) % 16 == 0);
    if (!vec) {
        pack_rows_generic_kernel<<<grid, block, 0, stream>>>(src, sh, sw, rows, len, range, out.scale, out.q,
                                                             out.rows_pad, out.k_pad);
        return hipGetLastError();
    }
    const int per_lane = ((len >> 2) + 63) / 64;  // float4 chunks per lane
#define QG_ROWS(Rv) pack_rows_vec_kernel<Rv><<<grid, block, 0, stream>>>(src, sh, rows, len, range, out.scale, out.q, out.rows_pad, out.k_pad)
    if (per_lane <= 1) QG_ROWS(1);
    else if (per_lane <= 2) QG_ROWS(2);
    else if (per_lane <= 4) QG_ROWS(4);
    else if (per_lane <= 8) QG_ROWS(8);
    else if (per_lane <= 16) QG_ROWS(16);
    else QG_ROWS(0);
#undef QG_ROWS
    return hipGetLastError();
}

hipError_t launch_pack_cols(const float *src, int64_t sh, int len, int cols, float range, PackedView out,
                            hipStream_t stream) {
    uint32_t *colmax = out.scratch;
    hipError_t e = hipMemsetAsync(colmax, 0, sizeof(uint32_t) * (size_t)cols, stream);
    if (e != hipSuccess) return e;
    const bool vec = (cols % 4 == 0) && (sh % 4 == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0);
    if (len > 1) {
        const dim3 g1((unsigned)((cols + kColStrip - 1) / kColStrip), (unsigned)((len - 1 + kColRows - 1) / kColRows));
        if (vec) colmax_kernel<true><<<g1, 256, 0, stream>>>(src, sh, len, cols, colmax);
        else colmax_kernel<false><<<g1, 256, 0, stream>>>(src, sh, len, cols, colmax);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const dim3 g2((unsigned)(out.rows_pad / kTc), (unsigned)(out.k_pad / kTk));
    if (vec) pack_cols_kernel<true><<<g2, 256, 0, stream>>>(src, sh, len, cols, range, colmax, out.scale, out.q, out.k_pad);
    else pack_cols_kernel<false><<<g2, 256, 0, stream>>>(src, sh, len, cols, range, colmax, out.scale, out.q, out.k_pad);
    return hipGetLastError();
}

hipError_t launch_fill_uniform(float *dst, int64_t count, uint64_t seed, float lo, float hi, hipStream_t stream) {
    if (count <= 0) return hipSuccess;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    fill_uniform_kernel<<<(unsigned)blocks, 256, 0, stream>>>(dst, count, seed, lo, hi);
    return hipGetLastError();
}

}  // namespace qgemm
