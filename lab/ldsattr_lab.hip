// ldsattr_lab.hip -- LAB: which role of the FFN-up single pass (pack_single_pass32_kernel<204>, 2048 x 4096 X and
// 4096 x 16384 W) produces its LDS bank-conflict cycles?  Launches, 10 each, in this order (tell them apart by
// grid size in the rocprofv3 counter CSV):
//   full   : the product launch (512 W strips + 128 X row blocks of 16 rows)      grid 640 x 1024
//   wonly  : the W strips alone                                                   grid 512 x 1024
//   xonly  : the X row blocks alone (n = rows_pad, no strips)                     grid 128 x 1024
//   lab_strip32_kernel<mode> (W strips only, 504 / 496 / 488 / 480 blocks for modes 0..3)
//   build/ldsattr_lab
#include <cstdio>
#include <cstdlib>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace qgemm {
// lab copies of the W-strip role (csrc/pack.hip pack_w_strip32_body) -- kMode 0: as the library; 1: a block barrier
// between the DMA wait and the first read-back (no read while other waves' DMA still lands); 2: no read-back in the
// column-max phase; 3: no read-back in the quantize phase (2 and 3 give wrong bytes: attribution only)
template <int kMode>
__device__ __forceinline__ void lab_strip32_body(int strip, const float *__restrict__ w, int64_t wsh, int k,
                                                    float range, float *__restrict__ scale, int8_t *__restrict__ q,
                                                    int64_t k_pad, uint8_t *lds, float *red) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c8 = t & 7, rq = t >> 3;  // columns n0 + 4*c8 .. +3; rows 4*rq + e + 512*i
    const int64_t n0 = (int64_t)strip * kW32Cols;
    const float w_seed = t < kW32Cols ? w[n0 + t] : 0.0f;  // W[0, j], issued first (used after the reduction)
    const auto src = buf_rsrc(w + n0, (uint32_t)(((int64_t)(k - 1) * wsh + kW32Cols) * 4));
    const uint32_t vrow = (uint32_t)((4 * rq * wsh + 4 * c8) * 4);
    // LDS part first (rows 512*kW32RegI ..): lane-linear DMA slots
#pragma unroll
    for (int i = 0; i < kW32LdsI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                src, (lds_void *)(lds + ((i * 4 + e) * 16 + wv) * 1024), 16,
                (int)(vrow + (uint32_t)((e + 512 * (i + kW32RegI)) * wsh * 4)), 0, 0, 0);
    float4 v[kW32RegI][4];
#pragma unroll
    for (int i = 0; i < kW32RegI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(src, vrow + (uint32_t)((e + 512 * i) * wsh * 4), 0, 0);
            v[i][e] = make_float4(__int_as_float(x[0]), __int_as_float(x[1]), __int_as_float(x[2]), __int_as_float(x[3]));
        }
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
    for (int i = 0; i < kW32RegI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 512 * i;
            if (r >= 1 && r < k) {
                p0 = cand_max(p0, v[i][e].x);
                p1 = cand_max(p1, v[i][e].y);
                p2 = cand_max(p2, v[i][e].z);
                p3 = cand_max(p3, v[i][e].w);
            }
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA slots have landed
    if constexpr (kMode == 1) __syncthreads();          // every wave's DMA has landed before any read-back
    const float4 *ls = reinterpret_cast<const float4 *>(lds) + wv * 64 + lane;
#pragma unroll
    for (int i = 0; i < kW32LdsI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 512 * (i + kW32RegI);
            if (r < k && kMode != 2) {
                const float4 x = ls[(i * 4 + e) * 16 * 64];
                p0 = cand_max(p0, x.x);
                p1 = cand_max(p1, x.y);
                p2 = cand_max(p2, x.z);
                p3 = cand_max(p3, x.w);
            }
        }
    // over the 8 lanes of the wave with the same c8 (lane bits 3..5), then over the 16 waves
#pragma unroll
    for (int off = 8; off < 64; off <<= 1) {
        p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
        p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
        p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
        p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
    }
    if (lane < 8) {
        red[wv * 32 + 4 * lane + 0] = p0;
        red[wv * 32 + 4 * lane + 1] = p1;
        red[wv * 32 + 4 * lane + 2] = p2;
        red[wv * 32 + 4 * lane + 3] = p3;
    }
    __syncthreads();
    float *s_sh = red + 16 * 32;
    if (t < kW32Cols) {
        float pm = red[t];
#pragma unroll
        for (int ww = 1; ww < 16; ++ww) pm = fmaxf(pm, red[ww * 32 + t]);  // -inf or >= +0: exact
        const float cw = absmax_finish(w_seed, pm);                       // seed = W[0, j]
        s_sh[t] = inv_divide(range, cw);
        scale[n0 + t] = cw;
    }
    __syncthreads();
    const float s0 = s_sh[4 * c8 + 0], s1 = s_sh[4 * c8 + 1], s2 = s_sh[4 * c8 + 2], s3 = s_sh[4 * c8 + 3];
    // the strip's 32 packed rows = two whole 16-row groups: one contiguous region of the fragment-major q
    // (dword stores: the quad transpose to 16-B pieces spilled here, 128 VGPRs, and measured slower)
    const auto dst = buf_rsrc(q + n0 * k_pad, (uint32_t)(kW32Cols * k_pad));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r0 = 4 * rq + 512 * i;
        if (r0 >= k_pad) continue;
        float4 x4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x4[e] = i < kW32RegI ? v[i < kW32RegI ? i : 0][e] : (kMode == 3 ? v[0][e] : ls[((i - kW32RegI) * 4 + e) * 16 * 64]);
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            int qe[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = cc == 0 ? x4[e].x : cc == 1 ? x4[e].y : cc == 2 ? x4[e].z : x4[e].w;
                const float sc = cc == 0 ? s0 : cc == 1 ? s1 : cc == 2 ? s2 : s3;
                qe[e] = (r0 + e < k) ? quant_i8(x, sc) : 0;
            }
            __builtin_amdgcn_raw_buffer_store_b32((int)pack4(qe[0], qe[1], qe[2], qe[3]), dst,
                                                  (uint32_t)fofs(4 * c8 + cc, r0, k_pad), 0, 0);
        }
    }
}

template <int kMode>
__global__ __launch_bounds__(1024) void lab_strip32_kernel(const float *__restrict__ w, int64_t wsh, int k, float range,
                                                          float *__restrict__ scale, int8_t *__restrict__ q, int64_t k_pad) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_w[kW32LdsBytes];
    __shared__ float red[16 * 32 + 32];
    lab_strip32_body<kMode>(blockIdx.x, w, wsh, k, range, scale, q, k_pad, lds_w, red);
}
}  // namespace qgemm

int main() {
    const int m = 2048, n = 16384, k = 4096;
    float *X, *W; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 1, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 2, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    const int nstrips = n / kW32Cols, nx = (int)(vx.rows_pad / 16);
    for (int v = 0; v < 3; ++v)
        for (int i = 0; i < 10; ++i) {
            const int g = v == 0 ? nstrips + nx : v == 1 ? nstrips : nx;
            const int ns = v == 2 ? 0 : nstrips;
            const int nn = v == 2 ? (int)vw.rows_pad : n;  // X-only: no strips and no padding strips
            pack_single_pass32_kernel<204><<<g, 1024>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, nn,
                                                        vw.scale, vw.q, vw.rows_pad, ns, 127.f, nullptr, 0);
            CK(hipGetLastError());
        }
    for (int v = 0; v < 4; ++v)
        for (int i = 0; i < 10; ++i) {
            // grid sizes 512 - 8 v strips (tell the modes apart in the counter CSV)
            const dim3 g(nstrips - 8 * (v + 1));
            if (v == 0) lab_strip32_kernel<0><<<g, 1024>>>(W, n, k, 127.f, vw.scale, vw.q, vw.k_pad);
            if (v == 1) lab_strip32_kernel<1><<<g, 1024>>>(W, n, k, 127.f, vw.scale, vw.q, vw.k_pad);
            if (v == 2) lab_strip32_kernel<2><<<g, 1024>>>(W, n, k, 127.f, vw.scale, vw.q, vw.k_pad);
            if (v == 3) lab_strip32_kernel<3><<<g, 1024>>>(W, n, k, 127.f, vw.scale, vw.q, vw.k_pad);
            CK(hipGetLastError());
        }
    CK(hipDeviceSynchronize());
    printf("ok\n");
    return 0;
}
