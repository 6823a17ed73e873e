// gemm_sd.h -- LAB: direct-load small-tile GEMM (gemm_i8_sd<TB, KW, D>), measured against the product's
// LDS-DMA small kernels (gemm_lab ... small, profiles/r03_sd_small_tiles_lab.log) and not adopted: equal or
// slower at the encoder shapes, faster only at M = 64, K = 4096.  Included by gemm_variants.h.
#pragma once
#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

// gemm_i8_sd<TB, KW, D>: TB x TB tiles (TB = 32 or 64) for the few-tile GEMMs (the encoder's M = 512
// linears, decode-sized M) on the 256-tile kernel's operand path: every MFMA operand one 1-KiB
// buffer_load_dwordx4 from the fragment-major packed layout straight into VGPRs, a ring of D sub-steps of
// operands in flight per wave, no LDS and no barrier in the k-loop.  (gemm_i8_small stages the same blocks
// by LDS-DMA through a barriered ring, and deeper rings did not speed it up: these GEMMs are latency- and
// issue-bound, not MFMA-bound.)
//   KW = 1: 4 waves as 2 x 2, each a (TB/2) x (TB/2) wave tile over all of K.
//   KW = 4: every wave the whole TB x TB tile over a quarter of the 64-deep k-blocks; the four int32
//           partials are summed through LDS (integer adds: exact in any order), then dequantized.
// Epilogue: the fp32 tile (bias / relu fused) into a padded LDS image, stored as full rows.
template <int TB, int KW>
struct SdTile {
    static constexpr int kThreads = 256;
    static constexpr int WT = KW == 1 ? TB / 2 : TB;  // wave tile rows = cols
    static constexpr int MI = WT / 16;
    static constexpr int TS = TB + 4;                 // fp32 image row (conflict-free column writes)
    static constexpr int kPartBytes = KW > 1 ? 4 * TB * TB * 4 : 0;
    static constexpr int kImgBytes = TB * TS * 4;
    static constexpr int kMainBytes = kPartBytes > kImgBytes ? kPartBytes : kImgBytes;
    static constexpr int kLdsBytes = kMainBytes + 3 * TB * 4;  // + Cx, Cw, bias
    static_assert(KW == 1 || KW == 4, "k split over 1 or 4 waves");
    static_assert(MI >= 1 && TB % 16 == 0, "whole 16-row fragments");
};

template <int TB, int KW, int D, int kEpi = kEpiNone>
__global__ __launch_bounds__(256) void gemm_i8_sd(GemmArgs p) {
    using T_ = SdTile<TB, KW>;
    constexpr int MI = T_::MI, WT = T_::WT, TS = T_::TS;
    __shared__ __attribute__((aligned(16))) int8_t lds[T_::kLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = KW == 1 ? wave >> 1 : 0, wn = KW == 1 ? (wave & 1) : 0, wk = KW == 1 ? 0 : wave;
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    int tm, tn;
    group_tiles(wid, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    // this wave's k-blocks [u0, u0 + nloc)
    const int u0 = __builtin_amdgcn_readfirstlane(wk * nsub / KW);
    const int nloc = __builtin_amdgcn_readfirstlane((wk + 1) * nsub / KW - u0);
    // the wave's MI row groups of A (B), k-block u0 on: block (i, u) at ((i * nsub) + u - u0) KiB
    const int bytes = MI * nsub * 1024 - u0 * 1024;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + ((int64_t)((tm * TB + wm * WT) >> 4) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + ((int64_t)((tn * TB + wn * WT) >> 4) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
    const int voff = lane * 16;

    v4i acc[MI][MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) acc[mi][ni] = v4i{};
    v4i fa[D][MI], fb[D][MI];
    auto ld = [&](v4i (&a)[MI], v4i (&b)[MI], int u) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            a[i] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, (i * nsub + u) * 1024, 0);
            b[i] = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, (i * nsub + u) * 1024, 0);
        }
    };
    auto mfmas = [&](const v4i (&a)[MI], const v4i (&b)[MI]) __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    };
    if (nloc > 0) {
        // D sub-steps in flight; the loads of a full trip are unconditional (index clamped to the last
        // sub-step, as in gemm_i8_fm), so the ring's registers stay fixed
#pragma unroll
        for (int d = 0; d < D; ++d) ld(fa[d], fb[d], d < nloc ? d : nloc - 1);
        int u = 0;
        for (; u + D <= nloc; u += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                mfmas(fa[d], fb[d]);
                const int un = u + d + D;
                ld(fa[d], fb[d], un < nloc ? un : nloc - 1);
            }
        }
        const int rest = nloc - u;  // sets 0 .. rest-1 hold sub-steps u .. nloc-1
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if (d < rest) mfmas(fa[d], fb[d]);
    }

    const int gi0 = tm * TB, gj0 = tn * TB;
    float *sCx = reinterpret_cast<float *>(lds + T_::kMainBytes);
    float *sCw = sCx + TB;
    float *sB = sCw + TB;
    if (tid < TB) {
        sCx[tid] = p.Cx[gi0 + tid];
        if constexpr (has_bias(kEpi)) sB[tid] = gj0 + tid < p.n ? p.bias[gj0 + tid] : 0.0f;
    } else if (tid < 2 * TB) {
        sCw[tid - TB] = p.Cw[gj0 + tid - TB];
    }
    float *T = reinterpret_cast<float *>(lds);  // [TB][TS] fp32 image
    const int lrow = lane & 15, kq = lane >> 4;
    if constexpr (KW > 1) {
        // the four partials in accumulator order: slot ((w * MI + mi) * MI + ni) * 64 + lane
        constexpr int kSlots = MI * MI * 64, kPer = kSlots / 256;
        v4i *part = reinterpret_cast<v4i *>(lds);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni) part[((wave * MI + mi) * MI + ni) * 64 + lane] = acc[mi][ni];
        __syncthreads();
        v4i tot[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int sl = tid + 256 * j;
            tot[j] = part[sl] + part[kSlots + sl] + part[2 * kSlots + sl] + part[3 * kSlots + sl];
        }
        __syncthreads();  // every partial read: the image may overwrite them
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int sl = tid + 256 * j, mi = sl / (MI * 64), ni = (sl / 64) % MI, ln = sl & 63;
            const int jl = ni * 16 + (ln & 15);
            const float cw = sCw[jl];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int il = mi * 16 + 4 * (ln >> 4) + r;
                T[il * TS + jl] = epi_extra<kEpi>(dequantize(tot[j][r], outer_product(sCx[il], cw), p.inv_r2), sB, jl);
            }
        }
    } else {
        __syncthreads();  // scales visible
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) {
            const int jl = wn * WT + ni * 16 + lrow;
            const float cw = sCw[jl];
#pragma unroll
            for (int mi = 0; mi < MI; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int il = wm * WT + mi * 16 + 4 * kq + r;
                    T[il * TS + jl] =
                        epi_extra<kEpi>(dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), p.inv_r2), sB, jl);
                }
        }
    }
    __syncthreads();
    float *C = static_cast<float *>(p.C);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) && gj0 + TB <= p.n;
    constexpr int kLanesPerRow = TB / 4;
    const int c4 = (tid % kLanesPerRow) * 4;
#pragma unroll
    for (int rr = tid / kLanesPerRow; rr < TB; rr += 256 / kLanesPerRow) {
        const int i = gi0 + rr;
        if (i >= p.m) break;
        const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
        const int j = gj0 + c4;
        if (full) {
            *reinterpret_cast<float4 *>(C + (int64_t)i * p.csh + j) = v;
        } else {
            const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
        }
    }
}


}  // namespace gemm
}  // namespace qgemm
