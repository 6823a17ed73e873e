// gemm_fk.h -- LAB: gemm_i8_fk, split-K inside one workgroup (round 4), measured and NOT adopted.
// Against the library's gemm_i8_fm<split-K> (lab/t2_lab.hip, lab/c3d_lab.hip; profiles/r04_fk_lab.log,
// profiles/r04_c3d_order_lab.log), bit-identical:
//   GEMM alone, back to back (operands warm):  2048x4096x16384 103.8 vs 109.2 us, x8192 59.5 vs 66.2, x4096 36.9 vs 44.5
//   inside the FFN-down drop-in call (after the two pack passes):  133-135 vs 120-124 us
// Each CU fetches 48 instead of 32 KiB per 64-deep sub-step from L2 (its two K halves share no operands); with the
// operands arriving from beyond L2 after the packs, that costs more than the slab traffic it removes.
#pragma once

#include <type_traits>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

// ------------------------------------------------------------------------------------------------
// gemm_i8_fk: split-K INSIDE one workgroup (round 4), for the long-K shapes with 128 256-tiles (FFN down
// 2048 x 16384 -> 4096: one 256-tile per CU would leave half the chip idle).  A block owns a 256 x 128 region --
// twice the blocks of the 256-tile plan, one per CU -- and its 4 waves are 2 row halves (wm) x 2 K halves (kh),
// each running gemm_i8_fm's main loop (128 x 128 wave tile, AGPR accumulators, fragment-major operands straight
// to VGPRs, three register sets) over its half of K.  The two K halves of a row half meet in LDS: wave
// (wm, kh) hands the half of its rows it does NOT finish (64 x 128 int32 = 32 KiB) to its partner (wm, 1 - kh),
// one barrier, and each wave adds the partner's partial sums to its own half (exact integer addition: bit-
// identical to any split) as it runs the dequant epilogue on its 64 rows.  Against gemm_i8_fm<split-K> (two
// blocks per 256-tile, int32 slabs through memory, arrival tickets, the last slice re-reading the other slab):
// no slab traffic (100 MB per FFN-down launch), no tickets, no workspace, one store tail.  The waves of a row
// half share its A panel (L1); the two K halves do not share operands, so the CU fetches 48 instead of 32 KiB
// per 64-deep sub-step from L2.
// p.tiles_n counts 128-column regions.
template <int kEpi = kEpiNone>
__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fk(GemmArgs p) {
    static_assert(kEpi != kEpiOutlier, "the outlier epilogue runs on gemm_i8_fm");
    constexpr int TS = 132;                   // padded row of a wave's epilogue image (conflict-free ds_write)
    constexpr int kBlockBytes = 64 * TS * 4;  // a wave's [64][132] fp32 image
    constexpr int kXBytes = 32 * 64 * 16;     // a wave's hand-off: 4 x 8 accumulators x 64 lanes x 16 B
    constexpr int kImgBytes = 4 * kBlockBytes > 4 * kXBytes ? 4 * kBlockBytes : 4 * kXBytes;
    __shared__ __attribute__((aligned(16))) int8_t lds[kImgBytes + 1536];  // + Cx[256], Cw[128]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, kh = wave >> 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    const int u0 = __builtin_amdgcn_readfirstlane(kh * nsub / 2);
    const int nloc = __builtin_amdgcn_readfirstlane((kh + 1) * nsub / 2 - u0);
    const int half_bytes = 8 * nsub * 1024 - u0 * 1024;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + (((int64_t)tm * 16 + wm * 8) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + (((int64_t)tn * 8) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const int voff = lane * 16;

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};
    v4i a0[8], b0[8], a1[8], b1[8], a2[8], b2[8];
    auto ld = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int u) __attribute__((always_inline)) {
        const int soff = ((j & 7) * nsub + u) * 1024;
        if (j < 8) fb[j] = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, soff, 0);
        else fa[j - 8] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, soff, 0);
    };
    auto substep = [&](v4i (&ca)[8], v4i (&cb)[8], v4i (&na)[8], v4i (&nb)[8], int un, bool more)
                       __attribute__((always_inline)) {
        un = un < nloc ? un : nloc - 1;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) mfma_agpr(acc[mi][ni], ca[mi], cb[ni]);
            if (more) {
                ld(na, nb, 2 * mi, un);
                ld(na, nb, 2 * mi + 1, un);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
    };
#pragma unroll
    for (int j = 0; j < 16; ++j) ld(a0, b0, j, 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) ld(a1, b1, j, nloc > 1 ? 1 : 0);
    int u = 0;
    for (; u + 3 <= nloc; u += 3) {
        substep(a0, b0, a2, b2, u + 2, true);
        substep(a1, b1, a0, b0, u + 3, true);
        substep(a2, b2, a1, b1, u + 4, true);
    }
    const int rest = nloc - u;
    if (rest > 0) {
        substep(a0, b0, a2, b2, 0, false);
        if (rest > 1) substep(a1, b1, a2, b2, 0, false);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

    // hand-off of the half this wave does not finish (rows 64 (1 - kh) .. of its 128), in MFMA lane order
    const int gi0 = tm * BM, gj0 = tn * 128;
    float *sCx = reinterpret_cast<float *>(lds + kImgBytes);
    float *sCw = sCx + BM;
    sCx[tid] = p.Cx[gi0 + tid];  // scales are padded to the 256-row tiles
    if (tid < 128) sCw[tid] = p.Cw[gj0 + tid];
    // the accumulator halves are indexed at compile time (a runtime index would send acc to scratch):
    // one instantiation per K half
    auto finish = [&](auto khc) __attribute__((always_inline)) {
        constexpr int KH = decltype(khc)::value, GIVE = 1 - KH;
        {
            int8_t *mine = lds + wave * kXBytes;
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int ni = 0; ni < 8; ++ni)
                    *reinterpret_cast<v4i *>(mine + ((mq * 8 + ni) * 64 + lane) * 16) = acc[4 * GIVE + mq][ni];
        }
        __syncthreads();
        const int8_t *theirs = lds + (wave ^ 2) * kXBytes;  // partner (wm, 1 - kh) handed over rows half kh
        const int lrow = lane & 15, kq = lane >> 4;
        const int r0 = wm * 128 + 64 * KH;  // this wave's 64 output rows in the region
        float cwv[8], bv[8], cxv[4][4];
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            cwv[ni] = sCw[ni * 16 + lrow];
            const int j = gj0 + ni * 16 + lrow;
            bv[ni] = has_bias(kEpi) && j < p.n ? p.bias[j] : 0.0f;
        }
#pragma unroll
        for (int mq = 0; mq < 4; ++mq)
#pragma unroll
            for (int r = 0; r < 4; ++r) cxv[mq][r] = sCx[r0 + mq * 16 + 4 * kq + r];
        // the sums, 16 rows at a time: the partner's partials of those rows from LDS (8 x 16 B per lane), added to
        // this wave's accumulators and dequantized into registers; every hand-off read retires before the
        // barrier, after which the epilogue images overwrite the hand-off area
        float o[4][8][4];
#pragma unroll
        for (int mq = 0; mq < 4; ++mq) {
            v4i oth[8];
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                oth[ni] = *reinterpret_cast<const v4i *>(theirs + ((mq * 8 + ni) * 64 + lane) * 16);
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = dequantize(acc[4 * KH + mq][ni][r] + oth[ni][r], outer_product(cxv[mq][r], cwv[ni]),
                                         p.inv_r2);
                    if constexpr (has_bias(kEpi)) v = __fadd_rn(v, bv[ni]);
                    if constexpr (kEpi == kEpiBiasRelu) v = (v < 0.0f) ? 0.0f : v;
                    o[mq][ni][r] = v;
                }
        }
        __syncthreads();
        float *T = reinterpret_cast<float *>(lds + wave * kBlockBytes);
#pragma unroll
        for (int mq = 0; mq < 4; ++mq)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) T[(mq * 16 + 4 * kq + r) * TS + ni * 16 + lrow] = o[mq][ni][r];
        const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                          gj0 + 128 <= p.n && gi0 + r0 + 64 <= p.m;
        const int c4 = (lane & 31) * 4;
        float *C = static_cast<float *>(p.C);
        if (full) {
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * it + (lane >> 5);
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
                typedef float v4f __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w},
                                            reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + rr) * p.csh + gj0 + c4));
            }
        } else {
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * it + (lane >> 5);
                const int i = gi0 + r0 + rr;
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
                const int j = gj0 + c4;
                if (i >= p.m) continue;
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
            }
        }
    };
    // kh is wave-uniform: both branches meet the same two barriers
    if (kh == 0) finish(std::integral_constant<int, 0>{});
    else finish(std::integral_constant<int, 1>{});
}

}  // namespace gemm
}  // namespace qgemm
