// gemm_ds.h -- LAB: gemm_i8_fm with the MFMA operands swapped so the accumulators come out TRANSPOSED, and an
// epilogue that stores straight from registers (no LDS image).
//
// Why (round 5): the store tail of gemm_i8_fm (block end - loop end, 6.1-10.2 us, mean 8.3, profiles/r05_spread.log)
// does not depend on when a block's loop ends (eta^2 0.025 by loop-end quartile): early finishers, which store
// while most of the chip still computes, take as long as late ones.  So the tail is the epilogue's own work, not
// HBM: per wave 256 accumulators x (v_accvgpr_read + cvt + 4 f32 VALU) = 1 536 VALU instructions (~6 k cycles),
// 128 ds_write2_b32 + 64 ds_read_b128 (512 KiB of LDS traffic per CU), then 64 1-KiB stores.
// v_mfma_i32_16x16x64_i8 D = Aop * Bop with lane (kq = lane >> 4, c = lane & 15) holding D[4 kq + r][c], r = 0..3.
// With Aop = the W fragment and Bop = the X fragment, D = C^T: the lane holds C[row 16 mi + c][cols 16 ni + 4 kq
// .. + 3] -- four CONSECUTIVE columns of one row, one 16-B store, no transpose.  The dequantize runs on packed
// f32 pairs (v_pk_mul_f32 / v_pk_add_f32: the same IEEE roundings as the scalar ops, two lanes of work each).
// Cost: a store instruction writes 16 rows x 64 B instead of 2 rows x 512 B.
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

enum DsFlags {
    kDsNt = 1,       // nontemporal output stores
    kDsPacked = 2,   // packed f32 dequantize (else the scalar helpers)
    kDsRowMajorOrder = 4,  // store loop: mi outer (16 rows x 512 B per 8 stores); else ni outer
    kDsStamp = 8,    // s_memrealtime at start / loop end / stores drained, per block (g_ds_stamp)
    kDsNoStore = 16, // the epilogue's arithmetic without its stores (one word per lane kept alive)
    kDsPair = 32,    // tiles ni, ni+1 exchanged between lanes c and c^8 (DPP row_ror:8): 8 rows x 128 B per store
};
__device__ unsigned long long g_ds_stamp[4096][4];

__device__ __forceinline__ void mfma_agpr_swapped(v4i &acc, const v4i &a, const v4i &b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

template <int kFlags = kDsNt | kDsPacked | kDsRowMajorOrder>
__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_ds(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) float sS[2 * BM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    int tm, tn;
    group_tiles(wid, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    const int nloc = nsub;
    const int half_bytes = 8 * nsub * 1024;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + ((int64_t)tm * 16 + wm * 8) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + ((int64_t)tn * 16 + wn * 8) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const int voff = lane * 16;
    const int gi0 = tm * BM, gj0 = tn * BN;
    if constexpr ((kFlags & kDsStamp) != 0)
        if (tid == 0) g_ds_stamp[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
    // the scales: loaded first (their latency hides under the operand prologue), staged in LDS
    const float sx = p.Cx[gi0 + tid], sw = p.Cw[gj0 + tid];

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
            for (int ni = 0; ni < 8; ++ni) mfma_agpr_swapped(acc[mi][ni], ca[mi], cb[ni]);
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
    sS[tid] = sx;
    sS[BM + tid] = sw;
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
    if constexpr ((kFlags & kDsStamp) != 0)
        if (tid == 0) g_ds_stamp[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // the scale image
    const int c = lane & 15, kq = lane >> 4;
    const int r0 = wm * 128, c0 = wn * 128;
    // lane's rows 16 mi + c, columns 16 ni + 4 kq .. + 3 of the wave tile
    float cx[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) cx[mi] = sS[r0 + 16 * mi + c];
    float4 cw[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) cw[ni] = *reinterpret_cast<const float4 *>(sS + BM + c0 + 16 * ni + 4 * kq);
    float *C = static_cast<float *>(p.C);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n && gi0 + BM <= p.m;
    typedef float v2f __attribute__((ext_vector_type(2)));
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v2f inv2 = {p.inv_r2, p.inv_r2};
    const v2f zero2 = {0.0f, 0.0f};
    auto tile_out = [&](int mi, int ni) __attribute__((always_inline)) -> v4f {
        const v4i a = acc[mi][ni];
        if constexpr (kFlags & kDsPacked) {
            const v2f x = {cx[mi], cx[mi]};
            const v2f w01 = {cw[ni].x, cw[ni].y}, w23 = {cw[ni].z, cw[ni].w};
            const v2f o01 = x * w01 + zero2, o23 = x * w23 + zero2;  // fl(cx * cw) + 0 (no contraction: -ffp-contract=off)
            const v2f f01 = {(float)a[0], (float)a[1]}, f23 = {(float)a[2], (float)a[3]};
            const v2f d01 = (f01 * o01) * inv2, d23 = (f23 * o23) * inv2;
            return v4f{d01.x, d01.y, d23.x, d23.y};
        } else {
            return v4f{dequantize(a[0], outer_product(cx[mi], cw[ni].x), p.inv_r2),
                       dequantize(a[1], outer_product(cx[mi], cw[ni].y), p.inv_r2),
                       dequantize(a[2], outer_product(cx[mi], cw[ni].z), p.inv_r2),
                       dequantize(a[3], outer_product(cx[mi], cw[ni].w), p.inv_r2)};
        }
    };
    // full tiles: one 16-B store per (mi, ni); the row base moves by 16 rows per mi
    auto put_full = [&](int mi, int ni) __attribute__((always_inline)) {
        const v4f o = tile_out(mi, ni);
        v4f *dst = reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + 16 * mi + c) * p.csh + gj0 + c0 + 16 * ni + 4 * kq);
        if constexpr (kFlags & kDsNt) __builtin_nontemporal_store(o, dst);
        else *dst = o;
    };
    if constexpr ((kFlags & kDsNoStore) != 0) {
        v4f s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const v4f o = tile_out(mi, ni);
                asm volatile("" : "+v"(s4) : "v"(o));  // keeps every output live, costs nothing
            }
        if (s4.x == 1.2345f) C[tid] = s4.y;
    } else if ((kFlags & kDsPair) != 0 && full) {
        const bool lo = c < 8;
#pragma unroll
        for (int it = 0; it < 32; ++it) {
                // kDsRowMajorOrder: mi outer (a 16-row group's 512 B per 4 pair stores); else np outer (one 128-B column
                // band down the quadrant's 128 rows, then the next)
                const int mi = (kFlags & kDsRowMajorOrder) ? it >> 2 : it & 7;
                const int np = (kFlags & kDsRowMajorOrder) ? it & 3 : it >> 3;
                const v4f o0 = tile_out(mi, 2 * np), o1 = tile_out(mi, 2 * np + 1);
                v4f x1, x2;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // lane c reads lane c ^ 8 of its 16-lane row (row_ror:8)
                    const float r0v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(o0[e]), 0x128, 0xf, 0xf, false));
                    const float r1v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(o1[e]), 0x128, 0xf, 0xf, false));
                    x1[e] = lo ? o0[e] : r1v;   // rows 0..7 of the group: tile 2np (c < 8), tile 2np+1 (c >= 8)
                    x2[e] = lo ? r0v : o1[e];   // rows 8..15
                }
                const int jc = gj0 + c0 + 32 * np + (lo ? 0 : 16) + 4 * kq;
                const int64_t ra = gi0 + r0 + 16 * mi + (c & 7);
                v4f *d1 = reinterpret_cast<v4f *>(C + ra * p.csh + jc);
                v4f *d2 = reinterpret_cast<v4f *>(C + (ra + 8) * p.csh + jc);
                if constexpr (kFlags & kDsNt) {
                    __builtin_nontemporal_store(x1, d1);
                    __builtin_nontemporal_store(x2, d2);
                } else {
                    *d1 = x1;
                    *d2 = x2;
                }
            }
    } else if (full) {
        if constexpr (kFlags & kDsRowMajorOrder) {
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                for (int ni = 0; ni < 8; ++ni) put_full(mi, ni);
        } else {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                for (int mi = 0; mi < 8; ++mi) put_full(mi, ni);
        }
    } else {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const v4f o = tile_out(mi, ni);
                const int64_t i = gi0 + r0 + 16 * mi + c;
                const int j = gj0 + c0 + 16 * ni + 4 * kq;
                if (i < p.m)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < p.n) C[i * p.csh + (int64_t)(j + e) * p.csw] = o[e];
            }
    }
    if constexpr ((kFlags & kDsStamp) != 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) g_ds_stamp[blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace gemm
}  // namespace qgemm
