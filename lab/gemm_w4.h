// gemm_w4.h -- LAB: the 256 x 256 int8 tile on 4 waves (one per SIMD) with 128 x 128 wave tiles.
//
// Why: the ping-pong kernel (gemm_i8_pp, 8 waves of 128 x 64) is power-bound -- its main loop holds
// 1.79 GHz against the 2.03 GHz of bare MFMA issue, and the LDS-DMA / LDS-read traffic is what the
// chip pays for (profiles/r02_mfma_peak.txt).  A 128 x 128 wave tile reads 16 fragments per 64-deep
// sub-step for 64 MFMAs (0.25 per MFMA) instead of 12 for 32 (0.375): a third fewer LDS read bytes
// per MAC.  Its 256 accumulators cannot share a SIMD with a partner wave, so each wave issues its
// own LDS reads and LDS-DMA between its MFMAs.
//
// Round 1's builtin version (lab gemm_variants.h v9) lost because hipcc kept the 256 accumulators in
// AGPRs but moved them around in the loop (56 v_accvgpr_read/write + 16 v_accvgpr_mov per k-step).
// Here every MFMA is an inline-asm statement with the accumulator as a tied "+a" operand, so each
// accumulator lives in ONE AGPR quad for the whole loop (audit: no v_accvgpr_* in the loop).
//
// Schedule (2-stage ring of 64 KiB stages, BK = 128, ONE barrier per k-step, in the middle):
//   k-step t, phase 1: 64 MFMAs on F0 (sub-step 0 of stage t, registers) + 16 ds_read of F1
//                      (sub-step 1 of stage t)
//            vmcnt(0) (stage t+1 landed: issued in phase 2 of k-step t-1), lgkmcnt(0) (F1 in
//            registers: every read of stage t's buffer is done), BARRIER
//            phase 2: 64 MFMAs on F1 + 16 ds_read of F0 <- stage t+1 (visible: every wave waited for
//                      its pieces before the barrier) + 16 LDS-DMA pieces of stage t+2 into stage
//                      t's buffer (every wave's last read of it retired before the barrier)
// Each wave stages rows [64w, 64w+64) of A and of B (8 + 8 pieces of 8 rows x 128 B).  LDS image and
// source swizzle as gemm_i8_pp (128-B rows, chunk g of row r in slot g ^ ((r>>1)&7)).
#pragma once

#include "gemm_legacy.h"

namespace qgemm {
namespace gemm {

enum W4Flags { kW4NoDma = 1, kW4NoRead = 2, kW4NoStore = 4, kW4Stamp = 8, kW4PadT = 16, kW4RowMajor = 32, kW4NoA = 64,
               kW4NoB = 128, kW4K1 = 256, kW4K4 = 512, kW4Sync = 1024,
               kW4Nt = 2048, kW4NoPrio = 4096, kW4Direct = 8192, kW4Rot = 16384, kW4GScale = 32768 };

#ifdef QGEMM_LAB
__device__ unsigned long long g_w4_stamp[4096 * 6];
#endif

// mfma_agpr (one MFMA, accumulator pinned to its AGPR quad) and uniform_ptr come from gemm_i8_kernels.h

constexpr int kW4Threads = 256;

constexpr int kW4TStride = 260;  // padded fp32 row of the epilogue image (conflict-free ds_write_b32)

template <int kFlags = kW4PadT>
__global__ __launch_bounds__(kW4Threads, 1) void gemm_i8_w4(GemmArgs p) {
    constexpr int TS = (kFlags & kW4PadT) ? kW4TStride : BN;
    constexpr int kImgBytes = 128 * TS * 4;
    constexpr int kRing = kLdsBytes > kImgBytes ? kLdsBytes : kImgBytes;
    __shared__ __attribute__((aligned(16))) int8_t lds[kRing + 2048];
#ifdef QGEMM_LAB
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kFlags & kW4Stamp)
            if (threadIdx.x == 0) {
                g_w4_stamp[blockIdx.x * 6 + 2 * i] = __builtin_amdgcn_s_memtime();
                g_w4_stamp[blockIdx.x * 6 + 2 * i + 1] = __builtin_amdgcn_s_memrealtime();
            }
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int nk = (int)(p.k_pad / BK);
    const int64_t kp = p.k_pad;
    const int8_t *Ablk = p.A + (int64_t)tm * BM * kp;
    const int8_t *Bblk = p.B + (int64_t)tn * BN * kp;
    // piece q (8 rows x 128 B): lane l writes LDS bytes 16l.. of rows 8q.. = row 8q + (l>>3), slot l&7,
    // holding global chunk (l&7) ^ (4(q&1) + (l>>4))
    uint32_t voff[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) voff[e] = (uint32_t)((lane >> 3) * kp) + ((((lane & 7) ^ (4 * e + (lane >> 4)))) << 4);
    auto piece = [&](int i, int kt, int buf) __attribute__((always_inline)) {
        // i < 8: A piece 8w + i; i >= 8: B piece 8w + i - 8
        const int q = 8 * wave + (i & 7);
        const int8_t *blk = i < 8 ? Ablk : Bblk;
        int8_t *dst = lds + buf * kStageBytes + (i < 8 ? 0 : kTileBytes) + q * 8 * BK;
        __builtin_amdgcn_global_load_lds((const void *)(blk + (int64_t)q * 8 * kp + (int64_t)kt * BK + voff[i & 1]),
                                         (void *)dst, 16, 0, 0);
    };

    const int lrow = lane & 15, kq = lane >> 4, swz = (lrow >> 1) & 7;
    const int a_row0 = (wm * 128 + lrow) * BK, b_row0 = (wn * 128 + lrow) * BK;
    const int off0 = (kq ^ swz) << 4, off1 = ((4 + kq) ^ swz) << 4;

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};
    v4i fa0[8], fb0[8], fa1[8], fb1[8];

    // fragment j of a set: j < 8 -> B fragment j, else A fragment j - 8 (B first: row 0 needs all of B)
    auto rd = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int buf, int off) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * kStageBytes;
        if (j < 8) fb[j] = *reinterpret_cast<const v4i *>(la + kTileBytes + b_row0 + j * 16 * BK + off);
        else fa[j - 8] = *reinterpret_cast<const v4i *>(la + a_row0 + (j - 8) * 16 * BK + off);
    };
    auto barrier = []() __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: stage 0 landed and visible, stage 1 in flight, F0 of stage 0 in registers
#pragma unroll
    for (int i = 0; i < 16; ++i) piece(i, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    if (nk > 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) piece(i, 1, 1);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) rd(fa0, fb0, j, 0, off0);

    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        // ---- phase 1: MFMAs on F0, reads of F1 (stage t) -- 2 reads after every row of 8 MFMAs
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) mfma_agpr(acc[mi][ni], fa0[mi], fb0[ni]);
            if (!(kFlags & kW4NoRead) || t == 0) {
                rd(fa1, fb1, 2 * mi, cur, off1);
                rd(fa1, fb1, 2 * mi + 1, cur, off1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
        // ---- phase 2: MFMAs on F1, reads of F0 <- stage t+1, LDS-DMA of stage t+2 into buffer cur
        const bool rd_next = t + 1 < nk && (!(kFlags & kW4NoRead) || t == 0);
        const bool dma = t + 2 < nk && (!(kFlags & kW4NoDma) || t == 0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) mfma_agpr(acc[mi][ni], fa1[mi], fb1[ni]);
            if (rd_next) {
                rd(fa0, fb0, 2 * mi, cur ^ 1, off0);
                rd(fa0, fb0, 2 * mi + 1, cur ^ 1, off0);
            }
            if (dma) {
                piece(2 * mi, t + 2, cur);
                piece(2 * mi + 1, t + 2, cur);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
    }
    stamp(1);
    // the last MFMAs' results are read by VALU below: the asm hides them from hipcc's hazard padding
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

    // ---- epilogue: dequantize into a [128][TS] fp32 LDS image one 128-row half at a time; every wave
    // instruction then stores one whole 1-KiB row (16 B per lane)
    const int gi0 = tm * BM, gj0 = tn * BN;
    float *sCx = reinterpret_cast<float *>(lds + kRing);
    float *sCw = sCx + BM;
    __syncthreads();
    sCx[tid] = p.Cx[gi0 + tid];
    sCw[tid] = p.Cw[gj0 + tid];
    float *T = reinterpret_cast<float *>(lds);
    float *C = static_cast<float *>(p.C);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n;
    if constexpr (kFlags & kW4NoStore) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
        if (x == 0x7fffffff && p.m < 0) C[tid] = (float)x;
        stamp(2);
        return;
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        __syncthreads();
        if (wm == half) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const int jl = wn * 128 + ni * 16 + lrow;
                const float cw = sCw[jl];
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int il = mi * 16 + 4 * kq + r;
                        T[il * TS + jl] = dequantize(acc[mi][ni][r], outer_product(sCx[half * 128 + il], cw), p.inv_r2);
                    }
            }
        }
        __syncthreads();
        const int c4 = lane * 4;
#pragma unroll 4
        for (int rr = wave; rr < 128; rr += 4) {
            const int i = gi0 + half * 128 + rr;
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
    stamp(2);
}


// ------------------------------------------------------------------------------------------------
// gemm_i8_w4s: the same 4-wave / 128 x 128 wave tile on a SUB-STEP ring, so the LDS-DMA gets two sub-steps
// of flight instead of one: a stage is one 64-deep sub-step (A 256 x 64 B + B 256 x 64 B = 32 KiB), the
// ring holds 4 of them (128 KiB).
//   sub-step u: 64 MFMAs on F(u) (registers) + 16 ds_read of F(u+1) from stage u+1 (landed and visible:
//               waited for before the previous barrier) + 8 LDS-DMA pieces of stage u+3 into the slot of
//               stage u-1 (read during sub-step u-2, retired before that sub-step's barrier)
//               -> vmcnt(8) (stage u+2 landed, stage u+3 in flight), lgkmcnt(0), BARRIER
// LDS rows are 64 B: row r's 16-B chunk c sits in slot c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}, which makes
// ds_read_b128's lane groups ({0-3,12-15,20-27}, ... MI355X_MICROARCH.md LDS table) hit 16 distinct
// (r & 3, slot) bank quads.  LDS-DMA: one piece = 16 rows x 64 B by buffer_load_dwordx4 ... lds (SGPR
// descriptor + soffset, one per-lane voffset); lane l holds row l >> 2, slot l & 3 = global chunk
// (l & 3) ^ g(l >> 4).
// Epilogue: per wave, two steps of 64 rows of its quadrant dequantized into its OWN padded [64][132]
// LDS block and stored from there as 512-B row segments -- no cross-wave hand-off, all 4 SIMDs busy.

template <int kFlags = 0>
__global__ __launch_bounds__(kW4Threads, 1) void gemm_i8_w4s(GemmArgs p) {
    constexpr int kSub = 64;                        // k per ring stage
    constexpr int kHalfTile = BM * kSub;            // 16 KiB: one operand of a stage
    constexpr int kStage = 2 * kHalfTile;           // 32 KiB
    constexpr int kDepth = 4;
    constexpr int kRing = kDepth * kStage;          // 128 KiB
    constexpr int TS = 132;                         // padded fp32 row of a wave's epilogue block
    constexpr int kBlockBytes = 64 * TS * 4;        // 33 792 B per wave
    constexpr int kImg = 4 * kBlockBytes;
    constexpr int kLds = (kRing > kImg ? kRing : kImg);
    __shared__ __attribute__((aligned(16))) int8_t lds[kLds + 2048];
#ifdef QGEMM_LAB
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kFlags & kW4Stamp)
            if (threadIdx.x == 0) {
                g_w4_stamp[blockIdx.x * 6 + 2 * i] = __builtin_amdgcn_s_memtime();
                g_w4_stamp[blockIdx.x * 6 + 2 * i + 1] = __builtin_amdgcn_s_memrealtime();
            }
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / kSub);
    const int kp = (int)p.k_pad;
    // descriptors over this tile's A and B panels (256 packed rows each)
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t *>(uniform_ptr(p.A + (int64_t)tm * BM * kp)), 0,
                                                       __builtin_amdgcn_readfirstlane(BM * kp), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t *>(uniform_ptr(p.B + (int64_t)tn * BN * kp)), 0,
                                                       __builtin_amdgcn_readfirstlane(BN * kp), 0x00020000);
    // per-lane voffset of a piece: row l>>2 of its 16, chunk (l&3) ^ g(l>>4)
    const int gl = (lane >> 4) == 0 ? 0 : (lane >> 4) == 1 ? 2 : (lane >> 4) == 2 ? 3 : 1;
    const int voff = (lane >> 2) * kp + (((lane & 3) ^ gl) << 4);
    typedef __attribute__((address_space(3))) void lds_void;
    auto piece = [&](int i, int u, int buf) __attribute__((always_inline)) {
        // i < 4: A piece 4w + i (rows 16(4w+i) ..); else B piece 4w + i - 4
        const int q = 4 * wave + (i & 3);
        int8_t *dst = lds + buf * kStage + (i < 4 ? 0 : kHalfTile) + q * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? rsA : rsB, (lds_void *)dst, 16, voff, q * 16 * kp + u * kSub,
                                                 0, 0);
    };
    const int lrow = lane & 15, kq = lane >> 4;
    const int gr = (lrow >> 2) == 0 ? 0 : (lrow >> 2) == 1 ? 2 : (lrow >> 2) == 2 ? 3 : 1;
    const int foff = (kq ^ gr) << 4;
    const int a_row0 = (wm * 128 + lrow) * kSub + foff, b_row0 = kHalfTile + (wn * 128 + lrow) * kSub + foff;

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};
    v4i fa0[8], fb0[8], fa1[8], fb1[8];
    auto rd = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int buf) __attribute__((always_inline)) {
        const int8_t *st = lds + buf * kStage;
        if (j < 8) fb[j] = *reinterpret_cast<const v4i *>(st + b_row0 + j * 16 * kSub);
        else fa[j - 8] = *reinterpret_cast<const v4i *>(st + a_row0 + (j - 8) * 16 * kSub);
    };
    auto barrier = []() __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // one sub-step: MFMAs on (ca, cb), reads into (na, nb) from slot (u+1)%4, DMA of stage u+3
    auto substep = [&](v4i (&ca)[8], v4i (&cb)[8], v4i (&na)[8], v4i (&nbf)[8], int u, bool rd_next, bool dma)
                       __attribute__((always_inline)) {
        const int nb = (u + 1) & 3, db = (u + 3) & 3;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) mfma_agpr(acc[mi][ni], ca[mi], cb[ni]);
            if (rd_next) {
                rd(na, nbf, 2 * mi, nb);
                rd(na, nbf, 2 * mi + 1, nb);
            }
            if (dma && mi < 4) {
                piece(2 * mi, u + 3, db);
                piece(2 * mi + 1, u + 3, db);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // prologue: stages 0, 1, 2 issued; 0 and 1 landed and visible; F(0) in set 0
#pragma unroll
    for (int s = 0; s < 3; ++s)
        if (s < nsub)
#pragma unroll
            for (int i = 0; i < 8; ++i) piece(i, s, s);
    // stages 0 and 1 landed (sub-step 0 reads stage 1), stage 2 may stay in flight
    if (nsub >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
#pragma unroll
    for (int j = 0; j < 16; ++j) rd(fa0, fb0, j, 0);
    // steady state in pairs of sub-steps (register set parity is static), then the tail
    int u = 0;
    for (; u + 4 <= nsub; u += 2) {
        // sub-steps u, u+1: both read ahead and stage u+3 / u+4 (< nsub since u + 4 <= nsub ... u+4 may == nsub)
        substep(fa0, fb0, fa1, fb1, u, true, !(kFlags & kW4NoDma) || u == 0);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
        const bool d1 = u + 4 < nsub && (!(kFlags & kW4NoDma));
        substep(fa1, fb1, fa0, fb0, u + 1, true, d1);
        if (d1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
    }
    // tail: 1..3 sub-steps left (u even), nothing more to stage; straight-line code (a runtime tail loop
    // switching register sets made hipcc spill the accumulators around it)
    const int rest = nsub - u;
    auto drain = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
    };
    substep(fa0, fb0, fa1, fb1, u, rest > 1, false);
    drain();
    if (rest > 1) {
        substep(fa1, fb1, fa0, fb0, u + 1, rest > 2, false);
        drain();
        if (rest > 2) {
            substep(fa0, fb0, fa1, fb1, u + 2, false, false);
            drain();
        }
    }
    stamp(1);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

    const int gi0 = tm * BM, gj0 = tn * BN;
    float *sCx = reinterpret_cast<float *>(lds + kLds);
    float *sCw = sCx + BM;
    float *C = static_cast<float *>(p.C);
    if constexpr (kFlags & kW4NoStore) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
        if (x == 0x7fffffff && p.m < 0) C[tid] = (float)x;
        stamp(2);
        return;
    }
    // (the loop's last barrier: every wave is done with the ring)
    sCx[tid] = p.Cx[gi0 + tid];
    sCw[tid] = p.Cw[gj0 + tid];
    __syncthreads();
    float *T = reinterpret_cast<float *>(lds + wave * kBlockBytes);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n;
    const int r0 = wm * 128, c0 = wn * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int jl = ni * 16 + lrow;
            const float cw = sCw[c0 + jl];
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int il = mq * 16 + 4 * kq + r;  // row within the 64-row step
                    T[il * TS + jl] = dequantize(acc[4 * s + mq][ni][r], outer_product(sCx[r0 + 64 * s + il], cw), p.inv_r2);
                }
        }
        // the wave's own block: its ds_writes precede its ds_reads (one wave's LDS ops stay in order)
        const int c4 = (lane & 31) * 4;
#pragma unroll 4
        for (int it = 0; it < 32; ++it) {
            const int rr = 2 * it + (lane >> 5);
            const int i = gi0 + r0 + 64 * s + rr;
            const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
            const int j = gj0 + c0 + c4;
            if (i >= p.m) continue;
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
    stamp(2);
}


// ------------------------------------------------------------------------------------------------
// FRAGMENT-MAJOR operand layout + an LDS-free main loop (gemm_i8_f4).
// F-layout of a packed operand (rows_pad x k_pad int8): 1-KiB blocks, block (rg, kg) = rows 16rg.. x
// k 64kg.. at byte ((rg * (k_pad / 64)) + kg) * 1024, lanes in MFMA order inside: lane l = 16 kc + r holds
// row 16rg + r, k 64kg + 16kc .. +15.  One v_mfma_i32_16x16x64_i8 operand = ONE contiguous 1-KiB
// buffer_load_dwordx4 (8 whole 128-B lines), straight into the fragment registers.
__global__ void relayout_f_kernel(const int8_t *__restrict__ src, int8_t *__restrict__ dst, int64_t rows_pad,
                                  int64_t k_pad) {
    const int64_t nkg = k_pad / 64;
    const int64_t blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blk >= (rows_pad / 16) * nkg) return;
    const int l = threadIdx.x & 63;
    const int64_t rg = blk / nkg, kg = blk % nkg;
    const int r = l & 15, kc = l >> 4;
    const v4i v = *reinterpret_cast<const v4i *>(src + (rg * 16 + r) * k_pad + kg * 64 + kc * 16);
    *reinterpret_cast<v4i *>(dst + blk * 1024 + l * 16) = v;
}

// 4 waves, 128 x 128 wave tiles, accumulators pinned in AGPRs, operands streamed from the F-layout
// straight into VGPRs (3 register sets: sub-step u computes while u+1 and u+2 are in flight), no LDS and
// no barrier in the main loop; the two waves that share an A (B) half read the same blocks (L1).
template <int kFlags = 0>
__global__ __launch_bounds__(kW4Threads, 1) void gemm_i8_f4(GemmArgs p) {
    constexpr int TS = 132;
    constexpr int kBlockBytes = 64 * TS * 4;
    __shared__ __attribute__((aligned(16))) int8_t lds[4 * kBlockBytes + 2048];
#ifdef QGEMM_LAB
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kFlags & kW4Stamp)
            if (threadIdx.x == 0) {
                g_w4_stamp[blockIdx.x * 6 + 2 * i] = __builtin_amdgcn_s_memtime();
                g_w4_stamp[blockIdx.x * 6 + 2 * i + 1] = __builtin_amdgcn_s_memrealtime();
            }
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    // this wave's half panels: 8 row groups x nsub blocks each (= 128 packed rows x k_pad bytes)
    const int half_bytes = 8 * nsub * 1024;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + ((int64_t)tm * 16 + wm * 8) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + ((int64_t)tn * 16 + wn * 8) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    // F-layout: lane l's 16 B at l*16 of each 1-KiB block; row-major (kW4RowMajor, lab): row l&15 of the
    // block's 16, bytes 16(l>>4).. of its 64
    constexpr bool kRM = (kFlags & kW4RowMajor) != 0;
    const int voff = kRM ? (lane & 15) * (int)p.k_pad + (lane >> 4) * 16 : lane * 16;

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};
    v4i a0[8], b0[8], a1[8], b1[8], a2[8], b2[8];
    // fragment loads of sub-step u: j < 8 -> B block j, else A block j - 8
    auto ld = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int u, bool pro = false) __attribute__((always_inline)) {
        const int soff = kRM ? ((j & 7) * 16 * nsub * 64 + u * 64) : (((j & 7) * nsub + u) * 1024);
        if (j < 8) {
            if (!(kFlags & kW4NoB) || pro) fb[j] = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, soff, 0);
        } else if (!(kFlags & kW4NoA) || pro) {
            fa[j - 8] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, soff, 0);
        }
    };
    // MFMAs on (ca, cb); loads of sub-step un into (na, nb) when `more`.  In the main loop the loads are
    // unconditional (the sub-step index clamped to the last one): a conditional register load makes hipcc
    // keep both values alive across the loop and spill a register set.
    auto substep = [&](v4i (&ca)[8], v4i (&cb)[8], v4i (&na)[8], v4i (&nb)[8], int un, bool more)
                       __attribute__((always_inline)) {
        un = un < nsub ? un : nsub - 1;
        if constexpr (kFlags & kW4K1) un = 0;   // ablation: every load re-reads sub-step 0 (L1 / L2 hits)
        if constexpr (kFlags & kW4K4) un &= 3;  // ablation: 4 sub-steps cycled (L2 hits)
        if constexpr (!(kFlags & kW4NoPrio)) __builtin_amdgcn_s_setprio(1);
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
        if constexpr (!(kFlags & kW4NoPrio)) __builtin_amdgcn_s_setprio(0);
    };
#pragma unroll
    for (int j = 0; j < 16; ++j) ld(a0, b0, j, 0, true);
#pragma unroll
    for (int j = 0; j < 16; ++j) ld(a1, b1, j, nsub > 1 ? 1 : 0, true);
    if constexpr (kFlags & (kW4NoA | kW4NoB)) {
#pragma unroll
        for (int j = 0; j < 16; ++j) ld(a2, b2, j, nsub > 2 ? 2 : 0, true);
    }
    int u = 0;
    for (; u + 3 <= nsub; u += 3) {
        constexpr bool kLd = !(kFlags & kW4NoRead);  // ablation: MFMAs on stale registers, no loads
        if constexpr (kFlags & kW4Sync) __builtin_amdgcn_s_barrier();  // keep the 4 waves within a step (L1 reuse)
        substep(a0, b0, a2, b2, u + 2, kLd);                  // u + 2 < nsub
        substep(a1, b1, a0, b0, u + 3, kLd);                  // clamped past the end
        substep(a2, b2, a1, b1, u + 4, kLd);
    }
    const int rest = nsub - u;  // 0, 1 or 2; sets 0 and (1) hold sub-steps u, u+1
    if (rest > 0) {
        substep(a0, b0, a2, b2, 0, false);
        if (rest > 1) substep(a1, b1, a2, b2, 0, false);
    }
    stamp(1);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

    const int gi0 = tm * BM, gj0 = tn * BN;
    float *sCx = reinterpret_cast<float *>(lds + 4 * kBlockBytes);
    float *sCw = sCx + BM;
    float *C = static_cast<float *>(p.C);
    if constexpr (kFlags & kW4NoStore) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
        if (x == 0x7fffffff && p.m < 0) C[tid] = (float)x;
        stamp(2);
        return;
    }
    // kW4GScale: each wave reads the scales it needs straight from global memory (no LDS copy, no barrier: a
    // wave whose k-loop ends first starts its epilogue at once)
    constexpr bool kGS = (kFlags & kW4GScale) != 0;
    if constexpr (!kGS) {
        sCx[tid] = p.Cx[gi0 + tid];
        sCw[tid] = p.Cw[gj0 + tid];
        __syncthreads();
    }
    float *T = reinterpret_cast<float *>(lds + wave * kBlockBytes);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n;
    const bool rows_full = gi0 + BM <= p.m;
    const int lrow = lane & 15, kq = lane >> 4;
    const int r0 = wm * 128, c0 = wn * 128;
    // the scales into registers first: T and the scales share the one LDS array, so a scale read between
    // T stores would be re-issued (and waited for) after every store
    float cwv[8], cxg[2][4][4];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) cwv[ni] = kGS ? p.Cw[gj0 + c0 + ni * 16 + lrow] : sCw[c0 + ni * 16 + lrow];
    if constexpr (kGS) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int r = 0; r < 4; ++r) cxg[h][mq][r] = p.Cx[gi0 + r0 + 64 * h + mq * 16 + 4 * kq + r];
    }
    if constexpr (kFlags & kW4Direct) {
        // ablation: dequantized straight from the accumulators, dword nontemporal stores (4 rows x 64 B per
        // wave instruction), no LDS image (full tiles only)
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            float cx4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) cx4[r] = sCx[r0 + mi * 16 + 4 * kq + r];
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    __builtin_nontemporal_store(
                        dequantize(acc[mi][ni][r], outer_product(cx4[r], cwv[ni]), p.inv_r2),
                        C + (int64_t)(gi0 + r0 + mi * 16 + 4 * kq + r) * p.csh + gj0 + c0 + ni * 16 + lrow);
        }
        stamp(2);
        return;
    }
    // kW4Rot: each tile starts its row-pair loop at its own offset (spreading the rows written at one time
    // over the chip; profiles/r03_f4_store_order_lab.log)
    const int rot = (kFlags & kW4Rot) ? ((tn * 7 + tm * 3) & 31) : 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        float cxv[4][4];
#pragma unroll
        for (int mq = 0; mq < 4; ++mq)
#pragma unroll
            for (int r = 0; r < 4; ++r) cxv[mq][r] = kGS ? cxg[s][mq][r] : sCx[r0 + 64 * s + mq * 16 + 4 * kq + r];
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int jl = ni * 16 + lrow;
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int il = mq * 16 + 4 * kq + r;
                    T[il * TS + jl] = dequantize(acc[4 * s + mq][ni][r], outer_product(cxv[mq][r], cwv[ni]), p.inv_r2);
                }
        }
        const int c4 = (lane & 31) * 4;
        if (full && rows_full) {
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * ((it + rot) & 31) + (lane >> 5);
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
                float4 *dst = reinterpret_cast<float4 *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + c0 + c4);
                if constexpr (kFlags & kW4Nt) {
                    typedef float v4f __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f *>(dst));
                } else {
                    *dst = v;
                }
            }
        } else {
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * it + (lane >> 5);
                const int i = gi0 + r0 + 64 * s + rr;
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
                const int j = gj0 + c0 + c4;
                if (i >= p.m) continue;
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
            }
        }
    }
    stamp(2);
}

}  // namespace gemm
}  // namespace qgemm
