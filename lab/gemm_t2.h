// gemm_t2.h -- LAB: the 256 x 256 tile on TWO teams of 4 waves (two waves per SIMD), direct operand loads.
//
// Why: gemm_i8_fm (4 waves, 128 x 128 wave tiles, 512 registers per lane) leaves its
// 64-MiB fp32 store tail exposed -- ~9-10 us of 56.6 -- because one wave per SIMD has nothing to run while
// it drains its stores (gfx950 counts a wave's loads and stores on one vmcnt).  Here waves w and w + 4
// share a SIMD: team 0 (waves 0-3) computes rows 0-127 of the tile, team 1 (waves 4-7) rows 128-255; each
// wave a 128 x 64 wave tile (8 x 4 accumulators = 128 AGPRs, 256 registers per lane).  If one team runs
// ahead of the other (a start-up sleep of team 1, or MFMA priority for team 0), the leading team's
// epilogue -- dequantize, LDS transpose, stores -- runs while its partner keeps the matrix pipe busy, and
// only the lagging team's half of the tile is stored after the last MFMA.
// Cost: 12 fragment loads per 32 MFMAs (0.375 per MFMA) against 16 per 64 (0.25) -- 1.5x the load
// instructions per CU; the unique bytes per CU (L1 -> L2) are unchanged (the teams share B, a team's
// waves share A).  The extra issue of one wave may hide under the other wave's MFMAs.
//
// Operands: fragment-major packed layout (qgemm_internal.h fofs), one MFMA operand = one 1-KiB
// buffer_load_dwordx4 straight into VGPRs.  Two register sets (3 do not fit in 256 registers): sub-step u
// computes on set u & 1 while set u + 1 lands; each A fragment is reloaded (for u + 2) right after the row
// of MFMAs that used it, the B fragments after the sub-step's last row.
// Epilogue: each wave on its own [64][64] fp32 LDS image (16 KiB; 8 waves = 128 KiB), rows read back as
// 16-B pieces (4 rows x 256 B per store instruction); scales straight from global memory (no block
// barrier: the teams never wait for each other).
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

enum T2Flags {
    kT2Stamp = 1,     // in-kernel stamps (lab)
    kT2NoStore = 2,   // ablation: no epilogue stores
    kT2Sleep = 4,     // team 1 sleeps g_t2_param[0] x 512 cycles before its k-loop
    kT2Prio = 8,      // team 0 at MFMA priority 2 for its first g_t2_param[1] sub-steps (team 1 at 1)
    kT2Nt = 16,       // nontemporal output stores (as the product)
    kT2NoLoad = 32,   // ablation: MFMAs on stale registers (prologue loads only)
    kT2NoPrio = 64,   // no s_setprio at all
    kT2Late = 128,    // reload A fragment mi after row mi + 2 (WAR distance 8 MFMAs) instead of mi + 1
};

#ifdef QGEMM_LAB
__device__ unsigned long long g_t2_stamp[4096 * 12];
__device__ int g_t2_param[4];
#endif

constexpr int kT2Threads = 512;

template <int kFlags = kT2Nt>
__global__ __launch_bounds__(kT2Threads, 1) void gemm_i8_t2(GemmArgs p) {
    constexpr int TS = 64;             // unpadded: ds_write_b32 2-way (free), ds_read_b128 conflict-free
    constexpr int kImg = 64 * TS * 4;  // 16 KiB per wave
    __shared__ __attribute__((aligned(16))) int8_t lds[8 * kImg];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int team = wave >> 2, wq = wave & 3;
#ifdef QGEMM_LAB
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kFlags & kT2Stamp)
            if (lane == 0 && wq == 0) {
                g_t2_stamp[blockIdx.x * 12 + team * 6 + 2 * i] = __builtin_amdgcn_s_memtime();
                g_t2_stamp[blockIdx.x * 12 + team * 6 + 2 * i + 1] = __builtin_amdgcn_s_memrealtime();
            }
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    // A: the team's 128 rows (8 row groups); B: the wave's 64 columns (4 row groups of the packed W^T)
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + ((int64_t)tm * 16 + team * 8) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(8 * nsub * 1024), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + ((int64_t)tn * 16 + wq * 4) * nsub * 1024)), 0,
        __builtin_amdgcn_readfirstlane(4 * nsub * 1024), 0x00020000);
    const int voff = lane * 16;

    v4i acc[8][4];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
    v4i a0[8], b0[4], a1[8], b1[4];
    auto ldA = [&](v4i &d, int mi, int u) __attribute__((always_inline)) {
        d = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, (mi * nsub + u) * 1024, 0);
    };
    auto ldB = [&](v4i &d, int ni, int u) __attribute__((always_inline)) {
        d = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, (ni * nsub + u) * 1024, 0);
    };
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) ldB(b0[ni], ni, 0);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) ldA(a0[mi], mi, 0);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) ldB(b1[ni], ni, 1);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) ldA(a1[mi], mi, 1);
#ifdef QGEMM_LAB
    if constexpr (kFlags & kT2Sleep)
        if (team == 1) {
            const int n = __builtin_amdgcn_readfirstlane(g_t2_param[0]);
            for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(8);
        }
    const int hi_until = (kFlags & kT2Prio) ? __builtin_amdgcn_readfirstlane(g_t2_param[1]) : 0;
#else
    const int hi_until = 0;
#endif
    constexpr bool kLd = !(kFlags & kT2NoLoad);
    constexpr int kLag = (kFlags & kT2Late) ? 2 : 1;
    // MFMAs of sub-step u on (ca, cb); reloads of the same set for sub-step un (clamped: unconditional
    // loads keep hipcc from holding two values of a set across the loop)
    auto substep = [&](v4i (&ca)[8], v4i (&cb)[4], int u, int un, bool more) __attribute__((always_inline)) {
        un = un < nsub ? un : nsub - 1;
        if constexpr (!(kFlags & kT2NoPrio)) {
            if constexpr (kFlags & kT2Prio) {
                if (team == 0 && u < hi_until) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(1);
            } else {
                __builtin_amdgcn_s_setprio(1);
            }
        }
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) mfma_agpr(acc[mi][ni], ca[mi], cb[ni]);
            if (more && kLd && mi >= kLag) ldA(ca[mi - kLag], mi - kLag, un);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (more && kLd) {
#pragma unroll
            for (int mi = 8 - kLag; mi < 8; ++mi) ldA(ca[mi], mi, un);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) ldB(cb[ni], ni, un);
        }
        if constexpr (!(kFlags & kT2NoPrio)) __builtin_amdgcn_s_setprio(0);
    };
    int u = 0;
    for (; u + 2 <= nsub; u += 2) {
        substep(a0, b0, u, u + 2, true);
        substep(a1, b1, u + 1, u + 3, true);
    }
    if (u < nsub) substep(a0, b0, u, 0, false);  // odd nsub: set 0 holds the last sub-step
    // the last MFMAs' results are read by VALU below; the asm statements hide them from hipcc's padding
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    stamp(1);

    const int gi0 = tm * BM + team * 128, gj0 = tn * BN + wq * 64;
    float *C = static_cast<float *>(p.C);
    if constexpr (kFlags & kT2NoStore) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) x ^= acc[mi][ni][0] ^ acc[mi][ni][1] ^ acc[mi][ni][2] ^ acc[mi][ni][3];
        if (x == 0x7fffffff && p.m < 0) C[tid] = (float)x;
        stamp(2);
        return;
    }
    const int lrow = lane & 15, kq = lane >> 4;
    float *T = reinterpret_cast<float *>(lds + wave * kImg);
    float cwv[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) cwv[ni] = p.Cw[gj0 + ni * 16 + lrow];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        float cxv[4][4];
#pragma unroll
        for (int mq = 0; mq < 4; ++mq)
#pragma unroll
            for (int r = 0; r < 4; ++r) cxv[mq][r] = p.Cx[gi0 + 64 * s + mq * 16 + 4 * kq + r];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    T[(mq * 16 + 4 * kq + r) * TS + ni * 16 + lrow] =
                        dequantize(acc[4 * s + mq][ni][r], outer_product(cxv[mq][r], cwv[ni]), p.inv_r2);
        // one wave's LDS ops stay in order: its ds_writes precede its ds_reads, which precede the next
        // half's ds_writes
#pragma unroll 4
        for (int it = 0; it < 16; ++it) {
            const int rr = 4 * it + kq;
            const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + lrow * 4);
            float4 *dst = reinterpret_cast<float4 *>(C + (int64_t)(gi0 + 64 * s + rr) * p.csh + gj0 + lrow * 4);
            if constexpr (kFlags & kT2Nt) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f *>(dst));
            } else {
                *dst = v;
            }
        }
    }
    stamp(2);
}

}  // namespace gemm
}  // namespace qgemm
