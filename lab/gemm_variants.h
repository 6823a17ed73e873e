// gemm_variants.h -- experimental GEMM structures kept for the lab's A/B runs (not built into the
// library).  Results of each are recorded in DESIGN.md "GEMM experiments".
#pragma once

#include <type_traits>

#include "gemm_legacy.h"
#include "gemm_sd.h"

namespace qgemm {
namespace gemm {

// ------------------------------------------------------------------------------------------------
// v2: register double-buffered fragments; the k-step's barrier sits before the LAST sub-step's
// MFMAs, so after it every wave has MFMA work in registers while the next tile's first fragments
// are read.  Per k-step t (buffer cur = t&1):
//   issue glds(t+1 -> cur^1)                         (cur^1 was last read before barrier B(t-1))
//   s0: read frags s1 | MFMA s0     s1: read s2 | MFMA s1     s2: read s3 | MFMA s2
//   vmcnt(0) ; barrier B(t)                          (tile t+1 visible; all reads of cur issued)
//   s3: read frags s0 of tile t+1 from cur^1 | MFMA s3
template <int kMode, bool kDequant, int kFlags = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v2(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) int8_t lds[kLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    Stager st;
    st.init(p.A, p.B, tm, tn, p.k_pad, wave, lane);
    const int lrow = lane & 31, khalf = lane >> 5, swz = (lrow >> 1) & 7;
    const int a_row0 = (wm * 128 + lrow) * BK, b_row0 = (wn * 64 + lrow) * BK;
    int off[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) off[s] = ((2 * s + khalf) ^ swz) << 4;

    v16i acc[4][2];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = v16i{};

    auto read_frags = [&](v4i (&a)[4], v4i (&b)[2], int buf, int s) {
        if constexpr (kFlags & kNoLdsRead) {
            if (s != 0 || buf != 0) return;
        }
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 32 * BK + off[s]);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 32 * BK + off[s]);
    };
    auto mfmas = [&](const v4i (&a)[4], const v4i (&b)[2]) {
        if constexpr (kFlags & kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        if constexpr (kFlags & kPrio) __builtin_amdgcn_s_setprio(0);
    };

    const int nk = (int)(p.k_pad / BK);
    v4i a0[4], b0[2], a1[4], b1[2];
    st.stage(lds, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    read_frags(a0, b0, 0, 0);
    if constexpr (kFlags & kNoLdsRead) read_frags(a1, b1, 0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nk;
        if (!(kFlags & kNoGlds) || kt == 0)
            if (more) st.stage(lds, kt + 1, cur ^ 1);
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        read_frags(a0, b0, cur, 2);
        mfmas(a1, b1);
        read_frags(a1, b1, cur, 3);
        mfmas(a0, b0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (more) read_frags(a0, b0, cur ^ 1, 0);
        mfmas(a1, b1);
    }
    epilogue<kMode, kDequant>(p, lds, acc, tm, tn, wm, wn, lane, tid);
}


// ------------------------------------------------------------------------------------------------
// v5: the production structure.
//  * v_mfma_i32_16x16x64_i8, s_setprio(1) around every MFMA cluster.
//  * Each 256 x 256 macro-tile is computed as two sequential 256 x 128 halves (8 waves as 4 (M) x
//    2 (N), 64 x 64 per wave = 4 x 4 MFMA tiles, 64 accumulators).  The dequantized fp32 results of
//    half 0 stay in 64 registers and are written DURING half 1's main loop, one 1-KiB store per wave
//    per k-step (4 rows x 256 B, bounced through a private 1-KiB LDS slot), so the HBM write of half
//    the tile overlaps MFMA work instead of forming a tail after it.
//  * kStages-deep LDS ring of 48-KiB stages (A 256 x 128 B + B 128 x 128 B), one stage in flight
//    beyond the one being waited for (kStages = 3), counted s_waitcnt vmcnt(N) and raw s_barrier:
//    no vmcnt(0) in the main loop.
//  * Fragment double buffering: sub-step 1's fragments are read under sub-step 0's MFMAs, and the
//    next k-step's sub-step 0 fragments under sub-step 1's MFMAs, after the k-step's one barrier.
namespace v5 {
constexpr int kStageA = BM * BK;             // 32 KiB
constexpr int kStage5 = kStageA + 128 * BK;  // + B half-tile 16 KiB = 48 KiB
constexpr int kGlds = 6;                     // glds instructions per wave per stage (4 A + 2 B)
template <int kStages>
constexpr int lds_bytes() { return kStages * kStage5 + 8 * 1024 + 2 * 1024; }
}  // namespace v5

__device__ __forceinline__ void wait_vm_barrier(int n) {
    // n = number of vector-memory ops allowed to stay in flight (youngest); then an LDS drain and a
    // raw barrier.  One asm statement with a memory clobber so no LDS access crosses it.
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 13: asm volatile("s_waitcnt vmcnt(13)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
}

template <int N>
struct IntC {
    static constexpr int value = N;
};

template <int kStages, int kFlags = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v5(GemmArgs p) {
    using namespace v5;
    static_assert(kStages == 2 || kStages == 3, "ring depth");
    __shared__ __attribute__((aligned(16))) int8_t lds[lds_bytes<kStages>()];
    float *bounce_all = reinterpret_cast<float *>(lds + kStages * kStage5);  // 8 x 1 KiB
    float *sCx = bounce_all + 8 * 256;                                        // 256 floats
    float *sCw = sCx + 256;                                                   // 256 floats

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int gi0 = tm * BM, gj0 = tn * BN;
    const int64_t k_pad = p.k_pad;
    const int nk = (int)(k_pad / BK);
    const int total = 2 * nk;  // k-steps over both halves

    // scales of this macro-tile -> LDS (ordinary loads; drained before the first glds is issued)
    if (tid < BM) sCx[tid] = p.Cx[gi0 + tid];
    else sCw[tid - BM] = p.Cw[gj0 + tid - BM];

    // ---- staging: wave w fills A rows [32w, 32w+32) (4 glds) and B rows [16w, 16w+16) (2 glds)
    const int8_t *Ablk = p.A + (int64_t)gi0 * k_pad;
    const int8_t *Bblk = p.B + (int64_t)gj0 * k_pad;
    int64_t offa[4], offb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wave * 32 + i * 8 + (lane >> 3);
        offa[i] = (int64_t)row * k_pad + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 16 + i * 8 + (lane >> 3);
        offb[i] = (int64_t)row * k_pad + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
    }
    // stage k-step t (both halves form one stream of 2*nk k-steps) into ring slot `slot`
    auto stage = [&](int t, int slot) __attribute__((always_inline)) {
        const int h = t >= nk ? 1 : 0;
        const int kt = t - h * nk;
        int8_t *la = lds + slot * kStage5;
        int8_t *lb = la + kStageA;
        const int8_t *ga = Ablk + (int64_t)kt * BK;
        const int8_t *gb = Bblk + (int64_t)h * 128 * k_pad + (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(ga + offa[i]), (void *)(la + (wave * 32 + i * 8) * BK), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(gb + offb[i]), (void *)(lb + (wave * 16 + i * 8) * BK), 16, 0, 0);
    };

    // ---- fragments (16x16x64: lane l holds row l&15, 16 bytes of k-chunk 4s + (l>>4))
    const int lrow = lane & 15, kq = lane >> 4, swz = (lrow >> 1) & 7;
    const int a_base = (wm * 64 + lrow) * BK, b_base = (wn * 64 + lrow) * BK;
    const int off0 = ((0 + kq) ^ swz) << 4, off1 = ((4 + kq) ^ swz) << 4;
    auto read_frags = [&](v4i (&a)[4], v4i (&b)[4], int slot, int off) __attribute__((always_inline)) {
        const int8_t *la = lds + slot * kStage5;
        const int8_t *lb = la + kStageA;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_base + ni * 16 * BK + off);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_base + mi * 16 * BK + off);
    };
    v4i acc[4][4];
    float o[4][4][4];  // [mi][ni][r]: dequantized results of the previous half, drained during the current one
    auto mfma_range = [&](const v4i (&a)[4], const v4i (&b)[4], int lo, int hi) __attribute__((always_inline)) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q >= lo && q < hi)
                acc[q >> 2][q & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q >> 2], b[q & 3], acc[q >> 2][q & 3], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    // ---- output group g = (mi, r): rows wm*64 + mi*16 + 4q + r (q = 0..3), the wave's 64 columns.
    // Transposed through the wave's private 1-KiB LDS slot by inline-asm LDS ops (invisible to the
    // compiler's LDS-DMA alias tracking, which would otherwise drain vmcnt to 0), then one 16-B store
    // per lane: 4 rows x 256 contiguous bytes per wave instruction.
    typedef __attribute__((address_space(3))) float lds_float;
    const uint32_t bounce_addr = (uint32_t)(uintptr_t)(lds_float *)(bounce_all + wave * 256);
    const uint32_t waddr = bounce_addr + (uint32_t)(kq * 64 + lrow) * 4;
    const uint32_t raddr = bounce_addr + (uint32_t)(kq * 64 + lrow * 4) * 4;
    float *C = static_cast<float *>(p.C);
    // uniform fast path: the whole macro-tile is in range and C is row-major, 16-B aligned rows
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gi0 + BM <= p.m && gj0 + BN <= p.n;
    float *Crow = C + (int64_t)(gi0 + wm * 64 + 4 * kq) * p.csh + gj0 + wn * 64 + lrow * 4;  // fast path base
    auto store_group = [&](int h, int mi, int r, float x0, float x1, float x2, float x3) __attribute__((always_inline)) {
        float4 v;
        asm volatile(
            "ds_write_b32 %1, %2\n\t"
            "ds_write_b32 %1, %3 offset:64\n\t"
            "ds_write_b32 %1, %4 offset:128\n\t"
            "ds_write_b32 %1, %5 offset:192\n\t"
            "ds_read_b128 %0, %6\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(v)
            : "v"(waddr), "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(raddr)
            : "memory");
        if (full) {
            *reinterpret_cast<float4 *>(Crow + (int64_t)(mi * 16 + r) * p.csh + h * 128) = v;
        } else {
            const int i = gi0 + wm * 64 + mi * 16 + 4 * kq + r;
            const int j = gj0 + h * 128 + wn * 64 + lrow * 4;
            const float vv[4] = {v.x, v.y, v.z, v.w};
            if (i < p.m) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
            }
        }
    };
    auto dequant_half = [&](int h) __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
            const float4 cx4 = *reinterpret_cast<const float4 *>(sCx + wm * 64 + mi * 16 + 4 * kq);
            const float cxv[4] = {cx4.x, cx4.y, cx4.z, cx4.w};
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const float cw = sCw[h * 128 + wn * 64 + ni * 16 + lrow];
#pragma unroll
                for (int r = 0; r < 4; ++r) o[mi][ni][r] = dequantize(acc[mi][ni][r], outer_product(cxv[r], cw), p.inv_r2);
            }
        }
    };

    v4i f0a[4], f0b[4], f1a[4], f1b[4];
    // one k-step t (ring slot `slot`); G >= 0: also drain output group G of the previous half
    auto kstep = [&](int t, int slot, auto G) __attribute__((always_inline)) {
        constexpr int g = decltype(G)::value;
        const int ahead = kStages == 3 ? (slot == 0 ? 2 : slot - 1) : (slot ^ 1);  // slot of t + kStages - 1
        const int nxt = kStages == 3 ? (slot == 2 ? 0 : slot + 1) : (slot ^ 1);   // slot of t + 1
        if (t + kStages - 1 < total) stage(t + kStages - 1, ahead);
        asm volatile("" ::: "memory");  // the glds stay ahead of this k-step's drain store (vmcnt order)
        read_frags(f1a, f1b, slot, off1);
        mfma_range(f0a, f0b, 0, 16);
        if constexpr (g >= 0) store_group(0, g >> 2, g & 3, o[g >> 2][0][g & 3], o[g >> 2][1][g & 3],
                                          o[g >> 2][2][g & 3], o[g >> 2][3][g & 3]);
        // stage t+1 must have landed: allow the younger stage (t+2) and this k-step's store
        const int pending = (kStages == 3 && t + 2 < total ? kGlds : 0) + (g >= 0 ? 1 : 0);
        wait_vm_barrier(pending);
        mfma_range(f1a, f1b, 0, 4);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < total) read_frags(f0a, f0b, nxt, off0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_range(f1a, f1b, 4, 16);
        return nxt;
    };
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
    };
#define QG_DRAIN(g) store_group(0, (g) >> 2, (g) & 3, o[(g) >> 2][0][(g) & 3], o[(g) >> 2][1][(g) & 3], \
                                o[(g) >> 2][2][(g) & 3], o[(g) >> 2][3][(g) & 3])

    // ---- prologue
    __syncthreads();  // sCx/sCw written (their global loads are drained here, before any glds)
#pragma unroll
    for (int s = 0; s < kStages - 1; ++s)
        if (s < total) stage(s, s);
    if constexpr (kStages == 3) {
        if (total > 1) wait_vm_barrier(kGlds);
        else wait_vm_barrier(0);
    } else {
        wait_vm_barrier(0);
    }
    read_frags(f0a, f0b, 0, off0);

    // ---- half 0
    zero_acc();
    int slot = 0, t = 0;
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt, ++t) slot = kstep(t, slot, IntC<-1>{});
    dequant_half(0);
    // ---- half 1: the first 16 k-steps each drain one output group of half 0
    zero_acc();
    if (nk >= 16) {
        slot = kstep(t++, slot, IntC<0>{});
        slot = kstep(t++, slot, IntC<1>{});
        slot = kstep(t++, slot, IntC<2>{});
        slot = kstep(t++, slot, IntC<3>{});
        slot = kstep(t++, slot, IntC<4>{});
        slot = kstep(t++, slot, IntC<5>{});
        slot = kstep(t++, slot, IntC<6>{});
        slot = kstep(t++, slot, IntC<7>{});
        slot = kstep(t++, slot, IntC<8>{});
        slot = kstep(t++, slot, IntC<9>{});
        slot = kstep(t++, slot, IntC<10>{});
        slot = kstep(t++, slot, IntC<11>{});
        slot = kstep(t++, slot, IntC<12>{});
        slot = kstep(t++, slot, IntC<13>{});
        slot = kstep(t++, slot, IntC<14>{});
        slot = kstep(t++, slot, IntC<15>{});
#pragma unroll 1
        for (int kt = 16; kt < nk; ++kt, ++t) slot = kstep(t, slot, IntC<-1>{});
    } else {
        // short K: drain half 0 up front (its stores then overlap half 1's few k-steps)
#pragma unroll
        for (int g = 0; g < 16; ++g) QG_DRAIN(g);
#pragma unroll 1
        for (int kt = 0; kt < nk; ++kt, ++t) slot = kstep(t, slot, IntC<-1>{});
    }
    dequant_half(1);
    // ---- tail: half 1's results
#pragma unroll
    for (int g = 0; g < 16; ++g)
        store_group(1, g >> 2, g & 3, o[g >> 2][0][g & 3], o[g >> 2][1][g & 3], o[g >> 2][2][g & 3], o[g >> 2][3][g & 3]);
#undef QG_DRAIN
}
// ------------------------------------------------------------------------------------------------
// v6: deeper staging.  256 x 256 macro-tile, 8 waves as 2 (M) x 4 (N), 128 x 64 per wave on
// v_mfma_i32_16x16x64_i8 (8 x 4 tiles, 128 accumulators).  k-step 64 bytes; ring of kNS stages of
// 32 KiB (A 256 x 64 B + B 256 x 64 B) with kNS-1 stages in flight (counted vmcnt, raw barrier).
// LDS rows are 64 B = 4 chunks; chunk c of row r sits at slot c ^ (((r >> 2) & 1) << 1), which
// makes the 16-row fragment reads conflict-free (each ds_read_b128 lane group hits 16 distinct
// 16-B slots).  Per k-step: 8 MFMAs, barrier, next k-step's 12 fragment reads under the other 24.
namespace v6 {
constexpr int BK6 = 64;
constexpr int kTile6 = BM * BK6;        // 16 KiB per operand
constexpr int kStage6 = 2 * kTile6;     // 32 KiB
constexpr int kGlds6 = 4;               // glds per wave per stage (2 A + 2 B)
}  // namespace v6

__device__ __forceinline__ void wait_vm_barrier6(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
}

// kTiled: packed operands stored as contiguous 1-KiB blocks of 16 rows x 64 bytes, block (rb, kb) at
// (rb * (k_pad/64) + kb) KiB -- every staging instruction then reads one contiguous KiB.
template <int kNS, int kMode, bool kTiled = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v6(GemmArgs p) {
    using namespace v6;
    static_assert(kNS == 3 || kNS == 4, "ring depth");
    __shared__ __attribute__((aligned(16))) int8_t lds[kNS * kStage6 + 2048];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int gi0 = tm * BM, gj0 = tn * BN;
    const int64_t k_pad = p.k_pad;
    const int nk = (int)(k_pad / BK6);

    // staging: wave w fills A rows [32w, 32w+32) and B rows [32w, 32w+32), 16 rows (1 KiB) per glds;
    // lane l -> row (l>>2) of the piece, slot l&3, holding global chunk slot ^ g(row)
    const int8_t *Ablk = p.A + (int64_t)gi0 * k_pad;
    const int8_t *Bblk = p.B + (int64_t)gj0 * k_pad;
    int64_t off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 32 + i * 16 + (lane >> 2);
        const int chunk = (lane & 3) ^ (((row >> 2) & 1) << 1);
        if constexpr (kTiled)
            off[i] = (int64_t)(row >> 4) * (k_pad / 64) * 1024 + (row & 15) * 64 + (chunk << 4);
        else
            off[i] = (int64_t)row * k_pad + (chunk << 4);
    }
    auto stage = [&](int t) __attribute__((always_inline)) {
        int8_t *la = lds + (t % kNS) * kStage6;
        int8_t *lb = la + kTile6;
        const int64_t kstep = kTiled ? (int64_t)t * 1024 : (int64_t)t * BK6;
        const int8_t *ga = Ablk + kstep;
        const int8_t *gb = Bblk + kstep;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(ga + off[i]), (void *)(la + (wave * 32 + i * 16) * BK6), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(gb + off[i]), (void *)(lb + (wave * 32 + i * 16) * BK6), 16, 0, 0);
    };
    // fragments: lane l reads row l&15 of each 16-row tile, chunk l>>4
    const int lrow = lane & 15, kq = lane >> 4;
    const int foff = (kq ^ (((lrow >> 2) & 1) << 1)) << 4;
    const int a_base = (wm * 128 + lrow) * BK6 + foff, b_base = (wn * 64 + lrow) * BK6 + foff;
    auto read_frags = [&](v4i (&a)[8], v4i (&b)[4], int t) __attribute__((always_inline)) {
        const int8_t *la = lds + (t % kNS) * kStage6;
        const int8_t *lb = la + kTile6;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_base + ni * 16 * BK6);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_base + mi * 16 * BK6);
    };
    v4i acc[8][4];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
    auto mfma_range = [&](const v4i (&a)[8], const v4i (&b)[4], int lo, int hi) __attribute__((always_inline)) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 32; ++q)
            if (q >= lo && q < hi)
                acc[q >> 2][q & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q >> 2], b[q & 3], acc[q >> 2][q & 3], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    v4i fa0[8], fb0[4], fa1[8], fb1[4];
    auto kstep = [&](int t, v4i (&ca)[8], v4i (&cb)[4], v4i (&na)[8], v4i (&nb)[4]) __attribute__((always_inline)) {
        if (t + kNS - 1 < nk) stage(t + kNS - 1);
        mfma_range(ca, cb, 0, 8);
        // stage t+1 must have landed; stages t+2 .. t+kNS-1 (if issued) may stay in flight
        int ahead = nk - 2 - t;  // stages beyond t+1 that exist
        ahead = ahead < 0 ? 0 : (ahead > kNS - 2 ? kNS - 2 : ahead);
        wait_vm_barrier6(ahead * kGlds6);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) read_frags(na, nb, t + 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_range(ca, cb, 8, 32);
    };

    // prologue: kNS-1 stages in flight, wait for stage 0
#pragma unroll
    for (int s = 0; s < kNS - 1; ++s)
        if (s < nk) stage(s);
    {
        int ahead = nk - 1;
        ahead = ahead < 0 ? 0 : (ahead > kNS - 2 ? kNS - 2 : ahead);
        wait_vm_barrier6(ahead * kGlds6);
    }
    read_frags(fa0, fb0, 0);
#pragma unroll 1
    for (int t = 0; t < nk; t += 2) {
        kstep(t, fa0, fb0, fa1, fb1);
        if (t + 1 < nk) kstep(t + 1, fa1, fb1, fa0, fb0);
    }

    // epilogue: C/D map of 16x16: col = lane&15, row = 4(lane>>4) + r
    if constexpr (kMode == kStoreNone) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) x ^= acc[mi][ni][r];
        if (x == 0x7fffffff && p.m < 0) static_cast<int *>(p.C)[tid] = x;
    } else if constexpr (kMode == kStoreDirect) {
        __syncthreads();
        float *sCx = reinterpret_cast<float *>(lds);
        float *sCw = sCx + BM;
        if (tid < BM) sCx[tid] = p.Cx[gi0 + tid];
        else sCw[tid - BM] = p.Cw[gj0 + tid - BM];
        __syncthreads();
        float *C = static_cast<float *>(p.C);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int jl = wn * 64 + ni * 16 + lrow;
            const int j = gj0 + jl;
            const float cw = sCw[jl];
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int il = wm * 128 + mi * 16 + 4 * kq + r;
                    const int i = gi0 + il;
                    const float o = dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), p.inv_r2);
                    if (i < p.m && j < p.n) C[(int64_t)i * p.csh + (int64_t)j * p.csw] = o;
                }
        }
    } else {
        // kStoreLds: dequantize into a [128][256] fp32 LDS image one 128-row half at a time, then
        // every wave instruction stores one full 1-KiB tile row (16 B per lane).
        float *T = reinterpret_cast<float *>(lds);                 // 128 KiB
        float *sCx = reinterpret_cast<float *>(lds + 128 * 1024);  // needs kNS*32 KiB >= 130 KiB
        float *sCw = sCx + BM;
        __syncthreads();
        if (tid < BM) sCx[tid] = p.Cx[gi0 + tid];
        else sCw[tid - BM] = p.Cw[gj0 + tid - BM];
        float *C = static_cast<float *>(p.C);
        const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                          gj0 + BN <= p.n;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            __syncthreads();
            if (wm == half) {
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    const int jl = wn * 64 + ni * 16 + lrow;
                    const float cw = sCw[jl];
#pragma unroll
                    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int il = mi * 16 + 4 * kq + r;
                            T[il * BN + jl] = dequantize(acc[mi][ni][r], outer_product(sCx[half * 128 + il], cw), p.inv_r2);
                        }
                }
            }
            __syncthreads();
            const int c4 = (tid & 63) * 4;
#pragma unroll 4
            for (int rr = tid >> 6; rr < 128; rr += kThreads / 64) {
                const int i = gi0 + half * 128 + rr;
                if (i >= p.m) break;
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * BN + c4);
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
    }
}


// ------------------------------------------------------------------------------------------------
// v7: v3's schedule with the next sub-step's fragment reads interleaved INTO the current MFMA cluster
// (sched_group_barrier: 2 MFMAs, 1 ds_read, ... then 8 MFMAs), so no read latency is exposed at the
// cluster boundary and the compiler has no reason for a blanket lgkmcnt(0) before the cluster.
// kDmaIn: also spread the next tile's 8 LDS-DMA issues over the first cluster.
template <int kRest, int J>
__device__ __forceinline__ void pin_reads() {
    if constexpr (J < 12) {
        __builtin_amdgcn_sched_group_barrier(0x0008, (kRest * (J + 1)) / 12 - (kRest * J) / 12, 0);
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
        pin_reads<kRest, J + 1>();
    }
}

// diagnostic in-kernel clock stamps (MI355X_MICROARCH.md 'DVFS give-back' item 6): per block,
// s_memtime / s_memrealtime at kernel start, after the main loop, after the epilogue
__device__ unsigned long long g_stamp[4096][6];
enum V7Flags { kV7Stamp = 32, kV7NoGlds = 64, kV7Early = 128 };

template <int kMode, bool kDmaIn, int kTail = 8, int kFlags = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v7(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) int8_t lds[kLdsBytes + 2048];
    const int tid = threadIdx.x, lane = tid & 63;
    if constexpr (kFlags & kV7Stamp)
        if (tid == 0) {
            g_stamp[blockIdx.x][0] = __builtin_amdgcn_s_memtime();
            g_stamp[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
        }
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    Stager st;
    st.init(p.A, p.B, tm, tn, p.k_pad, wave, lane);
    const int lrow = lane & 15, kq = lane >> 4, swz = (lrow >> 1) & 7;
    const int a_row0 = (wm * 128 + lrow) * BK, b_row0 = (wn * 64 + lrow) * BK;
    int off[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) off[s] = ((4 * s + kq) ^ swz) << 4;

    v4i acc[8][4];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};

    auto read_frags = [&](v4i (&a)[8], v4i (&b)[4], int buf, int s) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[s]);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[s]);
    };
    // no s_setprio inside: it is a scheduling boundary and would fence the reads off the MFMAs
    auto mfmas = [&](const v4i (&a)[8], const v4i (&b)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    };
    // pin the interleave: (32 - kTail) MFMAs paired with the 12 reads, then kTail MFMAs
    auto pin = [&](auto dma_c) __attribute__((always_inline)) {
        constexpr bool dma = decltype(dma_c)::value;
        if constexpr (dma) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);
            }
        }
        pin_reads<32 - kTail - (dma ? 8 : 0), 0>();
        __builtin_amdgcn_sched_group_barrier(0x0008, kTail, 0);
        __builtin_amdgcn_sched_barrier(0);  // nothing crosses into the next cluster
    };

    const int nk = (int)(p.k_pad / BK);
    v4i a0[8], b0[4], a1[8], b1[4];
    if constexpr (kFlags & kV7Early) {
        // early staging: buffer cur is free at barrier B(kt) (every read of tile kt has retired), so
        // tile kt+2 is issued right there and has a whole k-step to land (vs half a k-step)
        st.stage(lds, 0, 0);
        if (nk > 1) {
            st.stage(lds, 1, 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        read_frags(a0, b0, 0, 0);
        for (int kt = 0; kt < nk - 1; ++kt) {
            const int cur = kt & 1;
            read_frags(a1, b1, cur, 1);
            mfmas(a0, b0);
            pin(std::false_type{});
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (kt + 2 < nk) st.stage(lds, kt + 2, cur);
            read_frags(a0, b0, cur ^ 1, 0);
            mfmas(a1, b1);
            pin(std::false_type{});
        }
    } else {
    st.stage(lds, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    read_frags(a0, b0, 0, 0);
    // steady state: every k-step but the last stages the next tile (straight-line body, one block)
    for (int kt = 0; kt < nk - 1; ++kt) {
        const int cur = kt & 1;
        if constexpr (!(kFlags & kV7NoGlds)) st.stage(lds, kt + 1, cur ^ 1);
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        pin(std::integral_constant<bool, kDmaIn && !(kFlags & kV7NoGlds)>{});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        read_frags(a0, b0, cur ^ 1, 0);
        mfmas(a1, b1);
        pin(std::false_type{});
    }
    }
    {
        const int cur = (nk - 1) & 1;
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        pin(std::false_type{});
        mfmas(a1, b1);
    }
    if constexpr (kFlags & kV7Stamp)
        if (tid == 0) {
            __builtin_amdgcn_sched_barrier(0);
            g_stamp[blockIdx.x][2] = __builtin_amdgcn_s_memtime();
            g_stamp[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();
        }

    epilogue16<kMode>(p, lds, acc, tm, tn, wm, wn, lane, tid);
    if constexpr (kFlags & kV7Stamp)
        if (tid == 0) {
            g_stamp[blockIdx.x][4] = __builtin_amdgcn_s_memtime();
            g_stamp[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();
        }
}


// ------------------------------------------------------------------------------------------------
// v9: Tensile-style big wave tiles -- 4 waves (one per SIMD), 2x2, each 128x128 of the 256x256 tile
// (acc 8x8 16x16 tiles = 256 regs, AGPR-resident).  LDS read bytes per MAC drop by a third vs the
// 128x64 wave tile (1/128+1/128 vs 1/64+1/128).  Early staging and interleaved reads as in v7e.
template <int kRest, int kReads, int J>
__device__ __forceinline__ void pin_reads_n() {
    if constexpr (J < kReads) {
        __builtin_amdgcn_sched_group_barrier(0x0008, (kRest * (J + 1)) / kReads - (kRest * J) / kReads, 0);
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
        pin_reads_n<kRest, kReads, J + 1>();
    }
}

template <int kMode, int kTail = 16, int kFlags = 0>
__global__ __launch_bounds__(256, 1) void gemm_i8_v9(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) int8_t lds[kLdsBytes + 2048];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const int8_t *Ablk = p.A + (int64_t)tm * BM * p.k_pad;
    const int8_t *Bblk = p.B + (int64_t)tn * BN * p.k_pad;
    // wave w fills rows [64w, 64w+64) of both tiles, 8 rows (1 KiB) per glds, chunk-swizzled source
    int src_off[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = wave * 64 + i * 8 + (lane >> 3);
        const int g = (lane & 7) ^ ((row >> 1) & 7);
        src_off[i] = row * (int)p.k_pad + g * 16;
    }
    auto stage = [&](int kt, int buf) __attribute__((always_inline)) {
        int8_t *la = lds + buf * kStageBytes;
        int8_t *lb = la + kTileBytes;
        const int8_t *ga = Ablk + (int64_t)kt * BK;
        const int8_t *gb = Bblk + (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_global_load_lds((const void *)(ga + src_off[i]), (void *)(la + (wave * 64 + i * 8) * BK), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(gb + src_off[i]), (void *)(lb + (wave * 64 + i * 8) * BK), 16, 0, 0);
        }
    };
    const int lrow = lane & 15, kq = lane >> 4, swz = (lrow >> 1) & 7;
    const int a_row0 = (wm * 128 + lrow) * BK, b_row0 = (wn * 128 + lrow) * BK;
    int off[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) off[s] = ((4 * s + kq) ^ swz) << 4;

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};

    auto read_frags = [&](v4i (&a)[8], v4i (&b)[8], int buf, int s) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[s]);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[s]);
    };
    auto mfmas = [&](const v4i (&a)[8], const v4i (&b)[8]) __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    };
    auto pin = [&]() __attribute__((always_inline)) {
        pin_reads_n<64 - kTail, 16, 0>();
        __builtin_amdgcn_sched_group_barrier(0x0008, kTail, 0);
        __builtin_amdgcn_sched_barrier(0);
    };

    const int nk = (int)(p.k_pad / BK);
    v4i a0[8], b0[8], a1[8], b1[8];
    stage(0, 0);
    if (nk > 1) {
        stage(1, 1);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    read_frags(a0, b0, 0, 0);
    for (int kt = 0; kt < nk - 1; ++kt) {
        const int cur = kt & 1;
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        pin();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + 2 < nk) stage(kt + 2, cur);
        read_frags(a0, b0, cur ^ 1, 0);
        mfmas(a1, b1);
        pin();
    }
    {
        const int cur = (nk - 1) & 1;
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        pin();
        mfmas(a1, b1);
    }

    // epilogue
    const int gi0 = tm * BM, gj0 = tn * BN;
    if constexpr (kMode == kStoreNone) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) x ^= acc[mi][ni][r];
        if (x == 0x7fffffff && p.m < 0) static_cast<int *>(p.C)[tid] = x;
        return;
    } else {
        float *sCx = reinterpret_cast<float *>(lds + kLdsBytes);
        float *sCw = sCx + BM;
        float *C = static_cast<float *>(p.C);
        __syncthreads();
        sCx[tid] = p.Cx[gi0 + tid];
        sCw[tid] = p.Cw[gj0 + tid];
        float *T = reinterpret_cast<float *>(lds);  // [128][256] fp32
        const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                          gj0 + BN <= p.n;
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
                            T[il * BN + jl] = dequantize(acc[mi][ni][r], outer_product(sCx[half * 128 + il], cw), p.inv_r2);
                        }
                }
            }
            __syncthreads();
            const int c4 = (tid & 63) * 4;
#pragma unroll 4
            for (int rr = tid >> 6; rr < 128; rr += 4) {
                const int i = gi0 + half * 128 + rr;
                if (i >= p.m) break;
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * BN + c4);
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
    }
}

}  // namespace gemm
}  // namespace qgemm
