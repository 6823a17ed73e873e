// gemm_legacy.h -- LAB ONLY: the row-major-operand 256 x 256 kernels of rounds 1-2 and the ping-pong kernel,
// moved out of the product header in round 4 (the packed operands are fragment-major, so a row-major
// reader compiled into the library would read scrambled operands if it were ever launched on them; VERDICT r03
// item 5: gemm_i8_pp was reachable only through environment switches).  The lab harnesses (pp_lab, gemm_lab,
// w4_lab, overlap_lab, fused_lab, chain2_lab) still time them against the product gemm_i8_fm.
//   gemm_i8_v1 (32x32x32 MFMA, round 1), gemm_i8_v3 (16x16x64, LDS-DMA ring, round-1 product),
//   gemm_i8_pp (ping-pong 8-wave schedule, round-2 product; kPPLayoutF reads the fragment-major layout).
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

typedef int v16i __attribute__((ext_vector_type(16)));
constexpr int kThreads = 512;
constexpr int kTileBytes = BM * BK;          // 32 KiB per operand per stage
constexpr int kStageBytes = 2 * kTileBytes;  // A + B
constexpr int kLdsBytes = 2 * kStageBytes;   // 2-deep ring = 128 KiB
// epilogue16's fp32 image of a 128-row half: rows padded to 260 floats, so the ds_write_b32 of the
// accumulators (lanes 16 apart = rows 4 apart) fall on banks 16 apart instead of the same bank (r02 PMC:
// 6.7 % bank-conflict cycles in gemm_i8_pp); the scales and the rest of the epilogue's LDS follow it
constexpr int kTStride = 260;
constexpr int kTImgBytes = 128 * kTStride * 4;
constexpr int kEpiBase = kTImgBytes > kLdsBytes ? kTImgBytes : kLdsBytes;
// Epilogue variants
enum StoreMode { kStoreDirect = 0, kStoreLds = 1, kStoreNone = 2 };
// kEpiOutlier with <= kOutlierStaged outlier columns: the tile's xo [256 rows][8] and wo [8][256 cols] are
// staged in LDS behind the Cx / Cw slots (loads issued before the ring is released)
constexpr int kOutlierStaged = 8;
constexpr int kOutlierStageBytes = 2 * 256 * kOutlierStaged * 4;
constexpr int64_t kSlabInts = (int64_t)BM * BN;

// ------------------------------------------------------------------------------------------------
// Shared pieces
struct Stager {
    const int8_t *Ablk, *Bblk;
    int64_t src_off[4];
    int wave;
    __device__ __forceinline__ void init(const int8_t *A, const int8_t *B, int tm, int tn, int64_t k_pad, int wave_,
                                         int lane) {
        wave = wave_;
        Ablk = A + (int64_t)tm * BM * k_pad;
        Bblk = B + (int64_t)tn * BN * k_pad;
        // wave w fills rows [32w, 32w+32) of both tiles, 8 rows per glds; lane l of instruction i writes
        // LDS bytes [16l, 16l+16) of its 1-KiB piece = row 32w+8i+(l>>3), slot l&7, which must hold
        // global chunk g = slot ^ ((row>>1)&7).
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wave * 32 + i * 8 + (lane >> 3);
            const int g = (lane & 7) ^ ((row >> 1) & 7);
            src_off[i] = (int64_t)row * k_pad + g * 16;
        }
    }
    __device__ __forceinline__ void stage(int8_t *lds, int kt, int buf) const {
        int8_t *la = lds + buf * kStageBytes;
        int8_t *lb = la + kTileBytes;
        const int8_t *ga = Ablk + (int64_t)kt * BK;
        const int8_t *gb = Bblk + (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_global_load_lds((const void *)(ga + src_off[i]), (void *)(la + (wave * 32 + i * 8) * BK),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(gb + src_off[i]), (void *)(lb + (wave * 32 + i * 8) * BK),
                                             16, 0, 0);
        }
    }
};

// Epilogue for accumulators in the natural C/D map of v_mfma_*_32x32*: col = lane&31,
// row = (r&3) + 8(r>>2) + 4(lane>>5).  acc[mi][ni] covers rows wm*128+mi*32.., cols wn*64+ni*32..
template <int kMode, bool kDequant>
__device__ __forceinline__ void epilogue(const GemmArgs &p, int8_t *lds, v16i (&acc)[4][2], int tm, int tn, int wm,
                                         int wn, int lane, int tid) {
    const int gi0 = tm * BM, gj0 = tn * BN;
    const int lrow = lane & 31, khalf = lane >> 5;
    if constexpr (kMode == kStoreNone) {
        // keep the accumulators live without storing them (ablation only)
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int r = 0; r < 16; ++r) x ^= acc[mi][ni][r];
        if (x == 0x7fffffff && p.m < 0) static_cast<int *>(p.C)[tid] = x;
        return;
    } else if constexpr (kMode == kStoreDirect) {
        if constexpr (kDequant) {
            float *sCx = reinterpret_cast<float *>(lds);
            float *sCw = sCx + BM;
            __syncthreads();
            if (tid < BM) sCx[tid] = p.Cx[gi0 + tid];
            else sCw[tid - BM] = p.Cw[gj0 + tid - BM];
            __syncthreads();
            float *C = static_cast<float *>(p.C);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int jl = wn * 64 + ni * 32 + lrow;
                const int j = gj0 + jl;
                const float cw = sCw[jl];
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int il = wm * 128 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
                        const int i = gi0 + il;
                        const float o = dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), p.inv_r2);
                        if (i < p.m && j < p.n) C[(int64_t)i * p.csh + (int64_t)j * p.csw] = o;
                    }
            }
        } else {
            int32_t *C = static_cast<int32_t *>(p.C);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int j = gj0 + wn * 64 + ni * 32 + lrow;
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int i = gi0 + wm * 128 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
                        if (i < p.m && j < p.n) C[(int64_t)i * p.csh + (int64_t)j * p.csw] = acc[mi][ni][r];
                    }
            }
        }
    } else {
        // kStoreLds: stage one 128-row half of the 256x256 int32 tile in LDS ([128][256] = 128 KiB),
        // then every thread dequantizes 4 consecutive columns and writes them as one 16-B store:
        // a wave instruction covers one whole 1-KiB tile row.
        int32_t *T = reinterpret_cast<int32_t *>(lds);
        float *C = static_cast<float *>(p.C);
        const bool vec = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            __syncthreads();
            if (wm == half) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int il = mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;  // 0..127
                            const int jl = wn * 64 + ni * 32 + lrow;
                            T[il * BN + jl] = acc[mi][ni][r];
                        }
            }
            __syncthreads();
            const int c4 = (tid & 63) * 4;  // column within the tile
            float cw[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) cw[e] = p.Cw[gj0 + c4 + e];  // Cw is padded to n_pad
#pragma unroll 4
            for (int rr = tid >> 6; rr < 128; rr += kThreads / 64) {
                const int i = gi0 + half * 128 + rr;
                if (i >= p.m) continue;
                const v4i a = *reinterpret_cast<const v4i *>(T + rr * BN + c4);
                const float cx = p.Cx[i];
                if constexpr (kDequant) {
                    float4 o;
                    o.x = dequantize(a[0], outer_product(cx, cw[0]), p.inv_r2);
                    o.y = dequantize(a[1], outer_product(cx, cw[1]), p.inv_r2);
                    o.z = dequantize(a[2], outer_product(cx, cw[2]), p.inv_r2);
                    o.w = dequantize(a[3], outer_product(cx, cw[3]), p.inv_r2);
                    const int j = gj0 + c4;
                    if (vec && j + 3 < p.n) {
                        *reinterpret_cast<float4 *>(C + (int64_t)i * p.csh + j) = o;
                    } else {
                        const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = ov[e];
                    }
                }
            }
        }
    }
}

enum V2Flags { kPrio = 1, kNoGlds = 2, kNoLdsRead = 4, kNoBarrier = 8, kNoVmWait = 16, kNoSlab = 32 /* lab ablation */ };

// ------------------------------------------------------------------------------------------------
// v1: stage(kt+1) ; compute(kt) with just-in-time fragment reads ; vmcnt(0) ; barrier
template <int kMode, bool kDequant>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v1(GemmArgs p) {
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
    v16i acc[4][2];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = v16i{};
    const int nk = (int)(p.k_pad / BK);
    st.stage(lds, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) st.stage(lds, kt + 1, cur ^ 1);
        const int8_t *la = lds + cur * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            const int off = ((2 * s + khalf) ^ swz) << 4;
            v4i a[4], b[2];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 32 * BK + off);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 32 * BK + off);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    epilogue<kMode, kDequant>(p, lds, acc, tm, tn, wm, wn, lane, tid);
}

// Epilogue for 16x16 accumulators acc[8][4] (wave tile 128 x 64 at rows wm*128, cols wn*64):
// C/D map col = lane&15, row = 4(lane>>4) + r.
//   kStoreLds    : dequantize into a [128][256] fp32 LDS image one 128-row half at a time; every wave
//                  instruction then stores one whole 1-KiB tile row (16 B per lane).  Needs the
//                  128 KiB staging ring + 2 KiB for the scales.
//   kStoreDirect : one dword per lane per register (4 rows x 64 B per instruction).
//   kStoreNone   : ablation -- keep the accumulators live, store nothing.

// kEpiOutlier store of one 128-row half of the tile (rows i0 .. i0 + 127 in T): O = fl(O8 + fmaf chain
// from +0 over the outlier columns in ascending k).  A wave owns rows i0 + w + 8q, a lane 4 columns; the
// chain runs for 8 rows at once, 4 outlier columns per step: one load brings the 8 x 4 xo values (lane
// 8g + tt: row g, column tt), v_readlane hands each to the wave as a scalar, one float4 of wo per column
// serves the 8 rows.  Columns past n read wo's padding and are never stored.
// sX [256 tile rows][8] / sW [8][256 tile cols]: the staged xo / wo values when ocnt <= kOutlierStaged
// (nullptr otherwise); gi0 = the tile's first row.
// a 16-B output store, nontemporal when kNt (the 64-MiB output streams past the caches: the next launch's
// inputs are not evicted by it)
template <bool kNt>
__device__ __forceinline__ void st_f4(float *dst, float4 v) {
    if constexpr (kNt) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f *>(dst));
    } else {
        *reinterpret_cast<float4 *>(dst) = v;
    }
}

template <bool kNt = false>
__device__ __forceinline__ void epilogue_outlier_half(const GemmArgs &p, const float *T, int i0, int gj0, int c4,
                                                      int tid, bool full, const float *sX, const float *sW,
                                                      int gi0) {
    const int ocnt = *p.ocount;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int j = gj0 + c4;
    const float *wr = p.wo + j;
    float *C = static_cast<float *>(p.C);
#pragma unroll 1
    for (int q0 = 0; q0 < 16; q0 += 8) {
        const int ib = i0 + wv + 8 * q0;  // rows ib + 8g, g < 8
        if (ib >= p.m) break;
        if (sX) {  // staged: every operand from LDS (xo reads are wave-uniform: broadcast)
            float c[8][4];
#pragma unroll
            for (int g = 0; g < 8; ++g) c[g][0] = c[g][1] = c[g][2] = c[g][3] = 0.0f;
#pragma unroll
            for (int t = 0; t < kOutlierStaged; ++t) {
                if (t >= ocnt) break;
                const float4 w4 = *reinterpret_cast<const float4 *>(sW + t * 256 + c4);
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const float xs = sX[(ib + 8 * g - gi0) * kOutlierStaged + t];
                    c[g][0] = __fmaf_rn(xs, w4.x, c[g][0]);
                    c[g][1] = __fmaf_rn(xs, w4.y, c[g][1]);
                    c[g][2] = __fmaf_rn(xs, w4.z, c[g][2]);
                    c[g][3] = __fmaf_rn(xs, w4.w, c[g][3]);
                }
            }
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const int i = ib + 8 * g;
                if (i >= p.m) break;
                const float4 o = *reinterpret_cast<const float4 *>(T + (i - i0) * kTStride + c4);
                const float vv[4] = {__fadd_rn(o.x, c[g][0]), __fadd_rn(o.y, c[g][1]), __fadd_rn(o.z, c[g][2]),
                                     __fadd_rn(o.w, c[g][3])};
                if (full) {
                    st_f4<kNt>(C + (int64_t)i * p.csh + j, make_float4(vv[0], vv[1], vv[2], vv[3]));
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
                }
            }
            continue;
        }
        const float *xl = p.xo + (int64_t)min(ib + 8 * (lane >> 3), p.m - 1) * ocnt + (lane & 7);
        float c[8][4];
#pragma unroll
        for (int g = 0; g < 8; ++g) c[g][0] = c[g][1] = c[g][2] = c[g][3] = 0.0f;
        // 4 columns per step; step t0 + 4's loads are issued before step t0's arithmetic
        auto load_step = [&](int t0, float &xv, float4 (&w4)[4]) {
            const int tn = min(4, ocnt - t0);
            xv = (lane & 7) < tn ? xl[t0] : 0.0f;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt)
                w4[tt] = tt < tn ? *reinterpret_cast<const float4 *>(wr + (int64_t)(t0 + tt) * p.wo_ld)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        float xn;
        float4 wn[4];
        load_step(0, xn, wn);
#pragma unroll 1
        for (int t0 = 0; t0 < ocnt; t0 += 4) {
            const int tn = min(4, ocnt - t0);  // uniform
            const float xv = xn;
            float4 w4[4];
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) w4[tt] = wn[tt];
            if (t0 + 4 < ocnt) load_step(t0 + 4, xn, wn);
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) {
                if (tt >= tn) break;
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const float xs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), 8 * g + tt));
                    c[g][0] = __fmaf_rn(xs, w4[tt].x, c[g][0]);
                    c[g][1] = __fmaf_rn(xs, w4[tt].y, c[g][1]);
                    c[g][2] = __fmaf_rn(xs, w4[tt].z, c[g][2]);
                    c[g][3] = __fmaf_rn(xs, w4[tt].w, c[g][3]);
                }
            }
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const int i = ib + 8 * g;
            if (i >= p.m) break;
            const float4 o = *reinterpret_cast<const float4 *>(T + (i - i0) * kTStride + c4);
            const float vv[4] = {__fadd_rn(o.x, c[g][0]), __fadd_rn(o.y, c[g][1]), __fadd_rn(o.z, c[g][2]),
                                 __fadd_rn(o.w, c[g][3])};
            if (full) {
                st_f4<kNt>(C + (int64_t)i * p.csh + j, make_float4(vv[0], vv[1], vv[2], vv[3]));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j + e < p.n) C[(int64_t)i * p.csh + (int64_t)(j + e) * p.csw] = vv[e];
            }
        }
    }
}

template <int kMode, int kEpi = kEpiNone, bool kNt = false>
__device__ __forceinline__ void epilogue16(const GemmArgs &p, int8_t *lds, v4i (&acc)[8][4], int tm, int tn, int wm,
                                           int wn, int lane, int tid) {
    const int gi0 = tm * BM, gj0 = tn * BN;
    const int lrow = lane & 15, kq = lane >> 4;
    if constexpr (kMode == kStoreNone) {
        int x = 0;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) x ^= acc[mi][ni][r];
        if (x == 0x7fffffff && p.m < 0) static_cast<int *>(p.C)[tid] = x;
        return;
    }
    float *sCx = reinterpret_cast<float *>(lds + kEpiBase);
    float *sCw = sCx + BM;
    float *sB = sCw + BN;  // bias (kEpi >= 1): needs kEpiBase + 3 KiB
    float *C = static_cast<float *>(p.C);
    // kEpiOutlier, <= kOutlierStaged outlier columns: this tile's xo rows and wo columns are loaded here,
    // ahead of the barrier (their latency hides under the ring drain), and parked in LDS behind Cx / Cw
    float *sX = reinterpret_cast<float *>(lds + kEpiBase + 2048), *sW = sX + 256 * kOutlierStaged;
    bool staged = false;
    float xs4[4] = {0.f, 0.f, 0.f, 0.f};
    float4 ws4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kEpi == kEpiOutlier && kMode != kStoreDirect) {
        const int oc = *p.ocount;
        staged = oc > 0 && oc <= kOutlierStaged;
        if (staged) {
            const int64_t r = min(gi0 + (tid >> 1), p.m - 1);  // xo: tile row tid >> 1, columns 4 (tid & 1) ..
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 4 * (tid & 1) + e;
                xs4[e] = c < oc ? p.xo[r * oc + c] : 0.0f;
            }
            const int wrow = tid >> 6;  // wo: row tid >> 6, tile columns 4 (tid & 63) ..
            if (wrow < oc) ws4 = *reinterpret_cast<const float4 *>(p.wo + wrow * p.wo_ld + gj0 + 4 * (tid & 63));
        }
    }
    __syncthreads();  // every wave is done with the staging ring
    if (tid < BM) sCx[tid] = p.Cx[gi0 + tid];
    else sCw[tid - BM] = p.Cw[gj0 + tid - BM];
    if constexpr (has_bias(kEpi))
        if (tid < BN) sB[tid] = gj0 + tid < p.n ? p.bias[gj0 + tid] : 0.0f;
    if constexpr (kEpi == kEpiOutlier && kMode != kStoreDirect) {
        if (staged) {  // visible after the barrier that opens the first half
#pragma unroll
            for (int e = 0; e < 4; ++e) sX[(tid >> 1) * kOutlierStaged + 4 * (tid & 1) + e] = xs4[e];
            *reinterpret_cast<float4 *>(sW + (tid >> 6) * 256 + 4 * (tid & 63)) = ws4;
        }
    }
    if constexpr (kMode == kStoreDirect) {
        __syncthreads();
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
                    const float o =
                        epi_extra<kEpi>(dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), p.inv_r2), sB, jl);
                    if (i < p.m && j < p.n) C[(int64_t)i * p.csh + (int64_t)j * p.csw] = o;
                }
        }
    } else {
        float *T = reinterpret_cast<float *>(lds);  // [128][kTStride] fp32
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
                            T[il * kTStride + jl] = epi_extra<kEpi>(
                                dequantize(acc[mi][ni][r], outer_product(sCx[half * 128 + il], cw), p.inv_r2), sB, jl);
                        }
                }
            }
            __syncthreads();
            const int c4 = (tid & 63) * 4;
            if constexpr (kEpi == kEpiOutlier) {
                if (*p.ocount > 0) {
                    epilogue_outlier_half<kNt>(p, T, gi0 + half * 128, gj0, c4, tid, full, staged ? sX : nullptr, sW,
                                          gi0);
                    continue;
                }
            }
#pragma unroll 4
            for (int rr = tid >> 6; rr < 128; rr += kThreads / 64) {
                const int i = gi0 + half * 128 + rr;
                if (i >= p.m) break;
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * kTStride + c4);
                const int j = gj0 + c4;
                if (full) {
                    if constexpr (kNt) {
                        typedef float v4f __attribute__((ext_vector_type(4)));
                        __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w},
                                                    reinterpret_cast<v4f *>(C + (int64_t)i * p.csh + j));
                    } else {
                        *reinterpret_cast<float4 *>(C + (int64_t)i * p.csh + j) = v;
                    }
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

// v3: as v2 but on v_mfma_i32_16x16x64_i8 (16 x 16 output per MFMA, 64-deep k).  Per wave 128 x 64 =
// 8 x 4 tiles; per 64-deep sub-step 8 A + 4 B fragment reads (lane l: row l&15, 16 bytes of k-chunk
// 4s + (l>>4)) and 32 MFMAs.  C/D map: col = lane&15, row = 4(lane>>4) + reg.
// In-launch split-K combine (cdna_hip_programming.md s5 "In-launch split-K reduction", the counter
template <int kMode, bool kDequant, int kFlags = 0, int kEpi = kEpiNone>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_v3(GemmArgs p) {
    // + scales (and bias) for the epilogue
    __shared__ __attribute__((aligned(16))) int8_t lds[kEpiBase + (has_bias(kEpi) ? 3072 : 2048)];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    // XCD remap first, then tile = id / S, slice = id % S: a tile's slices share an XCD (their slabs
    // are read back at the same-XCD rate; placement is a speed choice only)
    const int S = p.splits > 1 ? p.splits : 1;
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = wid / S, slice = wid - tile * S;
    int tm, tn;
    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn);
    const int nk_all = (int)(p.k_pad / BK);
    const int kt0 = slice * nk_all / S;
    const int nk = (slice + 1) * nk_all / S - kt0;
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

    auto read_frags = [&](v4i (&a)[8], v4i (&b)[4], int buf, int s) {
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[s]);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[s]);
    };
    auto mfmas = [&](const v4i (&a)[8], const v4i (&b)[4]) {
        if constexpr (kFlags & kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        if constexpr (kFlags & kPrio) __builtin_amdgcn_s_setprio(0);
    };

    v4i a0[8], b0[4], a1[8], b1[4];
    st.stage(lds, kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    read_frags(a0, b0, 0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nk;
        if (!(kFlags & kNoGlds) || kt == 0)
            if (more) st.stage(lds, kt0 + kt + 1, cur ^ 1);
        read_frags(a1, b1, cur, 1);
        mfmas(a0, b0);
        if constexpr (!(kFlags & kNoVmWait)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (!(kFlags & kNoBarrier)) __syncthreads();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (more) read_frags(a0, b0, cur ^ 1, 0);
        mfmas(a1, b1);
    }

    if (S > 1 &&
        !splitk_combine<8, 4, 8, !(kFlags & kNoSlab)>(p, reinterpret_cast<unsigned *>(lds + kEpiBase), acc, tile, slice,
                                                     S, wave, lane, tid))
        return;
    epilogue16<kMode, kEpi>(p, lds, acc, tm, tn, wm, wn, lane, tid);
}

// ------------------------------------------------------------------------------------------------
// gemm_i8_pp: the 256 x 256 tile of gemm_i8_v3 on a PING-PONG schedule.  Waves w and w + 4 share a
// SIMD (a workgroup's waves are dealt over the 4 SIMDs cyclically), so the block is split into a LEAD
// half (waves 0-3: tile rows 0-127) and a LAG half (waves 4-7: rows 128-255) that runs one slot
// behind.  A k-step is two slots separated by raw s_barriers; in every slot one wave of each SIMD
// issues its 64 MFMAs (both 64-deep sub-steps, 1024 pipe cycles) while its partner stages and reads
// ALL of its next k-step's fragments (24 ds_read_b128) -- the MFMA pipe never waits for the partner's
// LDS-DMA issue, fragment reads or the barrier skew, which in v3 both waves of a SIMD pay together.
//
//   slot:     2t            2t+1          2t+2
//   lead:     R(t)          M(t)          R(t+1) ...
//   lag:      M(t-1)        R(t)          M(t)   ...
//
// 2-stage LDS ring (64 KiB stages).  Staging (kDma):
//   0: the lead waves issue stage t+1 whole in R(t) (16 LDS-DMA pieces each) and wait for it after
//      M(t) -- two slots of flight.
//   1: (RACY, lab only) the lead waves issue A of stage t+1 in R(t); lag wave wn issues B rows
//      [64wn, 64wn+64) of stage t+2 at the end of R(t).  The lead's A pieces for rows 128-255 land
//      in the buffer whose sub-step-1 A fragments the lag waves are still reading inside M(t-1) in
//      the same slot: correct only while the DMA is slower than ~28 MFMAs.
//   2: (product) every wave stages only rows that it and its SIMD partner, or its own half, read,
//      each after the last reads of the slot it overwrites:
//        lead wn, R(t):  A rows [32wn, 32wn+32) and B rows [64wn, 64wn+32) of stage t+1 (8 pieces),
//                        waited for (vmcnt(0)) after M(t);
//        lag wn,  R(t):  A rows [128+32wn, ..+32) of stage t+1 at the start of the slot (its own
//                        half's last reads of that buffer were in M(t-1), a barrier ago), waited for
//                        (vmcnt(4)) after M(t); B rows [64wn+32, 64wn+64) of stage t+2 after its own
//                        fragment reads of stage t retired (lgkmcnt(0)), waited for (vmcnt(8)) at the
//                        end of R(t+1).
// Every ds_read of a stage comes a barrier after the issuing wave's covering vmcnt; every LDS-DMA
// into a slot comes after the barrier that follows the last reads of it (lgkmcnt(0) before each
// R-slot barrier).  Barrier counts match: lead 1 + 2nk, lag 2 + 2nk - 1.
// lab-only flags (kPP*): in-kernel stamps, ablations
// kPPLayoutF: operands in the FRAGMENT-MAJOR packed layout (1-KiB blocks of 16 rows x 64 k in MFMA lane
// order, block (rg, kb) at ((rg * (k_pad / 64)) + kb) * 1024): every LDS-DMA piece is one contiguous block,
// the LDS image is block order, and a fragment read is one contiguous 1 KiB (no swizzle needed)
enum PPFlags { kPPStamp = 1, kPPNoDma = 2, kPPNoStore = 4, kPPNtStore = 8, kPPLayoutF = 16 };
#ifdef QGEMM_LAB
__device__ unsigned long long g_pp_stamp[4096 * 6];
#endif

// LDS bytes of the ping-pong body (staging ring + scales/bias/flag)
template <int kEpi>
constexpr int pp_lds_bytes() {
    return kEpiBase + (has_bias(kEpi) ? 3072 : 2048) + (kEpi == kEpiOutlier ? kOutlierStageBytes : 0);
}

// One 256 x 256 tile (k-slice `slice` of S) of the ping-pong GEMM on a 512-thread block; `lds` holds
// pp_lds_bytes<kEpi>() bytes.  The body of gemm_i8_pp and of the fused pack+GEMM launch.
template <int kDma, int kEpi = kEpiNone, int kFlags = 0>
__device__ __forceinline__ void pp_tile_body(const GemmArgs &p, int8_t *lds, int tile, int slice, int S) {
#ifdef QGEMM_LAB
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (kFlags & kPPStamp)
            if (threadIdx.x == 0) {
                g_pp_stamp[blockIdx.x * 6 + 2 * i] = __builtin_amdgcn_s_memtime();
                g_pp_stamp[blockIdx.x * 6 + 2 * i + 1] = __builtin_amdgcn_s_memrealtime();
            }
    };
#else
    static_assert((kFlags & ~(kPPNtStore | kPPLayoutF)) == 0, "lab flags need QGEMM_LAB");
    auto stamp = [](int) {};
#endif
    stamp(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const bool lead = wm == 0;
    int tm, tn;
    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn);
    const int nk_all = (int)(p.k_pad / BK);
    const int kt0 = slice * nk_all / S;
    const int nk = (slice + 1) * nk_all / S - kt0;
    const int64_t kp = p.k_pad;
    constexpr bool kF = (kFlags & kPPLayoutF) != 0;
    const int64_t nkg = kp / 64;  // F-layout: 1-KiB blocks per 16-row group
    const int8_t *Ablk = kF ? p.A + ((int64_t)tm * 16 * nkg + (int64_t)kt0 * 2) * 1024
                            : p.A + (int64_t)tm * BM * kp + (int64_t)kt0 * BK;
    const int8_t *Bblk = kF ? p.B + ((int64_t)tn * 16 * nkg + (int64_t)kt0 * 2) * 1024
                            : p.B + (int64_t)tn * BN * kp + (int64_t)kt0 * BK;
    // piece q (8 rows x 128 B, one wave instruction) of an operand: lane l writes LDS bytes 16l.. of
    // rows 8q.., i.e. row 8q + (l>>3), slot l&7, which holds global chunk (l&7) ^ (4(q&1) + (l>>4)).
    // F-layout: piece q = block (row group q >> 1, k-block q & 1) of the k-step, copied whole
    uint32_t voff[2];
#pragma unroll
    for (int e = 0; e < 2; ++e)
        voff[e] = kF ? (uint32_t)(lane * 16)
                     : (uint32_t)((lane >> 3) * kp) + ((((lane & 7) ^ (4 * e + (lane >> 4)))) << 4);
    auto piece_src = [&](const int8_t *blk, int q, int kt) __attribute__((always_inline)) -> const int8_t * {
        if constexpr (kF) return blk + ((int64_t)(q >> 1) * nkg + (int64_t)kt * 2 + (q & 1)) * 1024 + voff[0];
        else return blk + (int64_t)q * 8 * kp + (int64_t)kt * BK + voff[q & 1];
    };
    // wave-uniform part: 8 pieces starting at piece q0 of one operand, k-step kt, into LDS at dst
    auto pieces8 = [&](const int8_t *blk, int q0, int kt, int8_t *dst) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = q0 + i;
            __builtin_amdgcn_global_load_lds((const void *)piece_src(blk, q, kt), (void *)(dst + q * 8 * BK), 16, 0, 0);
        }
    };
    auto pieces4 = [&](const int8_t *blk, int q0, int kt, int8_t *dst) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = q0 + i;  // q0 even: piece parity = i & 1
            __builtin_amdgcn_global_load_lds((const void *)piece_src(blk, q, kt), (void *)(dst + q * 8 * BK), 16, 0, 0);
        }
    };
    // mode 2: this wave's A rows (its half: lead rows 0-127, lag rows 128-255) / its B half-strip
    auto stageA_own = [&](int kt, int buf) __attribute__((always_inline)) {
        pieces4(Ablk, 16 * wm + 4 * wn, kt, lds + buf * kStageBytes);
    };
    auto stageB_half = [&](int kt, int buf) __attribute__((always_inline)) {
        pieces4(Bblk, 8 * wn + 4 * wm, kt, lds + buf * kStageBytes + kTileBytes);
    };
    auto stageA = [&](int kt, int buf) __attribute__((always_inline)) {
        pieces8(Ablk, 8 * wn, kt, lds + buf * kStageBytes);
    };
    auto stageB = [&](int kt, int buf) __attribute__((always_inline)) {
        pieces8(Bblk, 8 * wn, kt, lds + buf * kStageBytes + kTileBytes);
    };

    const int lrow = lane & 15, kq = lane >> 4, swz = (lrow >> 1) & 7;
    // F-layout image: fragment (row block, sub-step s) = block ((rows >> 4), s) = lane's 16 B at lane * 16
    const int a_row0 = kF ? wm * 128 * BK + lane * 16 : (wm * 128 + lrow) * BK;
    const int b_row0 = kF ? wn * 64 * BK + lane * 16 : (wn * 64 + lrow) * BK;
    int off[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) off[s] = kF ? s * 1024 : ((4 * s + kq) ^ swz) << 4;

    v4i acc[8][4];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = v4i{};
    // R reads sub-step 0's fragments and sub-step 1's B fragments (64 VGPRs); sub-step 1's A
    // fragments are read inside M, each into the registers of the sub-step-0 A fragment whose four
    // MFMAs were just issued (LDS reads beside the wave's own MFMAs cost the pipe nothing; the
    // 128 accumulators + fragments then fit 256 VGPRs without spills)
    v4i a0[8], b0[4], b1[4];
    auto read_r = [&](int buf) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b0[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[0]);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a0[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[0]);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b1[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[1]);
    };
    auto mfmas = [&](int buf) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * kStageBytes;
        v4i a1[8];
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        // a1[mi] is read right after row mi's MFMAs (into a0[mi]'s registers); a1[7] goes out with
        // a1[6], so the first sub-step-1 MFMA does not wait for a read issued after the last
        // sub-step-0 MFMA
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0[mi], b0[ni], acc[mi][ni], 0, 0, 0);
            if (mi < 6) a1[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[1]);
            if (mi == 6) {
                a1[6] = *reinterpret_cast<const v4i *>(la + a_row0 + 6 * 16 * BK + off[1]);
                a1[7] = *reinterpret_cast<const v4i *>(la + a_row0 + 7 * 16 * BK + off[1]);
            }
        }
#pragma unroll
        for (int mi = 0; mi < 6; ++mi) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1[mi], b1[ni], acc[mi][ni], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto barrier = []() __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: stage 0 (+ B of stage 1 in mode 1, the lag's B half of stage 1 in mode 2) -> B0
    if constexpr (kDma == 2) {
        stageA_own(0, 0);
        stageB_half(0, 0);
        if (!lead && nk > 1) {
            stageB_half(1, 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else if constexpr (kDma == 0) {
        if (lead) {
            stageA(0, 0);
            stageB(0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        if (lead) {
            stageA(0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            stageB(0, 0);
            if (nk > 1) {
                stageB(1, 1);
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
    }
    barrier();
    if (!lead) barrier();  // the lag half idles through slot 0
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        // ---- R(t)
        const bool dma = !(kFlags & kPPNoDma) || t == 0;
        if constexpr (kDma == 2) {
            if (t + 1 < nk && dma) {
                stageA_own(t + 1, cur ^ 1);
                if (lead) stageB_half(t + 1, cur ^ 1);
            }
        } else if (lead && t + 1 < nk && dma) {
            stageA(t + 1, cur ^ 1);
            if constexpr (kDma == 0) stageB(t + 1, cur ^ 1);
        }
        read_r(cur);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (kDma == 2) {
            // lag: B half of stage t+2 over the rows just read; then B half of stage t+1 must have landed
            // (the lead reads it in R(t+1), the next slot)
            if (!lead) {
                if (t + 2 < nk && !(kFlags & kPPNoDma)) {
                    stageB_half(t + 2, cur);
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                } else if (t + 1 < nk && dma) {
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
        }
        if constexpr (kDma == 1) {
            if (!lead) {
                if (t + 2 < nk && !(kFlags & kPPNoDma)) {
                    stageB(t + 2, cur);
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
        }
        barrier();
        // ---- M(t)
        mfmas(cur);
        if (lead) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier();
        } else if (t + 1 < nk) {
            if constexpr (kDma == 2) {
                // lag: its A rows of stage t+1 (issued in R(t)) land before the barrier ahead of R(t+1)
                if (t + 2 < nk && !(kFlags & kPPNoDma)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
        }
    }

    stamp(1);
    if (S > 1 && !splitk_combine<8, 4, 8>(p, reinterpret_cast<unsigned *>(lds + kEpiBase), acc, tile, slice, S, wave,
                                          lane, tid))
        return;
    epilogue16<(kFlags & kPPNoStore) ? kStoreNone : kStoreLds, kEpi, (kFlags & kPPNtStore) != 0>(p, lds, acc, tm, tn, wm,
                                                                                                 wn, lane, tid);
    stamp(2);
}

template <int kDma, int kEpi = kEpiNone, int kFlags = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_pp(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) int8_t lds[pp_lds_bytes<kEpi>()];
    const int S = p.splits > 1 ? p.splits : 1;
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = wid / S;
    pp_tile_body<kDma, kEpi, kFlags>(p, lds, tile, wid - tile * S, S);
}


}  // namespace gemm
}  // namespace qgemm
