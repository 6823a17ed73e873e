// gemm_fm_r4.h -- LAB: the round-4 gemm_i8_fm (accumulators as the MFMA computes X x W, LDS-image epilogue, 512-B
// row stores, row rotation when wide_rows) kept for same-process A/B against the round-5 product kernel.
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

// Split-K modes of gemm_i8_fm (two K slices per tile, the only split the 256-tile plan makes; the rounds 2-3
// form where both slices stored a slab, and the XCD-pair map, are lab/splitk_both_pairxcd_experiment.patch):
//   kSplitFirst : (round 4) the ticket FIRST: only the slice that arrives first stores its slab (sc1 stores,
//                 drained, block barrier) and publishes it by adding 2 to the ticket; the second arriver stores
//                 nothing, waits for the published value (ticket == 4 in either arrival order: 0 -> 1 -> 3 -> 4 or
//                 0 -> 1 -> 2 -> 4), then reads the slab with sc1 loads -- the write-through hand-off of
//                 MI355X_MICROARCH.md (row 1 of the sc1 hand-off table: one lane's agent-scope add after every
//                 storing wave's vmcnt(0) and a block barrier, an sc1 poll, sc1 loads).  Slice 0 takes kFirst64/64
//                 of the k-steps, so it normally arrives first and its slab has landed before slice 1's loop ends:
//                 one slab per tile instead of two, off the critical path.  The waiting slice never waits on a
//                 block that is not running: the first arriver has already drawn its ticket.


// kNtC: the full-tile output stores are nontemporal (C2 bench, one box, interleaved: 11 598 vs 11 431 GEMMs/s, GEMM
// 58.2 vs 59.5 us by events; profiles/r03_ab_nt_c.log) -- the 64-MiB tail streams past the caches
template <int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>
__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm_r4(GemmArgs p) {
    static_assert(!(kI32 && kEpi != kEpiNone), "raw accumulators take no epilogue extras");
    static_assert(!(kI32 && kSplit), "raw accumulators are not split");
    static_assert(!(kEpi == kEpiOutlier && kSplit), "the outlier epilogue runs on unsplit plans");
    constexpr int TS = 132;                 // padded row of a wave's epilogue block (conflict-free ds_write)
    constexpr int kBlockBytes = 64 * TS * 4;
    __shared__ __attribute__((aligned(16))) int8_t lds[4 * kBlockBytes + 2048 + 16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    // XCD remap first, then tile = id / S, slice = id % S (split-K: a tile's slices share an XCD).  Measured
    // alternative (FFN down, kernel trace): XCD pairs taking one 4 x 8 patch of tiles for K half 0 / 1 cut the
    // operand fetch 404.7 -> 337.6 MB but ran 127.3 us vs 122-126 (the slab then crosses XCDs)
    const int S = kSplit ? 2 : 1;  // the 256-tile plan splits in two or not at all (host checks)
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = wid / S, slice = wid - tile * S;
    int tm, tn;
    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn);
    const int nsub = (int)(p.k_pad / 64);
    // this slice's sub-steps [u0, u0 + nloc) of the nsub 64-deep k-blocks (kSplitFirst: slice 0 the shorter one)
    int cut = slice * nsub / S, end = (slice + 1) * nsub / S;
    if constexpr (kSplit == kSplitFirst) {
        const int n0 = min(max(nsub * kFirst64 / 64, 1), nsub - 1);
        cut = slice ? n0 : 0;
        end = slice ? nsub : n0;
    }
    const int u0 = __builtin_amdgcn_readfirstlane(cut);
    const int nloc = __builtin_amdgcn_readfirstlane(end - cut);
    // this wave's half panels: 8 row groups x nsub blocks each (= 128 packed rows), from block u0 on
    const int half_bytes = 8 * nsub * 1024 - u0 * 1024;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.A + (((int64_t)tm * 16 + wm * 8) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int8_t *>(uniform_ptr(p.B + (((int64_t)tn * 16 + wn * 8) * nsub + u0) * 1024)), 0,
        __builtin_amdgcn_readfirstlane(half_bytes), 0x00020000);
    const int voff = lane * 16;
    // kEpiOutlier: the outlier-column count (device-side) and the lane's columns of the first two f32-MFMA steps
    // (t = 4 tt + kq), read before the k-loop so the epilogue's operand loads do not wait on them
    const int ocnt = kEpi == kEpiOutlier ? __builtin_amdgcn_readfirstlane(*p.ocount) : 0;
    int ocol[2] = {0, 0};
    if constexpr (kEpi == kEpiOutlier) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) ocol[tt] = 4 * tt + (lane >> 4) < ocnt ? p.ocols[4 * tt + (lane >> 4)] : 0;
    }

    v4i acc[8][8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = v4i{};
    v4i a0[8], b0[8], a1[8], b1[8], a2[8], b2[8];
    // fragment loads of sub-step u: j < 8 -> B block (row group j of the half, k-block u), else A
    auto ld = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int u) __attribute__((always_inline)) {
        const int soff = ((j & 7) * nsub + u) * 1024;
        if (j < 8) fb[j] = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, soff, 0);
        else fa[j - 8] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, soff, 0);
    };
    // MFMAs on (ca, cb), loads of sub-step un into (na, nb); in the main loop the loads are unconditional
    // (index clamped to the last sub-step: a conditional register load makes hipcc keep both values alive
    // across the loop and spill a register set)
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
    const int rest = nloc - u;  // 0, 1 or 2: sets 0 and 1 hold sub-steps u, u+1
    if (rest > 0) {
        substep(a0, b0, a2, b2, 0, false);
        if (rest > 1) substep(a1, b1, a2, b2, 0, false);
    }
    // the last MFMAs' results are read by VALU below; the asm statements hide them from hipcc's padding
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    if constexpr (kSplit == kSplitFirst) {
        unsigned *last = reinterpret_cast<unsigned *>(lds + 4 * kBlockBytes + 2048);
        if (tid == 0) *last = __hip_atomic_fetch_add(p.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (*last == 0u) {
            // first arriver: this slice's sums to the tile's ONE slab (write-through), then publish
            constexpr int kSlabBytes = 4 * 8 * 8 * 64 * 16;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char *>(p.slabs) + (int64_t)tile * kSlabBytes,
                                                              0, kSlabBytes, 0x00020000);
            const int lane_off = (wave * 64 * 64 + lane) * 16;
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                for (int ni = 0; ni < 8; ++ni)
                    __builtin_amdgcn_raw_buffer_store_b128(acc[mi][ni], rs, lane_off + (mi * 8 + ni) * 1024, 0, 16 /* sc1 */);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(p.tickets + tile, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        // second arriver: wait for the published slab (its producer drew its ticket before this block did)
        if (tid == 0) {
            while (__hip_atomic_load(p.tickets + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 4u)
                __builtin_amdgcn_s_sleep(2);
            if (p.reset_tickets) __hip_atomic_store(p.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: slab loads stay below
    }

    const int gi0 = tm * BM, gj0 = tn * BN;
    const int lrow = lane & 15, kq = lane >> 4;
    const int r0 = wm * 128, c0 = wn * 128;
    // kEpiOutlier: the operands of the first 8 outlier columns (two f32-MFMA steps) for both halves, loaded
    // together here so their latency is paid once: ow[step][ni] = W[col_t][j], ox[half][mq][step] = X[row][col_t]
    // with t = 4 step + kq; +0 / -0 past the count (see below)
    float ox[2][4][2], ow[2][8];
    if constexpr (kEpi == kEpiOutlier) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            const int t = 4 * tt + kq;
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const int j = gj0 + c0 + ni * 16 + lrow;
                ow[tt][ni] = t < ocnt ? (j < p.n ? p.wo[(int64_t)ocol[tt] * p.wo_ld + j] : 0.0f) : -0.0f;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int mq = 0; mq < 4; ++mq) {
                    const int i = gi0 + r0 + 64 * h + mq * 16 + lrow;
                    ox[h][mq][tt] = t < ocnt && i < p.m ? p.xo[(int64_t)i * p.xo_ld + ocol[tt]] : 0.0f;
                }
        }
    }
    float *sCx = reinterpret_cast<float *>(lds + 4 * kBlockBytes);
    float *sCw = sCx + BM;
    if constexpr (!kI32) {
        sCx[tid] = p.Cx[gi0 + tid];  // scales are padded to the 256-row tiles
        sCw[tid] = p.Cw[gj0 + tid];
    }
    __syncthreads();
    float *T = reinterpret_cast<float *>(lds + wave * kBlockBytes);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n && gi0 + BM <= p.m;
    // row-pair rotation of the full-tile stores (lab/w4_lab.hip `stride` mode, profiles/r03_f4_store_order_lab.log:
    // FFN-up output, 64-KiB rows, 121.6 -> 118.2 us; at 16-KiB rows it cost the 8192-row shard 2 us, hence host-set)
    const int rot = __builtin_amdgcn_readfirstlane(p.wide_rows ? ((tn * 7 + tm * 3) & 31) : 0);
    // the scales (and bias) into registers first: T and the scales share the one LDS array, so a scale read
    // between T stores would be re-issued and waited for after every store
    float cwv[8], bv[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
        cwv[ni] = kI32 ? 0.0f : sCw[c0 + ni * 16 + lrow];
        const int j = gj0 + c0 + ni * 16 + lrow;
        bv[ni] = has_bias(kEpi) && j < p.n ? p.bias[j] : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        // split-K reducer: the other slice's partial sums of this half (32 sc1 loads in flight, then the adds)
        v4i oth[4][8];
        if constexpr (kSplit) {
            constexpr int kSlabBytes = 4 * 8 * 8 * 64 * 16;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<char *>(p.slabs) + (int64_t)tile * kSlabBytes, 0, kSlabBytes, 0x00020000);
            const int lane_off = (wave * 64 * 64 + lane) * 16;
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int ni = 0; ni < 8; ++ni)
                    oth[mq][ni] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + ((4 * s + mq) * 8 + ni) * 1024,
                                                                        0, 16 /* sc1 */);
        }
        float cxv[4][4];
#pragma unroll
        for (int mq = 0; mq < 4; ++mq)
#pragma unroll
            for (int r = 0; r < 4; ++r) cxv[mq][r] = kI32 ? 0.0f : sCx[r0 + 64 * s + mq * 16 + 4 * kq + r];
        if constexpr (kEpi == kEpiOutlier) {
            // O = fl(O8 + Co), Co = the fp32 chain over the outlier columns from +0 in ascending t of
            // xo[i][t] * wo[t][j], on v_mfma_f32_16x16x4_f32 (its result is that k-ordered chain bit for bit,
            // as in the fp32 GEMMs): 4 columns per MFMA, D laid out as the int32 accumulators, one 16-row
            // block of the half at a time.  A step past the count multiplies +0 by -0: fma(+0, -0, c) = c for
            // every c, -0 included (+0 * +0 would turn a -0 sum into +0).
            // The first 8 columns' operands were loaded once, ahead of both halves (ox / ow); columns past 8
            // load per step.
            typedef float v4f_t __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int mq = 0; mq < 4; ++mq) {
                v4f_t oc[8];
#pragma unroll
                for (int ni = 0; ni < 8; ++ni) oc[ni] = v4f_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
                    if (4 * tt < ocnt)
#pragma unroll
                        for (int ni = 0; ni < 8; ++ni)
                            oc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(ox[s][mq][tt], ow[tt][ni], oc[ni], 0, 0, 0);
                const int ia = gi0 + r0 + 64 * s + mq * 16 + lrow;  // the A-operand row of this lane
#pragma unroll 1
                for (int t0 = 8; t0 < ocnt; t0 += 4) {
                    const int t = t0 + kq;  // the lane's k within the MFMA step
                    const int col = t < ocnt ? p.ocols[t] : 0;
                    const float xa = t < ocnt && ia < p.m ? p.xo[(int64_t)ia * p.xo_ld + col] : 0.0f;
                    float wb[8];
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) {
                        const int j = gj0 + c0 + ni * 16 + lrow;
                        wb[ni] = t < ocnt ? (j < p.n ? p.wo[(int64_t)col * p.wo_ld + j] : 0.0f) : -0.0f;
                    }
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) oc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, wb[ni], oc[ni], 0, 0, 0);
                }
                // no outlier column (count 0, wave-uniform): O = O8 with no add, as the oracle (qgemm_oracle.c
                // oracle_mm_outlier skips it) -- fl(-0 + +0) would turn an O8 of -0 into +0
#pragma unroll
                for (int ni = 0; ni < 8; ++ni)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float o8 = dequantize(acc[4 * s + mq][ni][r], outer_product(cxv[mq][r], cwv[ni]), p.inv_r2);
                        T[(mq * 16 + 4 * kq + r) * TS + ni * 16 + lrow] = ocnt > 0 ? __fadd_rn(o8, oc[ni][r]) : o8;
                    }
            }
        } else {
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int jl = ni * 16 + lrow;
#pragma unroll
            for (int mq = 0; mq < 4; ++mq)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int il = mq * 16 + 4 * kq + r;
                    float o;
                    if constexpr (kI32) {
                        o = __int_as_float(acc[4 * s + mq][ni][r]);  // the raw bits travel through LDS
                    } else {
                        const int a = kSplit ? acc[4 * s + mq][ni][r] + oth[mq][ni][r] : acc[4 * s + mq][ni][r];
                        o = dequantize(a, outer_product(cxv[mq][r], cwv[ni]), p.inv_r2);
                        if constexpr (has_bias(kEpi)) o = __fadd_rn(o, bv[ni]);
                        if constexpr (kEpi == kEpiBiasRelu) o = (o < 0.0f) ? 0.0f : o;
                    }
                    T[il * TS + jl] = o;
                }
        }
        }
        // the wave's own block: its ds_writes precede its ds_reads (one wave's LDS ops stay in order)
        const int c4 = (lane & 31) * 4;
        float *C = static_cast<float *>(p.C);
        if (full) {
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * ((it + rot) & 31) + (lane >> 5);
                const float4 v = *reinterpret_cast<const float4 *>(T + rr * TS + c4);
                float4 *dst = reinterpret_cast<float4 *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + c0 + c4);
                if constexpr (kNtC) {
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
}


}  // namespace gemm
}  // namespace qgemm
