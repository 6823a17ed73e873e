// gemm_i8_kernels.h -- the int8 MFMA GEMM kernels of the library (included by gemm_i8.hip and the lab harnesses).
//
// C[i,j] = dequant(sum_k A[i,k] * B[j,k]) with A = Xq [m_pad][k_pad], B = Wq^T [n_pad][k_pad]: the packed operands,
// k-contiguous, zero padded, stored FRAGMENT-MAJOR (qgemm_internal.h fofs: 1-KiB blocks of 16 rows x 64 k in the
// lane order of one v_mfma_i32_16x16x64_i8 operand).  Every kernel here reads that layout:
//   gemm_i8_fm      256 x 256 tiles, 4 waves of 128 x 128, operands straight to VGPRs, AGPR accumulators, fused
//                   dequant epilogue (+ bias / relu / the LLM.int8() outlier chain), optional 2-way split-K;
//   gemm_i8_small   TB x TB tiles (TB = 64 or 32) for few-tile shapes, LDS-DMA ring, split-K by tickets.
// The row-major kernels of rounds 1-2 (gemm_i8_v1/v3, the ping-pong gemm_i8_pp) live in lab/gemm_legacy.h.
#pragma once

#include "qgemm_internal.h"

namespace qgemm {
namespace gemm {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BK = 128;

static_assert(BM == kRowPad && BN == kRowPad && BK == kKPad, "packed layout must match the macro-tile");


// Block -> macro-tile.  Blocks b and b+8 are dispatched to the same XCD; give each XCD a contiguous
// range of logical ids (bijective for any grid size), then walk logical ids in groups of kGroupM
// tile-rows so one XCD's range covers a compact patch (shared A and B panels stay in its L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void group_tiles(int wgid, int tiles_m, int tiles_n, int &tm, int &tn, int kGroupM = 4) {
    const int per_group = kGroupM * tiles_n;
    const int group = wgid / per_group;
    const int first_m = group * kGroupM;
    const int gsz = min(tiles_m - first_m, kGroupM);
    const int w = wgid - group * per_group;
    tm = first_m + w % gsz;
    tn = w / gsz;
}

__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int &tm, int &tn) {
    group_tiles(xcd_remap(bid, nwg), tiles_m, tiles_n, tm, tn);
}

struct GemmArgs {
    const int8_t *A;
    const int8_t *B;
    const float *Cx;
    const float *Cw;
    void *C;
    int64_t csh, csw;
    int m, n;
    int64_t k_pad;
    int tiles_m, tiles_n;
    float inv_r2;
    // split-K (splits > 1): slice s of a tile runs k-steps [s*nk/S, (s+1)*nk/S); every slice stores its
    // int32 accumulators to slabs[tile][s] and draws a ticket; the last arriver sums the slabs (exact
    // integer addition, so any split gives bit-identical results) and runs the epilogue.
    int splits;
    int32_t *slabs;     // tiles x splits x (BM x BN) int32, MFMA-native order
    unsigned *tickets;  // tiles words, zeroed before every launch
    const float *bias;  // n floats, added after the dequantize (kEpi >= 1)
    int reset_tickets;  // the reducer re-zeroes its ticket (scratch zeroed once at allocation)
    // kEpiOutlier: the chain's operands where they lie -- xo = X (m x k, row stride xo_ld), wo = W (k x n, row stride
    // wo_ld) -- at the outlier columns ocols[0 .. cnt) (ascending), cnt = *ocount on the device
    const float *xo;
    const float *wo;
    const int *ocount;
    int64_t wo_ld;
    // gemm_i8_fm's full-tile stores for output rows of >= 64 KiB (set by the host): through a per-wave LDS image as
    // 512-B row segments in a per-tile rotated order; narrower rows take the paired register stores (see gemm_i8_fm)
    int wide_rows;
    int64_t xo_ld;
    const int *ocols;
};

// Epilogue extras for the encoder's linears (linear.cuh:52-54 then op_relu, transformer.cu:66):
// y = fl(O + b[j]) then relu(y) = (y < 0 ? 0 : y) -- each its own rounding, as the separate launches.
// kEpiOutlier: the LLM.int8() decomposition's fp32 part, O = fl(O8 + fmaf chain over the outlier
// columns in ascending k of xo[i][t] * wo[t][j]) (outlier.hip; the oracle's oracle_mm_outlier)
enum EpiMode { kEpiNone = 0, kEpiBias = 1, kEpiBiasRelu = 2, kEpiOutlier = 3 };
constexpr bool has_bias(int e) { return e == kEpiBias || e == kEpiBiasRelu; }


template <int kEpi>
__device__ __forceinline__ float epi_extra(float o, const float *sB, int jl) {
    if constexpr (has_bias(kEpi)) o = __fadd_rn(o, sB[jl]);
    if constexpr (kEpi == kEpiBiasRelu) o = (o < 0.0f) ? 0.0f : o;
    return o;
}

// ------------------------------------------------------------------------------------------------
// In-launch split-K combine of gemm_i8_small (cdna_hip_programming.md s5 "In-launch split-K reduction", the counter
// form of s6 Guideline 16), WRITE-THROUGH form: there is deliberately NO release fence and NO acquire
// fence (do not add them back: a buffer_wbl2 also writes back every dirty line of the XCD's L2 --
// other blocks' output tiles included -- and cost 14 us at 2048^3 split 2).  Instead
// every slab byte is stored with sc1 (write-through) 16-B buffer stores, every storing wave drains
// them (s_waitcnt vmcnt(0)) before the block barrier, lane 0 then draws the arrival ticket with a
// relaxed agent-scope atomic add, and the slice that draws S-1 is the reducer, which reads the other
// slabs with sc1 buffer loads (EVERY load of them).  Correct for any placement of a tile's slices over
// XCDs/CUs (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores drained before the counter,
// sc1 loads after it).  The "last arriver" word goes through the one LDS array (a second __shared__
// object can de-pipeline the main loop).  Returns true in the reducer, which then holds the complete
// sums in acc.
// MI x NI accumulator tiles per wave, kWaves waves: a slab is kWaves*MI*NI*64 v4i (= the tile's int32s).
template <int MI, int NI, int kWaves, bool kSlab = true>
__device__ __forceinline__ bool splitk_combine(const GemmArgs &p, unsigned *last, v4i (&acc)[MI][NI], int tile,
                                               int slice, int S, int wave, int lane, int tid) {
    constexpr int kSlabBytes = kWaves * MI * NI * 64 * 16;
    // one descriptor over this tile's S slabs (wave-uniform base)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char *>(p.slabs) + (int64_t)tile * S * kSlabBytes, 0, S * kSlabBytes, 0x00020000);
    const int lane_off = (wave * (MI * NI * 64) + lane) * 16;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
            if constexpr (kSlab) __builtin_amdgcn_raw_buffer_store_b128(acc[mi][ni], rsrc, slice * kSlabBytes + lane_off + (mi * NI + ni) * 1024,
                                                   0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned t = __hip_atomic_fetch_add(p.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = t;
        // every slice has arrived: nobody else touches this ticket in this launch
        if (t == (unsigned)(S - 1) && p.reset_tickets)
            __hip_atomic_store(p.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (*last != (unsigned)(S - 1)) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: loads stay below
    for (int s = 0; s < S; ++s) {
        if (s == slice || !kSlab) continue;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
                acc[mi][ni] += __builtin_amdgcn_raw_buffer_load_b128(rsrc, s * kSlabBytes + lane_off + (mi * NI + ni) * 1024,
                                                                     0, 16 /* sc1 */);
    }
    return true;
}

// ------------------------------------------------------------------------------------------------
// gemm_i8_fm: the product 256 x 256 tile (round 3).  4 waves (one per SIMD), each a 128 x 128 wave tile =
// 8 x 8 v_mfma_i32_16x16x64_i8 accumulators (256 registers, pinned in AGPRs: every MFMA is an inline-asm
// statement with its accumulator as a tied "+a" operand -- hipcc's builtin form kept them in AGPRs but
// moved them around the loop, lab gemm_variants.h v9), operands streamed from the FRAGMENT-MAJOR packed
// layout (qgemm_internal.h fofs) straight into VGPRs: one MFMA operand = one contiguous 1-KiB
// buffer_load_dwordx4.  No LDS and no barrier in the main loop: three register sets, sub-step u computes
// while u+1 and u+2 are in flight (hipcc's counted vmcnt waits).  The two waves that share an A (B) half
// read the same blocks (L1).  Measured against the ping-pong kernel (lab/w4_lab.hip, 4096^3, 5 boxes, bit-
// identical): 58.3-62.3 vs 62.7-64.9 us; its main loop holds 1.90-1.97 GHz (no LDS traffic) vs 1.77-1.83.
// The MFMAs take the W fragment as their first operand and the X fragment as their second, so each accumulator
// tile is C^T: lane (kq = lane >> 4, c = lane & 15) of tile (mi, ni) holds C[row 16 mi + c][columns 16 ni + 4 kq
// .. + 3] -- four consecutive columns of one row.  The epilogue dequantizes on packed f32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: the scalar roundings, two elements per instruction) and stores from registers, no LDS image:
// rows < 64 KiB exchange tiles ni, ni + 1 between lanes c and c ^ 8 (DPP row_ror:8) so one nontemporal store writes
// 8 rows x 128 B; wider rows (FFN up) go through a per-wave LDS image (one 16-B write per tile and lane) and leave as
// nontemporal 512-B row segments, each tile in its own rotated row order.  Lab (lab/ds_lab.hip,
// profiles/r05_ds_lab.log, same box, interleaved, bit-identical): 4096^3 57.76 -> 56.30 us (round-4 LDS epilogue ->
// paired register stores), the 8192-row shard 112.0 -> 110.0; FFN up's LDS image 120.45 vs 119.64 for round 4 (plain
// register stores ran 112.3 there but left the output in the caches: the whole call -6.4 %, profiles/
// r05_ab_epilogue.log).  The store tail is HBM-bound: the epilogue's arithmetic alone ends 1.7 us after the loop.
// kI32: the raw int32 accumulators (qgemm_mm_packed_i32) instead of the dequantized fp32.
__device__ __forceinline__ void mfma_agpr(v4i &acc, const v4i &a, const v4i &b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// a pointer the compiler can PROVE wave-uniform (cdna_hip_programming.md T20: a buffer descriptor built
// from anything it cannot prove uniform gets a waterfall loop around every buffer op)
__device__ __forceinline__ const int8_t *uniform_ptr(const int8_t *q) {
    const uint64_t v = reinterpret_cast<uint64_t>(q);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const int8_t *>(((uint64_t)hi << 32) | lo);
}

constexpr int kFmThreads = 256;

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
enum SplitMode { kSplitNone = 0, kSplitFirst = 2 };

// kNtC: the paired full-tile output stores (rows < 64 KiB) are nontemporal -- the 64-MiB tail streams past the
// caches (lab/ds_lab.hip: dsPn 56.30 vs plain pairs 56.99 us at 4096^3).  The wide-row LDS-image stores are
// nontemporal in every instantiation (qgemm_mm_packed_i32, the one kNtC = false caller, never sets wide_rows).
template <int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>
__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm(GemmArgs p) {
    static_assert(!(kI32 && kEpi != kEpiNone), "raw accumulators take no epilogue extras");
    static_assert(!(kI32 && kSplit), "raw accumulators are not split");
    static_assert(!(kEpi == kEpiOutlier && kSplit), "the outlier epilogue runs on unsplit plans");
    // the one LDS array: the tile's scales (Cx of its 256 rows, Cw of its 256 columns), the split-K ticket word,
    // (wide rows) each wave's padded [64][TS] image of half its quadrant, (kEpiOutlier) the chain's operands
    constexpr int TS = 132;  // padded image row (16-B aligned, conflict-free 16-B writes of 16 rows)
    // (kEpiOutlier) stage rows of OS floats: the 4 k-groups of a wave read rows t = 4 tt + kq at the same offsets,
    // so a row stride of BM would put them on the same banks
    constexpr int OS = BM + 16;
    constexpr int kOutlierStage = kEpi == kEpiOutlier ? 2 * 8 * OS : 0;
    __shared__ __attribute__((aligned(16))) float sS[2 * BM + 4 + 4 * 64 * TS + kOutlierStage];
    float *const sO = sS + 2 * BM + 4 + 4 * 64 * TS;  // [8][OS] X values, then [8][OS] W values
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
    // wide output rows (FFN up): groups of 8 tile-rows -- each XCD's patch 8 x 8 tiles instead of 4 x 16 (lab/epi_lab.hip,
    // profiles/r06_epi_lab.log: FFN-up GEMM 114.7-115.1 -> 110.2-110.6 us with the LDS-image stores, the whole call
    // +0.9 %; the reads are not the difference: without stores FFN up and the 8192-row shard both run 93.6 us).  Not
    // in the outlier epilogue's instantiation: there the runtime group size made hipcc move its accumulators (+186
    // v_accvgpr_mov, c2_outlier's GEMM 58.9 -> 61.8 us, same box)
    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn, kEpi != kEpiOutlier && p.wide_rows ? 8 : 4);
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
    const int gi0 = tm * BM, gj0 = tn * BN;
    // the scales are loaded first (scales are padded to the 256-row tiles): their latency hides under the operand
    // prologue, and they reach LDS before the k-loop.  (LDS-DMA here instead makes hipcc wait for vmcnt(0) before
    // the first MFMA: it orders the inline-asm MFMAs behind every pending LDS-DMA write.)
    const float sx = kI32 ? 0.0f : p.Cx[gi0 + tid], sw = kI32 ? 0.0f : p.Cw[gj0 + tid];
    // kEpiOutlier: the outlier-column count (device-side) and the operands of the chain's first 8 columns for this
    // tile -- X[row][col_t] of its 256 rows, W[col_t][j] of its 256 columns, +0 / -0 past the count (see the
    // epilogue) -- gathered first and staged in LDS after the operand prologue is in flight, so the epilogue reads
    // them from LDS and never waits on their latency (X's columns come from HBM: the pack streamed X past the caches)
    const int ocnt = kEpi == kEpiOutlier ? __builtin_amdgcn_readfirstlane(*p.ocount) : 0;
    float oxv[8], owv[8];
    if constexpr (kEpi == kEpiOutlier) {
        const int64_t i = gi0 + tid;
        const int j = gj0 + tid;
        // the column list through the constant address space: scalar loads (a vector load here would make every
        // column's gather wait for the ones before it)
        const __attribute__((address_space(4))) int *ocs = (const __attribute__((address_space(4))) int *)p.ocols;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int col = t < ocnt ? ocs[t] : 0;
            oxv[t] = t < ocnt && i < p.m ? p.xo[i * p.xo_ld + col] : 0.0f;
            owv[t] = t < ocnt ? (j < p.n ? p.wo[(int64_t)col * p.wo_ld + j] : 0.0f) : -0.0f;
        }
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
            // W first: the tile comes out C^T.  The row's two fragment loads go out before its MFMAs 2 and 6
            // (lab/ds_lab.hip + lab/gemm_fm_var.h, profiles/r05_ds_lab.log runs 8-10, same box, interleaved: both
            // after the row's 8 MFMAs (rounds 3-4) 57.2-57.8 us at 4096^3; after MFMAs 4 and 8 56.4, 109.4 at the
            // 8192-row shard; before MFMAs 0 / 1 / 2 / 3 and + 4: 56.1 / 55.2 / 55.1 / 55.2, shard 106.9-107.2)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                if (more && ni == 2) ld(na, nb, 2 * mi, un);
                if (more && ni == 6) ld(na, nb, 2 * mi + 1, un);
                mfma_agpr(acc[mi][ni], cb[ni], ca[mi]);
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
    if constexpr (kEpi == kEpiOutlier) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            sO[t * OS + tid] = oxv[t];
            sO[(8 + t) * OS + tid] = owv[t];
        }
    }
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
        unsigned *last = reinterpret_cast<unsigned *>(sS + 2 * BM);
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
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: slab loads stay below
    }
    __syncthreads();  // the scale image (and the split-K hand-off above)

    // lane (kq, c) of tile (mi, ni): row 16 mi + c, columns 16 ni + 4 kq .. + 3 of the wave's 128 x 128 quadrant
    const int c = lane & 15, kq = lane >> 4;
    const int r0 = wm * 128, c0 = wn * 128;
    // kEpiOutlier: the operands of the first 8 outlier columns (two f32-MFMA steps) from the LDS stage:
    // ow[step][ni] = W[col_t][j] (j = 16 ni + c), ox[mi][step] = X[row 16 mi + c][col_t], t = 4 step + kq
    float ox[8][2], ow[2][8];
    if constexpr (kEpi == kEpiOutlier) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            const int t = 4 * tt + kq;
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) ow[tt][ni] = sO[(8 + t) * OS + c0 + 16 * ni + c];
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) ox[mi][tt] = sO[t * OS + r0 + 16 * mi + c];
        }
    }
    typedef float v2f __attribute__((ext_vector_type(2)));
    typedef float v4f __attribute__((ext_vector_type(4)));
    // the scales (and bias) into registers
    float cx[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) cx[mi] = sS[r0 + 16 * mi + c];
    v4f cw[8], bv[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
        cw[ni] = *reinterpret_cast<const v4f *>(sS + BM + c0 + 16 * ni + 4 * kq);
        const int j = gj0 + c0 + 16 * ni + 4 * kq;
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = has_bias(kEpi) && j + r < p.n ? p.bias[j + r] : 0.0f;
    }
    const v2f inv2 = {p.inv_r2, p.inv_r2};
    const v2f zero2 = {0.0f, 0.0f};
    float *C = static_cast<float *>(p.C);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) &&
                      gj0 + BN <= p.n && gi0 + BM <= p.m;
    const bool pairs = full && !p.wide_rows;
    const bool image = full && p.wide_rows;
    const bool lo = c < 8;
    float *T = sS + 2 * BM + 4 + wave * 64 * TS;  // this wave's image (wide rows)
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
#pragma unroll
        for (int mq = 0; mq < 4; ++mq) {
            const int mi = 4 * s + mq;
            // kEpiOutlier: Co = the fp32 chain over the outlier columns from +0 in ascending t of xo[i][t] *
            // wo[t][j], on v_mfma_f32_16x16x4_f32 (its result is that k-ordered chain bit for bit, as in the fp32
            // GEMMs): 4 columns per MFMA, W first so D is laid out as the int32 accumulators, one 16-row block at a
            // time.  A step past the count multiplies -0 by +0: fma(-0, +0, c) = c for every c, -0 included (+0 *
            // +0 would turn a -0 sum into +0).  The first 8 columns' operands were loaded once (ox / ow); columns
            // past 8 load per step.
            v4f oc[8];
            if constexpr (kEpi == kEpiOutlier) {
#pragma unroll
                for (int ni = 0; ni < 8; ++ni) oc[ni] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
                    if (4 * tt < ocnt)
#pragma unroll
                        for (int ni = 0; ni < 8; ++ni)
                            oc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(ow[tt][ni], ox[mi][tt], oc[ni], 0, 0, 0);
                const int ia = gi0 + r0 + 16 * mi + c;  // the B-operand row (X row) of this lane
#pragma unroll 1
                for (int t0 = 8; t0 < ocnt; t0 += 4) {
                    const int t = t0 + kq;  // the lane's k within the MFMA step
                    const int col = t < ocnt ? p.ocols[t] : 0;
                    const float xa = t < ocnt && ia < p.m ? p.xo[(int64_t)ia * p.xo_ld + col] : 0.0f;
                    float wb[8];
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) {
                        const int j = gj0 + c0 + ni * 16 + c;
                        wb[ni] = t < ocnt ? (j < p.n ? p.wo[(int64_t)col * p.wo_ld + j] : 0.0f) : -0.0f;
                    }
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) oc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[ni], xa, oc[ni], 0, 0, 0);
                }
            }
            // the four outputs of tile (mi, ni) in this lane: O = fl(fl(float(acc) * (fl(Cx * Cw) + 0)) * inv_r2) on
            // packed pairs (-ffp-contract=off: no contraction), then the epilogue extras
            auto tile_out = [&](int ni) __attribute__((always_inline)) -> v4f {
                v4i a = acc[mi][ni];
                if constexpr (kSplit) a += oth[mq][ni];
                if constexpr (kI32) return v4f{__int_as_float(a[0]), __int_as_float(a[1]), __int_as_float(a[2]),
                                               __int_as_float(a[3])};  // the raw bits
                const v2f x = {cx[mi], cx[mi]};
                const v2f o01 = x * v2f{cw[ni][0], cw[ni][1]} + zero2, o23 = x * v2f{cw[ni][2], cw[ni][3]} + zero2;
                const v2f d01 = (v2f{(float)a[0], (float)a[1]} * o01) * inv2;
                const v2f d23 = (v2f{(float)a[2], (float)a[3]} * o23) * inv2;
                v4f o = {d01[0], d01[1], d23[0], d23[1]};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (has_bias(kEpi)) o[r] = __fadd_rn(o[r], bv[ni][r]);
                    if constexpr (kEpi == kEpiBiasRelu) o[r] = (o[r] < 0.0f) ? 0.0f : o[r];
                    // no outlier column (count 0, wave-uniform): O = O8 with no add, as the oracle
                    // (qgemm_oracle.c oracle_mm_outlier skips it) -- fl(-0 + +0) would turn an O8 of -0 into +0
                    if constexpr (kEpi == kEpiOutlier) o[r] = ocnt > 0 ? __fadd_rn(o[r], oc[ni][r]) : o[r];
                }
                return o;
            };
            const int64_t row = gi0 + r0 + 16 * mi + c;
#pragma unroll
            for (int np = 0; np < 4; ++np) {
                const v4f o0 = tile_out(2 * np), o1 = tile_out(2 * np + 1);
                if (pairs) {
                    // tiles 2 np and 2 np + 1 exchanged between lanes c and c ^ 8 (DPP row_ror:8): rows 16 mi + (c & 7)
                    // take store 1, rows 16 mi + 8 + (c & 7) store 2, each 8 rows x 128 B
                    v4f x1, x2;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float r0v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(o0[e]), 0x128, 0xf, 0xf, false));
                        const float r1v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(o1[e]), 0x128, 0xf, 0xf, false));
                        x1[e] = lo ? o0[e] : r1v;
                        x2[e] = lo ? r0v : o1[e];
                    }
                    const int64_t ra = gi0 + r0 + 16 * mi + (c & 7);
                    const int jc = gj0 + c0 + 32 * np + (lo ? 0 : 16) + 4 * kq;
                    v4f *d1 = reinterpret_cast<v4f *>(C + ra * p.csh + jc);
                    v4f *d2 = reinterpret_cast<v4f *>(C + (ra + 8) * p.csh + jc);
                    if constexpr (kNtC) {
                        __builtin_nontemporal_store(x1, d1);
                        __builtin_nontemporal_store(x2, d2);
                    } else {
                        *d1 = x1;
                        *d2 = x2;
                    }
                } else if (image) {
                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TS + 32 * np + 4 * kq) = o0;
                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TS + 32 * np + 16 + 4 * kq) = o1;
                } else {
                    const int j = gj0 + c0 + 32 * np + 4 * kq;  // tile 2 np; tile 2 np + 1 at j + 16
                    if (row < p.m) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            if (j + e < p.n) C[row * p.csh + (int64_t)(j + e) * p.csw] = o0[e];
                            if (j + 16 + e < p.n) C[row * p.csh + (int64_t)(j + 16 + e) * p.csw] = o1[e];
                        }
                    }
                }
            }
        }
        if (image) {
            // wide rows: the half's 64 rows read back from the wave's own image (one wave's LDS operations stay in
            // order) and stored as 512-B row segments, nontemporal: plain stores there leave the 128-MiB FFN-up output
            // in the caches and the next call's pack ran 15 us longer (same box, profiles/r05_ab_epilogue.log).  Each
            // tile starts its row-pair loop at its own offset (its rows otherwise meet the other tiles' on the same
            // memory channels; lab/rot_lab.hip, round 4: 122.3 -> 117.8 us).  Round 6, with the 8-tile-row XCD patches
            // (lab/epi_lab.hip rot*, profiles/r06_epi_lab.log run 4, both orders): (tn * 13 + tm * 7) 112.6 us against
            // the round-4 formula (tn * 7 + tm * 3) 113.9-114.0, no rotation 117.0-117.3
            const int rot = __builtin_amdgcn_readfirstlane((tn * 13 + tm * 7) & 31);
            const int c4 = (lane & 31) * 4;
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * ((it + rot) & 31) + (lane >> 5);
                const v4f v = *reinterpret_cast<const v4f *>(T + rr * TS + c4);
                __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + c0 + c4));
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// gemm_i8_small<TB>: TB x TB macro-tiles (TB = 128 or 64) for problems with few 256 x 256 tiles (the
// encoder's M = 512 linears, decode-sized M): 4 waves as 2 x 2, each (TB/2) x (TB/2) = MI x MI tiles
// of v_mfma_i32_16x16x64_i8, operands staged by LDS-DMA of whole 1-KiB fragment-major blocks (2-deep or
// deeper ring), split-K by splitk_combine; the epilogue writes the whole TB x TB fp32 tile through
// the ring at once.  TB = 128: 64-KiB ring, two blocks per CU; TB = 64: 32-KiB ring, four blocks per
// CU -- four times the tiles, so shapes whose 128-tiles leave most CUs idle spread over the chip.
// kDepth > 2: a kDepth-stage ring with kDepth - 1 k-steps in flight (each k-step then waits for the
// OLDEST stage only): these few-k-step GEMMs are bound by the LDS-DMA round trip, not by the MFMAs.
template <int TB, int kDepth = 2>
struct SmallTile {
    static constexpr int kThreads = 256;
    static constexpr int WT = TB / 2;                // wave tile rows = cols
    static constexpr int MI = WT / 16;               // 16 x 16 MFMA tiles per wave dimension
    static constexpr int kRowsPerWave = TB / 4;      // staged rows per wave per operand
    static constexpr int kPieces = kRowsPerWave / 8; // 1-KiB LDS-DMA pieces per operand per wave
    static constexpr int kTileBytes = TB * BK;
    static constexpr int kStageBytes = 2 * kTileBytes;
    static constexpr int kLdsBytes = kDepth * kStageBytes;
    static constexpr int kMinBlocks = TB == 128 || kDepth > 2 ? 2 : 4;
    static constexpr int kLoadsPerStage = 2 * kPieces;  // LDS-DMA instructions per wave per stage (vmcnt)
    static_assert(TB * TB * 4 <= kLdsBytes, "epilogue image fits the ring");
};
namespace t128 {  // the 128-tile constants (launch shape)
constexpr int TB = 128;
constexpr int kThreads = SmallTile<128>::kThreads;
}  // namespace t128

template <int TB, int kEpi = kEpiNone, int kDepth = 2>
__global__ __launch_bounds__((SmallTile<TB, kDepth>::kThreads), (SmallTile<TB, kDepth>::kMinBlocks)) void gemm_i8_small(
    GemmArgs p) {
    using T_ = SmallTile<TB, kDepth>;
    constexpr int MI = T_::MI, WT = T_::WT, RPW = T_::kRowsPerWave, NP = T_::kPieces;
    __shared__ __attribute__((aligned(16))) int8_t lds[T_::kLdsBytes + 4 * TB * 4];  // + Cx, Cw, bias, flag
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int S = p.splits > 1 ? p.splits : 1;
    const int wid = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = wid / S, slice = wid - tile * S;
    int tm, tn;
    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn);
    const int nk_all = (int)(p.k_pad / BK);
    const int kt0 = slice * nk_all / S;
    const int nk = (slice + 1) * nk_all / S - kt0;
    // staging (fragment-major operands, qgemm_internal.h fofs): a k-step of a TB-row tile is TB/16 row groups
    // x 2 k-blocks of 1 KiB; wave w copies blocks q = w NP + i (row group q >> 1, k-block q & 1) whole, one
    // LDS-DMA each, to LDS q * 1 KiB -- the LDS image is block order and a fragment read one contiguous 1 KiB
    const int8_t *Ablk = p.A + (int64_t)tm * TB * p.k_pad;  // = the tile's first row group (TB % 16 == 0)
    const int8_t *Bblk = p.B + (int64_t)tn * TB * p.k_pad;
    const int64_t nkg = p.k_pad / 64;
    int64_t src_off[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int q = wave * NP + i;
        src_off[i] = ((int64_t)(q >> 1) * nkg + (q & 1)) * 1024 + lane * 16;
    }
    auto stage = [&](int kt, int buf) __attribute__((always_inline)) {
        int8_t *la = lds + buf * T_::kStageBytes;
        int8_t *lb = la + T_::kTileBytes;
        const int8_t *ga = Ablk + (int64_t)kt * 2048;
        const int8_t *gb = Bblk + (int64_t)kt * 2048;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            __builtin_amdgcn_global_load_lds((const void *)(ga + src_off[i]), (void *)(la + (wave * RPW + i * 8) * BK), 16,
                                             0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(gb + src_off[i]), (void *)(lb + (wave * RPW + i * 8) * BK), 16,
                                             0, 0);
        }
    };
    const int lrow = lane & 15, kq = lane >> 4;
    // fragment (16 rows from r, sub-step s) = LDS block ((r >> 4), s): the lane's 16 B at lane * 16
    const int a_row0 = wm * WT * BK + lane * 16, b_row0 = wn * WT * BK + lane * 16;
    int off[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) off[s] = s * 1024;

    v4i acc[MI][MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) acc[mi][ni] = v4i{};
    auto read_frags = [&](v4i (&a)[MI], v4i (&b)[MI], int buf, int s) __attribute__((always_inline)) {
        const int8_t *la = lds + buf * T_::kStageBytes;
        const int8_t *lb = la + T_::kTileBytes;
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 16 * BK + off[s]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 16 * BK + off[s]);
    };
    auto mfmas = [&](const v4i (&a)[MI], const v4i (&b)[MI]) __attribute__((always_inline)) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    v4i a0[MI], b0[MI], a1[MI], b1[MI];
    if constexpr (kDepth == 2) {
        stage(kt0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        read_frags(a0, b0, 0, 0);
        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt & 1;
            const bool more = kt + 1 < nk;
            if (more) stage(kt0 + kt + 1, cur ^ 1);
            read_frags(a1, b1, cur, 1);
            mfmas(a0, b0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (more) read_frags(a0, b0, cur ^ 1, 0);
            mfmas(a1, b1);
        }
    } else {
        // kDepth - 1 stages in flight; k-steps past the slice re-load its last k-step (clamped), so every
        // trip waits for exactly kDepth - 2 younger stages
        const int last = kt0 + nk - 1;
#pragma unroll
        for (int s = 0; s < kDepth - 1; ++s) stage(min(kt0 + s, last), s);
        for (int kt = 0; kt < nk; ++kt) {
            // stage kt landed for this wave's pieces; a RAW barrier then makes it visible to every wave (and
            // every wave is done reading stage kt - 1's slot, which the DMA below refills).  Not
            // __syncthreads(): with LDS-DMA in flight its fence emits vmcnt(0), which drained the whole
            // ring every k-step (one stage in flight whatever kDepth was).
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDepth - 2) * T_::kLoadsPerStage) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            stage(min(kt0 + kt + kDepth - 1, last), (kt + kDepth - 1) % kDepth);
            const int cur = kt % kDepth;
            read_frags(a0, b0, cur, 0);
            read_frags(a1, b1, cur, 1);
            mfmas(a0, b0);
            mfmas(a1, b1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped re-loads land before the ring is reused
    }

    if (S > 1 &&
        !splitk_combine<MI, MI, 4>(p, reinterpret_cast<unsigned *>(lds + T_::kLdsBytes + 3 * TB * 4), acc, tile, slice, S,
                                   wave, lane, tid))
        return;

    // epilogue: the whole fp32 tile through LDS, then row stores (TB/4 lanes of 16 B per row)
    const int gi0 = tm * TB, gj0 = tn * TB;
    float *sCx = reinterpret_cast<float *>(lds + T_::kLdsBytes);
    float *sCw = sCx + TB;
    float *sB = sCw + TB;
    __syncthreads();  // every wave is done with the staging ring
    if (tid < TB) sCx[tid] = p.Cx[gi0 + tid];
    else if (tid < 2 * TB) sCw[tid - TB] = p.Cw[gj0 + tid - TB];
    if constexpr (has_bias(kEpi))
        if (tid < TB) sB[tid] = gj0 + tid < p.n ? p.bias[gj0 + tid] : 0.0f;
    __syncthreads();
    float *T = reinterpret_cast<float *>(lds);  // [TB][TB] fp32 in the ring
#pragma unroll
    for (int ni = 0; ni < MI; ++ni) {
        const int jl = wn * WT + ni * 16 + lrow;
        const float cw = sCw[jl];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int il = wm * WT + mi * 16 + 4 * kq + r;
                T[il * TB + jl] = epi_extra<kEpi>(dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), p.inv_r2), sB, jl);
            }
    }
    __syncthreads();
    float *C = static_cast<float *>(p.C);
    const bool full = p.csw == 1 && (p.csh % 4 == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0) && gj0 + TB <= p.n;
    constexpr int kLanesPerRow = TB / 4;
    const int c4 = (tid % kLanesPerRow) * 4;
#pragma unroll 4
    for (int rr = tid / kLanesPerRow; rr < TB; rr += T_::kThreads / kLanesPerRow) {
        const int i = gi0 + rr;
        if (i >= p.m) break;
        const float4 v = *reinterpret_cast<const float4 *>(T + rr * TB + c4);
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
