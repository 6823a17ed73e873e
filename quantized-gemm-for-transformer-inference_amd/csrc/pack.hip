// pack.hip -- absmax + quantize kernels (the reference's op_absmax / op_inv_divide / op_multiply
// steps, op_mm.cuh:75-89), fused into HBM-streaming passes that emit MFMA-ready int8 operands.
//
// A "packed operand" (include/qgemm.h) is [scale][scratch][q]: each packed row is one reduction
// vector -- a row of X (scale Cx) or a column of W (scale Cw, stored transposed so k is contiguous for
// the MFMA B fragment).  Padding rows and k >= len are zero.
//
//   pack_rows : the reduction vector is contiguous (X row-major, or W column-major).  One wave per
//               vector: absmax (wave shuffle reduction), IEEE range/absmax, truncating quantize.
//               Replaces op_reduction_kernel_colwise (op_reduction.cuh:71-92: one thread per row,
//               lanes 16 KiB apart) + the InvDivideConstFunc and MultiplyWithTypecastFunc launches.
//   pack_cols : the reduction vector is a column of a row-major matrix (W).  Pass 1 reduces
//               256-column x 256-row chunks (coalesced 1-KiB row reads) into one partial per
//               (chunk, column) -- no atomics and nothing to clear per call; pass 2 reduces the
//               partials, re-reads W (from the Infinity Cache at the sizes that matter), quantizes
//               and transposes 128 x 64 tiles through LDS.  Replaces op_reduction_kernel_rowwise
//               (op_reduction.cuh:96-117) + 2 elementwise launches.
//   pack_rows_and_colmax : pack_rows(A) and pass 1 of pack_cols(B) in ONE launch (block roles), so
//               the two HBM streams overlap and a launch boundary disappears.
#include <algorithm>
#include <atomic>

#include "qgemm_internal.h"

namespace qgemm {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_max(float p) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p = fmaxf(p, __shfl_xor(p, off, kWave));
    return p;
}

// running max of |x| candidates; maxnum returns the non-NaN operand, so NaN never wins, exactly as
// the reference's comparison (op_reduction.cuh:14-23) skips it
__device__ __forceinline__ float cand_max(float p, float x) { return fmaxf(p, absmax_candidate(x)); }

// partial encoding: candidates are >= +0 and NaN-free, so uint order of (bits + 1) is float order;
// 0 means "no candidate in this chunk"
__device__ __forceinline__ uint32_t enc_partial(float p) { return p >= 0.0f ? __float_as_uint(p) + 1u : 0u; }
__device__ __forceinline__ float dec_partial(uint32_t e) { return e ? __uint_as_float(e - 1u) : -INFINITY; }

// low bytes of a, b, c, d -> one dword (three v_perm_b32)
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)d, (uint32_t)c, 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// W strips hold 4 consecutive k of one column per dword; a 16-B piece of the fragment-major q (one packed row,
// 16 consecutive k) is the dwords d[col] of the 4 threads b = 0..3 of a quad (lanes qbase + stride * b) that
// hold k = 16a + 4b.  4 x 4 transpose among them: returns, in thread b, the piece of the quad's column b.
// Round rr: send d[(b - rr) & 3], receive from quad thread (b + rr) & 3 its d[b] = piece dword (b + rr) & 3.
__device__ __forceinline__ void quad_transpose(const uint32_t (&d)[4], int b, int qbase, int stride,
                                               uint32_t (&pc)[4]) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int si = (b - rr) & 3;
        const uint32_t x = si == 0 ? d[0] : si == 1 ? d[1] : si == 2 ? d[2] : d[3];
        const int from = (b + rr) & 3;
        const uint32_t y = (uint32_t)__shfl((int)x, qbase + stride * from, 64);
#pragma unroll
        for (int sl = 0; sl < 4; ++sl) pc[sl] = from == sl ? y : pc[sl];
    }
}

// wave-uniform buffer descriptor over [base, base + bytes): loads past the end return zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

// kWT (lab fused pack+GEMM launch only): the packed bytes and scales are handed to GEMM blocks of the SAME
// launch on other XCDs, so they are stored write-through (sc1; MI355X_MICROARCH.md inter-workgroup
// visibility) instead of staying dirty in this XCD's L2
template <bool kWT>
__device__ __forceinline__ void st_u32(uint32_t *p, uint32_t v) {
    if constexpr (kWT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <bool kWT>
__device__ __forceinline__ void st_f32(float *p, float v) {
    if constexpr (kWT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// 16-B load; kNt: non-temporal (the line is not kept in the Infinity Cache for a later reader)
template <bool kNt>
__device__ __forceinline__ float4 ld_f4(const float *p) {
    if constexpr (kNt) {
        typedef float v4f_nt __attribute__((ext_vector_type(4)));
        const v4f_nt v = __builtin_nontemporal_load(reinterpret_cast<const v4f_nt *>(p));
        return make_float4(v[0], v[1], v[2], v[3]);
    } else {
        return *reinterpret_cast<const float4 *>(p);
    }
}

// Blocks b and b + 8 run on one XCD.  For a role occupying blocks [base, base + count): a role-local index
// that gives every XCD ONE contiguous range (bijective).  Row packs index their rows with it: a 128-B line
// of the fragment-major q holds 16-B pieces of 8 consecutive rows (qgemm_internal.h fofs), and rows packed
// on 8 different XCDs would leave every line as 8 partial writes from 8 L2s (FFN-down X rows, one row per
// block: 116 vs 89 us before this mapping).
__device__ __forceinline__ int xcd_contig(int bid, int base, int count) {
    const int x = bid & 7;
    int start = 0;
#pragma unroll
    for (int y = 0; y < 7; ++y) {
        const int o = (y - base) & 7;
        if (y < x && o < count) start += (count - 1 - o) / 8 + 1;
    }
    return start + (bid - base - ((x - base) & 7)) / 8;
}

// The GEMM's split-K tickets live in the caller's workspace, whose contents are arbitrary: the pack
// launch that precedes the GEMM in the same stream zeroes them (block 0), which saves the GEMM a
// zeroing launch of its own.
__device__ __forceinline__ void zero_words_block0(uint32_t *words, int n) {
    if (n > 0 && blockIdx.x == 0)
        for (int i = threadIdx.x; i < n; i += blockDim.x) words[i] = 0u;
}

// ------------------------------------------------------------------------------------------------
// LLM.int8() decomposition inside the pack (outlier.hip builds the mask): feature k of X is an outlier
// column when bit k of `bits` is set.  The int8 chain runs on X' / W' = X / W with those columns /
// rows zeroed, so the packs treat them as +0 (absmax candidates, the signed seed and the quantized
// bytes alike, exactly as packing the zeroed copies).  The fp32 part reads the original values from X and W
// themselves (gemm_i8_fm<kEpiOutlier>), so nothing is written here but the column index.  The mask comes from the
// flags launch as nparts partial masks (outlier.hip outlier_colmask_kernel: partial[p][w] for row split p, every word
// written by it each call, so no state lives on between calls; nparts = 2 at K = 4096): word w = OR over p.  Each
// thread reads exactly the words of its own elements, issued ahead of its data: an X-row lane's chunk l + 64 j
// (columns 4 (l + 64 j) .. +3) is nibble l & 7 of word (l >> 3) + 8 j, a W-strip thread's rows 4 q + e + 1024 i
// are bits of word (4 q + 1024 i) >> 5.  Workgroup 0 also builds the column count and the ascending list for the
// GEMM (idx[0], idx[1 ..]).
struct OutlierMask {
    const uint32_t *partial;  // nparts x nwords partial mask words (bit 0 of word 0: column 0, the absmax seed)
    int nwords, nparts;
    int *idx;                 // out: [count][columns ascending]
    // mask words w[j] (0 where w[j] >= nwords): the ORs of their nparts partial words -- every load of split 0 issued
    // before any is waited for (nparts is 1 or 2 on the shapes the benchmarks run)
    template <int NW>
    __device__ __forceinline__ void words(const int (&w)[NW], uint32_t (&out)[NW]) const {
#pragma unroll
        for (int j = 0; j < NW; ++j) out[j] = w[j] < nwords ? partial[w[j]] : 0u;
        for (int p = 1; p < nparts; ++p)
#pragma unroll
            for (int j = 0; j < NW; ++j) out[j] |= w[j] < nwords ? partial[p * nwords + w[j]] : 0u;
    }
    __device__ __forceinline__ uint32_t word(int w) const {
        const int ws[1] = {w};
        uint32_t x[1];
        words(ws, x);
        return x[0];
    }
};
// workgroup 0 of the masked pack: idx[0] = the outlier columns, idx[1 ..] = them ascending (nwords <= blockDim)
__device__ __forceinline__ void outlier_column_list(const OutlierMask &om, int *wsum /* LDS, blockDim / 64 */) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nwave = blockDim.x >> 6;
    const uint32_t word = t < om.nwords ? om.word(t) : 0u;
    const int pc = __popc(word);
    int x = pc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(x, off, 64);
        if (lane >= off) x += v;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int below = x - pc, total = 0;
    for (int j = 0; j < nwave; ++j) {
        below += j < wave ? wsum[j] : 0;
        total += wsum[j];
    }
    int j = 0;
    for (uint32_t b = word; b; b &= b - 1, ++j) om.idx[1 + below + j] = 32 * t + __builtin_ctz(b);
    if (t == 0) om.idx[0] = total;
}

// ------------------------------------------------------------------------------------------------
// pack_rows, vector path: rows of `len` floats at src + r*sh, unit inner stride, 16-B aligned rows.
// R > 0: each lane keeps R float4 chunks in registers (len <= 256*R), one HBM read.
// R == 0: two streaming passes (second pass mostly L2 hits).  `blk` = kGroup-row group index.
// kStage: the packed row goes to `stage` (the wave's LDS row, dword c at stage[c]) instead of q; the caller
// writes the block's staged rows out as whole 128-B lines of the fragment-major q (write_staged_rows).
// kGroup: rows per `blk` (wave w of the block takes row blk * kGroup + w).
template <int R, bool kMask = false, bool kWT = false, bool kStage = false, int kGroup = 4>
__device__ __forceinline__ void pack_rows_vec_body(int64_t blk, const float *__restrict__ src, int64_t sh, int rows,
                                                   int len, float range, float *__restrict__ scale,
                                                   int8_t *__restrict__ q, int64_t rows_pad, int64_t k_pad,
                                                   const OutlierMask *om = nullptr, uint32_t *stage = nullptr) {
    static_assert(!kMask || R > 0, "the outlier mask needs the register-resident rows");
    const int lane = threadIdx.x & 63;
    const int64_t row = blk * kGroup + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    if (row >= rows_pad) return;
    // dword c of the packed row (k = 4c), fragment-major layout (qgemm_internal.h fofs), or of the LDS stage
    auto put = [&](int64_t c, uint32_t v) __attribute__((always_inline)) {
        if constexpr (kStage) stage[c] = v;
        else st_u32<kWT>(qword(q, row, 4 * c, k_pad), v);
    };
    const int64_t nq = k_pad >> 2;  // uint32 words per packed row
    if (row >= rows) {              // padding row
        for (int64_t c = lane; c < nq; c += kWave) put(c, 0u);
        if (lane == 0) st_f32<kWT>(scale + row, 0.0f);
        return;
    }
    const float *srow = src + row * sh;
    const float4 *s4 = reinterpret_cast<const float4 *>(srow);
    const int nfull = len >> 2;  // complete float4 chunks
    float seed = srow[0];

    float p = -INFINITY;
    float4 v[R > 0 ? R : 1];
    if constexpr (R > 0) {
        // buffer loads on one per-lane offset; chunks >= nfull lie past the descriptor and read as zeros
        typedef int v4i_t __attribute__((ext_vector_type(4)));
        const auto rs = buf_rsrc(srow, (uint32_t)nfull * 16);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(lane + j * kWave) * 16, 0, 0);
            v[j] = make_float4(__int_as_float(x[0]), __int_as_float(x[1]), __int_as_float(x[2]), __int_as_float(x[3]));
        }
        // the lane's mask words (chunk lane + 64 j: word (lane >> 3) + 8 j), issued behind the row's loads so that
        // both latencies overlap (a row split past the first ORs behind a wait)
        uint32_t mwd[R > 0 ? R : 1];
        uint32_t mw0 = 0u;  // word 0: its bit 0 masks the absmax seed
        if constexpr (kMask) {
            static_assert(R <= 16, "the mask words cover len <= 4096");
            // the wave loads the mask once (lane l: words l and l + 64), then each lane takes its words by
            // ds_bpermute: word (lane >> 3) + 8 j is < 64 exactly for j < 8
            const int wl[2] = {lane, lane + 64};
            uint32_t m2[2];
            om->words(wl, m2);
#pragma unroll
            for (int j = 0; j < R; ++j)
                mwd[j] = (uint32_t)__shfl((int)(j < 8 ? m2[0] : m2[1]), ((lane >> 3) + 8 * j) & 63, 64);
            mw0 = __builtin_amdgcn_readlane(m2[0], 0);
        }
        if constexpr (kMask) {
            // outlier columns: X' holds +0 there (the seed included); branch-free selects
            {
                if (mw0 & 1u) seed = 0.0f;
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const uint32_t nib = (mwd[j] >> (4 * (lane & 7))) & 15u;
                    v[j].x = (nib & 1u) ? 0.0f : v[j].x;
                    v[j].y = (nib & 2u) ? 0.0f : v[j].y;
                    v[j].z = (nib & 4u) ? 0.0f : v[j].z;
                    v[j].w = (nib & 8u) ? 0.0f : v[j].w;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int c = lane + j * kWave;
            if (c < nfull) {
                p = (c == 0) ? p : cand_max(p, v[j].x);  // element 0 is the seed
                p = cand_max(p, v[j].y);
                p = cand_max(p, v[j].z);
                p = cand_max(p, v[j].w);
            }
        }
    } else {
        for (int c = lane; c < nfull; c += kWave) {
            float4 x = s4[c];
            p = (c == 0) ? p : cand_max(p, x.x);
            p = cand_max(p, x.y);
            p = cand_max(p, x.z);
            p = cand_max(p, x.w);
        }
    }
    const int tail0 = nfull << 2;  // scalar tail elements [tail0, len)
    if (tail0 + lane < len && tail0 + lane > 0) p = cand_max(p, srow[tail0 + lane]);
    p = wave_max(p);
    const float cx = absmax_finish(seed, p);
    const float s = inv_divide(range, cx);

    if constexpr (R > 0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int c = lane + j * kWave;
            if (c < nfull)
                put(c, pack4(quant_i8(v[j].x, s), quant_i8(v[j].y, s), quant_i8(v[j].z, s), quant_i8(v[j].w, s)));
        }
    } else {
        for (int c = lane; c < nfull; c += kWave) {
            float4 x = s4[c];
            put(c, pack4(quant_i8(x.x, s), quant_i8(x.y, s), quant_i8(x.z, s), quant_i8(x.w, s)));
        }
    }
    // partial tail word, then zero padding words
    const int64_t first_zero = nfull + ((len & 3) ? 1 : 0);
    if ((len & 3) && lane == 0) {
        int b[4] = {0, 0, 0, 0};
        for (int e = 0; e < (len & 3); ++e) b[e] = quant_i8(srow[tail0 + e], s);
        put(nfull, pack4(b[0], b[1], b[2], b[3]));
    }
    for (int64_t c = first_zero + lane; c < nq; c += kWave) put(c, 0u);
    if (lane == 0) st_f32<kWT>(scale + row, cx);
}

// Staged packed rows: kRows (8 or 16) consecutive packed rows row0 .. (row0 % 8 == 0), one per wave, in LDS
// at stage + r * rsw dwords (rsw = k_pad / 4 + 16: the 16-B reads below are conflict-free in ds_read_b128's
// lane groups for k_pad / 4 = 0 or 32 mod 64; + 8 left 2-way conflicts, 6.5 % of the pack's LDS cycles), written out as whole 128-B lines of the fragment-major q: line (L, h) = the 16-B pieces
// of k 16L .. 16L+15 of rows 8h .. 8h+7; one wave store instruction = 8 lines.  After a block barrier.
constexpr int kStageRowWordsMax = 4096 / 4 + 16;
template <int kRows>
__device__ __forceinline__ void write_staged_rows(const uint32_t *stage, int rsw, int8_t *__restrict__ q, int64_t row0,
                                                  int64_t k_pad) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int nl = (int)(k_pad >> 4);  // 16-B pieces per row (a multiple of 8)
    const int units = nl * (kRows / 8);
    for (int u = wv * 8 + (lane >> 3); u < units; u += kRows * 8) {
        const int h = u / nl, L = u - h * nl;
        const int r = h * 8 + (lane & 7);
        const uint4 v = *reinterpret_cast<const uint4 *>(stage + r * rsw + 4 * L);
        *reinterpret_cast<uint4 *>(q + fofs(row0 + r, 16 * L, k_pad)) = v;
    }
}

// pack_rows, long rows (4096 < len <= 16384): ONE 256-thread block per row, up to 16 float4 per
// thread in registers (4-KiB coalesced loads per block instruction), block-wide absmax (shuffle + LDS),
// quantized from the registers -- one HBM read of the row.  `red` holds >= 5 floats of LDS.
constexpr int kLongRowMax = 16384;
template <bool kNt = false>
__device__ __forceinline__ void pack_row_block_body(int64_t row, const float *__restrict__ src, int64_t sh, int rows,
                                                    int len, float range, float *__restrict__ scale,
                                                    int8_t *__restrict__ q, int64_t rows_pad, int64_t k_pad,
                                                    float *red) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (row >= rows_pad) return;
    auto qrow = [&](int64_t c) __attribute__((always_inline)) -> uint32_t & { return *qword(q, row, 4 * c, k_pad); };
    const int64_t nq = k_pad >> 2;
    if (row >= rows) {  // padding row
        for (int64_t c = t; c < nq; c += 256) qrow(c) = 0u;
        if (t == 0) scale[row] = 0.0f;
        return;
    }
    const float *srow = src + row * sh;
    const int nfull = len >> 2;
    float4 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int c = t + 256 * j;
        v[j] = (c < nfull) ? ld_f4<kNt>(srow + 4 * (int64_t)c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float p = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int c = t + 256 * j;
        if (c < nfull) {
            p = (c == 0) ? p : cand_max(p, v[j].x);  // element 0 is the seed
            p = cand_max(p, v[j].y);
            p = cand_max(p, v[j].z);
            p = cand_max(p, v[j].w);
        }
    }
    const int tail0 = nfull << 2;
    if (tail0 + t < len && tail0 + t > 0) p = cand_max(p, srow[tail0 + t]);
    p = wave_max(p);
    if (lane == 0) red[wv] = p;
    if (t == 0) red[4] = nfull > 0 ? v[0].x : srow[0];  // the seed
    __syncthreads();
    p = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));  // -inf or >= +0: exact
    const float cx = absmax_finish(red[4], p);
    const float sc = inv_divide(range, cx);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int c = t + 256 * j;
        if (c < nfull)
            qrow(c) = pack4(quant_i8(v[j].x, sc), quant_i8(v[j].y, sc), quant_i8(v[j].z, sc), quant_i8(v[j].w, sc));
    }
    const int64_t first_zero = nfull + ((len & 3) ? 1 : 0);
    if ((len & 3) && t == 0) {
        int b[4] = {0, 0, 0, 0};
        for (int e = 0; e < (len & 3); ++e) b[e] = quant_i8(srow[tail0 + e], sc);
        qrow(nfull) = pack4(b[0], b[1], b[2], b[3]);
    }
    for (int64_t c = first_zero + t; c < nq; c += 256) qrow(c) = 0u;
    if (t == 0) scale[row] = cx;
}

__global__ __launch_bounds__(256) void pack_rows_block_kernel(const float *__restrict__ src, int64_t sh, int rows,
                                                              int len, float range, float *__restrict__ scale,
                                                              int8_t *__restrict__ q, int64_t rows_pad,
                                                              int64_t k_pad) {
    __shared__ float red[8];
    pack_row_block_body(xcd_contig(blockIdx.x, 0, gridDim.x), src, sh, rows, len, range, scale, q, rows_pad, k_pad, red);
}

// R > 0 (rows of <= 4096 floats): 8 rows per 512-thread block, one wave per row, staged in LDS and written out
// as whole 128-B lines of the fragment-major q (a line = 16-B pieces of 8 rows).  R == 0 (streaming rows): 4
// rows per 256-thread block, stored directly.
template <int R>
__global__ __launch_bounds__(R > 0 ? 512 : 256) void pack_rows_vec_kernel(const float *__restrict__ src, int64_t sh,
                                                                          int rows, int len, float range,
                                                                          float *__restrict__ scale,
                                                                          int8_t *__restrict__ q, int64_t rows_pad,
                                                                          int64_t k_pad) {
    const int b = xcd_contig(blockIdx.x, 0, gridDim.x);
    if constexpr (R > 0) {
        __shared__ __attribute__((aligned(16))) uint32_t xstage[8 * kStageRowWordsMax];
        const int rsw = (int)(k_pad >> 2) + 16;
        pack_rows_vec_body<R, false, false, true>(2 * (int64_t)b, src, sh, rows, len, range, scale, q, rows_pad, k_pad,
                                                  nullptr, xstage + (threadIdx.x >> 6) * rsw);
        __syncthreads();
        write_staged_rows<8>(xstage, rsw, q, 8 * (int64_t)b, k_pad);
    } else {
        pack_rows_vec_body<R>(b, src, sh, rows, len, range, scale, q, rows_pad, k_pad);
    }
}

// R > 0 with fewer staged 8-row blocks than CUs (rows_pad < 2 048: the encoder's activations): 2 rows per 128-thread
// block, each wave's dwords stored straight into the fragment-major q -- 4x the blocks, so 4x the CUs pull rows
// (lab/rowpack_lab.hip, profiles/r06_rowpack_lab.log: 512 x 4 096 4.28 vs 5.38 us, 512 x 1 024 3.03-3.15 vs 3.23 us;
// at 2 048 rows the staged lines are as fast or faster)
template <int R>
__global__ __launch_bounds__(128) void pack_rows_pair_kernel(const float *__restrict__ src, int64_t sh, int rows, int len,
                                                             float range, float *__restrict__ scale,
                                                             int8_t *__restrict__ q, int64_t rows_pad, int64_t k_pad) {
    pack_rows_vec_body<R, false, false, false, 2>(xcd_contig(blockIdx.x, 0, gridDim.x), src, sh, rows, len, range, scale,
                                                  q, rows_pad, k_pad);
}

// pack_rows, generic strides (any sh, sw): scalar loads, two passes.
__global__ __launch_bounds__(256) void pack_rows_generic_kernel(const float *__restrict__ src, int64_t sh,
                                                                int64_t sw, int rows, int len, float range,
                                                                float *__restrict__ scale, int8_t *__restrict__ q,
                                                                int64_t rows_pad, int64_t k_pad) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)xcd_contig(blockIdx.x, 0, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (row >= rows_pad) return;
    auto qrow = [&](int64_t c) __attribute__((always_inline)) -> int8_t & { return q[fofs(row, c, k_pad)]; };
    if (row >= rows) {
        for (int64_t c = lane; c < k_pad; c += kWave) qrow(c) = 0;
        if (lane == 0) scale[row] = 0.0f;
        return;
    }
    const float *srow = src + row * sh;
    const float seed = srow[0];
    float p = -INFINITY;
    for (int64_t c = 1 + lane; c < len; c += kWave) p = cand_max(p, srow[c * sw]);
    p = wave_max(p);
    const float cx = absmax_finish(seed, p);
    const float s = inv_divide(range, cx);
    for (int64_t c = lane; c < k_pad; c += kWave) qrow(c) = (c < len) ? (int8_t)quant_i8(srow[c * sw], s) : 0;
    if (lane == 0) scale[row] = cx;
}

// ------------------------------------------------------------------------------------------------
// pack_cols pass 1: for a [len x cols] row-major matrix (row stride sh, unit column stride), block
// (cb, part) reduces |x| over rows [1 + 256*part, 1 + 256*(part+1)) of columns [256*cb, 256*cb+256)
// (row 0 is the seed, combined in pass 2) and writes partial[part][col].  4 waves x 64 rows; each
// lane owns 4 columns (VEC: contiguous float4 -> 1 KiB per wave load; else stride-64 scalars).
constexpr int kColBlock = 256;  // columns per pass-1 block

template <bool VEC, int kUnroll = 8>
__device__ __forceinline__ void colmax_body(int cb, int part, const float *__restrict__ src, int64_t sh, int len,
                                            int cols, uint32_t *__restrict__ partial, int64_t rows_pad,
                                            float *red /* 4 x 256 floats of LDS */) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t r0 = 1 + (int64_t)part * kColChunk + w * 64;
    const int64_t r1 = min((int64_t)len, r0 + 64);
    const int64_t c0 = (int64_t)cb * kColBlock;
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
    if constexpr (VEC) {
        const int64_t c = c0 + lane * 4;
        if (c < cols) {
            const float *base = src + c;
#pragma unroll kUnroll
            for (int64_t r = r0; r < r1; ++r) {
                const float4 x = *reinterpret_cast<const float4 *>(base + r * sh);
                p0 = cand_max(p0, x.x);
                p1 = cand_max(p1, x.y);
                p2 = cand_max(p2, x.z);
                p3 = cand_max(p3, x.w);
            }
        }
        red[w * 256 + lane * 4 + 0] = p0;
        red[w * 256 + lane * 4 + 1] = p1;
        red[w * 256 + lane * 4 + 2] = p2;
        red[w * 256 + lane * 4 + 3] = p3;
    } else {
        float pv[4] = {p0, p1, p2, p3};
        for (int64_t r = r0; r < r1; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t c = c0 + lane + 64 * j;
                if (c < cols) pv[j] = cand_max(pv[j], src[r * sh + c]);
            }
#pragma unroll
        for (int j = 0; j < 4; ++j) red[w * 256 + lane + 64 * j] = pv[j];
    }
    __syncthreads();
    const int t = threadIdx.x;  // column within the block
    float m = red[t];
    m = fmaxf(m, red[256 + t]);  // all values are -inf or >= +0: fmaxf is exact here
    m = fmaxf(m, red[512 + t]);
    m = fmaxf(m, red[768 + t]);
    if (c0 + t < cols) partial[(int64_t)part * rows_pad + c0 + t] = enc_partial(m);
}

template <bool VEC>
__global__ __launch_bounds__(256) void colmax_kernel(const float *__restrict__ src, int64_t sh, int len, int cols,
                                                     uint32_t *__restrict__ partial, int64_t rows_pad) {
    __shared__ float red[4 * 256];
    colmax_body<VEC>(blockIdx.x, blockIdx.y, src, sh, len, cols, partial, rows_pad, red);
}

// Fused: blocks [0, ncol) run pass 1 of pack_cols(B), blocks [ncol, ncol + nrow) run pack_rows(A).
// kXFirst: the X-row blocks come first in dispatch order and W's column-max sweep last, so W's rows are the most
// recent bytes in the Infinity Cache when pass 2 starts (it re-reads them in reverse: pack_cols_kernel<.., true>)
template <int R, bool kXFirst = false>
__global__ __launch_bounds__(256) void pack_rows_and_colmax_kernel(
    const float *__restrict__ a, int64_t ash, int m, int k, float *__restrict__ a_scale, int8_t *__restrict__ a_q,
    int64_t a_rows_pad, int64_t k_pad, const float *__restrict__ b, int64_t bsh, int n,
    uint32_t *__restrict__ b_partial, int64_t b_rows_pad, int col_blocks, int ncol, float range, uint32_t *zero_words,
    int nzero) {
    __shared__ float red[4 * 256];
    const int nrow = (int)gridDim.x - ncol;
    // role index: column-max blocks [0, ncol), X-row blocks [ncol, ncol + nrow) (rotated when kXFirst)
    const int bid = kXFirst ? ((int)blockIdx.x < nrow ? (int)blockIdx.x + ncol : (int)blockIdx.x - nrow) : (int)blockIdx.x;
    zero_words_block0(zero_words, nzero);
    if (bid < ncol) {
        // unrolled 4 deep: pack3_lab `call_u4` 140.9-146.0 vs 143.6-149.4 us for 8 (FFN down, pass 1 + pass 2)
        colmax_body<true, 4>(bid % col_blocks, bid / col_blocks, b, bsh, k, n, b_partial, b_rows_pad, red);
    } else if constexpr (R < 0) {
        pack_row_block_body(kXFirst ? xcd_contig(blockIdx.x, 0, nrow) : xcd_contig(bid, ncol, nrow), a, ash, m, k, range,
                            a_scale, a_q, a_rows_pad, k_pad, red);
    } else {
        pack_rows_vec_body<R>(kXFirst ? xcd_contig(blockIdx.x, 0, nrow) : xcd_contig(bid, ncol, nrow), a, ash, m, k, range,
                              a_scale, a_q, a_rows_pad, k_pad);
    }
}

// pack_cols pass 2: finish the column scale from the partials, quantize, transpose a [128 k][64 col]
// tile through LDS and write 64 packed rows x 128 bytes.  Grid: (rows_pad/64, k_pad/128).
constexpr int kTc = 64;             // output rows (= input columns) per block
constexpr int kTk = 128;            // k per block
constexpr int kTStride = kTk + 4;   // LDS row stride: 33 dwords (odd) -> transpose writes 2-way, reads conflict-free

template <bool VEC, bool kNt = false>
__device__ __forceinline__ void load_col_tile(float4 (&x)[2][4], const float *__restrict__ src, int64_t sh, int len,
                                              int cols, int64_t c, int64_t k0, int rg) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t kk = k0 + 4 * rg + 64 * h + i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (kk < len) {
                const float *rp = src + kk * sh + c;
                if constexpr (VEC) {
                    if (c < cols) v = ld_f4<kNt>(rp);
                } else {
                    if (c + 0 < cols) v.x = rp[0];
                    if (c + 1 < cols) v.y = rp[1];
                    if (c + 2 < cols) v.z = rp[2];
                    if (c + 3 < cols) v.w = rp[3];
                }
            }
            x[h][i] = v;
        }
}

// Block = 64 output rows (input columns) x kTilesPerBlock k-tiles of 128: the column scales are
// computed once, and tile kt+1's loads are in flight while tile kt is quantized, transposed and
// stored.  Grid: (rows_pad/64, ceil(k_pad/128 / kTilesPerBlock)).  lab/pack3_lab.hip at 4096 x 16384
// (FFN down W): 2 / 4 / 8 / 16 / 32 tiles per block 70.1 / 74.7 / 69.2 / 68.9 / 87.8 us.
constexpr int kTilesPerBlock = 8;

// kRev: the k-ranges in reverse dispatch order (bottom rows of W first): pass 1 swept W top to bottom, so its
// last rows are the ones still in the Infinity Cache
// block (bx, by): packed rows [64 bx, 64 bx + 64) x k-tiles [kTPB by, kTPB by + kTPB); tile = 2 x kTc x kTStride
// bytes of LDS (two [64 packed rows][132 B] buffers), s_sh = kTc floats
template <bool VEC, int kTPB, bool kNt = false>
__device__ __forceinline__ void pack_cols_body(int bx, int by, const float *__restrict__ src, int64_t sh, int len,
                                               int cols, float range, const uint32_t *__restrict__ partial,
                                               int64_t parts, int64_t rows_pad, float *__restrict__ scale,
                                               int8_t *__restrict__ q, int64_t k_pad, uint8_t (*tile)[kTc * kTStride],
                                               float *s_sh) {
    const int t = threadIdx.x;
    const int64_t n0 = (int64_t)bx * kTc;
    const int64_t nkt = k_pad / kTk;
    const int64_t kt0 = (int64_t)by * kTPB;
    const int64_t kt1 = min(nkt, kt0 + kTPB);
    const int col4 = t & 15;  // 4 input columns n0 + 4*col4 .. +3
    const int rg = t >> 4;    // rows k0 + 4*rg + 64*h + {0..3}
    const int64_t c = n0 + 4 * col4;
    // first tile's loads before the scale reduction (their latency overlaps it)
    float4 x[2][4], xn[2][4];
    load_col_tile<VEC, kNt>(x, src, sh, len, cols, c, kt0 * kTk, rg);
    if (t < kTc) {
        const int64_t j = n0 + t;
        float cx = 0.0f, s = 0.0f;
        if (j < cols) {
            float p = -INFINITY;
#pragma unroll 16
            for (int64_t part = 0; part < parts; ++part) p = fmaxf(p, dec_partial(partial[part * rows_pad + j]));
            cx = absmax_finish(src[j], p);  // seed = row 0 (op_reduction.cuh:105)
            s = inv_divide(range, cx);
        }
        s_sh[t] = s;
        if (by == 0) scale[j] = cx;
    }
    __syncthreads();
    const float s0 = s_sh[4 * col4 + 0], s1 = s_sh[4 * col4 + 1], s2 = s_sh[4 * col4 + 2], s3 = s_sh[4 * col4 + 3];
    const int n = t >> 2;         // packed row within the tile (write-out role)
    const int kc = (t & 3) * 32;  // byte offset within the 128-byte k slice
    for (int64_t kt = kt0; kt < kt1; ++kt) {
        const int64_t k0 = kt * kTk;
        if (kt + 1 < kt1) load_col_tile<VEC, kNt>(xn, src, sh, len, cols, c, k0 + kTk, rg);
        uint8_t *tb = tile[(kt - kt0) & 1];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int qv[4][4];  // [row i][col e]
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t kk = k0 + 4 * rg + 64 * h + i;
                qv[i][0] = (kk < len && c + 0 < cols) ? quant_i8(x[h][i].x, s0) : 0;
                qv[i][1] = (kk < len && c + 1 < cols) ? quant_i8(x[h][i].y, s1) : 0;
                qv[i][2] = (kk < len && c + 2 < cols) ? quant_i8(x[h][i].z, s2) : 0;
                qv[i][3] = (kk < len && c + 3 < cols) ? quant_i8(x[h][i].w, s3) : 0;
            }
            // packed rows >= 32 (col4 >= 8) have their dwords XOR-swizzled by 2: with the 33-dword stride rows
            // 4 col4 and 4 (col4 + 8) otherwise share a bank in ds_write_b32's 32-bank lane groups (2-way; r02
            // PMC 33 % bank-conflict cycles); the read below undoes it (a bijection inside every 8-dword run)
            const int swz = (col4 >> 3) * 8;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                *reinterpret_cast<uint32_t *>(tb + (4 * col4 + e) * kTStride + ((4 * rg + 64 * h) ^ swz)) =
                    pack4(qv[0][e], qv[1][e], qv[2][e], qv[3][e]);
        }
        __syncthreads();  // tile tb complete (and, double-buffered, the other one is free to rewrite next)
        const uint32_t *lp = reinterpret_cast<const uint32_t *>(tb + n * kTStride + kc);  // 4-B aligned only
        const int rs = (n >> 5) * 2;  // the write's dword swizzle of rows >= 32
        *reinterpret_cast<uint4 *>(q + fofs(n0 + n, k0 + kc, k_pad)) =
            make_uint4(lp[0 ^ rs], lp[1 ^ rs], lp[2 ^ rs], lp[3 ^ rs]);
        *reinterpret_cast<uint4 *>(q + fofs(n0 + n, k0 + kc + 16, k_pad)) =
            make_uint4(lp[4 ^ rs], lp[5 ^ rs], lp[6 ^ rs], lp[7 ^ rs]);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) x[h][i] = xn[h][i];
    }
}

template <bool VEC, int kTPB = kTilesPerBlock, bool kRev = false>
__global__ __launch_bounds__(256) void pack_cols_kernel(const float *__restrict__ src, int64_t sh, int len, int cols,
                                                        float range, const uint32_t *__restrict__ partial,
                                                        int64_t parts, int64_t rows_pad, float *__restrict__ scale,
                                                        int8_t *__restrict__ q, int64_t k_pad) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][kTc * kTStride];  // [64 packed rows][132 B], 2 buffers
    __shared__ float s_sh[kTc];
    const int by = kRev ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y;
    pack_cols_body<VEC, kTPB>(blockIdx.x, by, src, sh, len, cols, range, partial, parts, rows_pad, scale, q, k_pad, tile,
                              s_sh);
}

// Pass 2 of the long-row two-pass pack (4096 < K <= 16384, round 4) with X's rows packed at its END: blocks
// [0, gx * gy) run pack_cols bottom-up (the rows a W-only pass 1 read last first: they are still in the Infinity
// Cache), blocks [gx * gy, + rows_pad) one X row each (pack_row_block_body); block 0 zeroes zero_words (the GEMM's
// split-K tickets).  Pass 1 is colmax_kernel alone: a clean sweep of W.  lab/c3d_lab.hip, FFN down, one box,
// interleaved (profiles/r04_c3d_xrows.log): passes 97.3 + 63.5 -> 50.9 + 95.2 us, call 281.2 -> 267.5 us; the GEMM
// after it unchanged (121.3 vs 120.3 us).
// kNtW / kNtX: W's and X's fp32 loads non-temporal (the product sets both).  This pass is the last reader of them,
// and with default loads their 384 MiB push the packed operands the GEMM reads next out of the Infinity Cache: the
// FFN-down GEMM takes 108-110 us with its operands resident and 120-123 us after any 512-MiB sweep
// (lab/c3g_lab.hip, profiles/r04_c3g_lab.log: non-temporal sweeps leave them resident, default or sc1 ones do not).
// Call 264.9 -> 248.3 us: pass 2 94.2 -> 87.3, GEMM 120.8 -> 109.4 (profiles/r04_c3d_nt.log).
template <bool kNtW = false, bool kNtX = false>
__global__ __launch_bounds__(256) void pack_cols_then_rows_kernel(
    const float *__restrict__ w, int64_t wsh, int k, int n, float range, const uint32_t *__restrict__ partial,
    int64_t parts, int64_t w_rows_pad, float *__restrict__ w_scale, int8_t *__restrict__ w_q, int64_t k_pad, int gx,
    int gy, const float *__restrict__ x, int64_t xsh, int m, float *__restrict__ x_scale, int8_t *__restrict__ x_q,
    int64_t x_rows_pad, uint32_t *zero_words, int nzero) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][kTc * kTStride];
    __shared__ float s_sh[kTc];
    zero_words_block0(zero_words, nzero);
    const int bid = blockIdx.x, ncb = gx * gy;
    if (bid < ncb) {
        pack_cols_body<true, kTilesPerBlock, kNtW>(bid % gx, gy - 1 - bid / gx, w, wsh, k, n, range, partial, parts,
                                                   w_rows_pad, w_scale, w_q, k_pad, tile, s_sh);
    } else {
        pack_row_block_body<kNtX>(xcd_contig(bid, ncb, (int)gridDim.x - ncb), x, xsh, m, k, range, x_scale, x_q, x_rows_pad,
                            k_pad, s_sh);
    }
}

// ------------------------------------------------------------------------------------------------
// Single-pass packing for the common shapes (row-major X and W, K <= 4096, N % 16 == 0), ONE launch
// of 1024-thread blocks with two roles:
//   W strip (blocks [0, n/16)): 16 columns x all K rows of W held in registers (16 float4 per
//       thread), column absmax reduced on chip (shuffle + LDS), scales computed, quantized from the
//       registers, stored as dwords of the 16 packed rows (4 k-bytes of one column each).
//       W is read from HBM exactly once (the two-pass path reads it twice).
//   X rows (remaining blocks): one wave per row, 16 rows per block (pack_rows_vec_body<16>).
// Thread t of a W strip: c4 = t & 3 (columns n0 + 4*c4 .. +3), rq = t >> 2 (0..255): rows
// 4*rq + e + 1024*i (e, i = 0..3); one wave instruction reads 16 rows x 64 B.
constexpr int kWsCols = 16;
constexpr int kWsMaxK = 4096;

__device__ __forceinline__ void pack_w_strip_body(int strip, const float *__restrict__ w, int64_t wsh, int k,
                                                  int n, float range, float *__restrict__ scale,
                                                  int8_t *__restrict__ q, int64_t k_pad, uint8_t *lds) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c4 = t & 3, rq = t >> 2;
    const int64_t n0 = (int64_t)strip * kWsCols;
    const float w_seed = t < kWsCols ? w[n0 + t] : 0.0f;  // W[0, j], issued first (used after the reduction)
    float *red = reinterpret_cast<float *>(lds);                 // [16 waves][16 cols]
    float *s_sh = red + 16 * 16;                                 // [16] scales
    float4 v[4][4];                                              // [i][e]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            v[i][e] = (r < k) ? *reinterpret_cast<const float4 *>(w + (int64_t)r * wsh + n0 + 4 * c4)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    // column candidates over rows >= 1 (row 0 is the seed)
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            if (r >= 1 && r < k) {
                p0 = cand_max(p0, v[i][e].x);
                p1 = cand_max(p1, v[i][e].y);
                p2 = cand_max(p2, v[i][e].z);
                p3 = cand_max(p3, v[i][e].w);
            }
        }
    // reduce over the 16 lanes of the wave with the same c4 (lane bits 2..5), then over the 16 waves
#pragma unroll
    for (int off = 4; off < 64; off <<= 1) {
        p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
        p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
        p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
        p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
    }
    if (lane < 4) {
        red[wv * 16 + 4 * lane + 0] = p0;
        red[wv * 16 + 4 * lane + 1] = p1;
        red[wv * 16 + 4 * lane + 2] = p2;
        red[wv * 16 + 4 * lane + 3] = p3;
    }
    __syncthreads();
    if (t < kWsCols) {
        float p = red[t];
#pragma unroll
        for (int ww = 1; ww < 16; ++ww) p = fmaxf(p, red[ww * 16 + t]);  // -inf or >= +0: exact
        const float cw = absmax_finish(w_seed, p);                      // seed = W[0, j]
        s_sh[t] = inv_divide(range, cw);
        scale[n0 + t] = cw;
    }
    __syncthreads();
    const float s0 = s_sh[4 * c4 + 0], s1 = s_sh[4 * c4 + 1], s2 = s_sh[4 * c4 + 2], s3 = s_sh[4 * c4 + 3];
    // quantize; 4 consecutive rows of one column = one dword of packed row n0 + 4 c4 + cc.  The quad of threads
    // rq = 4a .. 4a+3 with the same c4 (lanes 4 rq + c4) hold the 16 k of a fragment-major piece: after the quad
    // transpose thread b = rq & 3 stores the piece of packed row n0 + 4 c4 + b, and one wave store instruction
    // writes a whole 1-KiB block (16 rows x 64 k).
    const auto dst = buf_rsrc(q + n0 * k_pad, (uint32_t)(16 * k_pad));
    const int b = rq & 3;
    const int qbase = lane - 4 * b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r0 = 4 * rq + 1024 * i;
        uint32_t d[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            int qe[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = cc == 0 ? v[i][e].x : cc == 1 ? v[i][e].y : cc == 2 ? v[i][e].z : v[i][e].w;
                const float sc = cc == 0 ? s0 : cc == 1 ? s1 : cc == 2 ? s2 : s3;
                qe[e] = (r0 + e < k) ? quant_i8(x, sc) : 0;
            }
            d[cc] = pack4(qe[0], qe[1], qe[2], qe[3]);
        }
        uint32_t pc[4] = {0u, 0u, 0u, 0u};
        quad_transpose(d, b, qbase, 4, pc);
        const int kp = r0 - 4 * b;
        if (kp < k_pad) {
            typedef int v4i_t __attribute__((ext_vector_type(4)));
            const v4i_t val = {(int)pc[0], (int)pc[1], (int)pc[2], (int)pc[3]};
            __builtin_amdgcn_raw_buffer_store_b128(val, dst, (uint32_t)fofs(4 * c4 + b, kp, k_pad), 0, 0);
        }
    }
}

__global__ __launch_bounds__(1024) void pack_single_pass_kernel(
    const float *__restrict__ x, int64_t xsh, int m, int k, float *__restrict__ x_scale, int8_t *__restrict__ x_q,
    int64_t x_rows_pad, int64_t k_pad, const float *__restrict__ w, int64_t wsh, int n, float *__restrict__ w_scale,
    int8_t *__restrict__ w_q, int64_t w_rows_pad, int nstrips, float range, uint32_t *zero_words, int nzero) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    zero_words_block0(zero_words, nzero);
    // roles by block id: [W strips][zero padding strips][X rows] (lab, 4096^3: 30.4 us; X rows first
    // 31.5 us; W and X interleaved in groups of 8 blocks 35.1 us)
    const int bid = blockIdx.x;
    if (bid < nstrips) {
        // blocks b and b+8 run on one XCD: give them adjacent strips, so each 128-B line of W (two
        // 64-B strip segments) is fetched into that XCD's L2 once (bijective for any nstrips)
        const int xcd = bid & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
        const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        pack_w_strip_body(strip, w, wsh, k, n, range, w_scale, w_q, k_pad, dyn_lds);
    } else if (bid < nstrips + (int)((w_rows_pad - n) / kWsCols)) {
        // padding rows of packed W: zero rows, zero scales
        const int64_t n0 = n + (int64_t)(bid - nstrips) * kWsCols;
        zero_packed_rows(w_q, n0, kWsCols, k_pad, threadIdx.x, 1024);
        if (threadIdx.x < kWsCols) w_scale[n0 + threadIdx.x] = 0.0f;
    } else {
        // X rows: 16 rows per 1024-thread block = four 4-row groups of the 256-thread body (rows 16xb + (t>>6)),
        // staged in LDS and written out as whole 1-KiB blocks of the fragment-major q
        const int64_t xb = bid - nstrips - (int)((w_rows_pad - n) / kWsCols);
        const int rsw = (int)(k_pad >> 2) + 16;
        uint32_t *xstage = reinterpret_cast<uint32_t *>(dyn_lds);
        pack_rows_vec_body<16, false, false, true>(xb * 4, x, xsh, m, k, range, x_scale, x_q, x_rows_pad, k_pad, nullptr,
                                                   xstage + (threadIdx.x >> 6) * rsw);
        __syncthreads();
        write_staged_rows<16>(xstage, rsw, x_q, xb * 16, k_pad);
    }
}

// ------------------------------------------------------------------------------------------------
// Single pass for WIDE W (n >= 16384, 2048 < K <= 4096): 32-column strips, so each row segment of W a
// block reads is 128 B -- the 16-column pass's 64-B segments stream at 3.8-3.9 TB/s at n = 16384 / 32768
// (row strides of 64 / 128 KiB).  A 32-column strip of 4096 rows is 512 KiB: one 1024-thread block per
// CU holds rows < 3072 in registers (24 float4 per thread, 96 VGPRs) and rows 3072..4095 in LDS (128 KiB
// through buffer_load ... lds; a lane's slot is the one its own DMA writes, so it reads its rows back
// conflict-free after its own vmcnt, no barrier).  Thread t: c8 = t & 7 (columns n0 + 4*c8 .. +3), rq =
// t >> 3: rows 4*rq + e + 512*i -- one wave instruction reads 8 rows x 128 B.  lab/pack32_lab.hip
// (2048 x n x 4096, µs, 16-column vs 32-column): n = 16384 98.0 -> 85.2, 32768 182.7 -> 162.6, 24576
// 125.3 -> 119.2 (1024 rows: 93.2 -> 87.7); narrower W stays on the 16- / 8-column passes (12288: 59.2 vs
// 62.4, 8192: 43.1 vs 44.5, 4096: 28.7 vs 34.4; 20480 106.8 vs 110.3; K = 2048 37.7 vs 38.9).
constexpr int kW32Cols = 32;
constexpr int kW32RegI = 6;                      // row blocks of 512 held in registers
constexpr int kW32LdsI = 8 - kW32RegI;           // row blocks of 512 held in LDS
constexpr int kW32LdsBytes = kW32LdsI * 4 * 16 * 1024;  // [i][e][wave] x 1 KiB

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void pack_w_strip32_body(int strip, const float *__restrict__ w, int64_t wsh, int k,
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
    const float4 *ls = reinterpret_cast<const float4 *>(lds) + wv * 64 + lane;
#pragma unroll
    for (int i = 0; i < kW32LdsI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 512 * (i + kW32RegI);
            if (r < k) {
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
        for (int e = 0; e < 4; ++e) {
            if (i < kW32RegI) {
                x4[e] = v[i < kW32RegI ? i : 0][e];
            } else {
                // one ds_read_b128 per slot (volatile: hipcc had split the first of these reads into
                // ds_read2_b32 + 2 ds_read_b32, whose lane-linear 16-B stride is a 4-way bank conflict per
                // dword -- all of this pack's LDS bank-conflict cycles, lab/ldsattr_lab.hip)
                typedef float v4f_t __attribute__((ext_vector_type(4)));
                typedef __attribute__((address_space(3))) const volatile v4f_t lds_v4f_t;
                const v4f_t y = *(lds_v4f_t *)(ls + ((i - kW32RegI) * 4 + e) * 16 * 64);
                x4[e] = make_float4(y.x, y.y, y.z, y.w);
            }
        }
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

// kMap (block -> strip order; lab A/B): 0 = XCD-contiguous strip ranges, 1 = strip = block, 2 = even strips
// first then odd, 3 = strips 4j, then 4j + 1, ... (the blocks on the chip at one time spread over the row)
template <int kMap = 0>
__global__ __launch_bounds__(1024) void pack_single_pass32_kernel(
    const float *__restrict__ x, int64_t xsh, int m, int k, float *__restrict__ x_scale, int8_t *__restrict__ x_q,
    int64_t x_rows_pad, int64_t k_pad, const float *__restrict__ w, int64_t wsh, int n, float *__restrict__ w_scale,
    int8_t *__restrict__ w_q, int64_t w_rows_pad, int nstrips, float range, uint32_t *zero_words, int nzero) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_w[kW32LdsBytes];
    __shared__ float red[16 * 32 + 32];
    zero_words_block0(zero_words, nzero);
    const int bid = blockIdx.x;
    const int npad = (int)((w_rows_pad - n) / kW32Cols);
    if (bid < nstrips) {
        int strip;
        if constexpr (kMap == 0) {
            const int xcd = bid & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
            strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        } else if constexpr (kMap == 1) {
            strip = bid;
        } else if constexpr (kMap == 2) {
            const int h = nstrips >> 1;
            strip = (nstrips & 1) ? bid : (bid < h ? 2 * bid : 2 * (bid - h) + 1);
        } else if constexpr (kMap == 3) {
            const int q = nstrips >> 2;
            strip = (nstrips & 3) ? bid : (bid % q) * 4 + bid / q;
        } else {
            // kMap = 100 c + P: P phases over groups of c adjacent strips; phase ph takes groups ph, ph + P, ...
            constexpr int c = kMap / 100, P = kMap % 100;
            if (nstrips % (c * P)) {
                strip = bid;
            } else {
                const int per = nstrips / P, g = bid % c, j = (bid % per) / c, ph = bid / per;
                strip = (j * P + ph) * c + g;
            }
        }
        pack_w_strip32_body(strip, w, wsh, k, range, w_scale, w_q, k_pad, lds_w, red);
    } else if (bid < nstrips + npad) {
        const int64_t n0 = n + (int64_t)(bid - nstrips) * kW32Cols;
        zero_packed_rows(w_q, n0, kW32Cols, k_pad, threadIdx.x, 1024);
        if (threadIdx.x < kW32Cols) w_scale[n0 + threadIdx.x] = 0.0f;
    } else {
        // 16 rows per block, staged in LDS (the strip role's DMA region) and written out as whole 1-KiB blocks
        const int64_t xb = bid - nstrips - npad;
        const int rsw = (int)(k_pad >> 2) + 16;
        uint32_t *xstage = reinterpret_cast<uint32_t *>(lds_w);
        pack_rows_vec_body<16, false, false, true>(xb * 4, x, xsh, m, k, range, x_scale, x_q, x_rows_pad, k_pad, nullptr,
                                                   xstage + (threadIdx.x >> 6) * rsw);
        __syncthreads();
        write_staged_rows<16>(xstage, rsw, x_q, xb * 16, k_pad);
    }
}

// ------------------------------------------------------------------------------------------------
// Single pass at TWO blocks per CU (K <= 4096, n % 8 == 0): 512-thread blocks with the same 16 float4
// per thread, so a block fits in 88 VGPRs (5 waves/SIMD) and a second block on the CU streams its
// loads while the first reduces, quantizes and stores (the 1024-thread single pass leaves the CU's HBM
// stream idle through those phases).  Roles:
//   W strip (blocks [0, n/8)): 8 columns x all K rows; thread t: c2 = t & 1 (columns n0 + 4*c2 .. +3),
//       rows 4*(t>>1) + e + 1024*i (e, i = 0..3).  One wave instruction reads 32 rows x 32 B; the four
//       strips sharing a 128-B line of W run on one XCD (blocks b, b+8, b+16, b+24 get adjacent strips)
//       so the line is fetched once.  Loads and stores are buffer instructions on a wave-uniform
//       descriptor with ONE per-lane offset; rows >= K lie past the descriptor and read as zeros.
//   X rows (the rest): 8 rows per block, one wave per row (pack_rows_vec_body<16>).
// Measured (lab/pack2_lab.hip, 4096^3): 28.0 us vs 31.7 us for the 16-column single pass; better up to
// n = 8192 at K >= 2048, worse for wider W (n = 12288, 16384) and short K, where the 16-column pass stays.
constexpr int kWs8Cols = 8;

template <bool kMask = false, bool kWT = false>
__device__ __forceinline__ void pack_w_strip8_body(int strip, const float *__restrict__ w, int64_t wsh, int k,
                                                   float range, float *__restrict__ scale, int8_t *__restrict__ q,
                                                   int64_t k_pad, float *red /* [8 waves][8 cols] + [8] */,
                                                   const OutlierMask *om = nullptr) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c2 = t & 1, rq = t >> 1;
    const int64_t n0 = (int64_t)strip * kWs8Cols;
    const float w_seed = t < kWs8Cols ? w[n0 + t] : 0.0f;  // W[0, j], issued first (used after the reduction)
    const auto src = buf_rsrc(w + n0, (uint32_t)(((int64_t)(k - 1) * wsh + kWs8Cols) * 4));
    const uint32_t vrow = (uint32_t)((4 * rq * wsh + 4 * c2) * 4);
    float4 v[4][4];  // [i][e]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(src, vrow + (uint32_t)((e + 1024 * i) * wsh * 4), 0, 0);
            v[i][e] = make_float4(__int_as_float(x[0]), __int_as_float(x[1]), __int_as_float(x[2]), __int_as_float(x[3]));
        }
    // the mask words of the thread's rows (4 rq + e + 1024 i: word (4 rq + 1024 i) >> 5), issued behind the strip's
    // loads
    uint32_t mw[4] = {0u, 0u, 0u, 0u}, mw0 = 0u;  // mw0: word 0, whose bit 0 masks the absmax seed
    if constexpr (kMask) {
        // the wave's 16 words (rq >> 3 = 4 wv .. 4 wv + 3, + 32 i) are loaded once, lane b + 4 i holding word
        // 4 wv + b + 32 i, lane 16 word 0; each thread takes its 4 by ds_bpermute
        const int b0 = (rq >> 3) - 4 * wv;
        const int wl[1] = {lane < 16 ? 4 * wv + (lane & 3) + 32 * (lane >> 2) : (lane == 16 ? 0 : om->nwords)};
        uint32_t m1[1];
        om->words(wl, m1);
#pragma unroll
        for (int i = 0; i < 4; ++i) mw[i] = (uint32_t)__shfl((int)m1[0], b0 + 4 * i, 64);
        mw0 = __builtin_amdgcn_readlane(m1[0], 16);
    }
    bool seed_masked = false;
    if constexpr (kMask) {
        // outlier rows of W (outlier feature columns of X): W' holds +0 there; branch-free selects
        {
            seed_masked = mw0 & 1u;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * rq + e + 1024 * i;
                    const bool z = r < k && ((mw[i] >> (r & 31)) & 1u);
                    v[i][e].x = z ? 0.0f : v[i][e].x;
                    v[i][e].y = z ? 0.0f : v[i][e].y;
                    v[i][e].z = z ? 0.0f : v[i][e].z;
                    v[i][e].w = z ? 0.0f : v[i][e].w;
                }
        }
    }
    // column candidates over rows >= 1 (row 0 is the seed)
    float p0 = -INFINITY, p1 = -INFINITY, p2 = -INFINITY, p3 = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * rq + e + 1024 * i;
            if (r >= 1 && r < k) {
                p0 = cand_max(p0, v[i][e].x);
                p1 = cand_max(p1, v[i][e].y);
                p2 = cand_max(p2, v[i][e].z);
                p3 = cand_max(p3, v[i][e].w);
            }
        }
    // over the 32 lanes of the wave with the same c2 (lane bits 1..5), then over the 8 waves
#pragma unroll
    for (int off = 2; off < 64; off <<= 1) {
        p0 = fmaxf(p0, __shfl_xor(p0, off, 64));
        p1 = fmaxf(p1, __shfl_xor(p1, off, 64));
        p2 = fmaxf(p2, __shfl_xor(p2, off, 64));
        p3 = fmaxf(p3, __shfl_xor(p3, off, 64));
    }
    if (lane < 2) {
        red[wv * 8 + 4 * lane + 0] = p0;
        red[wv * 8 + 4 * lane + 1] = p1;
        red[wv * 8 + 4 * lane + 2] = p2;
        red[wv * 8 + 4 * lane + 3] = p3;
    }
    __syncthreads();
    float *s_sh = red + 8 * 8;
    if (t < kWs8Cols) {
        float pm = red[t];
#pragma unroll
        for (int ww = 1; ww < 8; ++ww) pm = fmaxf(pm, red[ww * 8 + t]);  // -inf or >= +0: exact
        const float cw = absmax_finish(seed_masked ? 0.0f : w_seed, pm);  // seed = W[0, j] (W'[0, j])
        s_sh[t] = inv_divide(range, cw);
        st_f32<kWT>(scale + n0 + t, cw);
    }
    __syncthreads();
    const float s0 = s_sh[4 * c2 + 0], s1 = s_sh[4 * c2 + 1], s2 = s_sh[4 * c2 + 2], s3 = s_sh[4 * c2 + 3];
    // 4 consecutive rows of one column = one dword of packed row n0 + 4*c2 + cc.  The strip's 8 packed rows are
    // half of a 16-row group of the fragment-major q (descriptor over the group), and a 16-B piece of it (one
    // packed row, 16 consecutive k) is the dwords of the 4 threads rq = 4a .. 4a+3 with the same c2 (lanes
    // 2 rq + c2).  A 4 x 4 transpose among those lanes (4 shuffles) leaves thread b = rq & 3 holding the piece of
    // packed row 4 c2 + b, so one wave store instruction writes 16 B per lane = 8 whole 128-B lines (rows 0-7
    // of the group, 2 k-blocks x 4 k-chunks), not 4-B pieces of 16 lines.
    const int64_t g0 = n0 & ~(int64_t)15;
    const auto dst = buf_rsrc(q + g0 * k_pad, (uint32_t)(16 * k_pad));
    const int b = rq & 3;
    const int qbase = lane - 2 * b;  // lane of this quad's b = 0 thread
    const int prow = (int)(n0 - g0) + 4 * c2 + b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r0 = 4 * rq + 1024 * i;
        uint32_t d[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            int qe[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = cc == 0 ? v[i][e].x : cc == 1 ? v[i][e].y : cc == 2 ? v[i][e].z : v[i][e].w;
                const float sc = cc == 0 ? s0 : cc == 1 ? s1 : cc == 2 ? s2 : s3;
                qe[e] = (r0 + e < k) ? quant_i8(x, sc) : 0;
            }
            d[cc] = pack4(qe[0], qe[1], qe[2], qe[3]);
        }
        uint32_t pc[4] = {0u, 0u, 0u, 0u};
        quad_transpose(d, b, qbase, 2, pc);
        const int kp = r0 - 4 * b;  // the piece's first k (a multiple of 16)
        if (kp < k_pad) {
            typedef int v4i_t __attribute__((ext_vector_type(4)));
            const v4i_t val = {(int)pc[0], (int)pc[1], (int)pc[2], (int)pc[3]};
            __builtin_amdgcn_raw_buffer_store_b128(val, dst, (uint32_t)fofs(prow, kp, k_pad), 0, kWT ? 16 /* sc1 */ : 0);
        }
    }
}

// Roles by block id: [W strips][W padding][X rows] (measured against W / X alternating and X rows first:
// 29.1 vs 35.6 / 30.5 µs at 4096^3, 41.0 vs 42.2 / 43.0 at 8192 x 4096^2; profiles/r03_pack8_order_lab.log)
template <int kWavesPerEu, bool kMask = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(kWavesPerEu, kWavesPerEu))) void pack_single_pass8_kernel(
    const float *__restrict__ x, int64_t xsh, int m, int k, float *__restrict__ x_scale, int8_t *__restrict__ x_q,
    int64_t x_rows_pad, int64_t k_pad, const float *__restrict__ w, int64_t wsh, int n, float *__restrict__ w_scale,
    int8_t *__restrict__ w_q, int64_t w_rows_pad, int nstrips, float range, uint32_t *zero_words, int nzero,
    OutlierMask om = OutlierMask{}) {
    __shared__ float red[8 * 8 + 8];
    __shared__ __attribute__((aligned(16))) uint32_t xstage[8 * kStageRowWordsMax];  // X rows, LDS-staged
    zero_words_block0(zero_words, nzero);
    const int npad = (int)((w_rows_pad - n) / kWs8Cols);
    const int bid = blockIdx.x;
    if (bid < nstrips) {
        // blocks b, b+8, ... run on one XCD: XCD-contiguous strip ranges (bijective for any nstrips)
        const int xcd = bid & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
        const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        pack_w_strip8_body<kMask>(strip, w, wsh, k, range, w_scale, w_q, k_pad, red, &om);
        if constexpr (kMask)
            if (bid == 0) {
                __syncthreads();  // red is reused as the scan's wave sums
                outlier_column_list(om, reinterpret_cast<int *>(red));
            }
    } else if (bid < nstrips + npad) {
        const int64_t n0 = n + (int64_t)(bid - nstrips) * kWs8Cols;
        zero_packed_rows(w_q, n0, kWs8Cols, k_pad, threadIdx.x, 512);
        if (threadIdx.x < kWs8Cols) w_scale[n0 + threadIdx.x] = 0.0f;
    } else {
        // rows 8xb + (t>>6): two 4-row groups of the 256-thread body, staged in LDS and written out as whole
        // 128-B lines of the fragment-major q (a line = 8 rows x 16 B: exactly this block's rows)
        const int64_t xb = bid - nstrips - npad;
        const int rsw = (int)(k_pad >> 2) + 16;
        pack_rows_vec_body<16, kMask, false, true>(xb * 2, x, xsh, m, k, range, x_scale, x_q, x_rows_pad, k_pad, &om,
                                                   xstage + (threadIdx.x >> 6) * rsw);
        __syncthreads();
        write_staged_rows<8>(xstage, rsw, x_q, xb * 8, k_pad);
    }
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fill_uniform_kernel(float *__restrict__ dst, int64_t count, uint64_t seed,
                                                           float lo, float hi) {
    const uint64_t key = mix64(seed + 0x9E3779B97F4A7C15ULL);
    const float span = __fsub_rn(hi, lo);
    const float shift = __fdiv_rn(lo, span);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t z = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        const float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
        dst[i] = __fmul_rn(__fadd_rn(u, shift), span);
    }
}

bool rows_vec_ok(const float *src, int64_t sh, int64_t sw, int rows) {
    return sw == 1 && (sh % 4 == 0 || rows == 1) && (reinterpret_cast<uintptr_t>(src) % 16 == 0);
}

bool cols_vec_ok(const float *src, int64_t sh, int cols) {
    return (cols % 4 == 0) && (sh % 4 == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0);
}

int rows_regs(int len) {  // float4 chunks per lane -> register-resident variant (-1 = block per row, 0 = streaming)
    const int per_lane = ((len >> 2) + 63) / 64;
    if (per_lane > 16) return len <= kLongRowMax ? -1 : 0;
    return per_lane <= 1 ? 1 : per_lane <= 2 ? 2 : per_lane <= 4 ? 4 : per_lane <= 8 ? 8 : 16;
}

}  // namespace

hipError_t launch_pack_rows(const float *src, int64_t sh, int64_t sw, int rows, int len, float range, PackedView out,
                            hipStream_t stream) {
    const dim3 grid((unsigned)(out.rows_pad / 4)), block(256);
    if (!rows_vec_ok(src, sh, sw, rows)) {
        pack_rows_generic_kernel<<<grid, block, 0, stream>>>(src, sh, sw, rows, len, range, out.scale, out.q,
                                                             out.rows_pad, out.k_pad);
        return hipGetLastError();
    }
    const bool pairs = out.rows_pad < 2048;  // fewer than 256 staged 8-row blocks
#define QG_ROWS(Rv)                                                                                                   \
    if ((Rv) > 0 && pairs)                                                                                            \
        pack_rows_pair_kernel<((Rv) > 0 ? (Rv) : 1)><<<(unsigned)(out.rows_pad / 2), 128, 0, stream>>>(                 \
            src, sh, rows, len, range, out.scale, out.q, out.rows_pad, out.k_pad);                                    \
    else                                                                                                              \
        pack_rows_vec_kernel<Rv><<<(Rv) > 0 ? (unsigned)(out.rows_pad / 8) : grid.x, (Rv) > 0 ? 512 : 256, 0, stream>>>( \
            src, sh, rows, len, range, out.scale, out.q, out.rows_pad, out.k_pad)
    if (rows_regs(len) < 0) {
        pack_rows_block_kernel<<<(unsigned)out.rows_pad, 256, 0, stream>>>(src, sh, rows, len, range, out.scale, out.q,
                                                                           out.rows_pad, out.k_pad);
        return hipGetLastError();
    }
    switch (rows_regs(len)) {
        case 1: QG_ROWS(1); break;
        case 2: QG_ROWS(2); break;
        case 4: QG_ROWS(4); break;
        case 8: QG_ROWS(8); break;
        case 16: QG_ROWS(16); break;
        default: QG_ROWS(0); break;
    }
#undef QG_ROWS
    return hipGetLastError();
}

hipError_t launch_pack_cols_pass2(const float *src, int64_t sh, int len, int cols, float range, PackedView out,
                                  hipStream_t stream) {
    const dim3 g2((unsigned)(out.rows_pad / kTc), (unsigned)((out.k_pad / kTk + kTilesPerBlock - 1) / kTilesPerBlock));
    const int64_t parts = len > 1 ? out.parts : 0;  // K = 1: no candidates, Cw = seed
    // bottom rows of W first: pass 1 swept W top to bottom, so its last rows are still in the Infinity Cache
    // (lab/c3d_lab.hip, FFN down: pass 2 72.5 -> 64.2 us with X-first pass 1, profiles/r04_c3d_order_lab.log)
    if (cols_vec_ok(src, sh, cols))
        pack_cols_kernel<true, kTilesPerBlock, true><<<g2, 256, 0, stream>>>(src, sh, len, cols, range, out.scratch,
                                                                             parts, out.rows_pad, out.scale, out.q,
                                                                             out.k_pad);
    else
        pack_cols_kernel<false, kTilesPerBlock, true><<<g2, 256, 0, stream>>>(src, sh, len, cols, range, out.scratch,
                                                                              parts, out.rows_pad, out.scale, out.q,
                                                                              out.k_pad);
    return hipGetLastError();
}

hipError_t launch_pack_cols(const float *src, int64_t sh, int len, int cols, float range, PackedView out,
                            hipStream_t stream) {
    if (len > 1) {
        const dim3 g1((unsigned)((cols + kColBlock - 1) / kColBlock), (unsigned)out.parts);
        if (cols_vec_ok(src, sh, cols)) colmax_kernel<true><<<g1, 256, 0, stream>>>(src, sh, len, cols, out.scratch, out.rows_pad);
        else colmax_kernel<false><<<g1, 256, 0, stream>>>(src, sh, len, cols, out.scratch, out.rows_pad);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_pack_cols_pass2(src, sh, len, cols, range, out, stream);
}

// kind: 0 = choose (the 8-column two-blocks-per-CU pass where it measured faster, else 16 columns),
// 8 or 16 = force that strip width (lab)
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) of pack_single_pass_kernel, once per device
static hipError_t pack16_lds_attr() {
    constexpr int kMaxDev = 64;
    static std::atomic<int> set[kMaxDev];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    if (set[dev].load(std::memory_order_acquire)) return hipSuccess;
    e = hipFuncSetAttribute(reinterpret_cast<const void *>(pack_single_pass_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 4 * kStageRowWordsMax);
    if (e == hipSuccess) set[dev].store(1, std::memory_order_release);
    return e;
}

hipError_t launch_pack_single_pass_kind(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                        int64_t wsh, int n, PackedView outw, float range, hipStream_t stream, int kind,
                                        uint32_t *zero_words, int nzero) {
    if (k < 1 || k > kWsMaxK || !rows_vec_ok(x, xsh, 1, m) || !cols_vec_ok(w, wsh, n)) return hipErrorNotSupported;
    const bool can8 = n % kWs8Cols == 0 && ((int64_t)k * wsh + kWs8Cols) * 4 < ((int64_t)1 << 31);
    const bool can16 = n % kWsCols == 0;
    const bool can32 = n % kW32Cols == 0 && ((int64_t)k * wsh + kW32Cols) * 4 < ((int64_t)1 << 31);
    if (kind == 0) kind = (can32 && n >= 16384 && k > 2048) ? 32 : (can8 && n <= 8192 && k > 1024) || !can16 ? 8 : 16;
    if (kind == 32) {
        if (!can32) return hipErrorNotSupported;
        const int nstrips = n / kW32Cols;
        const int npad = (int)((outw.rows_pad - n) / kW32Cols);
        const int nx = (int)(outx.rows_pad / 16);
        // strip order: groups of 2 adjacent strips, 4 phases (lab/pack32_lab.hip at 2048 x 16384 x 4096: 85.8-86.2
        // vs 90.9-91.2 us for XCD-contiguous ranges, the <0> instantiation the lab keeps)
        pack_single_pass32_kernel<204><<<nstrips + npad + nx, 1024, 0, stream>>>(
            x, xsh, m, k, outx.scale, outx.q, outx.rows_pad, outx.k_pad, w, wsh, n, outw.scale, outw.q, outw.rows_pad,
            nstrips, range, zero_words, nzero);
        return hipGetLastError();
    }
    if (kind == 8) {
        if (!can8) return hipErrorNotSupported;
        const int nstrips = n / kWs8Cols;
        const int npad = (int)((outw.rows_pad - n) / kWs8Cols);
        const int nx = (int)(outx.rows_pad / 8);
        pack_single_pass8_kernel<5><<<nstrips + npad + nx, 512, 0, stream>>>(x, xsh, m, k, outx.scale, outx.q,
                                                                          outx.rows_pad, outx.k_pad, w, wsh, n,
                                                                          outw.scale, outw.q, outw.rows_pad, nstrips,
                                                                          range, zero_words, nzero);
        return hipGetLastError();
    }
    if (!can16) return hipErrorNotSupported;
    const int nstrips = n / kWsCols;
    const int npad = (int)((outw.rows_pad - n) / kWsCols);
    const int nx = (int)(outx.rows_pad / 16);
    // W strips: [16 waves][16 cols] partial maxima + 16 scales; X rows: 16 staged packed rows
    const size_t lds = std::max<size_t>(4096, (size_t)16 * 4 * (outx.k_pad / 4 + 16));
    // above 64 KiB of dynamic LDS (K > 4032) the kernel needs the attribute -- set once per DEVICE (one process may
    // drive every GPU of a node, qgemm_node_mm_quantize); a failure is returned, not remembered
    if (lds > 65536) {
        const hipError_t lds_attr = pack16_lds_attr();
        if (lds_attr != hipSuccess) return lds_attr;
    }
    pack_single_pass_kernel<<<nstrips + npad + nx, 1024, lds, stream>>>(x, xsh, m, k, outx.scale, outx.q, outx.rows_pad,
                                                                         outx.k_pad, w, wsh, n, outw.scale, outw.q,
                                                                         outw.rows_pad, nstrips, range, zero_words,
                                                                         nzero);
    return hipGetLastError();
}

bool pack_single_pass_outlier_ok(const float *x, int64_t xsh, int m, int k, const float *w, int64_t wsh, int n) {
    return k >= 1 && k <= kWsMaxK && !(k & 3) && rows_vec_ok(x, xsh, 1, m) && cols_vec_ok(w, wsh, n) &&
           n % kWs8Cols == 0 && ((int64_t)k * wsh + kWs8Cols) * 4 < ((int64_t)1 << 31);
}

hipError_t launch_pack_single_pass_outlier(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                           int64_t wsh, int n, PackedView outw, float range, const uint32_t *partial,
                                           int nparts, int nwords, int *idx, hipStream_t stream) {
    if (!pack_single_pass_outlier_ok(x, xsh, m, k, w, wsh, n)) return hipErrorNotSupported;
    const int nstrips = n / kWs8Cols;
    const int npad = (int)((outw.rows_pad - n) / kWs8Cols);
    const int nx = (int)(outx.rows_pad / 8);
    if (nwords > 128 || nparts < 1 || nparts > 16) return hipErrorNotSupported;  // K <= 4096: the single pass's envelope
    const OutlierMask om{partial, nwords, nparts, idx};
    // a 4-waves-per-SIMD register budget (102 VGPRs, the same two blocks per CU): at 5 the masked body spilled
    // 20 B per lane (profiles/r03_ab_maskpack_wpe.log)
    pack_single_pass8_kernel<4, true><<<nstrips + npad + nx, 512, 0, stream>>>(
        x, xsh, m, k, outx.scale, outx.q, outx.rows_pad, outx.k_pad, w, wsh, n, outw.scale, outw.q, outw.rows_pad,
        nstrips, range, nullptr, 0, om);
    return hipGetLastError();
}

hipError_t launch_pack_single_pass(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                   int64_t wsh, int n, PackedView outw, float range, hipStream_t stream,
                                   uint32_t *zero_words, int nzero) {
    return launch_pack_single_pass_kind(x, xsh, m, k, outx, w, wsh, n, outw, range, stream, 0, zero_words, nzero);
}

hipError_t launch_fill_uniform(float *dst, int64_t count, uint64_t seed, float lo, float hi, hipStream_t stream) {
    if (count <= 0) return hipSuccess;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    fill_uniform_kernel<<<(unsigned)blocks, 256, 0, stream>>>(dst, count, seed, lo, hi);
    return hipGetLastError();
}

hipError_t launch_pack_two_pass(const float *a, int64_t ash, int m, int k, PackedView outa, const float *b, int64_t bsh,
                                int n, PackedView outb, float range, hipStream_t stream, uint32_t *zero_words, int nzero) {
    if (k < 2 || !rows_vec_ok(a, ash, 1, m) || !cols_vec_ok(b, bsh, n)) return hipErrorNotSupported;
    if (rows_regs(k) < 0) {
        // long rows: W-only pass 1 (column maxima), then pass 2 bottom-up with X's rows at its end, both read
        // non-temporally (they would displace the packed operands from the Infinity Cache)
        const int col_blocks = (n + kColBlock - 1) / kColBlock;
        colmax_kernel<true><<<dim3((unsigned)col_blocks, (unsigned)outb.parts), 256, 0, stream>>>(b, bsh, k, n, outb.scratch,
                                                                                               outb.rows_pad);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const unsigned gx = (unsigned)(outb.rows_pad / kTc);
        const unsigned gy = (unsigned)((outb.k_pad / kTk + kTilesPerBlock - 1) / kTilesPerBlock);
        pack_cols_then_rows_kernel<true, true><<<gx * gy + (unsigned)outa.rows_pad, 256, 0, stream>>>(
            b, bsh, k, n, range, outb.scratch, outb.parts, outb.rows_pad, outb.scale, outb.q, outb.k_pad, (int)gx, (int)gy,
            a, ash, m, outa.scale, outa.q, outa.rows_pad, zero_words, nzero);
        return hipGetLastError();
    }
    hipError_t e = launch_pack_rows_and_colmax(a, ash, m, k, outa, b, bsh, n, outb, range, stream, zero_words, nzero);
    if (e != hipSuccess) return e;
    return launch_pack_cols_pass2(b, bsh, k, n, range, outb, stream);
}

hipError_t launch_pack_rows_and_colmax(const float *a, int64_t ash, int m, int k, PackedView outa, const float *b,
                                         int64_t bsh, int n, PackedView outb, float range, hipStream_t stream,
                                         uint32_t *zero_words, int nzero) {
    if (k < 2 || !rows_vec_ok(a, ash, 1, m) || !cols_vec_ok(b, bsh, n)) return hipErrorNotSupported;
    const int col_blocks = (n + kColBlock - 1) / kColBlock;
    const int ncol = col_blocks * (int)outb.parts;
    const int rr = rows_regs(k);
    const int nrow = (int)(rr < 0 ? outa.rows_pad : outa.rows_pad / 4);  // block per row / 4 rows per block
    // X's row blocks first, W's column-max sweep last: W's rows are then the most recent bytes in the Infinity Cache
    // when pass 2 re-reads them bottom-up (lab/c3d_lab.hip, FFN down, one box, interleaved: call 291.1 -> 282.9 us)
#define QG_FUSED(Rv)                                                                                            \
    pack_rows_and_colmax_kernel<Rv, true><<<ncol + nrow, 256, 0, stream>>>(a, ash, m, k, outa.scale, outa.q,          \
                                                                     outa.rows_pad, outa.k_pad, b, bsh, n,       \
                                                                     outb.scratch, outb.rows_pad, col_blocks,    \
                                                                     ncol, range, zero_words, nzero)
    switch (rr) {
        case -1: QG_FUSED(-1); break;
        case 1: QG_FUSED(1); break;
        case 2: QG_FUSED(2); break;
        case 4: QG_FUSED(4); break;
        case 8: QG_FUSED(8); break;
        case 16: QG_FUSED(16); break;
        default: QG_FUSED(0); break;
    }
#undef QG_FUSED
    return hipGetLastError();
}

}  // namespace qgemm
