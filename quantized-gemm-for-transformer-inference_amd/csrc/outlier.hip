// outlier.hip -- LLM.int8() mixed-precision decomposition: the feature columns of X
// that hold an outlier are multiplied in fp32, the rest through the int8 absmax path, so the outliers
// no longer set the row scales Cx.  The reference carries only the building blocks, unused:
// op_outlier_extractor / AbsCompareLTEConstFunc (op_elemwise.cuh:293-306, 698-708) and op_round_int8
// (:167-176, 685-695).  Definition (DESIGN.md "Outlier decomposition"; the oracle restates it):
//   outlier column k  : some X[i,k] is not (|x| <= t)  -- AbsCompareLTEConstFunc returns 1 (NaN: 1)
//   O8  = op_quantized_mm(X', W'), X' = X with the outlier columns zeroed, W' = W with those rows zeroed
//   Co  = fmaf chain from +0 over the outlier columns in ascending k: X[i,k] * W[k,j]
//   O   = fl(O8 + Co)            (no outlier columns: O = O8, the plain path)
//
// One call, fast path (row-major operands on the single-pass pack + 256-tile GEMM): three launches --
//   outlier_colmask: X read once; workgroup (w, p) reads columns 32 w .. +31 over row split p and writes mask word w
//                    of that split with one plain store (2 splits at K = 4096) -- every word written every
//                    call, so no state lives on between calls (no counters, no accumulator, no zeroing)
//   the pack       : the single pass with the mask (pack.hip): X'/W' quantized without materialising them, every
//                    thread reading the mask words of its own elements; its workgroup 0 writes the outlier count
//                    and the ascending column list
//   the GEMM       : the int8 part with the fp32 chain added in its store epilogue (gemm_i8_kernels.h), its
//                    operands read from X's outlier columns and W's outlier rows where they lie
// Other shapes: the state zeroed, flags + index (built by the last-arriving flags workgroup), X'/W' materialised by
// a masking pass, the plain drop-in on them, and a correction kernel adding the chain to O.
#include <algorithm>

#include "qgemm_internal.h"

namespace qgemm {

// The fallback's flags launch keeps per-call state in the caller's outlier scratch (scratch_view), right after the
// index: 9 arrival counters (8 per-XCD + 1 global, each on a 128-B line of its own) and, for K <= 32 768 (kAccWords
// words of 32 columns), the mask accumulator -- each flags workgroup ORs its nonzero mask words into it with
// agent-scope atomics (performed at the memory side, coherent across XCDs), so the last workgroup reads nwords words
// instead of every chunk's partial words.  outlier_zero_state_kernel zeroes it at the start of every such call:
// calls with different workspaces (streams, graph replays) share nothing, and a failed call leaves nothing behind.
constexpr int kCounterWords = 32, kTicketWords = 9 * kCounterWords;
constexpr int kAccWords = 1024;

namespace {

constexpr int kChunkRows = 64;     // rows per flags block
constexpr int kFlagCols = 1024;    // columns per flags block (256 threads x 4)

// AbsCompareLTEConstFunc (op_elemwise.cuh:296-304): 0 when a in [-b, b], else 1 (NaN -> 1)
__device__ __forceinline__ bool is_outlier(float a, float b) {
    return !(((a >= 0) & (a <= b)) | ((a <= 0) & (-a <= b)));
}

// bits[w] = OR of the chunk masks, rank[w] = set bits below word w, idx[1 + ...] = the outlier columns in
// ascending order, idx[0] = their count -- by the ONE workgroup of outlier_flags_kernel that arrives last.  P
// adjacent threads share a word (each ORs every P-th chunk, 16 sc1 loads in flight, then a shuffle-OR),
// kThreads / P words per pass; the ranks by a wave scan + a scan of the wave sums.
template <int P, int kThreads>
__device__ __forceinline__ void build_index(const uint32_t *__restrict__ partial, int nchunks, int nwords,
                                            uint32_t *__restrict__ bits, int *__restrict__ rank, int *__restrict__ idx,
                                            int *wsum, int *base) {
    constexpr int kWaves = kThreads / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s = tid % P;
    int run = 0;  // count of outlier columns in the words already done (the same in every thread)
    for (int w0 = 0; w0 < nwords; w0 += kThreads / P) {
        const int w = w0 + tid / P;
        uint32_t word = 0;
        if (w < nwords) {
            int ch = s;
            // the partial words are the other workgroups' sc1 stores: every load of them is an sc1 load
            for (; ch + 15 * P < nchunks; ch += 16 * P) {
                uint32_t u[16];
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    u[e] = __hip_atomic_load(partial + (int64_t)(ch + e * P) * nwords + w, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int e = 0; e < 16; ++e) word |= u[e];
            }
            for (; ch < nchunks; ch += P)
                word |= __hip_atomic_load(partial + (int64_t)ch * nwords + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int off = 1; off < P; off <<= 1) word |= (uint32_t)__shfl_xor((int)word, off, 64);
        const int pc = (s == 0 && w < nwords) ? __popc(word) : 0;
        int x = pc;  // inclusive scan over the block in thread order (= word order)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(x, off, 64);
            if (lane >= off) x += v;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        int before = run;
        for (int j = 0; j < wave; ++j) before += wsum[j];
        const int below = before + x - pc;
        if (s == 0 && w < nwords) {
            bits[w] = word;
            rank[w] = below;
            int j = 0;
            for (uint32_t b = word; b; b &= b - 1, ++j) idx[1 + below + j] = 32 * w + __builtin_ctz(b);
        }
#pragma unroll
        for (int j = 0; j < kWaves; ++j) run += wsum[j];
        __syncthreads();  // wsum is rewritten by the next pass
    }
    if (tid == 0) *base = run;
}

// (fallback) Mask word w of a 64-row chunk: bit c set when column 32w + c holds an outlier in the chunk's rows.  1024
// threads = 4 row groups x 256 column threads: thread (g, t) reads columns 1024 bx + 4t .. +3 of rows 16 g .. 16 g + 15
// of the chunk (16 float4 loads in flight per thread, 16 waves per CU), the groups' nibbles meet in LDS.  kAcc:
// nonzero words are ORed into the call's accumulator (agent-scope atomics); else every word is stored
// to partial[chunk][word] (sc1).  Then each workgroup, after every wave's stores / atomics have drained, arrives
// on its XCD's counter (one lane, agent scope), and the last of each XCD on the global counter -- sharded, because
// ≈ 12 ns per arrival serialise on one counter (MI355X_MICROARCH.md fan-in row); the write-through hand-off of the
// sc1 table, row 1, at each level.  The workgroup that arrives last overall
// builds the column mask, ranks, list and count (build_index over the accumulator or the partial words) -- no
// separate index launch.
constexpr int kFlagThreads = 1024, kFlagGroups = 4, kGroupRows = kChunkRows / kFlagGroups;
template <bool VEC, bool kAcc>
__global__ __launch_bounds__(kFlagThreads) void outlier_flags_kernel(const float *__restrict__ X, int64_t xsh, int m,
                                                                     int k, float t, uint32_t *__restrict__ partial,
                                                                     int nwords, unsigned *ticket, uint32_t *acc,
                                                                     uint32_t *__restrict__ bits, int *__restrict__ rank,
                                                                     int *__restrict__ idx) {
    // ticket: counter x (x < 8: per XCD, 8: global) at x * kCounterWords; acc: nwords mask words (kAcc)
    __shared__ int wsum[kFlagThreads / 64];
    __shared__ uint32_t nibs[kFlagGroups - 1][256];
    __shared__ unsigned last;
    __shared__ int count;
    const int tid = threadIdx.x, ct = tid & 255, g = tid >> 8;
    const int c = blockIdx.x * kFlagCols + 4 * ct;
    const int r0 = blockIdx.y * kChunkRows + g * kGroupRows, r1 = min(m, r0 + kGroupRows);
    uint32_t nib = 0;
    if (c < k) {
        if constexpr (VEC) {
            const float *p = X + (int64_t)r0 * xsh + c;
#pragma unroll 16
            for (int r = r0; r < r1; ++r, p += xsh) {
                const float4 x = *reinterpret_cast<const float4 *>(p);
                nib |= (is_outlier(x.x, t) ? 1u : 0u) | (is_outlier(x.y, t) ? 2u : 0u) | (is_outlier(x.z, t) ? 4u : 0u) |
                       (is_outlier(x.w, t) ? 8u : 0u);
            }
        } else {
            for (int r = r0; r < r1; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (c + e < k && is_outlier(X[(int64_t)r * xsh + c + e], t)) nib |= 1u << e;
        }
    }
    if (g > 0) nibs[g - 1][ct] = nib;
    __syncthreads();
    if (g == 0) {
#pragma unroll
        for (int j = 0; j < kFlagGroups - 1; ++j) nib |= nibs[j][ct];
        // eight consecutive lanes hold one 32-column word
        uint32_t word = nib << (4 * (ct & 7));
        word |= __shfl_xor(word, 1, 64);
        word |= __shfl_xor(word, 2, 64);
        word |= __shfl_xor(word, 4, 64);
        const int w = blockIdx.x * (kFlagCols / 32) + (ct >> 3);
        if ((ct & 7) == 0 && w < nwords) {
            if constexpr (kAcc) {
                if (word) __hip_atomic_fetch_or(acc + w, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(partial + (int64_t)blockIdx.y * nwords + w, word, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
        // blocks b, b + 8, ... share an XCD (round-robin dispatch); the last of each XCD arrives globally
        const unsigned total = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x, xcd = bid & 7;
        const unsigned on_xcd = (total - xcd + 7) / 8, xcds = total < 8 ? total : 8;
        unsigned fin = 0;
        unsigned *mine = ticket + xcd * kCounterWords, *all = ticket + 8 * kCounterWords;
        if (__hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == on_xcd - 1 &&
            __hip_atomic_fetch_add(all, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == xcds - 1)
            fin = 1;
        last = fin;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the sc1 loads stay below
    if constexpr (kAcc) build_index<1, kFlagThreads>(acc, 1, nwords, bits, rank, idx, wsum, &count);
    else build_index<1, kFlagThreads>(partial, (int)gridDim.y, nwords, bits, rank, idx, wsum, &count);
    __syncthreads();
    if (tid == 0) idx[0] = count;
}

// the flags launch's counters and accumulator (scratch_view: state, state_words) to zero, ahead of it in the stream
__global__ __launch_bounds__(256) void outlier_zero_state_kernel(uint32_t *__restrict__ state, int words) {
    for (int i = threadIdx.x; i < words; i += 256) state[i] = 0u;
}

// Fast path: the column mask with no cross-workgroup combine.  Workgroup (w, p) owns mask word w (columns
// 32 w .. +31) over row split p (rows [p rps, (p + 1) rps)): 1024 threads, thread t reads the 16-B piece t & 7 of rows
// (t >> 3) + 128 i (a wave-instruction = 8 rows x 128 B; 16 loads in flight per thread), ORs its nibbles, the 128
// row-threads of each piece meet by shuffles and LDS, and ONE plain store writes partial[p][w].  Every partial word is
// written every call: no counters, no accumulator, nothing kept between calls (2 splits at K = 4096: the pack ORs
// two words per mask word).
constexpr int kColmaskRowsPerPass = kFlagThreads / 8;  // 128
__global__ __launch_bounds__(kFlagThreads) void outlier_colmask_kernel(const float *__restrict__ X, int64_t xsh, int m,
                                                                       int k, float t, int rps,
                                                                       uint32_t *__restrict__ partial, int nwords) {
    __shared__ uint32_t nibs[kFlagThreads / 64][8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, piece = tid & 7;
    const int c = blockIdx.x * 32 + 4 * piece;
    const int r0 = blockIdx.y * rps, r1 = min(m, r0 + rps);
    uint32_t nib = 0;
    if (c < k) {
        const float *p = X + (int64_t)(r0 + (tid >> 3)) * xsh + c;
        const int64_t step = (int64_t)kColmaskRowsPerPass * xsh;
#pragma unroll 16
        for (int r = r0 + (tid >> 3); r < r1; r += kColmaskRowsPerPass, p += step) {
            const float4 x = *reinterpret_cast<const float4 *>(p);
            nib |= (is_outlier(x.x, t) ? 1u : 0u) | (is_outlier(x.y, t) ? 2u : 0u) | (is_outlier(x.z, t) ? 4u : 0u) |
                   (is_outlier(x.w, t) ? 8u : 0u);
        }
    }
    // the wave's 8 row-threads of each piece (lane bits 3..5), then the 16 waves
    nib |= (uint32_t)__shfl_xor((int)nib, 8, 64);
    nib |= (uint32_t)__shfl_xor((int)nib, 16, 64);
    nib |= (uint32_t)__shfl_xor((int)nib, 32, 64);
    if (lane < 8) nibs[wave][lane] = nib;
    __syncthreads();
    if (tid < 8) {
        uint32_t x = 0u;
#pragma unroll
        for (int v = 0; v < kFlagThreads / 64; ++v) x |= nibs[v][tid];
        uint32_t word = x << (4 * tid);
        word |= (uint32_t)__shfl_xor((int)word, 1, 64);
        word |= (uint32_t)__shfl_xor((int)word, 2, 64);
        word |= (uint32_t)__shfl_xor((int)word, 4, 64);
        if (tid == 0) partial[(int64_t)blockIdx.y * nwords + blockIdx.x] = word;
    }
}

// the fast path's row splits: about 256 workgroups for the stream (128 at K = 4096 read 64 MiB in 16.0 us, 256 in
// 11.x), each split a multiple of 128 rows, at most 16
int colmask_splits(int m, int nwords, int *rps) {
    int splits = std::min(16, std::max(1, (256 + nwords - 1) / nwords));
    splits = std::min(splits, std::max(1, (m + kColmaskRowsPerPass - 1) / kColmaskRowsPerPass));
    *rps = (int)round_up((m + splits - 1) / splits, kColmaskRowsPerPass);
    return (m + *rps - 1) / *rps;
}

__device__ __forceinline__ bool bit_of(const uint32_t *bits, int64_t c) { return (bits[c >> 5] >> (c & 31)) & 1u; }

// X' (outlier columns zeroed) and W' (outlier rows zeroed), contiguous outputs; block = one row of X (the
// first m blocks) or of W
__global__ __launch_bounds__(256) void outlier_mask_kernel(const float *__restrict__ X, int64_t xsh, int m, int k,
                                                           const float *__restrict__ W, int64_t wsh, int n,
                                                           const uint32_t *__restrict__ bits, float *__restrict__ Xm,
                                                           float *__restrict__ Wm) {
    const int64_t row = blockIdx.x;
    if (row < m) {
        for (int c = threadIdx.x; c < k; c += 256) Xm[row * k + c] = bit_of(bits, c) ? 0.0f : X[row * xsh + c];
    } else {
        const int64_t r = row - m;
        const bool z = bit_of(bits, r);
        for (int c = threadIdx.x; c < n; c += 256) Wm[r * n + c] = z ? 0.0f : W[r * wsh + c];
    }
}

// O[i,j] = fl(O[i,j] + fmaf-chain over the outlier columns), one thread per output (j fastest)
__global__ __launch_bounds__(256) void outlier_mm_kernel(const float *__restrict__ X, int64_t xsh,
                                                         const float *__restrict__ W, int64_t wsh,
                                                         const int *__restrict__ idx,
                                                         const int *__restrict__ count, float *__restrict__ O,
                                                         int64_t osh, int m, int n) {
    const int cnt = *count;
    if (cnt == 0) return;
    const int i = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (i >= m || j >= n) return;
    float acc = 0.0f;
    for (int t = 0; t < cnt; ++t) {
        const int c = idx[t];
        acc = __fmaf_rn(X[(int64_t)i * xsh + c], W[(int64_t)c * wsh + j], acc);
    }
    O[(int64_t)i * osh + j] = __fadd_rn(O[(int64_t)i * osh + j], acc);
}

struct OutlierScratch {
    uint32_t *partial, *bits;
    int *rank, *idx;    // idx[0] = count, idx[1 ..] = the outlier columns ascending
    float *xm, *wm;     // X' / W' (fallback)
    uint32_t *state;    // the flags launch's counters (kTicketWords) then its accumulator (acc_words)
    int nchunks, nwords, acc_words, state_words;
    unsigned *ticket() const { return state; }
    uint32_t *acc() const { return acc_words ? state + kTicketWords : nullptr; }
};

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// [idx: count + list, k + 1 ints][state: counters + accumulator][bits][rank][partial][X'][W']: the count's offset
// depends on nothing (qgemm_outlier_count)
size_t state_words_for(int k) {
    const int nwords = (k + 31) / 32;
    return kTicketWords + (nwords <= kAccWords ? nwords : 0);
}

OutlierScratch scratch_view(void *scratch, int m, int k) {
    OutlierScratch v;
    v.nchunks = (m + kChunkRows - 1) / kChunkRows;
    v.nwords = (k + 31) / 32;
    v.acc_words = v.nwords <= kAccWords ? v.nwords : 0;
    v.state_words = (int)state_words_for(k);
    char *p = static_cast<char *>(scratch);
    v.idx = reinterpret_cast<int *>(p);
    p += a256(sizeof(int) * ((size_t)k + 1));
    v.state = reinterpret_cast<uint32_t *>(p);
    p += a256(sizeof(uint32_t) * (size_t)v.state_words);
    v.bits = reinterpret_cast<uint32_t *>(p);
    p += a256(sizeof(uint32_t) * v.nwords);
    v.rank = reinterpret_cast<int *>(p);
    p += a256(sizeof(int) * v.nwords);
    v.partial = reinterpret_cast<uint32_t *>(p);
    p += a256(sizeof(uint32_t) * (size_t)v.nchunks * v.nwords);
    v.xm = reinterpret_cast<float *>(p);
    p += a256(sizeof(float) * (size_t)m * k);
    v.wm = reinterpret_cast<float *>(p);
    return v;
}

template <bool VEC>
void launch_flags(hipStream_t s, const float *X, int64_t xsh, int m, int k, float t, const OutlierScratch &v) {
    const dim3 grid((unsigned)((k + kFlagCols - 1) / kFlagCols), (unsigned)v.nchunks);
    // K <= 32 768: the accumulator (the last workgroup reads nwords words); else every chunk's partial words
    auto go = [&](auto kern) { kern<<<grid, kFlagThreads, 0, s>>>(X, xsh, m, k, t, v.partial, v.nwords, v.ticket(),
                                                                  v.acc(), v.bits, v.rank, v.idx); };
    if (!v.acc_words) go(outlier_flags_kernel<VEC, false>);
    else go(outlier_flags_kernel<VEC, true>);
}

bool x_vec_ok(const float *X, int64_t xsh, int k) {
    return (k % 4 == 0) && (xsh % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0);
}

// (fallback) column mask, ranks, index list and count of X's outlier columns: the state zeroed, then ONE flags launch
// (its last workgroup builds the index)
hipError_t outlier_scan(const float *X, int64_t xsh, int m, int k, float t, const OutlierScratch &v, hipStream_t s) {
    if (v.nchunks > 65535) return hipErrorNotSupported;
    outlier_zero_state_kernel<<<1, 256, 0, s>>>(v.state, v.state_words);
    if (x_vec_ok(X, xsh, k)) launch_flags<true>(s, X, xsh, m, k, t, v);
    else launch_flags<false>(s, X, xsh, m, k, t, v);
    return hipGetLastError();
}

}  // namespace

size_t outlier_scratch_bytes(int m, int n, int k) {
    const size_t nwords = (size_t)(k + 31) / 32;
    const size_t nchunks = (size_t)(m + kChunkRows - 1) / kChunkRows;
    return a256(sizeof(uint32_t) * nchunks * nwords) + a256(sizeof(uint32_t) * nwords) + a256(sizeof(int) * nwords) +
           a256(sizeof(int) * ((size_t)k + 1)) + a256(sizeof(uint32_t) * state_words_for(k)) +
           a256(sizeof(float) * (size_t)m * k) +
           a256(sizeof(float) * (size_t)k * (size_t)round_up(n, 256));
}

// Fast path: the partial masks, the masked single-pass pack (mask, count and column list), the 256-tile GEMM with the
// fp32 chain in its epilogue.  hipErrorNotSupported (nothing launched) outside its envelope.
hipError_t outlier_fast(const float *X, const float *W, float *O, int m, int n, int k, float t, void *scratch,
                        PackedView va, PackedView vb, float range, hipStream_t s) {
    if (!gemm_outlier_ok(m, n, (int)va.k_pad) || !pack_single_pass_outlier_ok(X, k, m, k, W, n, n)) return hipErrorNotSupported;
    const OutlierScratch v = scratch_view(scratch, m, k);
    int rps = 0;
    const int splits = colmask_splits(m, v.nwords, &rps);
    // the partial words (splits x nwords <= 16 x 128) fit the fallback's chunk words (nchunks >= splits)
    if (v.nwords > 128 || splits > v.nchunks || !x_vec_ok(X, k, k)) return hipErrorNotSupported;
    outlier_colmask_kernel<<<dim3((unsigned)v.nwords, (unsigned)splits), kFlagThreads, 0, s>>>(X, k, m, k, t, rps,
                                                                                              v.partial, v.nwords);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_pack_single_pass_outlier(X, k, m, k, va, W, n, n, vb, range, v.partial, splits, v.nwords, v.idx, s);
    if (e == hipErrorNotSupported) return hipErrorUnknown;  // the mask already enqueued: the envelope checks disagree
    if (e != hipSuccess) return e;
    const float inv_r2 = 1.0f / (range * range);
    // the fp32 chain reads the outlier columns of X and rows of W where they lie (the column list idx + 1); a compact
    // copy of X's outlier values written by the pack measured slower (profiles/r05_maskpack_lab_xo_staged.log)
    return launch_gemm_dequant_outlier(va, vb, O, n, m, n, inv_r2, X, k, W, n, v.idx + 1, v.idx, s);
}

// Fallback phase 1: flags, indices, X', W' into scratch; the caller then runs the int8 chain on (X', W')
// and phase 2 (outlier_finish) adds the fp32 outlier products.
hipError_t outlier_prepare(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, float t,
                           void *scratch, float **Xm, float **Wm, hipStream_t s) {
    const OutlierScratch v = scratch_view(scratch, m, k);
    *Xm = v.xm;
    *Wm = v.wm;
    hipError_t e = outlier_scan(X, xsh, m, k, t, v, s);
    if (e != hipSuccess) return e;
    outlier_mask_kernel<<<(unsigned)(m + k), 256, 0, s>>>(X, xsh, m, k, W, wsh, n, v.bits, v.xm, v.wm);
    return hipGetLastError();
}

hipError_t outlier_finish(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, void *scratch,
                          float *O, int64_t osh, hipStream_t s) {
    const OutlierScratch v = scratch_view(scratch, m, k);
    outlier_mm_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)m), 256, 0, s>>>(X, xsh, W, wsh, v.idx + 1, v.idx,
                                                                                     O, osh, m, n);
    return hipGetLastError();
}

int outlier_count_slot(int k, const void *scratch, int *count_host) {
    (void)k;  // the count leads the scratch
    return (int)hipMemcpy(count_host, scratch, sizeof(int), hipMemcpyDeviceToHost);
}

}  // namespace qgemm
