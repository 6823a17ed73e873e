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
//   outlier_flags  : X read once in full-row float4 loads; per 64-row chunk a bitmask of its outlier
//                    columns (every word written: nothing to clear per call); the workgroup that arrives
//                    last ORs the chunk masks into the column mask, the per-word ranks, the ascending list
//                    of outlier columns and their count (stays on the device; round 5: no index launch)
//   the pack       : the single pass with the mask (pack.hip): X'/W' quantized without materialising
//                    them (per-lane nibble / row-bit tables the flags launch builds: no shuffles, no stores)
//   the GEMM       : the int8 part with the fp32 chain added in its store epilogue (gemm_i8_kernels.h), its
//                    operands read from X's outlier columns and W's outlier rows where they lie
// Other shapes: flags + index, X'/W' materialised by a masking pass, the plain drop-in on them, and a
// correction kernel adding the chain to O.
#include <algorithm>
#include <map>
#include <mutex>

#include "qgemm_internal.h"

namespace qgemm {

// The flags launch's arrival tickets: a zero-initialised array of the code object (per device), one 128-B line per
// slot, one slot per stream (outlier_ticket_slot).  Each launch's last workgroup re-zeroes its slot, so a slot is 0
// between calls -- without any allocation or memset, so the first call on a stream may be inside a graph capture.
// a slot = 9 counters (8 per-XCD + 1 global), each on a 128-B line of its own
constexpr int kTicketSlots = 256, kCounterWords = 32, kTicketStride = 9 * kCounterWords;
__device__ unsigned g_flags_ticket[kTicketSlots * kTicketStride];
// K <= 32 768 (kAccWords words of 32 columns): each flags workgroup ORs its nonzero mask words into the slot's
// accumulator with agent-scope atomics (performed at the memory side, coherent across XCDs), so the last workgroup
// reads nwords words instead of every chunk's partial words; it re-zeroes them for the next call.
constexpr int kAccWords = 1024;
__device__ uint32_t g_flags_acc[kTicketSlots * kAccWords];

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

// Mask word w of a 64-row chunk: bit c set when column 32w + c holds an outlier in the chunk's rows.  1024 threads =
// 4 row groups x 256 column threads: thread (g, t) reads columns 1024 bx + 4t .. +3 of rows 16 g .. 16 g + 15 of
// the chunk (16 float4 loads in flight per thread, 16 waves per CU), the groups' nibbles meet in LDS.  kAcc:
// nonzero words are ORed into the stream's accumulator g_flags_acc (agent-scope atomics); else every word is stored
// to partial[chunk][word] (sc1).  Then each workgroup, after every wave's stores / atomics have drained, arrives
// on its XCD's counter of the stream's ticket slot (one lane, agent scope), and the last of each XCD on the slot's
// global counter -- sharded, because ≈ 12 ns per arrival serialise on one counter (MI355X_MICROARCH.md fan-in row);
// the write-through hand-off of the sc1 table, row 1, at each level.  The workgroup that arrives last overall
// builds the column mask, ranks, list and count (build_index over the accumulator or the partial words) and
// re-zeroes the counters and the accumulator for the next call -- no separate index launch.
constexpr int kFlagThreads = 1024, kFlagGroups = 4, kGroupRows = kChunkRows / kFlagGroups;
template <bool VEC, bool kAcc, bool kIndex>
__global__ __launch_bounds__(kFlagThreads) void outlier_flags_kernel(const float *__restrict__ X, int64_t xsh, int m,
                                                                     int k, float t, uint32_t *__restrict__ partial,
                                                                     int nwords, int slot, uint32_t *__restrict__ bits,
                                                                     int *__restrict__ rank, int *__restrict__ idx) {
    static_assert(kAcc || kIndex, "the partial words need the index build");
    unsigned *ticket = g_flags_ticket + slot * kTicketStride;  // counter x (x < 8: per XCD, 8: global) at x * 32
    uint32_t *acc = g_flags_acc + slot * kAccWords;
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
        if constexpr (!kIndex) return;  // the fast path: the masked pack reads the accumulator itself
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (!kIndex) return;
    __syncthreads();
    if (tid == 0) {
        // blocks b, b + 8, ... share an XCD (round-robin dispatch); the last of each XCD arrives globally
        const unsigned total = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x, xcd = bid & 7;
        const unsigned on_xcd = (total - xcd + 7) / 8, xcds = total < 8 ? total : 8;
        unsigned fin = 0;
        unsigned *mine = ticket + xcd * kCounterWords, *all = ticket + 8 * kCounterWords;
        if (__hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == on_xcd - 1) {
            __hip_atomic_store(mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(all, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == xcds - 1) {
                __hip_atomic_store(all, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fin = 1;
            }
        }
        last = fin;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the sc1 loads stay below
    if constexpr (kAcc) build_index<1, kFlagThreads>(acc, 1, nwords, bits, rank, idx, wsum, &count);
    else build_index<1, kFlagThreads>(partial, (int)gridDim.y, nwords, bits, rank, idx, wsum, &count);
    __syncthreads();  // every accumulator word has been read
    if (tid == 0) idx[0] = count;
    if constexpr (kAcc)
        for (int i = tid; i < nwords; i += kFlagThreads)
            __hip_atomic_store(acc + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// the stream's ticket slot (host bookkeeping only: no HIP call, so it is capture-safe); -1 when all are taken
int outlier_ticket_slot(hipStream_t s) {
    static std::mutex mu;
    static std::map<hipStream_t, int> slots;
    std::lock_guard<std::mutex> lk(mu);
    auto it = slots.find(s);
    if (it != slots.end()) return it->second;
    if ((int)slots.size() >= kTicketSlots) return -1;
    const int id = (int)slots.size();
    slots.emplace(s, id);
    return id;
}

struct OutlierScratch {
    uint32_t *partial, *bits;
    int *rank, *idx;    // idx[0] = count, idx[1 ..] = the outlier columns ascending
    float *xm, *wm;     // X' / W' (fallback)
    int nchunks, nwords;
};

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// [idx: count + list, k + 1 ints][bits][rank][partial][X' or xo][W' or wo]: the count's offset depends on
// k only (qgemm_outlier_count)
OutlierScratch scratch_view(void *scratch, int m, int k) {
    OutlierScratch v;
    v.nchunks = (m + kChunkRows - 1) / kChunkRows;
    v.nwords = (k + 31) / 32;
    char *p = static_cast<char *>(scratch);
    v.idx = reinterpret_cast<int *>(p);
    p += a256(sizeof(int) * ((size_t)k + 1));
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
void launch_flags(hipStream_t s, const float *X, int64_t xsh, int m, int k, float t, const OutlierScratch &v,
                  int slot, bool index) {
    const dim3 grid((unsigned)((k + kFlagCols - 1) / kFlagCols), (unsigned)v.nchunks);
    // K <= 32 768: the accumulator (the last workgroup reads nwords words, or -- !index, the fast path -- the pack
    // reads them itself); else every chunk's partial words
    auto go = [&](auto kern) { kern<<<grid, kFlagThreads, 0, s>>>(X, xsh, m, k, t, v.partial, v.nwords, slot, v.bits,
                                                                  v.rank, v.idx); };
    if (v.nwords > kAccWords) go(outlier_flags_kernel<VEC, false, true>);
    else if (index) go(outlier_flags_kernel<VEC, true, true>);
    else go(outlier_flags_kernel<VEC, true, false>);
}

// the device address of the stream's accumulator slot (hipGetSymbolAddress once per device; not a stream operation)
uint32_t *flags_acc(int slot) {
    constexpr int kMaxDev = 64;
    static uint32_t *base[kMaxDev];
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!base[dev]) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_flags_acc)) != hipSuccess) return nullptr;
        base[dev] = static_cast<uint32_t *>(p);
    }
    return base[dev] + (size_t)slot * kAccWords;
}

// column mask, ranks, index list and count of X's outlier columns: ONE launch (the last flags workgroup
// builds the index)
hipError_t outlier_scan(const float *X, int64_t xsh, int m, int k, float t, const OutlierScratch &v, hipStream_t s,
                        bool index = true) {
    const int slot = outlier_ticket_slot(s);
    if (slot < 0) return hipErrorOutOfMemory;  // more streams than ticket slots
    if (v.nchunks > 65535) return hipErrorNotSupported;
    const bool vec = (k % 4 == 0) && (xsh % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0);
    if (vec) launch_flags<true>(s, X, xsh, m, k, t, v, slot, index);
    else launch_flags<false>(s, X, xsh, m, k, t, v, slot, index);
    return hipGetLastError();
}

}  // namespace

size_t outlier_scratch_bytes(int m, int n, int k) {
    const size_t nchunks = (size_t)(m + kChunkRows - 1) / kChunkRows, nwords = (size_t)(k + 31) / 32;
    return a256(sizeof(uint32_t) * nchunks * nwords) + a256(sizeof(uint32_t) * nwords) + a256(sizeof(int) * nwords) +
           a256(sizeof(int) * ((size_t)k + 1)) + a256(sizeof(float) * (size_t)m * k) +
           a256(sizeof(float) * (size_t)k * (size_t)round_up(n, 256));
}

// Fast path: flags + index, the masked single-pass pack, the 256-tile GEMM with the fp32 chain in its
// epilogue.  hipErrorNotSupported (nothing launched) outside its envelope.
hipError_t outlier_fast(const float *X, const float *W, float *O, int m, int n, int k, float t, void *scratch,
                        PackedView va, PackedView vb, float range, hipStream_t s) {
    if (!gemm_outlier_ok(m, n, (int)va.k_pad) || !pack_single_pass_outlier_ok(X, k, m, k, W, n, n)) return hipErrorNotSupported;
    const OutlierScratch v = scratch_view(scratch, m, k);
    const int slot = outlier_ticket_slot(s);
    uint32_t *acc = slot < 0 ? nullptr : flags_acc(slot);
    if (!acc || v.nwords > 128) return hipErrorNotSupported;  // nothing enqueued yet: the fallback runs
    // flags: the mask words ORed into the stream's accumulator, no index; the masked pack reads the words itself and
    // its workgroup 0 writes the count and column list; the GEMM's workgroup 0 zeroes the accumulator after them
    hipError_t e = outlier_scan(X, k, m, k, t, v, s, /*index=*/false);
    if (e != hipSuccess) return e;
    e = launch_pack_single_pass_outlier(X, k, m, k, va, W, n, n, vb, range, acc, v.nwords, v.idx, s);
    if (e == hipErrorNotSupported) return hipErrorUnknown;  // scan already enqueued: the envelope checks above disagree
    if (e != hipSuccess) return e;
    const float inv_r2 = 1.0f / (range * range);
    // the fp32 chain reads the outlier columns of X and rows of W where they lie (the column list idx + 1); a compact
    // copy of X's outlier values written by the pack measured slower (profiles/r05_maskpack_lab_xo_staged.log)
    return launch_gemm_dequant_outlier(va, vb, O, n, m, n, inv_r2, X, k, W, n, v.idx + 1, v.idx, acc, v.nwords, s);
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
