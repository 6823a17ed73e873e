// qgemm_internal.h -- shared definitions of the gfx950 quantized-GEMM kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qgemm {

// Packed operand geometry (include/qgemm.h): rows padded to the GEMM macro-tile, k to its k-step.
constexpr int kRowPad = 256;
constexpr int kKPad = 128;

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Column-absmax partials: pack_cols' pass 1 reduces chunks of kColChunk rows (k >= 1) and writes one
// partial per (chunk, column); pass 2 reduces the partials.  No atomics, nothing to zero per call.
constexpr int kColChunk = 256;
__host__ __device__ inline int64_t colmax_parts(int64_t k) { return k > 1 ? (k - 1 + kColChunk - 1) / kColChunk : 1; }

// Layout of one packed operand buffer:
//   [scale: rows_pad f32][scratch: parts x rows_pad u32][q: rows_pad x k_pad i8, FRAGMENT-MAJOR]
// The scratch holds pack_cols' column-absmax partials (pass 1 -> pass 2).
//
// q is stored fragment-major: 1-KiB blocks of 16 packed rows x 64 k-bytes, block (rg, kb) at byte
// (rg * (k_pad / 64) + kb) * 1024, and inside a block the bytes in the lane order of one
// v_mfma_i32_16x16x64_i8 operand: lane l = 16 kc + r holds row 16 rg + r, k = 64 kb + 16 kc .. +15.  So a
// GEMM wave loads a whole MFMA fragment as ONE contiguous 1-KiB buffer_load_dwordx4 (gemm_i8_f4), and
// an LDS-DMA piece is one block (no source swizzle, conflict-free fragment reads).  Any 4-byte group
// k .. k+3 with k % 4 == 0 (and any aligned 16-byte group) of one row stays contiguous.
__host__ __device__ inline int64_t fofs(int64_t row, int64_t k, int64_t k_pad) {
    return ((row >> 4) * (k_pad >> 6) + (k >> 6)) * 1024 + ((((k >> 4) & 3) << 4) + (row & 15)) * 16 + (k & 15);
}
struct PackedView {
    float *scale;       // rows_pad floats (Cx or Cw)
    uint32_t *scratch;  // parts x rows_pad words
    int8_t *q;          // rows_pad x k_pad
    int64_t rows_pad, k_pad, parts;
};

inline PackedView packed_view(const void *base, int rows, int k) {
    PackedView v;
    v.rows_pad = round_up(rows, kRowPad);
    v.k_pad = round_up(k, kKPad);
    v.parts = colmax_parts(k);
    char *p = static_cast<char *>(const_cast<void *>(base));
    v.scale = reinterpret_cast<float *>(p);
    v.scratch = reinterpret_cast<uint32_t *>(p + v.rows_pad * 4);
    v.q = reinterpret_cast<int8_t *>(p + round_up(v.rows_pad * 4 * (1 + v.parts), 256));
    return v;
}

inline size_t packed_bytes(int rows, int k) {
    const int64_t rp = round_up(rows, kRowPad);
    return (size_t)round_up(rp * 4 * (1 + colmax_parts(k)), 256) + (size_t)rp * round_up(k, kKPad);
}

// the dword of packed row `row` holding k .. k+3 (k % 4 == 0)
__device__ __forceinline__ uint32_t *qword(int8_t *q, int64_t row, int64_t k, int64_t k_pad) {
    return reinterpret_cast<uint32_t *>(q + fofs(row, k, k_pad));
}
// zero packed rows [r0, r0 + nrows) over all k_pad bytes, 16 B per thread-step (threads t of nt)
__device__ __forceinline__ void zero_packed_rows(int8_t *q, int64_t r0, int nrows, int64_t k_pad, int t, int nt) {
    const int64_t per = k_pad >> 4;
    for (int64_t i = t; i < (int64_t)nrows * per; i += nt)
        *reinterpret_cast<uint4 *>(q + fofs(r0 + i / per, (i % per) << 4, k_pad)) = make_uint4(0, 0, 0, 0);
}

// ---- the reference's per-element arithmetic, pinned to single IEEE operations ----------------

// AbsMaxFunc (op_reduction.cuh:11-24) on an element that is not the seed: |x|, skipping NaN.
// Returned as a candidate for a running maximum started at -inf; the caller combines candidates
// with strict ">" so NaN never enters.
__device__ __forceinline__ float absmax_candidate(float x) { return fabsf(x); }

// Final combine with the signed seed (the reduction kernels' first element, op_reduction.cuh:80/105):
// acc = seed; if (p > acc) acc = p.  A NaN seed sticks, exactly as in the sequential functor.
__device__ __forceinline__ float absmax_finish(float seed, float p) { return (p > seed) ? p : seed; }

// InvDivideConstFunc (op_elemwise.cuh:131-143): correctly rounded range / C.
__device__ __forceinline__ float inv_divide(float range, float c) { return __fdiv_rn(range, c); }

// MultiplyWithTypecastFunc<float,int8_t> (op_elemwise.cuh:106-114): static_cast<int8_t>(x*s),
// truncation toward zero; saturation and NaN->0 where C++ leaves the cast undefined.
// v_cvt_i32_f32 truncates toward zero, turns NaN into 0 and saturates out-of-range values, so
// after the clamp (v_med3_i32) this equals clamping the float first: 3 VALU per element.
__device__ __forceinline__ int quant_i8(float x, float s) {
    const float v = __fmul_rn(x, s);
    int i;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(i) : "v"(v));
    return min(max(i, -128), 127);
}

// op_mm(Cx, Cw) with K = 1 (op_mm.cuh:96-97): res = 0; res += Cx*Cw -> fl(Cx*Cw) + 0 (turns -0 into +0).
__device__ __forceinline__ float outer_product(float cx, float cw) { return __fadd_rn(__fmul_rn(cx, cw), 0.0f); }

// op_dequantize (DequantizeFunc, op_elemwise.cuh:93-103) then op_multiply(O, 1/(range*range))
// (op_mm.cuh:99): two separate launches in the reference, so two roundings, no contraction.
__device__ __forceinline__ float dequantize(int acc, float outer, float inv_r2) {
    return __fmul_rn(__fmul_rn((float)acc, outer), inv_r2);
}

// The running value of the lane to the LEFT (DPP wave_ror:1: lane l reads lane l - 1, lane 0 reads lane 63),
// for sequential fp32 sums that hop from lane to lane (encoder_ops.hip lane_chain_sum, attention.hip).  With
// old = 0 and bound_ctrl set, hipcc folds the move into the consuming v_add_f32 (v_add_f32_dpp).
__device__ __forceinline__ float hop_left(float s) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x13C /* wave_ror:1 */, 0xf, 0xf, true));
}

// Counter-based generator shared with oracle_uniform_at (oracle/qgemm_oracle.c).
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// ---- launchers (defined in the .hip files) ------------------------------------------------------
hipError_t launch_pack_rows(const float *src, int64_t sh, int64_t sw, int rows, int len, float range,
                            PackedView out, hipStream_t stream);
hipError_t launch_pack_cols(const float *src, int64_t sh, int len, int cols, float range, PackedView out,
                            hipStream_t stream);
// The two-pass pack of a row-major A and B (B's columns reduced in pass 1, quantized in pass 2; A's rows in one of
// the passes): long rows (4096 < K <= 16384) as a W-only pass 1 + pass 2 with A's rows at its end, shorter rows as
// launch_pack_rows_and_colmax + launch_pack_cols_pass2.  hipErrorNotSupported when the layouts do not allow it.
hipError_t launch_pack_two_pass(const float *a, int64_t ash, int m, int k, PackedView outa, const float *b, int64_t bsh,
                                int n, PackedView outb, float range, hipStream_t stream, uint32_t *zero_words = nullptr,
                                int nzero = 0);
// One launch: pack_rows of a row-major A (vector path) and pass 1 of pack_cols of a row-major B.
// Returns hipErrorNotSupported when the layouts do not allow it (caller falls back).
hipError_t launch_pack_rows_and_colmax(const float *a, int64_t ash, int m, int k, PackedView outa, const float *b,
                                       int64_t bsh, int n, PackedView outb, float range, hipStream_t stream,
                                       uint32_t *zero_words = nullptr, int nzero = 0);
// One launch, W read once: single-pass W strips (K <= 4096, n % 8 == 0: 8-column strips at two blocks
// per CU, or 16-column strips) + X rows.  hipErrorNotSupported when the shape/layout is outside that
// (caller falls back).
// zero_words/nzero: words zeroed by block 0 of the launch (the GEMM's split-K tickets)
hipError_t launch_pack_single_pass(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                   int64_t wsh, int n, PackedView outw, float range, hipStream_t stream,
                                   uint32_t *zero_words = nullptr, int nzero = 0);
// kind 8 / 16 forces the strip width (lab); 0 chooses.
hipError_t launch_pack_single_pass_kind(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                        int64_t wsh, int n, PackedView outw, float range, hipStream_t stream, int kind,
                                        uint32_t *zero_words = nullptr, int nzero = 0);
// The single-pass pack (8-column W strips) of the LLM.int8() decomposition's int8 part: outlier columns
// of X / rows of W packed as +0 (the mask = OR of the flags launch's nparts x nwords partial words partial[p][w],
// bit c of word w = column 32 w + c); workgroup 0 writes idx[0] = the outlier count, idx[1 ..] = the columns
// ascending.  hipErrorNotSupported outside the single pass's envelope (K % 4 == 0 too) or for nparts > 16 (nothing
// launched).
bool pack_single_pass_outlier_ok(const float *x, int64_t xsh, int m, int k, const float *w, int64_t wsh, int n);
hipError_t launch_pack_single_pass_outlier(const float *x, int64_t xsh, int m, int k, PackedView outx, const float *w,
                                           int64_t wsh, int n, PackedView outw, float range, const uint32_t *partial,
                                           int nparts, int nwords, int *idx, hipStream_t stream);
hipError_t launch_pack_cols_pass2(const float *src, int64_t sh, int len, int cols, float range, PackedView out,
                                  hipStream_t stream);
hipError_t launch_fill_uniform(float *dst, int64_t count, uint64_t seed, float lo, float hi, hipStream_t stream);
// Split-K for shapes with too few 256x256 tiles to fill the chip: gemm_splits() slices per tile and
// the scratch (tickets + int32 slabs) they need; 1 / 0 when the shape is not split.
int gemm_splits(int m, int n, int k);
// the plan's tile edge and kernel name (qgemm_gemm_plan); returns the splits
int gemm_plan_info(int m, int n, int k, int *tile, const char **kernel);
size_t gemm_scratch_bytes(int m, int n, int k);
// scratch: gemm_scratch_bytes(m, n, k) bytes, or nullptr (then no split: correct, slower)
// bias (n floats) != nullptr: y = fl(O + b[j]) (+ relu): the encoder's linear layers.
// tickets_zeroed: the split-K scratch is library-owned, zeroed once at allocation; the launch's
// reducers re-zero their tickets instead of a memset ahead of every launch.
// bytes at the start of the split-K scratch that must be zero before a split launch (0: no split)
size_t gemm_ticket_bytes(int m, int n, int k);
hipError_t launch_gemm_dequant(const PackedView &a, const PackedView &b, float *C, int64_t csh, int64_t csw,
                               int m, int n, float inv_r2, void *scratch, size_t scratch_bytes, hipStream_t stream,
                               const float *bias = nullptr, bool relu = false, bool tickets_zeroed = false);
// The LLM.int8() decomposition's GEMM: int8 part + the outlier columns' fp32 products in the epilogue, read from
// X (m x k, row stride xsh) and W (k x n, row stride wsh) at the columns / rows ocols[0 .. *ocount) (ascending).
// Only where the plan is the 256-tile GEMM without split-K (gemm_outlier_ok); hipErrorNotSupported otherwise.
bool gemm_outlier_ok(int m, int n, int k);
hipError_t launch_gemm_dequant_outlier(const PackedView &a, const PackedView &b, float *C, int64_t csh, int m, int n,
                                       float inv_r2, const float *x, int64_t xsh, const float *w, int64_t wsh,
                                       const int *ocols, const int *ocount, hipStream_t stream);
hipError_t launch_gemm_i32(const PackedView &a, const PackedView &b, int32_t *Acc, int m, int n,
                           hipStream_t stream);
hipError_t launch_mm_f32(const float *A, int64_t ash, int64_t asw, const float *B, int64_t bsh, int64_t bsw, float *C,
                         int64_t csh, int64_t csw, int m, int n, int k, hipStream_t stream);
// batch of independent GEMMs (blockIdx.z), operand i at base + i * batch stride (attention heads)
hipError_t launch_mm_f32_batched(const float *A, int64_t ash, int64_t asw, int64_t a_bs, const float *B, int64_t bsh,
                                 int64_t bsw, int64_t b_bs, float *C, int64_t csh, int64_t csw, int64_t c_bs, int m,
                                 int n, int k, int batch, hipStream_t stream);
// Encoder row ops (encoder_ops.hip): the reference's op_softmax (after op_multiply by `scale`) and
// op_add + op_layernorm, one row per wave, sums in the reference's sequential order.
// S = QK^T, softmax(S * scale), heads = PV for every head in one launch (S in LDS), bit-identical to
// the three separate kernels; hipErrorNotSupported outside d_k <= 64, seq <= 512 (caller falls back).
// qkv: seq x 3d ([Q | K | V], head h at columns h*d_k of each third); heads: seq x d.
hipError_t launch_attention_fused(const float *qkv, int seq, int d, int n_heads, float scale, float *heads,
                                  hipStream_t stream);
hipError_t launch_softmax_rows(const float *S, float *P, int64_t rows, int w, float scale, hipStream_t stream);
hipError_t launch_add_layernorm_rows(const float *A, const float *B, float *Y, int64_t rows, int w,
                                     hipStream_t stream);
// the same, also writing Y's rows packed (Cx + int8) for the next quantized linear (pack_rows fused)
hipError_t launch_add_layernorm_rows_pack(const float *A, const float *B, float *Y, int64_t rows, int w, float range,
                                          PackedView out, hipStream_t stream);
// LLM.int8() outlier decomposition (outlier.hip).
size_t outlier_scratch_bytes(int m, int n, int k);
hipError_t outlier_prepare(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, float t,
                           void *scratch, float **Xm, float **Wm, hipStream_t s);
hipError_t outlier_finish(const float *X, int64_t xsh, const float *W, int64_t wsh, int m, int n, int k, void *scratch,
                          float *O, int64_t osh, hipStream_t s);
int outlier_count_slot(int k, const void *scratch, int *count_host);
// fast path (flags, indices, masked single-pass pack, GEMM with the fp32 chain in its epilogue) into the
// packed views va / vb; hipErrorNotSupported (nothing launched) outside its envelope (row-major operands)
hipError_t outlier_fast(const float *X, const float *W, float *O, int m, int n, int k, float t, void *scratch,
                        PackedView va, PackedView vb, float range, hipStream_t s);
// The encoder counterpart (encoder.hip).
struct Encoder;
uint64_t encoder_weight_seed(uint64_t base, int block, int kind, int head);
float encoder_init_bound(int n);
hipError_t encoder_create(int d_model, int n_heads, int d_ff, int n_blocks, int max_seq, uint64_t seed, Encoder **out);
hipError_t encoder_forward(Encoder *E, const float *X, float *Y, int seq, hipStream_t s);
void encoder_destroy(Encoder *E);
const char *gemm_config_name();
// Quantization-error statistics on the device (error_stats.hip); scratch = error_stats_scratch_bytes().
size_t error_stats_scratch_bytes();
hipError_t launch_error_stats(const float *C, const float *O, int64_t n, bool reference_order, double *stats,
                              void *scratch, hipStream_t stream);

// Diagnostics: events to record exactly around the next GEMM kernel (hipExtLaunchKernelGGL), set
// through qgemm_set_gemm_events() and consumed by one launch.  Thread-local.
struct GemmEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
GemmEvents take_gemm_events();
void set_gemm_events(hipEvent_t start, hipEvent_t stop);
void set_gemm_event_mode(int mode);

}  // namespace qgemm
