/*
 * qgemm.h -- C-ABI of the MI355X-native (gfx950) int8 absmax quantized GEMM.
 *
 * Drop-in for the reference's quantized matrix multiply
 *     template<typename T> void op_quantized_mm(const Tensor<T>& X, const Tensor<T>& W,
 *                                               Tensor<T>& O, T range)
 *     (/root/reference/src/ops/op_mm.cuh:67-101, instantiated only at T = float,
 *      called from test_quantize.cu:78 and inlined in timing_quantize.cu:38-58)
 * as the flat C entry point the north star names, op_mm_quantize(A, B, C, M, N, K).
 *
 * Semantics (bit-exact with the reference chain, see DESIGN.md "Semantics"):
 *   Cx[i] = absmax of row i of A with the reference's signed-first-element seed
 *   Cw[j] = absmax of column j of B, same seed rule
 *   Aq = trunc_sat_i8(A * fl(range/Cx)), Bq = trunc_sat_i8(B * fl(range/Cw))
 *   C[i,j] = fl(fl(float(sum_k Aq[i,k]*Bq[k,j]) * (fl(Cx[i]*Cw[j]) + 0)) * fl(1/fl(range*range)))
 *
 * Conventions
 *   - All matrix pointers are DEVICE pointers (the reference asserts on_device, op_mm.cuh:72).
 *   - Return value: 0 on success, otherwise a hipError_t code (hipErrorInvalidValue = 1 for
 *     bad shapes / null pointers -- where the reference would assert(), op_mm.cuh:71-72).
 *   - Work is enqueued asynchronously; the plain entry point uses the null stream, like the
 *     reference's launches (legacy default stream).
 *   - No parameter is named N: the reference's op_elemwise.cuh:10 does "#define N 256".
 *   - The entry points without a workspace argument use a grow-only device buffer cached per
 *     (device, stream) -- per calling thread as well for hipStreamPerThread -- so calls on
 *     different streams never share it; the reference allocates per call (op_mm.cuh:76-93).
 *     Growing it allocates (not allowed inside a hipGraph capture) and waits for that stream;
 *     at most 8 such buffers are kept per device (the least recently used one is freed, after
 *     a device synchronisation, when a ninth stream arrives).  Pass an explicit workspace
 *     (op_mm_quantize_ws) for capture or to bound memory.
 */
#ifndef QGEMM_H_
#define QGEMM_H_

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define QGEMM_API __attribute__((visibility("default")))
#else
#define QGEMM_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces op_quantized_mm<float>(X, W, O, 127.0f) (op_mm.cuh:67-101).
 * A = X: m x k, row-major fp32.  B = W: k x n, row-major fp32.  C = O: m x n, row-major fp32. */
QGEMM_API int op_mm_quantize(const float *A, const float *B, float *C, int m, int n, int k);

/* Strided form: element (r, c) of a matrix lives at ptr[r*stride_h + c*stride_w], exactly the
 * reference's Index() macro (tensor.cuh:14), so transposed views (tensor.cuh:121-133) work.
 * range is the reference's `range` argument (127 at every reference call site). stream is a
 * hipStream_t (NULL = null stream). */
QGEMM_API int op_mm_quantize_ex(const float *A, int64_t a_stride_h, int64_t a_stride_w,
                      const float *B, int64_t b_stride_h, int64_t b_stride_w,
                      float *C, int64_t c_stride_h, int64_t c_stride_w,
                      int m, int n, int k, float range, void *stream);

/* Same, with caller-owned device workspace (no allocation inside: safe for hipGraph capture and
 * for concurrent calls on different streams).  ws_bytes >= op_mm_quantize_workspace_size(m,n,k). */
QGEMM_API size_t op_mm_quantize_workspace_size(int m, int n, int k);
QGEMM_API int op_mm_quantize_ws(const float *A, int64_t a_stride_h, int64_t a_stride_w,
                      const float *B, int64_t b_stride_h, int64_t b_stride_w,
                      float *C, int64_t c_stride_h, int64_t c_stride_w,
                      int m, int n, int k, float range,
                      void *workspace, size_t ws_bytes, void *stream);

/* ---- The chain's stages (the reference's L2 primitives, fused MI355X-style) ----------------
 * Packed operand = the quantized operand in MFMA-ready form, in ONE device buffer:
 *   [ scale: rows_pad f32 ][ reserved: parts x rows_pad u32, padded to 256 B ][ q: rows_pad x k_pad int8,
 *     zero padded ]   with parts = max(1, ceil((k-1)/256))
 * The q region is OPAQUE to callers: it is stored FRAGMENT-MAJOR (1-KiB blocks of 16 packed rows x 64 k,
 * bytes in the lane order of one v_mfma_i32_16x16x64_i8 operand; csrc/qgemm_internal.h fofs), so the GEMM
 * loads each MFMA operand with one contiguous 1-KiB load.  Treat a packed buffer as a handle: produce it
 * with qgemm_pack_a / qgemm_pack_b, consume it with qgemm_mm_packed / qgemm_linear / the prepacked drop-in.
 * rows_pad = round_up(rows, 256), k_pad = round_up(k, 128).  For A, rows = m and the scale is
 * Cx (op_absmax(X,Cx), op_mm.cuh:76-77) and q = X_int8 (op_mm.cuh:86-87).  For B, rows = n
 * (B is stored transposed, k contiguous) and the scale is Cw (op_mm.cuh:78-79), q = W_int8^T.
 * Packing B once and reusing it is the LLM.int8() weight-cache pattern. */
QGEMM_API size_t qgemm_packed_size(int rows, int k);
QGEMM_API int qgemm_pack_a(const float *A, int64_t a_stride_h, int64_t a_stride_w, int m, int k, float range,
                 void *packed_a, void *stream);
QGEMM_API int qgemm_pack_b(const float *B, int64_t b_stride_h, int64_t b_stride_w, int k, int n, float range,
                 void *packed_b, void *stream);
/* int8 x int8 -> int32 MFMA GEMM with the fused dequantize epilogue (op_mm.cuh:92-99). */
QGEMM_API int qgemm_mm_packed(const void *packed_a, const void *packed_b, float *C, int64_t c_stride_h,
                    int64_t c_stride_w, int m, int n, int k, float range, void *stream);
/* The weight-cache form of the drop-in (op_mm_quantize_prepacked): B was packed once
 * with qgemm_pack_b(range 127); every call quantizes A (op_mm.cuh:76-77, 82-87) and runs the int8 GEMM
 * with the fused dequantize (op_mm.cuh:92-99) -- bit-identical to op_mm_quantize(A, B, C, m, n, k) on the
 * B that was packed.  A: m x k (row stride a_stride_h, unit column stride), C: m x n (row stride
 * c_stride_h).  The plain form uses the library's workspace and the null stream.
 * Range: A is quantized with range 127 and O dequantized with fl(1/127^2), as op_mm_quantize does, so
 * packed_b must come from qgemm_pack_b(..., range = 127, ...); a B packed with another range gives
 * results that differ from op_mm_quantize (the packed buffer does not record its range). */
QGEMM_API int op_mm_quantize_prepacked(const float *A, const void *packed_b, float *C, int m, int n, int k);
QGEMM_API size_t op_mm_quantize_prepacked_workspace_size(int m, int n, int k);
QGEMM_API int op_mm_quantize_prepacked_ws(const float *A, int64_t a_stride_h, const void *packed_b, float *C,
                                int64_t c_stride_h, int m, int n, int k, void *workspace, size_t ws_bytes,
                                void *stream);
/* Debug/parity view of the raw int32 accumulator (op_mm<int8_t,int>, op_mm.cuh:92-93):
 * Acc is m x n row-major int32. */
QGEMM_API int qgemm_mm_packed_i32(const void *packed_a, const void *packed_b, int32_t *Acc, int m, int n, int k,
                        void *stream);

/* The reference's UNQUANTIZED op_mm<float,float> (op_mm.cuh:49-65), bit-exact: sequential-k fmaf from +0.
 * Used for the reference's error metric (timing_quantize.cu:67-70) and its unquantized timing line. */
QGEMM_API int qgemm_mm_fp32(const float *A, int64_t a_stride_h, int64_t a_stride_w,
                  const float *B, int64_t b_stride_h, int64_t b_stride_w,
                  float *C, int64_t c_stride_h, int64_t c_stride_w, int m, int n, int k, void *stream);

/* ---- The encoder counterpart (transformer.cu:14-77, BASELINE config 5) ----------
 * Linear layer on the quantized path (linear.cuh:50-54): Y = quantized_mm(X, W) [+ b] [relu], where
 * W (k x n) was packed once with qgemm_pack_b.  X is m x k row-major (row stride x_stride_h), Y m x n
 * (row stride y_stride_h).  bias = NULL: no bias (relu requires a bias, as the reference's FFN).
 * y = fl(O + b[j]) then (y < 0 ? 0 : y) (op_add, op_relu: op_elemwise.cuh:57-65, 181-195). */
QGEMM_API size_t qgemm_linear_workspace_size(int m, int n, int k);
QGEMM_API int qgemm_linear(const float *X, int64_t x_stride_h, int m, int k, const void *packed_w, int n,
                 const float *bias, int relu, float *Y, int64_t y_stride_h, void *workspace, size_t ws_bytes,
                 void *stream);
/* op_multiply(S, scale) then op_softmax (attention.cuh:65-68, op_softmax.cuh:6-29), per row of w
 * contiguous floats (w <= 4096); P may equal S.  exp is the correctly rounded fp32 exp. */
QGEMM_API int qgemm_softmax_rows(const float *S, float *P, int64_t rows, int w, float scale, void *stream);
/* op_add(A, B) then op_layernorm (transformer.cu:58-59, op_layernorm.cuh:6-33) as written:
 * (y - mean) / var, sums in column order, pow(d, 2) = fl32(d*d); rows of w <= 4096 floats. */
QGEMM_API int qgemm_add_layernorm_rows(const float *A, const float *B, float *Y, int64_t rows, int w, void *stream);
/* Encoder stack with seeded weights drawn once and packed (the weight cache, s8f f2).  X, Y: seq x
 * d_model row-major fp32 device arrays, seq <= max_seq <= 4096, d_model <= 4096, d_model % n_heads == 0.
 * Weight tensor t of block i is the qgemm_fill_uniform stream encoder_weight_seed(seed, i, kind, head)
 * = seed*1000003 + i*4099 + kind*131 + head, kind 0..7 = Wq, Wk, Wv, W_O, W1, b1, W2, b2, with the
 * reference's init bounds (DESIGN.md "Encoder"). */
QGEMM_API int qgemm_encoder_create(int d_model, int n_heads, int d_ff, int n_blocks, int max_seq, uint64_t seed,
                         void **encoder);
QGEMM_API int qgemm_encoder_forward(void *encoder, const float *X, float *Y, int seq, void *stream);
QGEMM_API int qgemm_encoder_destroy(void *encoder);

/* ---- LLM.int8() outlier decomposition ------------------------------------------
 * Feature columns k of A (= rows of B) holding an element with NOT(|x| <= threshold) (the reference's
 * AbsCompareLTEConstFunc, op_elemwise.cuh:293-306; NaN counts as an outlier) are multiplied in fp32,
 * the rest by the int8 chain, so outliers no longer set the absmax scales:
 *   C = fl( op_quantized_mm(A', B') + fmaf-chain over the outlier columns in ascending k )
 * with A' / B' = A / B with those columns / rows zeroed (no outlier column: the plain op_mm_quantize).
 * A: m x k, B: k x n, C: m x n, row-major contiguous, device pointers.  threshold: 6.0 in LLM.int8(). */
QGEMM_API size_t qgemm_mm_outlier_workspace_size(int m, int n, int k);
QGEMM_API int qgemm_mm_outlier(const float *A, const float *B, float *C, int m, int n, int k, float threshold,
                     void *workspace, size_t ws_bytes, void *stream);
/* number of outlier columns found by the last qgemm_mm_outlier on this workspace (synchronizes) */
QGEMM_API int qgemm_outlier_count(int k, const void *workspace, int *count);

/* The reference's quantization-error metric on the device: E = fl(C - O) per
 * element (op_subtract, op_elemwise.cuh:531-542), C = the unquantized product, O = the quantized one;
 * count elements, contiguous.  stats = DEVICE array of 5 doubles:
 *   [0] the reference's "Mean Quantization error" (tensor.cuh:201-211: signed, summed sequentially in
 *       fp32, / (float)count) -- computed only when reference_order != 0 (one lane, slow), else NaN
 *   [1] signed mean (fp64)  [2] mean |E|  [3] max |E|  [4] mean |C|   (relative error = [2] / [4])
 * Deterministic (fixed reduction tree for a given count). */
QGEMM_API int qgemm_error_stats(const float *C, const float *O, int64_t count, int reference_order, double *stats,
                      void *stream);

/* Deterministic U[lo,hi) fill, bit-identical to oracle_fill_uniform (stands in for the
 * reference's cuRAND op_uniform_init, op_elemwise.cuh:728-744). */
QGEMM_API int qgemm_fill_uniform(float *dst, int64_t count, uint64_t seed, float lo, float hi, void *stream);

/* Diagnostics: record hipEvent_t start_event / stop_event exactly at the start and end of the GEMM
 * kernel of the NEXT op_mm_quantize* / qgemm_mm_packed call made by this thread (then cleared).
 * Used by bench.py to time the dominant kernel inside its timed region.  NULL, NULL = off. */
QGEMM_API int qgemm_set_gemm_events(void *start_event, void *stop_event);
/* How those events are taken: 0 = hipExtLaunchKernel start/stop (default), 1 = hipEventRecord on the
 * stream right before / after the GEMM launch. */
QGEMM_API int qgemm_set_event_mode(int mode);

/* Diagnostics: the int8 GEMM launch plan op_mm_quantize* / qgemm_mm_packed use for an m x n x k call:
 * returns the number of K slices (1 = no split-K; < 0 on invalid sizes) and, when non-NULL, the
 * macro-tile edge (256, 64 or 32) and a static string naming the kernel. */
QGEMM_API int qgemm_gemm_plan(int m, int n, int k, int *tile, const char **kernel);

/* Library identification: "qgemm <version> gfx950 <kernel config>". */
QGEMM_API const char *qgemm_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QGEMM_H_ */
