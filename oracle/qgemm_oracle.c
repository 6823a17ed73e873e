/*
 * qgemm_oracle.c -- CPU restatement of the reference's int8 quantized GEMM chain.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library under
 * quantized-gemm-for-transformer-inference_amd/) links, loads or calls this file.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it,
 * and only as the checker / the CPU baseline -- never as the thing measured.
 *
 * It restates, element for element, the arithmetic of
 *   /root/reference/src/ops/op_mm.cuh:67-101  op_quantized_mm<float>(X, W, O, range)
 * as the reference's ten kernel launches perform it (citations per function below).
 * The reference itself cannot be built here (its headers need cuda_runtime.h /
 * curand.h, which this image lacks), so this restatement is pinned by the reference's
 * own fixture (test_quantize.cu:38-62, outputs recorded in SURVEY.md s4 KAT-1) and by
 * an independent pure-Python literal restatement (oracle/literal.py).  See DESIGN.md
 * "Oracle".
 *
 * Semantics:
 *   Cx[i] = seed X[i,0], then for k>=1: if |X[i,k]| > acc: acc = |X[i,k]|      (quirk)
 *   sx[i] = fl(range / Cx[i])                              (IEEE division)
 *   Xq[i,k] = sat_i8(trunc(fl(X[i,k] * sx[i])))   NaN -> 0  (reference: static_cast)
 *   Acc[i,j] = sum_k Xq[i,k] * Wq[k,j]                     exact int32
 *   Outer[i,j] = fl(Cx[i] * Cw[j]) + 0.0f                  (K=1 fp32 op_mm)
 *   O[i,j] = fl(fl((float)Acc * Outer) * fl(1/fl(range*range)))
 *
 * Build: see oracle/Makefile (gcc -O3 -ffp-contract=off -fopenmp, no fast-math).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <omp.h>

#define ORACLE_TILE 32 /* TILE_WIDTH, op_mm.cuh:6 -- sets the zero-padding of the fp32 k loop */

/* ---------------------------------------------------------------------------------
 * Deterministic input generator (shared bit-for-bit with the HIP fill kernel).
 * Restates op_uniform_init (op_elemwise.cuh:728-744) on our own counter-based
 * generator: u in [0,1) with 24 random bits, then t = fl(u + fl(lo/(hi-lo))),
 * x = fl(t * fl(hi-lo)).  For (lo,hi) = (-1,1) this is exactly 2u-1.
 * ------------------------------------------------------------------------------- */
static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

float oracle_uniform_at(uint64_t seed, uint64_t i, float lo, float hi)
{
    uint64_t key = mix64(seed + 0x9E3779B97F4A7C15ULL);
    uint64_t z = mix64(key + (i + 1) * 0x9E3779B97F4A7C15ULL);
    float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
    float span = hi - lo;
    float shift = lo / span;
    float t = u + shift;
    return t * span;
}

void oracle_fill_uniform(float *out, int64_t n, uint64_t seed, float lo, float hi)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
        out[i] = oracle_uniform_at(seed, (uint64_t)i, lo, hi);
}

/* ---------------------------------------------------------------------------------
 * AbsMaxFunc (op_reduction.cuh:7-25) applied as the reduction kernels do:
 * accumulator seeded with the SIGNED first element (colwise :80 / rowwise :105),
 * then the functor for i >= 1 (:81-83 / :106-108).  Reproduced literally, including
 * which zero sign survives and that NaN at i>=1 is skipped while a NaN seed sticks.
 * ------------------------------------------------------------------------------- */
static inline void absmax_step(float x, float *acc)
{
    if (x > 0) {
        if (x > *acc) *acc = x;
    } else {
        if (-x > *acc) *acc = -x;
    }
}

/* Cx[i] = AbsMax over row i of X[M x K] (op_absmax(X, Cx), op_mm.cuh:76-77 -> colwise kernel). */
void oracle_absmax_rows(const float *X, int M, int K, float *Cx)
{
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i) {
        const float *row = X + (int64_t)i * K;
        float acc = row[0];
        for (int k = 1; k < K; ++k) absmax_step(row[k], &acc);
        Cx[i] = acc;
    }
}

/* Cw[j] = AbsMax over column j of W[K x N] (op_absmax(W, Cw), op_mm.cuh:78-79 -> rowwise kernel).
 * K == 1 is undefined in the reference (it takes the colwise branch and leaves Cw[1..]
 * uninitialised); we define Cw[j] = W[0,j], the per-column seed. */
void oracle_absmax_cols(const float *W, int K, int N, float *Cw)
{
    for (int j = 0; j < N; ++j) Cw[j] = W[j];
    for (int k = 1; k < K; ++k) {
        const float *row = W + (int64_t)k * N;
        for (int j = 0; j < N; ++j) absmax_step(row[j], &Cw[j]);
    }
}

/* InvDivideConstFunc (op_elemwise.cuh:131-143): s = range / C, correctly rounded. */
void oracle_inv_divide(const float *C, int n, float range, float *s)
{
    for (int i = 0; i < n; ++i) s[i] = range / C[i];
}

/* MultiplyWithTypecastFunc<float,int8_t> (op_elemwise.cuh:106-114): static_cast<int8_t>(x*a).
 * The cast truncates toward zero; outside [-128,127] (reachable only through the absmax
 * quirk) and for NaN it is undefined in C++ -- we define saturation and NaN -> 0, the
 * behaviour of a saturating hardware convert.  Written without UB. */
static inline int8_t quant_i8(float x, float s)
{
    float v = x * s;
    if (v != v) return 0;
    if (v >= 127.0f) return 127;
    if (v <= -128.0f) return -128;
    return (int8_t)(int)v; /* |v| < 128: truncation, defined */
}

/* op_multiply(X, sx, X_int8) (op_mm.cuh:86-87): row broadcast of sx (bcast kernel :416-418). */
void oracle_quantize_rows(const float *X, const float *sx, int M, int K, int8_t *Xq)
{
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i)
        for (int k = 0; k < K; ++k)
            Xq[(int64_t)i * K + k] = quant_i8(X[(int64_t)i * K + k], sx[i]);
}

/* op_multiply(W, sw, W_int8) (op_mm.cuh:88-89): column broadcast of sw (bcast kernel :412-414). */
void oracle_quantize_cols(const float *W, const float *sw, int K, int N, int8_t *Wq)
{
#pragma omp parallel for schedule(static)
    for (int k = 0; k < K; ++k)
        for (int j = 0; j < N; ++j)
            Wq[(int64_t)k * N + j] = quant_i8(W[(int64_t)k * N + j], sw[j]);
}

/* op_mm<int8_t,int>(X_int8, W_int8, O_int32) (op_mm.cuh:92-93 -> op_matmul_kernel :9-46),
 * restated as the exact int32 dot product.  The reference accumulates through fp32 FMA
 * (int res; res += (float)a*(float)b, :37-39), identical to this while every partial sum
 * stays below 2^24 in magnitude; oracle_int8_mm_fp32emu below restates that literally
 * and the tests check both agree on every input they use. */
void oracle_int8_mm(const int8_t *Xq, const int8_t *Wq, int M, int N, int K, int32_t *Acc)
{
    int8_t *WqT = (int8_t *)malloc((size_t)N * (size_t)K + 1);
    for (int k = 0; k < K; ++k)
        for (int j = 0; j < N; ++j) WqT[(int64_t)j * K + k] = Wq[(int64_t)k * N + j];
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = 0; i < M; ++i) {
        const int8_t *a = Xq + (int64_t)i * K;
        for (int j = 0; j < N; ++j) {
            const int8_t *b = WqT + (int64_t)j * K;
            int32_t s = 0;
            for (int k = 0; k < K; ++k) s += (int16_t)a[k] * (int16_t)b[k];
            Acc[(int64_t)i * N + j] = s;
        }
    }
    free(WqT);
}

/* Literal restatement of op_matmul_kernel<int8_t,int>: per 32-wide k tile, res += A*B with
 * the operands staged as float (op_mm.cuh:16-17) and the += contracted to an fma (nvcc
 * default), then converted back to int (truncation).  Zero-padded tail products as the
 * kernel loads them (:21-33).  Slow; small sizes only. */
void oracle_int8_mm_fp32emu(const int8_t *Xq, const int8_t *Wq, int M, int N, int K, int32_t *Acc)
{
    int ntiles = (K - 1) / ORACLE_TILE + 1;
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            int res = 0;
            for (int t = 0; t < ntiles * ORACLE_TILE; ++t) {
                float a = t < K ? (float)Xq[(int64_t)i * K + t] : 0.0f;
                float b = t < K ? (float)Wq[(int64_t)t * N + j] : 0.0f;
                res = (int)fmaf(a, b, (float)res);
            }
            Acc[(int64_t)i * N + j] = res;
        }
}

/* op_mm<float,float>(Cx, Cw, Outer) with K = 1 (op_mm.cuh:96-97): res = 0, then 32 products
 * of which 31 are the zero padding; = fl(Cx*Cw) + 0.0f (a -0 product becomes +0). */
static inline float outer_at(float cx, float cw)
{
    float r = fmaf(cx, cw, 0.0f);
    return r + 0.0f;
}

/* op_dequantize (op_elemwise.cuh:614-625, DequantizeFunc :93-103) then
 * op_multiply(O, 1/(range*range), O) (op_mm.cuh:99, MultiplyConstFunc :118-129). */
static inline float dequant(int32_t acc, float cx, float cw, float inv_r2)
{
    float o = (float)acc * outer_at(cx, cw);
    return o * inv_r2;
}

void oracle_dequantize(const int32_t *Acc, const float *Cx, const float *Cw, int M, int N,
                       float range, float *O)
{
    float inv_r2 = 1.0f / (range * range);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j)
            O[(int64_t)i * N + j] = dequant(Acc[(int64_t)i * N + j], Cx[i], Cw[j], inv_r2);
}

/* Whole chain, op_quantized_mm (op_mm.cuh:67-101).  Optional intermediates (may be NULL). */
void oracle_quantized_mm_ex(const float *X, const float *W, float *O, int M, int N, int K, float range,
                            float *Cx_out, float *Cw_out, int8_t *Xq_out, int8_t *Wq_out, int32_t *Acc_out)
{
    float *Cx = Cx_out ? Cx_out : (float *)malloc(sizeof(float) * (size_t)M);
    float *Cw = Cw_out ? Cw_out : (float *)malloc(sizeof(float) * (size_t)N);
    float *sx = (float *)malloc(sizeof(float) * (size_t)M);
    float *sw = (float *)malloc(sizeof(float) * (size_t)N);
    int8_t *Xq = Xq_out ? Xq_out : (int8_t *)malloc((size_t)M * (size_t)K + 1);
    int8_t *Wq = Wq_out ? Wq_out : (int8_t *)malloc((size_t)K * (size_t)N + 1);
    int32_t *Acc = Acc_out ? Acc_out : (int32_t *)malloc(sizeof(int32_t) * (size_t)M * (size_t)N);

    oracle_absmax_rows(X, M, K, Cx);
    oracle_absmax_cols(W, K, N, Cw);
    oracle_inv_divide(Cx, M, range, sx);
    oracle_inv_divide(Cw, N, range, sw);
    oracle_quantize_rows(X, sx, M, K, Xq);
    oracle_quantize_cols(W, sw, K, N, Wq);
    oracle_int8_mm(Xq, Wq, M, N, K, Acc);
    oracle_dequantize(Acc, Cx, Cw, M, N, range, O);

    if (!Cx_out) free(Cx);
    if (!Cw_out) free(Cw);
    free(sx);
    free(sw);
    if (!Xq_out) free(Xq);
    if (!Wq_out) free(Wq);
    if (!Acc_out) free(Acc);
}

void oracle_quantized_mm(const float *X, const float *W, float *O, int M, int N, int K, float range)
{
    oracle_quantized_mm_ex(X, W, O, M, N, K, range, NULL, NULL, NULL, NULL, NULL);
}

/* The chain for a SUBSET of output rows: rows are independent given Cw, so a full-size
 * GPU result can be checked bit-exactly on sampled rows in seconds.  O_rows is [nrows x N]. */
void oracle_quantized_mm_rows(const float *X, const float *W, float *O_rows, int M, int N, int K,
                              float range, const int *rows, int nrows)
{
    (void)M;
    float *Cw = (float *)malloc(sizeof(float) * (size_t)N);
    float *sw = (float *)malloc(sizeof(float) * (size_t)N);
    int8_t *WqT = (int8_t *)malloc((size_t)N * (size_t)K + 1);
    oracle_absmax_cols(W, K, N, Cw);
    oracle_inv_divide(Cw, N, range, sw);
#pragma omp parallel for schedule(static)
    for (int j = 0; j < N; ++j)
        for (int k = 0; k < K; ++k) WqT[(int64_t)j * K + k] = quant_i8(W[(int64_t)k * N + j], sw[j]);
    float inv_r2 = 1.0f / (range * range);
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; ++r) {
        const float *x = X + (int64_t)rows[r] * K;
        float cx;
        oracle_absmax_rows(x, 1, K, &cx);
        float sx = range / cx;
        int8_t *xq = (int8_t *)malloc((size_t)K + 1);
        for (int k = 0; k < K; ++k) xq[k] = quant_i8(x[k], sx);
        for (int j = 0; j < N; ++j) {
            const int8_t *b = WqT + (int64_t)j * K;
            int32_t s = 0;
            for (int k = 0; k < K; ++k) s += (int16_t)xq[k] * (int16_t)b[k];
            O_rows[(int64_t)r * N + j] = dequant(s, cx, Cw[j], inv_r2);
        }
        free(xq);
    }
    free(Cw);
    free(sw);
    free(WqT);
}

/* op_mm<float,float>(X, W, C) (op_mm.cuh:49-65 -> op_matmul_kernel<float,float>): the
 * unquantized path.  res starts at +0 and is accumulated sequentially in k with fmaf
 * (nvcc contracts :38), including the zero-padded products of the last 32-wide tile. */
void oracle_mm_fp32(const float *X, const float *W, float *C, int M, int N, int K)
{
    int kpad = ((K - 1) / ORACLE_TILE + 1) * ORACLE_TILE;
#pragma omp parallel
    {
        float *acc = (float *)malloc(sizeof(float) * (size_t)N);
#pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < M; ++i) {
            for (int j = 0; j < N; ++j) acc[j] = 0.0f;
            /* i-k-j order: each acc[j] still sees its k terms in ascending order */
            for (int k = 0; k < K; ++k) {
                float a = X[(int64_t)i * K + k];
                const float *w = W + (int64_t)k * N;
                for (int j = 0; j < N; ++j) acc[j] = fmaf(a, w[j], acc[j]);
            }
            for (int k = K; k < kpad; ++k)
                for (int j = 0; j < N; ++j) acc[j] = fmaf(0.0f, 0.0f, acc[j]);
            memcpy(C + (int64_t)i * N, acc, sizeof(float) * (size_t)N);
        }
        free(acc);
    }
}

/* op_subtract(C, qC, err) then err.toHost().mean() (tensor.cuh:201-211): a SIGNED mean,
 * summed sequentially in fp32 and divided by h*w (an int converted to float). */
float oracle_signed_mean_error(const float *C, const float *O, int64_t n)
{
    float sum = 0.0f;
    for (int64_t i = 0; i < n; ++i) {
        float d = C[i] - O[i];
        sum += d;
    }
    return sum / (float)(int)n;
}

/* Error statistics beyond the reference's metric: mean|E|, max|E|, and sum|C| (for relative). */
void oracle_error_stats(const float *C, const float *O, int64_t n, double *mean_abs, double *max_abs,
                        double *mean_abs_ref)
{
    double s = 0.0, m = 0.0, r = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double d = fabs((double)C[i] - (double)O[i]);
        s += d;
        if (d > m) m = d;
        r += fabs((double)C[i]);
    }
    *mean_abs = s / (double)n;
    *max_abs = m;
    *mean_abs_ref = r / (double)n;
}

/* =================================================================================
 * Encoder counterpart: transformer.cu:14-77 with the quantized linears,
 * restated with the decisions documented in DESIGN.md "Encoder" (the reference's Encoder does
 * not compile: arity at transformer.cu:37, ffnOut size at :62).
 * ================================================================================= */

/* op_mm<float,float> on strided views (Index(), tensor.cuh:14): res = +0, then fmaf over k
 * ascending, then the zero products of the last 32-wide tile (op_mm.cuh:9-46). */
static void mm_f32_strided(const float *A, int64_t ash, int64_t asw, const float *B, int64_t bsh, int64_t bsw,
                           float *C, int64_t csh, int64_t csw, int m, int n, int k)
{
    int kpad = ((k - 1) / ORACLE_TILE + 1) * ORACLE_TILE;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            float r = 0.0f;
            for (int kk = 0; kk < k; ++kk) r = fmaf(A[i * ash + kk * asw], B[kk * bsh + j * bsw], r);
            for (int kk = k; kk < kpad; ++kk) r = fmaf(0.0f, 0.0f, r);
            C[i * csh + j * csw] = r;
        }
}

/* op_multiply(S, scale) (attention.cuh:65) then op_softmax (op_softmax.cuh:6-29) per row:
 * max seeded with the first element, strict '>'; exp as the correctly rounded fp32 exp
 * fl32(exp((double)x)); sum in column order; divide. */
void oracle_softmax_rows(const float *S, float *P, int64_t rows, int w, float scale)
{
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
        const float *s = S + r * w;
        float *p = P + r * w;
        float mx = s[0] * scale;
        for (int c = 1; c < w; ++c) {
            float x = s[c] * scale;
            if (x > mx) mx = x;
        }
        float sum = 0.0f;
        for (int c = 0; c < w; ++c) {
            float e = (float)exp((double)(s[c] * scale - mx));
            p[c] = e;
            sum += p[c];
        }
        for (int c = 0; c < w; ++c) p[c] = p[c] / sum;
    }
}

/* op_add(A, B) (transformer.cu:58) then op_layernorm as written (op_layernorm.cuh:6-33):
 * mean = sum/w, var = sum of pow(y-mean, 2) with CUDA's float pow(float,int) = fl(d*d), / w,
 * out = (y - mean) / var. */
void oracle_add_layernorm_rows(const float *A, const float *B, float *Y, int64_t rows, int w)
{
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
        const float *a = A + r * w, *b = B + r * w;
        float *y = Y + r * w;
        float mean = 0.0f, var = 0.0f;
        for (int c = 0; c < w; ++c) mean += a[c] + b[c];
        mean = mean / (float)w;
        for (int c = 0; c < w; ++c) {
            float d = (a[c] + b[c]) - mean;
            var += d * d;
        }
        var = var / (float)w;
        for (int c = 0; c < w; ++c) y[c] = ((a[c] + b[c]) - mean) / var;
    }
}

/* LinearLayer.forward on the quantized path (linear.cuh:50-54, + op_relu): y = fl(O + b[j]),
 * relu = (y < 0 ? 0 : y).  W is K x N row-major; b may be NULL. */
void oracle_linear(const float *X, const float *W, const float *b, int relu, float *Y, int M, int N, int K)
{
    oracle_quantized_mm(X, W, Y, M, N, K, 127.0f);
    if (!b) return;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            float y = Y[(int64_t)i * N + j] + b[j];
            if (relu && y < 0) y = 0;
            Y[(int64_t)i * N + j] = y;
        }
}

/* Seed of encoder weight tensor (block, kind, head), kind 0..7 = Wq Wk Wv Wo W1 b1 W2 b2
 * (include/qgemm.h qgemm_encoder_create). */
uint64_t oracle_encoder_weight_seed(uint64_t base, int block, int kind, int head)
{
    return base * 1000003ULL + (uint64_t)block * 4099ULL + (uint64_t)kind * 131ULL + (uint64_t)head;
}

/* "float max = 1.0f / std::sqrt(n)" with an int n (attention.cuh:38, linear.cuh:35) */
static float init_bound(int n) { return (float)(1.0 / sqrt((double)n)); }

void oracle_encoder_forward(const float *X, float *Y, int seq, int d, int H, int dff, int nblocks, uint64_t seed)
{
    const int dk = d / H;
    const float scale = (float)(1.0 / sqrt((double)dk));
    size_t S = (size_t)seq;
    float *qkv = (float *)malloc(sizeof(float) * S * 3 * d);
    float *scores = (float *)malloc(sizeof(float) * (size_t)H * S * S);
    float *heads = (float *)malloc(sizeof(float) * S * d);
    float *t = (float *)malloc(sizeof(float) * S * d);
    float *x1 = (float *)malloc(sizeof(float) * S * d);
    float *ffn = (float *)malloc(sizeof(float) * S * dff);
    float *cur = (float *)malloc(sizeof(float) * S * d);
    float *w = (float *)malloc(sizeof(float) * (size_t)(d > dff ? d : dff) * (size_t)(3 * d > dff ? 3 * d : dff));
    float *one = (float *)malloc(sizeof(float) * (size_t)d * dk);
    float *b = (float *)malloc(sizeof(float) * (size_t)(d > dff ? d : dff));
    const float *in = X;
    for (int i = 0; i < nblocks; ++i) {
        float *out = (i == nblocks - 1) ? Y : cur;
        /* [Wq | Wk | Wv], one d x dk tensor per (kind, head) (attention.cuh:37-41, :54-56) */
        for (int kind = 0; kind < 3; ++kind)
            for (int h = 0; h < H; ++h) {
                float bd = init_bound(dk);
                oracle_fill_uniform(one, (int64_t)d * dk, oracle_encoder_weight_seed(seed, i, kind, h), -bd, bd);
                for (int r = 0; r < d; ++r)
                    memcpy(w + (size_t)r * 3 * d + kind * d + h * dk, one + (size_t)r * dk, sizeof(float) * dk);
            }
        oracle_quantized_mm(in, w, qkv, seq, 3 * d, d, 127.0f);
        for (int h = 0; h < H; ++h)   /* S_h = Q_h K_h^T (attention.cuh:58-60) */
            mm_f32_strided(qkv + h * dk, 3 * d, 1, qkv + d + h * dk, 1, 3 * d, scores + (size_t)h * S * S, seq, 1,
                           seq, seq, dk);
        oracle_softmax_rows(scores, scores, (int64_t)H * seq, seq, scale);
        for (int h = 0; h < H; ++h)   /* heads[:, h*dk..] = P_h V_h (attention.cuh:69, transformer.cu:43-50) */
            mm_f32_strided(scores + (size_t)h * S * S, seq, 1, qkv + 2 * d + h * dk, 3 * d, 1, heads + h * dk, d, 1,
                           seq, dk, seq);
        /* output = multiHeadOut @ W_O (transformer.cu:52-54), W_O ~ U(-1, 1) */
        oracle_fill_uniform(w, (int64_t)d * d, oracle_encoder_weight_seed(seed, i, 3, 0), -1.0f, 1.0f);
        oracle_quantized_mm(heads, w, t, seq, d, d, 127.0f);
        oracle_add_layernorm_rows(t, heads, x1, seq, d);   /* :58-59 */
        /* FFN (transformer.cu:62-71, linear.cuh:34-39 bounds) */
        float bd = init_bound(d), bf = init_bound(dff);
        oracle_fill_uniform(w, (int64_t)d * dff, oracle_encoder_weight_seed(seed, i, 4, 0), -bd, bd);
        oracle_fill_uniform(b, dff, oracle_encoder_weight_seed(seed, i, 5, 0), -bd, bd);
        oracle_linear(x1, w, b, 1, ffn, seq, dff, d);
        oracle_fill_uniform(w, (int64_t)dff * d, oracle_encoder_weight_seed(seed, i, 6, 0), -bf, bf);
        oracle_fill_uniform(b, d, oracle_encoder_weight_seed(seed, i, 7, 0), -bf, bf);
        oracle_linear(ffn, w, b, 0, t, seq, d, dff);
        oracle_add_layernorm_rows(t, heads, out, seq, d);  /* :74-75 */
        in = out;
    }
    free(qkv);
    free(scores);
    free(heads);
    free(t);
    free(x1);
    free(ffn);
    free(cur);
    free(w);
    free(one);
    free(b);
}

/* =================================================================================
 * LLM.int8() outlier decomposition (the reference's unused hooks
 * AbsCompareLTEConstFunc op_elemwise.cuh:293-306 and op_outlier_extractor :698-708).
 * Column k of X is an outlier column when some X[i,k] is not in [-t, t] (NaN included);
 * O = fl(quantized_mm(X', W') + fmaf chain over the outlier columns in ascending k), X'/W' with
 * those columns/rows zeroed.  Returns the number of outlier columns.
 * ================================================================================= */
int oracle_mm_outlier(const float *X, const float *W, float *O, int M, int N, int K, float t)
{
    unsigned char *flag = (unsigned char *)calloc((size_t)K, 1);
    for (int i = 0; i < M; ++i)
        for (int k = 0; k < K; ++k) {
            float a = X[(int64_t)i * K + k];
            int inside = ((a >= 0) & (a <= t)) | ((a <= 0) & (-a <= t));
            if (!inside) flag[k] = 1;
        }
    int *idx = (int *)malloc(sizeof(int) * (size_t)K);
    int cnt = 0;
    for (int k = 0; k < K; ++k)
        if (flag[k]) idx[cnt++] = k;
    float *Xm = (float *)malloc(sizeof(float) * (size_t)M * K);
    float *Wm = (float *)malloc(sizeof(float) * (size_t)K * N);
    for (int64_t e = 0; e < (int64_t)M * K; ++e) Xm[e] = flag[e % K] ? 0.0f : X[e];
    for (int64_t e = 0; e < (int64_t)K * N; ++e) Wm[e] = flag[e / N] ? 0.0f : W[e];
    oracle_quantized_mm(Xm, Wm, O, M, N, K, 127.0f);
    if (cnt) {
#pragma omp parallel for schedule(static)
        for (int i = 0; i < M; ++i)
            for (int j = 0; j < N; ++j) {
                float acc = 0.0f;
                for (int q = 0; q < cnt; ++q)
                    acc = fmaf(X[(int64_t)i * K + idx[q]], W[(int64_t)idx[q] * N + j], acc);
                O[(int64_t)i * N + j] = O[(int64_t)i * N + j] + acc;
            }
    }
    free(flag);
    free(idx);
    free(Xm);
    free(Wm);
    return cnt;
}

/* The thread count of the OpenMP regions above (bench.py's cpu_baseline sets it from the measured host CPU
 * share, so `cores` is what ran, not an environment default). */
void oracle_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
}
