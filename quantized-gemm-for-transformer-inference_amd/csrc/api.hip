// api.hip -- the C-ABI of include/qgemm.h: argument checks, layout dispatch, workspace, stream order.
//
// op_quantized_mm (/root/reference/src/ops/op_mm.cuh:67-101) runs ten launches and allocates eight
// temporaries per call.  Here a call is two or three stream-ordered launches on caller memory plus a
// grow-only workspace cached per (device, stream):
//   pack A  (Cx + X_int8)          -- op_mm.cuh:76-77, 82-83, 86-87
//   pack B  (Cw + W_int8^T)        -- op_mm.cuh:78-79, 84-85, 88-89
//   MFMA GEMM + dequant epilogue   -- op_mm.cuh:92-99
#include <map>
#include <mutex>
#include <thread>
#include <stdio.h>

#include "../../include/qgemm.h"
#include "qgemm_internal.h"

using namespace qgemm;

namespace {

constexpr float kDefaultRange = 127.0f;  // `range` at every reference call site (test_quantize.cu:76)

int err(hipError_t e) { return (int)e; }

bool dims_ok(int m, int n, int k) { return m >= 0 && n >= 0 && k >= 1; }

// Which packing pass serves a matrix whose reduction vectors are its rows (row_stride, elem_stride)?
//   elem_stride == 1       : the vectors are contiguous        -> pack_rows (vector path)
//   row_stride  == 1       : the vectors are columns of a row-major image -> pack_cols
//   anything else          : pack_rows generic (scalar, strided)
hipError_t pack_vectors(const float *src, int64_t row_stride, int64_t elem_stride, int rows, int len, float range,
                        PackedView out, hipStream_t stream) {
    if (elem_stride == 1) return launch_pack_rows(src, row_stride, 1, rows, len, range, out, stream);
    if (row_stride == 1 && len > 1) return launch_pack_cols(src, elem_stride, len, rows, range, out, stream);
    return launch_pack_rows(src, row_stride, elem_stride, rows, len, range, out, stream);
}

// Grow-only cached buffers for the entry points without an explicit workspace, one per (device, stream, use): a
// buffer is only reused in its stream's order, so calls on different streams never share packed operands or split-K
// tickets (the reference allocates its temporaries per call, op_mm.cuh:76-93).  hipStreamPerThread names a different
// stream in every host thread, so it is keyed by the calling thread as well.  Growth waits for the owning stream only.
// At most kMaxCachedStreams buffers per (device, use): a process that cycles through many streams does not keep one
// workspace per stream it ever used -- the least recently used buffer is freed after a device synchronisation (its
// stream may no longer exist), which only happens when a new stream arrives.
enum CacheUse { kUseWorkspace = 0, kUseSplitK = 1, kUseErrorStats = 2 };  // never shared: split-K tickets stay zero
constexpr int kMaxCachedStreams = 8;
struct CacheKey {
    int dev;
    hipStream_t stream;
    std::thread::id thread;
    int use;
    bool operator<(const CacheKey &o) const {
        if (dev != o.dev) return dev < o.dev;
        if (stream != o.stream) return stream < o.stream;
        if (thread != o.thread) return thread < o.thread;
        return use < o.use;
    }
};
struct CachedBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    uint64_t last_use = 0;
};
std::mutex g_cache_mu;
std::map<CacheKey, CachedBuf> g_cache;
uint64_t g_cache_clock = 0;

// frees the least recently used buffer of (dev, use) other than `keep` once there are more than kMaxCachedStreams
hipError_t evict_cached(int dev, int use, const CacheKey &keep) {
    int n = 0;
    auto victim = g_cache.end();
    for (auto it = g_cache.begin(); it != g_cache.end(); ++it) {
        if (it->first.dev != dev || it->first.use != use) continue;
        ++n;
        if (!(it->first < keep) && !(keep < it->first)) continue;
        if (victim == g_cache.end() || it->second.last_use < victim->second.last_use) victim = it;
    }
    if (n <= kMaxCachedStreams || victim == g_cache.end()) return hipSuccess;
    hipError_t e = hipSuccess;
    if (victim->second.ptr) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
        e = hipFree(victim->second.ptr);
    }
    g_cache.erase(victim);
    return e;
}

// zero_new: the buffer is zeroed when (re)allocated (split-K tickets start at zero; the launches re-zero them)
hipError_t cached_buffer(size_t need, hipStream_t stream, int use, bool zero_new, size_t headroom, void **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const std::thread::id th = stream == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
    std::lock_guard<std::mutex> lk(g_cache_mu);
    const CacheKey key{dev, stream, th, use};
    const bool fresh = g_cache.find(key) == g_cache.end();
    CachedBuf &w = g_cache[key];
    w.last_use = ++g_cache_clock;
    if (fresh && (e = evict_cached(dev, use, key)) != hipSuccess) return e;
    if (w.bytes < need) {
        if (w.ptr) {
            // earlier calls on this stream may still be using it
            if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
            if ((e = hipFree(w.ptr)) != hipSuccess) return e;
            w.ptr = nullptr;
            w.bytes = 0;
        }
        const size_t grow = need + headroom;
        if ((e = hipMalloc(&w.ptr, grow)) != hipSuccess) return e;
        if (zero_new && (e = hipMemset(w.ptr, 0, grow)) != hipSuccess) return e;
        w.bytes = grow;
    }
    *out = w.ptr;
    return hipSuccess;
}

hipError_t cached_workspace(size_t need, hipStream_t stream, void **out) {
    return cached_buffer(need, stream, kUseWorkspace, false, need / 8 /* headroom for nearby shapes */, out);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split-K scratch of qgemm_mm_packed and the error-statistics scratch (no workspace argument): zeroed at allocation.
hipError_t cached_scratch(size_t need, hipStream_t stream, int use, void **out) {
    return cached_buffer(need, stream, use, true, 0, out);
}

hipError_t mm_packed_impl(const void *packed_a, const void *packed_b, float *C, int64_t c_stride_h,
                          int64_t c_stride_w, int m, int n, int k, float range, void *scratch, size_t scratch_bytes,
                          hipStream_t stream, bool tickets_zeroed = false) {
    const float inv_r2 = 1.0f / (range * range);  // op_mm.cuh:99, one rounding per operation (host IEEE)
    return launch_gemm_dequant(packed_view(packed_a, m, k), packed_view(packed_b, n, k), C, c_stride_h, c_stride_w, m,
                               n, inv_r2, scratch, scratch_bytes, stream, nullptr, false, tickets_zeroed);
}

}  // namespace

extern "C" {

size_t qgemm_packed_size(int rows, int k) {
    if (rows < 0 || k < 1) return 0;
    return packed_bytes(rows, k);
}

size_t op_mm_quantize_workspace_size(int m, int n, int k) {
    if (!dims_ok(m, n, k)) return 0;
    // [split-K scratch (0 unless the shape has too few tiles)][packed A][packed B]
    return align256(gemm_scratch_bytes(m, n, k)) + align256(packed_bytes(m, k)) + align256(packed_bytes(n, k));
}

int qgemm_pack_a(const float *A, int64_t a_stride_h, int64_t a_stride_w, int m, int k, float range, void *packed_a,
                 void *stream) {
    if (!A || !packed_a || m < 0 || k < 1) return err(hipErrorInvalidValue);
    if (m == 0) return 0;
    // reduction vectors = rows of A: (row stride, element stride) = (stride_h, stride_w)
    return err(pack_vectors(A, a_stride_h, a_stride_w, m, k, range, packed_view(packed_a, m, k),
                            static_cast<hipStream_t>(stream)));
}

int qgemm_pack_b(const float *B, int64_t b_stride_h, int64_t b_stride_w, int k, int n, float range, void *packed_b,
                 void *stream) {
    if (!B || !packed_b || n < 0 || k < 1) return err(hipErrorInvalidValue);
    if (n == 0) return 0;
    // reduction vectors = columns of B: (vector stride, element stride) = (stride_w, stride_h)
    return err(pack_vectors(B, b_stride_w, b_stride_h, n, k, range, packed_view(packed_b, n, k),
                            static_cast<hipStream_t>(stream)));
}

int qgemm_mm_packed(const void *packed_a, const void *packed_b, float *C, int64_t c_stride_h, int64_t c_stride_w,
                    int m, int n, int k, float range, void *stream) {
    if (!packed_a || !packed_b || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    void *scratch = nullptr;
    const size_t sb = gemm_scratch_bytes(m, n, k);
    if (sb) {
        hipError_t e = cached_scratch(sb, s, kUseSplitK, &scratch);
        if (e != hipSuccess) return err(e);
    }
    return err(mm_packed_impl(packed_a, packed_b, C, c_stride_h, c_stride_w, m, n, k, range, scratch, sb, s,
                              /*tickets_zeroed=*/true));
}

int qgemm_mm_packed_i32(const void *packed_a, const void *packed_b, int32_t *Acc, int m, int n, int k, void *stream) {
    if (!packed_a || !packed_b || !Acc || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    return err(launch_gemm_i32(packed_view(packed_a, m, k), packed_view(packed_b, n, k), Acc, m, n,
                               static_cast<hipStream_t>(stream)));
}

int op_mm_quantize_ws(const float *A, int64_t a_stride_h, int64_t a_stride_w, const float *B, int64_t b_stride_h,
                      int64_t b_stride_w, float *C, int64_t c_stride_h, int64_t c_stride_w, int m, int n, int k,
                      float range, void *workspace, size_t ws_bytes, void *stream) {
    // op_mm.cuh:71-72: shape agreement and device residency are asserted by the reference
    if (!A || !B || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    const size_t need = op_mm_quantize_workspace_size(m, n, k);
    if (!workspace || ws_bytes < need) return err(hipErrorInvalidValue);
    char *scratch = static_cast<char *>(workspace);
    const size_t sb = gemm_scratch_bytes(m, n, k);
    char *pa = scratch + align256(sb);
    char *pb = pa + align256(packed_bytes(m, k));
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto gemm = [&](bool tickets_zeroed) {
        return err(mm_packed_impl(pa, pb, C, c_stride_h, c_stride_w, m, n, k, range, scratch, sb, s, tickets_zeroed));
    };
    // the pack launch zeroes the split-K tickets at the start of the workspace (the GEMM then needs no
    // zeroing launch of its own)
    uint32_t *tickets = reinterpret_cast<uint32_t *>(scratch);
    const int ntickets = (int)(gemm_ticket_bytes(m, n, k) / 4);
    // Common case (row-major X and W): X's row pass and W's column-absmax pass share one launch,
    // then W's quantize/transpose pass, then the GEMM -- three launches in all.
    if (a_stride_w == 1 && b_stride_w == 1 && k > 1) {
        const PackedView va = packed_view(pa, m, k), vb = packed_view(pb, n, k);
        // K <= 4096: W read once (single-pass strips) -- two launches in all
        hipError_t e = launch_pack_single_pass(A, a_stride_h, m, k, va, B, b_stride_h, n, vb, range, s, tickets, ntickets);
        if (e == hipSuccess) return gemm(true);
        if (e != hipErrorNotSupported) return err(e);
        e = launch_pack_two_pass(A, a_stride_h, m, k, va, B, b_stride_h, n, vb, range, s, tickets, ntickets);
        if (e == hipSuccess) return gemm(true);
        if (e != hipErrorNotSupported) return err(e);
    }
    int rc = qgemm_pack_a(A, a_stride_h, a_stride_w, m, k, range, pa, stream);
    if (rc) return rc;
    rc = qgemm_pack_b(B, b_stride_h, b_stride_w, k, n, range, pb, stream);
    if (rc) return rc;
    return gemm(false);
}

int op_mm_quantize_ex(const float *A, int64_t a_stride_h, int64_t a_stride_w, const float *B, int64_t b_stride_h,
                      int64_t b_stride_w, float *C, int64_t c_stride_h, int64_t c_stride_w, int m, int n, int k,
                      float range, void *stream) {
    if (!A || !B || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    const size_t need = op_mm_quantize_workspace_size(m, n, k);
    void *ws = nullptr;
    hipError_t e = cached_workspace(need, static_cast<hipStream_t>(stream), &ws);
    if (e != hipSuccess) return err(e);
    return op_mm_quantize_ws(A, a_stride_h, a_stride_w, B, b_stride_h, b_stride_w, C, c_stride_h, c_stride_w, m, n, k,
                             range, ws, need, stream);
}

int op_mm_quantize(const float *A, const float *B, float *C, int m, int n, int k) {
    return op_mm_quantize_ex(A, k, 1, B, n, 1, C, n, 1, m, n, k, kDefaultRange, nullptr);
}

int qgemm_mm_fp32(const float *A, int64_t a_stride_h, int64_t a_stride_w, const float *B, int64_t b_stride_h,
                  int64_t b_stride_w, float *C, int64_t c_stride_h, int64_t c_stride_w, int m, int n, int k,
                  void *stream) {
    if (!A || !B || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    return err(launch_mm_f32(A, a_stride_h, a_stride_w, B, b_stride_h, b_stride_w, C, c_stride_h, c_stride_w, m, n, k,
                             static_cast<hipStream_t>(stream)));
}

int qgemm_error_stats(const float *C, const float *O, int64_t count, int reference_order, double *stats,
                      void *stream) {
    if (!C || !O || !stats || count < 1) return err(hipErrorInvalidValue);
    hipStream_t s = static_cast<hipStream_t>(stream);
    void *scratch = nullptr;
    hipError_t e = cached_scratch(error_stats_scratch_bytes(), s, kUseErrorStats, &scratch);
    if (e != hipSuccess) return err(e);
    return err(launch_error_stats(C, O, count, reference_order != 0, stats, scratch, s));
}

int qgemm_linear(const float *X, int64_t x_stride_h, int m, int k, const void *packed_w, int n, const float *bias,
                 int relu, float *Y, int64_t y_stride_h, void *workspace, size_t ws_bytes, void *stream) {
    if (!X || !packed_w || !Y || m < 0 || n < 0 || k < 1 || (relu && !bias)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    const size_t need = qgemm_linear_workspace_size(m, n, k);
    if (!workspace || ws_bytes < need) return err(hipErrorInvalidValue);
    hipStream_t s = static_cast<hipStream_t>(stream);
    char *scratch = static_cast<char *>(workspace);
    const size_t sb = gemm_scratch_bytes(m, n, k);
    char *pa = scratch + align256(sb);
    const PackedView va = packed_view(pa, m, k);
    hipError_t e = pack_vectors(X, x_stride_h, 1, m, k, kDefaultRange, va, s);
    if (e != hipSuccess) return err(e);
    const float inv_r2 = 1.0f / (kDefaultRange * kDefaultRange);
    return err(launch_gemm_dequant(va, packed_view(packed_w, n, k), Y, y_stride_h, 1, m, n, inv_r2, scratch, sb, s, bias,
                                   relu != 0));
}

size_t qgemm_linear_workspace_size(int m, int n, int k) {
    if (m < 0 || n < 0 || k < 1) return 0;
    return align256(gemm_scratch_bytes(m, n, k)) + align256(packed_bytes(m, k));
}

size_t op_mm_quantize_prepacked_workspace_size(int m, int n, int k) { return qgemm_linear_workspace_size(m, n, k); }

int op_mm_quantize_prepacked_ws(const float *A, int64_t a_stride_h, const void *packed_b, float *C, int64_t c_stride_h,
                                int m, int n, int k, void *workspace, size_t ws_bytes, void *stream) {
    // op_mm.cuh:71-72: shape agreement and device residency are asserted by the reference
    if (!A || !packed_b || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    return qgemm_linear(A, a_stride_h, m, k, packed_b, n, nullptr, 0, C, c_stride_h, workspace, ws_bytes, stream);
}

int op_mm_quantize_prepacked(const float *A, const void *packed_b, float *C, int m, int n, int k) {
    if (!A || !packed_b || !C || !dims_ok(m, n, k)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    const size_t need = qgemm_linear_workspace_size(m, n, k);
    void *ws = nullptr;
    hipError_t e = cached_workspace(need, nullptr, &ws);
    if (e != hipSuccess) return err(e);
    return op_mm_quantize_prepacked_ws(A, k, packed_b, C, n, m, n, k, ws, need, nullptr);
}

int qgemm_softmax_rows(const float *S, float *P, int64_t rows, int w, float scale, void *stream) {
    if (!S || !P) return err(hipErrorInvalidValue);
    return err(launch_softmax_rows(S, P, rows, w, scale, static_cast<hipStream_t>(stream)));
}

int qgemm_add_layernorm_rows(const float *A, const float *B, float *Y, int64_t rows, int w, void *stream) {
    if (!A || !B || !Y) return err(hipErrorInvalidValue);
    return err(launch_add_layernorm_rows(A, B, Y, rows, w, static_cast<hipStream_t>(stream)));
}

int qgemm_encoder_create(int d_model, int n_heads, int d_ff, int n_blocks, int max_seq, uint64_t seed,
                         void **encoder) {
    if (!encoder) return err(hipErrorInvalidValue);
    Encoder *E = nullptr;
    hipError_t e = encoder_create(d_model, n_heads, d_ff, n_blocks, max_seq, seed, &E);
    *encoder = E;
    return err(e);
}

int qgemm_encoder_forward(void *encoder, const float *X, float *Y, int seq, void *stream) {
    return err(encoder_forward(static_cast<Encoder *>(encoder), X, Y, seq, static_cast<hipStream_t>(stream)));
}

int qgemm_encoder_destroy(void *encoder) {
    encoder_destroy(static_cast<Encoder *>(encoder));
    return 0;
}

size_t qgemm_mm_outlier_workspace_size(int m, int n, int k) {
    if (!dims_ok(m, n, k)) return 0;
    return align256(outlier_scratch_bytes(m, n, k)) + op_mm_quantize_workspace_size(m, n, k);
}

int qgemm_mm_outlier(const float *A, const float *B, float *C, int m, int n, int k, float threshold, void *workspace,
                     size_t ws_bytes, void *stream) {
    if (!A || !B || !C || !dims_ok(m, n, k) || !(threshold >= 0.0f)) return err(hipErrorInvalidValue);
    if (m == 0 || n == 0) return 0;
    const size_t need = qgemm_mm_outlier_workspace_size(m, n, k);
    if (!workspace || ws_bytes < need) return err(hipErrorInvalidValue);
    hipStream_t s = static_cast<hipStream_t>(stream);
    char *scratch = static_cast<char *>(workspace);
    char *ws2 = scratch + align256(outlier_scratch_bytes(m, n, k));
    {
        // fast path: the packed operands in the plain chain's slots of ws2 (no split-K: no tickets)
        char *pa = ws2 + align256(gemm_scratch_bytes(m, n, k));
        char *pb = pa + align256(packed_bytes(m, k));
        const hipError_t e = outlier_fast(A, B, C, m, n, k, threshold, scratch, packed_view(pa, m, k),
                                          packed_view(pb, n, k), kDefaultRange, s);
        if (e != hipErrorNotSupported) return err(e);
    }
    float *Xm = nullptr, *Wm = nullptr;
    hipError_t e = outlier_prepare(A, k, B, n, m, n, k, threshold, scratch, &Xm, &Wm, s);
    if (e != hipSuccess) return err(e);
    // the int8 part on the outlier-free operands (their scales no longer see the outliers)
    const int rc = op_mm_quantize_ws(Xm, k, 1, Wm, n, 1, C, n, 1, m, n, k, kDefaultRange, ws2,
                                     op_mm_quantize_workspace_size(m, n, k), stream);
    if (rc) return rc;
    return err(outlier_finish(A, k, B, n, m, n, k, scratch, C, n, s));
}

int qgemm_outlier_count(int k, const void *workspace, int *count) {
    if (!workspace || !count || k < 1) return err(hipErrorInvalidValue);
    return outlier_count_slot(k, workspace, count);
}

int qgemm_set_gemm_events(void *start_event, void *stop_event) {
    set_gemm_events(static_cast<hipEvent_t>(start_event), static_cast<hipEvent_t>(stop_event));
    return 0;
}

int qgemm_set_event_mode(int mode) {
    if (mode != 0 && mode != 1) return err(hipErrorInvalidValue);
    set_gemm_event_mode(mode);
    return 0;
}

int qgemm_fill_uniform(float *dst, int64_t count, uint64_t seed, float lo, float hi, void *stream) {
    if (!dst || count < 0) return err(hipErrorInvalidValue);
    return err(launch_fill_uniform(dst, count, seed, lo, hi, static_cast<hipStream_t>(stream)));
}

int qgemm_gemm_plan(int m, int n, int k, int *tile, const char **kernel) {
    if (m < 1 || n < 1 || k < 1) return -(int)hipErrorInvalidValue;
    return gemm_plan_info(m, n, round_up(k, kKPad), tile, kernel);
}

#ifndef QGEMM_SRC_HASH
#define QGEMM_SRC_HASH "unknown"
#endif

// the same hash as a tagged literal in the file itself, so a build step can compare a binary with the tree
// without loading it (qgemm_amd.file_hash)
__attribute__((used)) static const char kSrcHashTag[] = "QGEMM_SRC_HASH=" QGEMM_SRC_HASH;

const char *qgemm_version(void) {
    static char buf[192];
    snprintf(buf, sizeof buf, "qgemm 0.1.0 gfx950 %s src=%s", gemm_config_name(), QGEMM_SRC_HASH);
    return buf;
}

}  // extern "C"
