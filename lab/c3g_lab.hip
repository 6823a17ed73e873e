// c3g_lab.hip -- LAB: why does the FFN-down GEMM (2048 x 16384 -> 4096, ticket-first split-K) take ~106 us back to
// back but ~120 us right after the two pack passes of the drop-in call?  The GEMM is timed by events after each of
// these predecessors (interleaved rounds, one process):
//   b2b      : the GEMM itself (operands clean in the Infinity Cache, translations warm)
//   pack     : the product's pass 1 + pass 2 (the drop-in call)
//   rewrite  : a kernel that reads and rewrites the packed operands in place (96 MiB left dirty, same bytes)
//   sweep    : a 512-MiB read of an unrelated buffer (operands evicted, nothing dirty)
//   sweep_rw : the sweep, then the rewrite
//   wother   : 96 MiB written to an unrelated buffer (other data dirty, operands untouched)
//   wsweep   : a 384-MiB read + 96-MiB write of unrelated buffers (the pack's byte counts, operands untouched)
//   sweep_rd : the sweep, then a read of the packed operands (back in the cache, clean)
//   spin     : ~100 us of VALU work on every CU, no memory
//   icread   : a 128-MiB buffer read 4 times (Infinity-Cache hits after the first)
//   sweep128 : a 128-MiB read of an unrelated buffer
//   sweep_idle: the 512-MiB sweep, then ~40 us of s_sleep on every CU
//   sw_rw_aN : the sweep, then the rewrite with buffer stores of cache-policy bits N (0 plain, 2 nt, 16 sc1,
//              17 sc0 sc1, 18 sc1 nt, 3 sc0 nt)
//   sw_rw_rd : the sweep, the rewrite, then a read of the operands
//   (rewrite_kernel's `v = p[i]; p[i] = v` compiles to nothing: "rewrite" and "sweep_rw" are no-ops after the sweep)
//   swpol_aN : the 512-MiB sweep with buffer loads of cache-policy bits N (does it evict the resident operands?)
//   build/c3g_lab [rounds]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void rewrite_kernel(uint4 *p, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        p[i] = v;
    }
}
__global__ __launch_bounds__(256) void read_kernel(const uint4 *p, int64_t n16, int *sink) {
    uint32_t x = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        x ^= v.x ^ v.w;
    }
    if (x == 0x12345679u) sink[0] = (int)x;
}
__global__ __launch_bounds__(256) void write_kernel(uint4 *p, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

template <int kAux>
__global__ __launch_bounds__(256) void read_pol_kernel(const uint4 *p, int64_t n16, int *sink) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4 *>(p), 0, 0xffffffffu, 0x00020000);
    int x = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v4i_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(i * 16), 0, kAux);
        x ^= v[0] ^ v[3];
    }
    if (x == 0x12345679) sink[0] = x;
}

template <int kAux>
__global__ __launch_bounds__(256) void rewrite_pol_kernel(uint4 *p, int64_t n16) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, (uint32_t)(n16 * 16), 0x00020000);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v4i_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(i * 16), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(i * 16), 0, kAux);
    }
}

__global__ __launch_bounds__(256) void spin_kernel(float *sink, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) {
        a = __builtin_fmaf(a, b, 1e-7f);
        b = __builtin_fmaf(b, 0.99999f, 1e-6f);
    }
    if (a == 12345.f) sink[0] = a;
}
__global__ __launch_bounds__(64) void sleep_kernel(int iters) {
    for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

int main(int argc, char **argv) {
    const int m = 2048, n = 4096, k = 16384;
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, reps = 10;
    float *X, *W, *C; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4)); CK(hipMalloc(&C, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    uint4 *big, *wbuf; int *sink;
    CK(hipMalloc(&big, (size_t)512 << 20)); CK(hipMalloc(&wbuf, (size_t)96 << 20)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(big, 3, (size_t)512 << 20));
    const int tiles_m = m / 256, tiles_n = n / 256, tiles = tiles_m * tiles_n;
    int32_t *slabs; unsigned *tickets;
    CK(hipMalloc(&slabs, (size_t)tiles * 256 * 256 * 4)); CK(hipMalloc(&tickets, 4096));
    CK(hipMemset(tickets, 0, 4096));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    const int col_blocks = (n + kColBlock - 1) / kColBlock, nrow = (int)vx.rows_pad;
    const float range = 127.f;
    const dim3 g2((unsigned)(vw.rows_pad / kTc), (unsigned)((vw.k_pad / kTk + kTilesPerBlock - 1) / kTilesPerBlock));
    auto pack = [&]() {
        colmax_kernel<true><<<dim3(col_blocks, (unsigned)vw.parts), 256, 0, s0>>>(W, n, k, n, vw.scratch, vw.rows_pad);
        pack_cols_then_rows_kernel<<<g2.x * g2.y + nrow, 256, 0, s0>>>(
            W, n, k, n, range, vw.scratch, vw.parts, vw.rows_pad, vw.scale, vw.q, vw.k_pad, (int)g2.x, (int)g2.y, X, k, m,
            vx.scale, vx.q, vx.rows_pad, reinterpret_cast<uint32_t *>(tickets), 1024);
    };
    auto gemm = [&]() {
        GemmArgs p{};
        p.A = vx.q; p.B = vw.q; p.Cx = vx.scale; p.Cw = vw.scale; p.C = C; p.csh = n; p.csw = 1; p.m = m; p.n = n;
        p.k_pad = vx.k_pad; p.tiles_m = tiles_m; p.inv_r2 = 1.0f / (range * range);
        p.tiles_n = tiles_n; p.splits = 2; p.slabs = slabs; p.tickets = tickets; p.reset_tickets = 1;
        gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 31><<<tiles * 2, 256, 0, s0>>>(p);
    };
    const int64_t nx16 = (int64_t)(vx.rows_pad * vx.k_pad / 16), nw16 = (int64_t)(vw.rows_pad * vw.k_pad / 16);
    auto rewrite = [&]() {
        rewrite_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<uint4 *>(vw.q), nw16);
        rewrite_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<uint4 *>(vx.q), nx16);
    };
    auto sweep = [&](int64_t bytes) { read_kernel<<<2048, 256, 0, s0>>>(big, bytes / 16, sink); };
    auto wother = [&]() { write_kernel<<<2048, 256, 0, s0>>>(wbuf, ((int64_t)96 << 20) / 16); };
    struct V { std::string name; int mode; };
    std::vector<V> vs = {{"b2b", 0}, {"pack", 1}, {"rewrite", 2}, {"sweep", 3}, {"sweep_rw", 4}, {"wother", 5},
                         {"wsweep", 6}, {"sweep_rd", 7}, {"spin", 8}, {"icread", 9}, {"sweep128", 10}, {"sweep_idle", 11},
                         {"sw_rw_a0", 20}, {"sw_rw_a2", 22}, {"sw_rw_a16", 36}, {"sw_rw_a17", 37}, {"sw_rw_a18", 38},
                         {"sw_rw_a3", 23}, {"sw_rw_rd", 12}, {"swpol_a0", 40}, {"swpol_a1", 41}, {"swpol_a2", 42},
                         {"swpol_a3", 43}, {"swpol_a16", 56}, {"swpol_a17", 57}, {"swpol_a18", 58}, {"swpol_a19", 59}};
    const int spin_iters = argc > 2 ? atoi(argv[2]) : 20000, sleep_iters = argc > 3 ? atoi(argv[3]) : 12;
    auto pre = [&](int mode) {
        if (mode == 1) pack();
        if (mode == 2) rewrite();
        if (mode == 3) sweep((int64_t)512 << 20);
        if (mode == 4) { sweep((int64_t)512 << 20); rewrite(); }
        if (mode == 5) wother();
        if (mode == 6) { sweep((int64_t)384 << 20); wother(); }
        if (mode == 7) {
            sweep((int64_t)512 << 20);
            read_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<const uint4 *>(vw.q), nw16, sink);
            read_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<const uint4 *>(vx.q), nx16, sink);
        }
        if (mode == 8) spin_kernel<<<256 * 8, 256, 0, s0>>>(reinterpret_cast<float *>(sink), spin_iters);
        if (mode == 9) for (int j = 0; j < 4; ++j) sweep((int64_t)128 << 20);
        if (mode == 10) sweep((int64_t)128 << 20);
        if (mode == 11) { sweep((int64_t)512 << 20); sleep_kernel<<<256, 64, 0, s0>>>(sleep_iters); }
        if (mode == 12) {
            sweep((int64_t)512 << 20); rewrite();
            read_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<const uint4 *>(vw.q), nw16, sink);
            read_kernel<<<2048, 256, 0, s0>>>(reinterpret_cast<const uint4 *>(vx.q), nx16, sink);
        }
        if (mode >= 40) {
            const int64_t c = ((int64_t)512 << 20) / 16;
            if (mode == 40) read_pol_kernel<0><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 41) read_pol_kernel<1><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 42) read_pol_kernel<2><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 43) read_pol_kernel<3><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 56) read_pol_kernel<16><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 57) read_pol_kernel<17><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 58) read_pol_kernel<18><<<2048, 256, 0, s0>>>(big, c, sink);
            if (mode == 59) read_pol_kernel<19><<<2048, 256, 0, s0>>>(big, c, sink);
        } else if (mode >= 20) {
            sweep((int64_t)512 << 20);
            for (int b = 0; b < 2; ++b) {
                uint4 *q = reinterpret_cast<uint4 *>(b ? vx.q : vw.q);
                const int64_t c = b ? nx16 : nw16;
                if (mode == 20) rewrite_pol_kernel<0><<<2048, 256, 0, s0>>>(q, c);
                if (mode == 22) rewrite_pol_kernel<2><<<2048, 256, 0, s0>>>(q, c);
                if (mode == 36) rewrite_pol_kernel<16><<<2048, 256, 0, s0>>>(q, c);
                if (mode == 37) rewrite_pol_kernel<17><<<2048, 256, 0, s0>>>(q, c);
                if (mode == 38) rewrite_pol_kernel<18><<<2048, 256, 0, s0>>>(q, c);
                if (mode == 23) rewrite_pol_kernel<3><<<2048, 256, 0, s0>>>(q, c);
            }
        }
    };
    pack(); gemm();
    CK(hipStreamSynchronize(s0)); CK(hipGetLastError());
    std::vector<float> ref((size_t)m * n), got(ref.size());
    CK(hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
    hipEvent_t e1, e2;
    CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    std::vector<std::vector<float>> tg(vs.size());
    for (int i = 0; i < 200; ++i) { pack(); gemm(); }  // clocks up
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            float ag = 0;
            for (int j = 0; j < reps + 2; ++j) {
                pre(vs[i].mode);
                CK(hipEventRecord(e1, s0)); gemm();
                CK(hipEventRecord(e2, s0)); CK(hipEventSynchronize(e2));
                float x; CK(hipEventElapsedTime(&x, e1, e2));
                if (j >= 2) ag += x;
            }
            tg[i].push_back(ag * 1000 / reps);
        }
    CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
    // durations of the predecessors themselves (calibration of spin / sleep lengths)
    for (int mode : {3, 8, 9, 11}) {
        pre(mode);
        CK(hipEventRecord(e1, s0)); pre(mode); CK(hipEventRecord(e2, s0)); CK(hipEventSynchronize(e2));
        float x; CK(hipEventElapsedTime(&x, e1, e2));
        printf("predecessor mode %d takes %.1f us\n", mode, x * 1000);
    }
    printf("output after the timed runs: %s\n", memcmp(ref.data(), got.data(), ref.size() * 4) ? "DIFF" : "same");
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = tg[i]; std::sort(v.begin(), v.end());
        printf("GEMM after %-9s median %7.2f us  min %7.2f  max %7.2f\n", vs[i].name.c_str(), v[v.size() / 2], v[0],
               v.back());
    }
    return 0;
}
