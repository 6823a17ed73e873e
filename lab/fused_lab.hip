// fused_lab.hip -- LAB (not part of the library): the dependency-respecting ONE-launch pack || GEMM of
// op_mm_quantize at 4096^3, against the library's serial call (pack launch, then
// GEMM launch), bit-compared and timed in interleaved rounds in one process.
//
// One launch, 512-thread blocks at one per CU (the GEMM role's 232 VGPRs), roles by blockIdx in
// dispatch order:
//   W strips (8 columns x all K rows, pack_w_strip8_body) -> X groups (8 rows, pack_rows_vec_body) ->
//   GEMM tiles (pp_tile_body<2>, the product's 256 x 256 ping-pong tile)
// Orders: 0 = [all W][all X][all tiles] (the serial call without its kernel boundary);
//         1 = [all W] then per X panel p: [its 32 X groups][its 16 tiles] (a tile is dispatched as soon as
//             a CU frees up after its panel's groups were dispatched, while later panels still pack).
// Hand-off (MI355X_MICROARCH.md inter-workgroup visibility): pack blocks store the packed bytes and scales
// write-through (sc1), every wave drains (vmcnt(0)), a block barrier, then lane 0 adds 1 to the W counter or
// to its panel's counter (relaxed, agent scope).  A tile's lane 0 polls its two counters with relaxed
// agent loads (s_sleep between polls, bounded: on timeout it raises an error word and goes on), then ONE
// agent acquire, vmcnt(0), block barrier, and the tile's LDS-DMA loads.  Pack blocks never wait, and every
// pack block is dispatched before the tiles that depend on it, so the waits end.
//   build/fused_lab [rounds]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>
#include <string>
#include <functional>

#define QGEMM_LAB 1
#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "gemm_legacy.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kPanels = 16;      // 4096 / 256
constexpr int kGroupsPerPanel = 32;  // 256 rows / 8
constexpr int kErrWord = 64;

struct Fused {
    GemmArgs g;
    const float *x, *w;
    int m, n, k;
    PackedView vx, vw;
    unsigned *sync;  // [0] W strips done, [1 + p] groups of X panel p done, [kErrWord] timeouts
    int order;
};

__device__ __forceinline__ void signal(unsigned *ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores have landed
    __syncthreads();                                   // ... and every other wave's
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(512, 2) void fused_kernel(Fused f) {
    __shared__ __attribute__((aligned(16))) int8_t lds[pp_lds_bytes<kEpiNone>()];
    const int b = blockIdx.x;
    const int nstrips = f.n / 8, ngroups = f.m / 8;
    // role of block b
    int role = 0, idx = 0;  // role 0 = W strip, 1 = X group, 2 = tile
    if (b < nstrips) {
        role = 0;
        idx = b;
    } else if (f.order == 0) {
        const int r = b - nstrips;
        if (r < ngroups) { role = 1; idx = r; }
        else { role = 2; idx = r - ngroups; }
    } else {
        const int r = b - nstrips, per = kGroupsPerPanel + 16, p = r / per, o = r % per;
        if (o < kGroupsPerPanel) { role = 1; idx = p * kGroupsPerPanel + o; }
        else { role = 2; idx = p * 16 + (o - kGroupsPerPanel); }  // panel p, tile column o - 32
    }
    if (role == 0) {
        // the product's XCD-contiguous strip map: blocks b, b+8, ... share an XCD
        const int xcd = idx & 7, q8 = nstrips >> 3, r8 = nstrips & 7;
        const int strip = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (idx >> 3);
        pack_w_strip8_body<false, true>(strip, f.w, f.n, f.k, 127.f, f.vw.scale, f.vw.q, f.vw.k_pad,
                                        reinterpret_cast<float *>(lds));
        signal(f.sync);
        return;
    }
    if (role == 1) {
        pack_rows_vec_body<16, false, true>((int64_t)idx * 2, f.x, f.k, f.m, f.k, 127.f, f.vx.scale, f.vx.q,
                                            f.vx.rows_pad, f.vx.k_pad);
        signal(f.sync + 1 + (idx * 8) / 256);
        return;
    }
    // tile: order 0 -> the product's tile order (XCD-aware); order 1 -> panel tm = idx / 16, column idx % 16
    int tile;
    int tm;
    if (f.order == 0) {
        tile = xcd_remap(idx, kPanels * 16);
        int tn;
        group_tiles(tile, f.g.tiles_m, f.g.tiles_n, tm, tn);
    } else {
        tm = idx / 16;
        const int tn = idx % 16;
        tile = (tm / 4) * 64 + tn * 4 + (tm % 4);  // group_tiles(tile) = (tm, tn)
    }
    if (threadIdx.x == 0) {
        long spins = 0;
        while (__hip_atomic_load(f.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nstrips ||
               __hip_atomic_load(f.sync + 1 + tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)kGroupsPerPanel) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > 20000000) {  // ~> 1 s: give up (error word), so the grid still drains
                __hip_atomic_fetch_add(f.sync + kErrWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    pp_tile_body<2, kEpiNone, kPPLayoutF>(f.g, lds, tile, 0, 1);
}

int main(int argc, char **argv) {
    const int m = 4096, n = 4096, k = 4096;
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, reps = 20;
    float *X, *W, *C, *Cref;
    void *PX, *PW;
    unsigned *sync;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(hipMalloc(&sync, 4096));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    GemmArgs g{vx.q, vw.q, vx.scale, vw.scale, C, n, 1, m, n, vx.k_pad, m / 256, n / 256, 1.0f / (127.0f * 127.0f),
               1, nullptr, nullptr, nullptr, 0};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto serial = [&] {
        CK(launch_pack_single_pass_kind(X, k, m, k, vx, W, n, n, vw, 127.f, s, 0));
        gemm_i8_pp<2, kEpiNone, kPPLayoutF><<<g.tiles_m * g.tiles_n, kThreads, 0, s>>>(g);
    };
    const int nblocks = n / 8 + m / 8 + (m / 256) * (n / 256);
    auto fused = [&](int order) {
        CK(hipMemsetAsync(sync, 0, 4096, s));
        Fused f{g, X, W, m, n, k, vx, vw, sync, order};
        fused_kernel<<<nblocks, 512, 0, s>>>(f);
    };
    // reference: the serial call
    serial();
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(Cref, C, (size_t)m * n * 4, hipMemcpyDeviceToDevice));
    std::vector<float> href((size_t)m * n), hgot((size_t)m * n);
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (int order = 0; order < 2; ++order)
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(C, 0xff, (size_t)m * n * 4, s));
            CK(hipMemsetAsync(PX, 0x5a, packed_bytes(m, k), s));
            CK(hipMemsetAsync(PW, 0x5a, packed_bytes(n, k), s));
            fused(order);
            CK(hipStreamSynchronize(s));
            unsigned err = 0;
            CK(hipMemcpy(&err, sync + kErrWord, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < href.size(); ++i) bad += memcmp(&href[i], &hgot[i], 4) != 0;
            printf("check fused order %d rep %d mismatches %zu timeouts %u\n", order, rep, bad, err);
        }
    struct V { const char *name; std::function<void()> f; };
    std::vector<V> vs = {{"serial", serial}, {"fused_order0", [&] { fused(0); }}, {"fused_order1", [&] { fused(1); }},
                         {"memset_only", [&] { CK(hipMemsetAsync(sync, 0, 4096, s)); }}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            for (int w = 0; w < 3; ++w) vs[i].f();
            CK(hipEventRecord(e0, s));
            for (int j = 0; j < reps; ++j) vs[i].f();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1000 / reps);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i];
        std::sort(v.begin(), v.end());
        printf("%-14s median %8.2f us  min %8.2f us\n", vs[i].name, v[v.size() / 2], v[0]);
    }
    unsigned err = 0;
    CK(hipMemcpy(&err, sync + kErrWord, 4, hipMemcpyDeviceToHost));
    printf("timeouts after timing: %u\n", err);
    return 0;
}
