// gemm_i8.hip -- launchers of the int8 MFMA GEMM (kernels in gemm_i8_kernels.h).
//
// Replaces three reference launches (op_mm.cuh:92-99):
//   op_matmul_kernel<int8_t,int>   (op_mm.cuh:9-46; fp32 VALU emulation, 3 VALU/MAC, byte loads)
//   op_matmul_kernel<float,float>  (K = 1 outer product Cx*Cw, a full M x N fp32 write + read back)
//   op_dequantize + op_multiply    (two more M x N passes)
// by one kernel that reads the packed int8 operands once per macro-tile and writes fp32 O once.
#include <hip/hip_ext.h>

#include "gemm_i8_kernels.h"

namespace qgemm {

using namespace gemm;

const char *gemm_config_name() { return "i8mfma16x16x64_t256x256_w4_wt128x128_fragmajor_direct_agpr"; }

static thread_local GemmEvents t_events;
static int g_event_mode = 0;  // 0: hipExtLaunchKernel events, 1: hipEventRecord around the launch
void set_gemm_event_mode(int mode) { g_event_mode = mode; }
void set_gemm_events(hipEvent_t start, hipEvent_t stop) { t_events = GemmEvents{start, stop}; }
GemmEvents take_gemm_events() {
    GemmEvents e = t_events;
    t_events = GemmEvents{};
    return e;
}

static bool shape_ok(const PackedView &a, const PackedView &b) {
    return a.k_pad == b.k_pad && a.rows_pad % BM == 0 && b.rows_pad % BN == 0 && a.k_pad % BK == 0;
}

// Launch plan.  256 x 256 tiles (gemm_i8_fm) while they give >= 128 blocks, with split-K below 160
// tiles when K is long: S = min(256 / tiles, k-steps / 8, 8) -- every slice keeps >= 8 k-steps
// (scripts/split_probe.py: the slab round trip costs ~3-5 us); 128 <= tiles < 160 makes S <= 2.  Fewer 256-tiles: 64 x 64 tiles
// (gemm_i8_small<64>, four blocks per CU) with S = min(512 / tiles, k-steps / 16, 4) slices -- splits
// only for K >= 4096.  Measured (gemm_lab small mode, us, 128-tiles vs 64-tiles at the chosen S):
// 512x3072x1024 11.8 -> 7.6, 512x1024x1024 11.1 -> 6.1, 512x4096x1024 12.2 -> 8.1,
// 512x1024x4096 16.8 (S4) -> 10.9 (S2), 256x4096x4096 20.2 (S2) -> 13.2 (S2), 2048^3 20.7 -> 18.5;
// split-K never helped at K = 1024.  Fewer than 256 64-tiles: 32-tiles where they fill the chip (below).
struct GemmPlan {
    int tile;       // 256, 64 or 32
    int tiles_m, tiles_n;
    int splits;
};

static GemmPlan gemm_plan(int m, int n, int k) {
    GemmPlan g{256, (int)(round_up(m, 256) / 256), (int)(round_up(n, 256) / 256), 1};
    if (m <= 0 || n <= 0 || k <= 0) return g;
    const int nk = (int)(round_up(k, BK) / BK);
    int64_t tiles = (int64_t)g.tiles_m * g.tiles_n;
    if (tiles >= 128) {
        if (tiles >= 160) return g;
        int sp = (int)(256 / tiles);
        sp = sp < nk / 8 ? sp : nk / 8;
        sp = sp < 8 ? sp : 8;
        g.splits = sp > 1 ? sp : 1;
        return g;
    }
    g = GemmPlan{64, (int)(round_up(m, 64) / 64), (int)(round_up(n, 64) / 64), 1};
    tiles = (int64_t)g.tiles_m * g.tiles_n;
    // fewer 64-tiles than CUs: 32 x 32 tiles (gemm_i8_small<32>, 4-stage ring, no split) where they give
    // >= 512 blocks, or >= 256 at K <= 2048 (gemm_lab ... small, us, best 64-tile plan -> 32-tiles:
    // 512x1024x1024 5.65 -> 4.79, 512x1024x4096 10.07 -> 8.67, 256x1024x1024 5.50 -> 4.08, 128x2048x2048
    // 7.58 -> 5.96, 256x2048x4096 10.05 -> 8.66, 512x1024x2048 7.73 -> 6.07; but 64x4096x4096 11.55 -> 15.21)
    if (tiles < 256) {
        const GemmPlan g32{32, (int)(round_up(m, 32) / 32), (int)(round_up(n, 32) / 32), 1};
        const int64_t tiles32 = (int64_t)g32.tiles_m * g32.tiles_n;
        if (tiles32 >= 512 || (tiles32 >= 256 && k <= 2048)) return g32;
    }
    int sp = tiles >= 512 ? 1 : (int)(512 / tiles);
    sp = sp < nk / 16 ? sp : nk / 16;
    sp = sp < 4 ? sp : 4;
    g.splits = sp > 1 ? sp : 1;
    return g;
}

int gemm_splits(int m, int n, int k) { return gemm_plan(m, n, k).splits; }

int gemm_plan_info(int m, int n, int k, int *tile, const char **kernel) {
    const GemmPlan g = gemm_plan(m, n, k);
    if (tile) *tile = g.tile;
    if (kernel) {
        if (g.tile == 32) *kernel = "gemm_i8_small<32> (32x32 tiles, 4 waves of 16x16, 4-stage LDS-DMA ring)";
        else if (g.tile == 64)
            *kernel = g.splits > 1 ? "gemm_i8_small<64> (64x64 tiles, LDS-DMA ring, split-K)"
                                   : "gemm_i8_small<64> (64x64 tiles, LDS-DMA ring)";
        else
            *kernel = g.splits > 1 ? "gemm_i8_fm<split-K> (256x256 tiles, 4 waves of 128x128, fragment-major operands "
                                     "straight to VGPRs, AGPR accumulators, ticket-first split-K: one int32 slab per tile)"
                                   : "gemm_i8_fm (256x256 tiles, 4 waves of 128x128, fragment-major operands straight to "
                                     "VGPRs, AGPR accumulators, fused dequant epilogue)";
    }
    return g.splits;
}

// One fixed ticket region at the start of every split-K scratch (splits happen only below 320 tiles):
// shapes that share a library-owned scratch then never write slabs over each other's tickets.
constexpr size_t kTicketBytes = 4096;
static size_t ticket_bytes(int64_t tiles) {
    (void)tiles;
    return kTicketBytes;
}

size_t gemm_ticket_bytes(int m, int n, int k) { return gemm_plan(m, n, k).splits > 1 ? kTicketBytes : 0; }

size_t gemm_scratch_bytes(int m, int n, int k) {
    const GemmPlan g = gemm_plan(m, n, k);
    if (g.splits <= 1) return 0;
    const int64_t tiles = (int64_t)g.tiles_m * g.tiles_n;
    // the 256-tile split (gemm_i8_fm, ticket-first) keeps ONE slab per tile; the small tiles one per slice
    const int slabs = g.tile == 256 ? 1 : g.splits;
    return ticket_bytes(tiles) + (size_t)tiles * slabs * g.tile * g.tile * 4;
}

// zeroes the ticket region ahead of a split launch.  A kernel rather than hipMemsetAsync: inside a
// captured HIP graph the memset node left the tickets unzeroed on replay (every slice then saw a
// nonzero ticket and no tile was written) -- a kernel node replays as launched.
__global__ __launch_bounds__(256) void zero_tickets_kernel(unsigned *__restrict__ t, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) t[i] = 0u;
}

// 256 x 256 tiles: gemm_i8_fm (4 waves of 128 x 128, operands straight from the fragment-major packed
// layout, no LDS in the main loop) for every plan -- unsplit, 2-way split-K and the LLM.int8() outlier
// epilogue.  (The ping-pong kernel gemm_i8_pp of round 2 is in lab/gemm_legacy.h: the 256-tile plan splits
// in two or not at all, so no shape reached it without an environment switch)
template <typename Launch>
static hipError_t launch_timed(dim3 grid, dim3 block, hipStream_t stream, const GemmArgs &p, Launch kernel) {
    const GemmEvents ev = take_gemm_events();
    if ((ev.start || ev.stop) && g_event_mode == 0) {
        hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, ev.start, ev.stop, 0, p);
        return hipGetLastError();
    }
    if (ev.start) (void)hipEventRecord(ev.start, stream);
    kernel<<<grid, block, 0, stream>>>(p);
    hipError_t e = hipGetLastError();
    if (ev.stop) (void)hipEventRecord(ev.stop, stream);
    return e;
}

template <int kEpi>
static hipError_t launch_v3(const GemmArgs &p, dim3 grid, hipStream_t stream) {
    if constexpr (kEpi != kEpiOutlier) {
        // ticket-first split-K, slice 0 = 31/64 of the k-steps (lab/t2_lab.hip, lab/c3d_lab.hip; profiles/
        // r04_splitfirst_*.log: FFN-down GEMM alone 110.5 -> 105.8 us, the whole drop-in call 284.7 -> 279.7 us)
        if (p.splits == 2)
            return launch_timed(grid, dim3(kFmThreads), stream, p, gemm_i8_fm<kEpi, false, kSplitFirst, true, 31>);
        if (p.splits > 2) return hipErrorNotSupported;  // gemm_plan never makes one (tiles in [128, 160) -> S <= 2)
    }
    return launch_timed(grid, dim3(kFmThreads), stream, p, gemm_i8_fm<kEpi>);
}

template <int TB, int kEpi, int kDepth>
static hipError_t launch_small(const GemmArgs &p, dim3 grid, hipStream_t stream) {
    const GemmEvents ev = take_gemm_events();
    if ((ev.start || ev.stop) && g_event_mode == 0) {
        hipExtLaunchKernelGGL((gemm_i8_small<TB, kEpi, kDepth>), grid, dim3(SmallTile<TB, kDepth>::kThreads), 0, stream,
                              ev.start, ev.stop, 0, p);
        return hipGetLastError();
    }
    if (ev.start) (void)hipEventRecord(ev.start, stream);
    gemm_i8_small<TB, kEpi, kDepth><<<grid, dim3(SmallTile<TB, kDepth>::kThreads), 0, stream>>>(p);
    hipError_t e = hipGetLastError();
    if (ev.stop) (void)hipEventRecord(ev.stop, stream);
    return e;
}

hipError_t launch_gemm_dequant(const PackedView &a, const PackedView &b, float *C, int64_t csh, int64_t csw, int m,
                               int n, float inv_r2, void *scratch, size_t scratch_bytes, hipStream_t stream,
                               const float *bias, bool relu, bool tickets_zeroed) {
    if (!shape_ok(a, b)) return hipErrorInvalidValue;
    const GemmPlan g = gemm_plan(m, n, (int)a.k_pad);
    GemmArgs p{a.q, b.q, a.scale, b.scale, C, csh, csw, m, n, a.k_pad, g.tiles_m, g.tiles_n,
               inv_r2, 1, nullptr, nullptr, bias, tickets_zeroed ? 1 : 0};
    const int64_t tiles = (int64_t)g.tiles_m * g.tiles_n;
    // output rows of >= 64 KiB (FFN up's 16 384 columns): gemm_i8_fm's LDS-image stores (512-B nontemporal row
    // segments, rotated per tile); its paired nontemporal register stores ran 122.6 vs 112.3 us there
    // (lab/ds_lab.hip) and plain ones left the output in the caches
    p.wide_rows = (csw == 1 && csh >= 16384) ? 1 : 0;
    if (g.splits > 1 && scratch && scratch_bytes >= gemm_scratch_bytes(m, n, (int)a.k_pad)) {
        p.splits = g.splits;
        p.tickets = static_cast<unsigned *>(scratch);
        p.slabs = reinterpret_cast<int32_t *>(static_cast<char *>(scratch) + ticket_bytes(tiles));
        // the tickets are polled state: zeroed ahead of every launch unless the scratch is
        // library-owned, zeroed at allocation and re-zeroed by each launch's reducers
        if (!tickets_zeroed) {
            const int nt = (int)(ticket_bytes(tiles) / sizeof(unsigned));
            zero_tickets_kernel<<<(nt + 255) / 256, 256, 0, stream>>>(p.tickets, nt);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    const dim3 grid((unsigned)(tiles * p.splits));
    if (g.tile == 32) {
        if (!bias) return launch_small<32, kEpiNone, 4>(p, grid, stream);
        return relu ? launch_small<32, kEpiBiasRelu, 4>(p, grid, stream) : launch_small<32, kEpiBias, 4>(p, grid, stream);
    }
    if (g.tile == 64) {
        // at most two 64-tiles per CU: a 3-stage ring (two k-steps in flight, three blocks per CU); more
        // tiles: the 2-stage ring, four blocks per CU (gemm_lab ... small, us: 512x1024x1024 6.10 -> 5.67,
        // 512x1024x4096 S2 10.73 -> 9.91, 512x3072x1024 7.43 -> 7.20; 2048^3 18.1 -> 22.3 with 3 stages)
        if (tiles <= 512) {
            if (!bias) return launch_small<64, kEpiNone, 3>(p, grid, stream);
            return relu ? launch_small<64, kEpiBiasRelu, 3>(p, grid, stream) : launch_small<64, kEpiBias, 3>(p, grid, stream);
        }
        if (!bias) return launch_small<64, kEpiNone, 2>(p, grid, stream);
        return relu ? launch_small<64, kEpiBiasRelu, 2>(p, grid, stream) : launch_small<64, kEpiBias, 2>(p, grid, stream);
    }
    if (!bias) return launch_v3<kEpiNone>(p, grid, stream);
    return relu ? launch_v3<kEpiBiasRelu>(p, grid, stream) : launch_v3<kEpiBias>(p, grid, stream);
}

bool gemm_outlier_ok(int m, int n, int k) {
    const GemmPlan g = gemm_plan(m, n, k);
    return g.tile == 256 && g.splits == 1;
}

hipError_t launch_gemm_dequant_outlier(const PackedView &a, const PackedView &b, float *C, int64_t csh, int m, int n,
                                       float inv_r2, const float *x, int64_t xsh, const float *w, int64_t wsh,
                                       const int *ocols, const int *ocount, hipStream_t stream) {
    if (!shape_ok(a, b) || !gemm_outlier_ok(m, n, (int)a.k_pad)) return hipErrorNotSupported;
    const GemmPlan g = gemm_plan(m, n, (int)a.k_pad);
    GemmArgs p{a.q, b.q, a.scale, b.scale, C, csh, 1, m, n, a.k_pad, g.tiles_m, g.tiles_n,
               inv_r2, 1, nullptr, nullptr, nullptr, 0, x, w, ocount, wsh};
    p.wide_rows = csh >= 16384 ? 1 : 0;
    p.xo_ld = xsh;
    p.ocols = ocols;
    return launch_v3<kEpiOutlier>(p, dim3((unsigned)(g.tiles_m * g.tiles_n)), stream);
}

hipError_t launch_gemm_i32(const PackedView &a, const PackedView &b, int32_t *Acc, int m, int n, hipStream_t stream) {
    if (!shape_ok(a, b)) return hipErrorInvalidValue;
    GemmArgs p{a.q, b.q, a.scale, b.scale, Acc, n, 1, m, n, a.k_pad, (int)(a.rows_pad / BM), (int)(b.rows_pad / BN),
               0.0f, 1, nullptr, nullptr, nullptr, 0};
    gemm_i8_fm<kEpiNone, true><<<dim3(p.tiles_m * p.tiles_n), dim3(kFmThreads), 0, stream>>>(p);
    return hipGetLastError();
}

}  // namespace qgemm
