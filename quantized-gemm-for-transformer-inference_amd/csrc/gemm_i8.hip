// gemm_i8.hip -- int8 x int8 -> int32 GEMM on CDNA4 matrix cores with the dequantize fused into the
// epilogue.  Replaces three reference launches (op_mm.cuh:92-99):
//   op_matmul_kernel<int8_t,int>   (op_mm.cuh:9-46; fp32 VALU emulation, 3 VALU/MAC, byte loads)
//   op_matmul_kernel<float,float>  (K = 1 outer product Cx*Cw, a full M x N fp32 write + read back)
//   op_dequantize + op_multiply    (two more M x N passes)
// by one kernel that reads the packed int8 operands once per macro-tile and writes fp32 O once.
//
// Operands (include/qgemm.h packed form): A = Xq [m_pad][k_pad], B = Wq^T [n_pad][k_pad], both
// k-contiguous and zero padded, so the kernel has no bounds checks except on the C store.
//
// Geometry: 256 x 256 macro-tile, k-step 128 (bytes), 512 threads = 8 waves as 2 (M) x 4 (N); each
// wave owns a 128 x 64 sub-tile = 4 x 2 accumulators of v_mfma_i32_32x32x32_i8 (16 i32 each).
// Staging: global_load_lds_dwordx4 (1 KiB per wave-instruction = 8 rows x 128 B) into a 2-deep LDS
// ring (2 x 64 KiB).  LDS rows are 128 B; 16-B chunk g of row r is stored at slot g ^ ((r>>1)&7)
// (swizzle applied on the per-lane SOURCE address, the LDS image stays lane-linear), which makes the
// ds_read_b128 fragment reads (32 consecutive rows, one chunk) bank-conflict free.
#include "qgemm_internal.h"

namespace qgemm {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int BM = 256, BN = 256, BK = 128;
constexpr int kThreads = 512;
constexpr int kTileBytes = BM * BK;             // 32 KiB per operand per stage
constexpr int kStageBytes = 2 * kTileBytes;     // A + B
constexpr int kLdsBytes = 2 * kStageBytes;      // 2-deep ring = 128 KiB

static_assert(BM == kRowPad && BN == kRowPad && BK == kKPad, "packed layout must match the macro-tile");

// Block -> macro-tile.  Blocks b and b+8 are dispatched to the same XCD; give each XCD a contiguous
// range of logical ids (bijective for any grid size), then walk logical ids in groups of kGroupM
// tile-rows so one XCD's range covers a compact patch (shared A and B panels stay in its L2).
__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int &tm, int &tn) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    constexpr int kGroupM = 4;
    const int per_group = kGroupM * tiles_n;
    const int group = wgid / per_group;
    const int first_m = group * kGroupM;
    const int gsz = min(tiles_m - first_m, kGroupM);
    const int w = wgid - group * per_group;
    tm = first_m + w % gsz;
    tn = w / gsz;
}

template <bool kDequant>
__global__ __launch_bounds__(kThreads, 2) void gemm_i8_kernel(const int8_t *__restrict__ A, const int8_t *__restrict__ B,
                                                              const float *__restrict__ Cx, const float *__restrict__ Cw,
                                                              void *__restrict__ Cout, int64_t csh, int64_t csw, int m,
                                                              int n, int64_t k_pad, int tiles_m, int tiles_n,
                                                              float inv_r2) {
    __shared__ __attribute__((aligned(16))) int8_t lds[kLdsBytes];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2;  // 0..1 : 128-row half
    const int wn = wave & 3;   // 0..3 : 64-column quarter

    int tm, tn;
    tile_coords(blockIdx.x, gridDim.x, tiles_m, tiles_n, tm, tn);
    const int8_t *Ablk = A + (int64_t)tm * BM * k_pad;
    const int8_t *Bblk = B + (int64_t)tn * BN * k_pad;

    // ---- staging addresses: wave w fills rows [32w, 32w+32) of the A and B tiles, 8 rows per glds.
    // Lane l of instruction i writes LDS bytes [16l, 16l+16) of that 1-KiB piece: row 32w+8i+(l>>3),
    // slot l&7, which must hold global chunk g = slot ^ ((row>>1)&7).
    int64_t src_off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wave * 32 + i * 8 + (lane >> 3);
        const int g = (lane & 7) ^ ((row >> 1) & 7);
        src_off[i] = (int64_t)row * k_pad + g * 16;
    }
    auto stage = [&](int kt, int buf) {
        int8_t *la = lds + buf * kStageBytes;
        int8_t *lb = la + kTileBytes;
        const int8_t *ga = Ablk + (int64_t)kt * BK;
        const int8_t *gb = Bblk + (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_global_load_lds((const void *)(ga + src_off[i]), (void *)(la + (wave * 32 + i * 8) * BK),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(gb + src_off[i]), (void *)(lb + (wave * 32 + i * 8) * BK),
                                             16, 0, 0);
        }
    };

    // ---- fragment addresses.  v_mfma_i32_32x32x32_i8: lane l holds A[row l&31][16 k's of half l>>5]
    // and B^T[col l&31][same k's]; A and B share the k map, so 16 contiguous bytes per lane suffice.
    const int lrow = lane & 31;
    const int khalf = lane >> 5;
    const int swz = (lrow >> 1) & 7;  // (row>>1)&7 for every fragment row (bases are multiples of 32)
    const int a_row0 = (wm * 128 + lrow) * BK;
    const int b_row0 = (wn * 64 + lrow) * BK;

    v16i acc[4][2];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = v16i{};

    auto compute = [&](int buf) {
        const int8_t *la = lds + buf * kStageBytes;
        const int8_t *lb = la + kTileBytes;
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            const int off = ((2 * s + khalf) ^ swz) << 4;
            v4i a[4], b[2];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[mi] = *reinterpret_cast<const v4i *>(la + a_row0 + mi * 32 * BK + off);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[ni] = *reinterpret_cast<const v4i *>(lb + b_row0 + ni * 32 * BK + off);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    };

    // ---- main loop: stage k-step kt+1 while computing kt (2-deep ring, one barrier per k-step)
    const int nk = (int)(k_pad / BK);
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
        compute(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue: C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    const int gi0 = tm * BM, gj0 = tn * BN;
    if constexpr (kDequant) {
        float *sCx = reinterpret_cast<float *>(lds);
        float *sCw = sCx + BM;
        if (tid < BM) sCx[tid] = Cx[gi0 + tid];
        else sCw[tid - BM] = Cw[gj0 + tid - BM];
        __syncthreads();
        float *C = static_cast<float *>(Cout);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int jl = wn * 64 + ni * 32 + lrow;
            const int j = gj0 + jl;
            const float cw = sCw[jl];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int il = wm * 128 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
                    const int i = gi0 + il;
                    const float o = dequantize(acc[mi][ni][r], outer_product(sCx[il], cw), inv_r2);
                    if (i < m && j < n) C[(int64_t)i * csh + (int64_t)j * csw] = o;
                }
            }
        }
    } else {
        int32_t *C = static_cast<int32_t *>(Cout);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int j = gj0 + wn * 64 + ni * 32 + lrow;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = gi0 + wm * 128 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
                    if (i < m && j < n) C[(int64_t)i * csh + (int64_t)j * csw] = acc[mi][ni][r];
                }
        }
    }
}

}  // namespace

const char *gemm_config_name() { return "i8mfma32x32x32_t256x256x128_w8_glds2"; }

static hipError_t launch_gemm(const PackedView &a, const PackedView &b, void *C, int64_t csh, int64_t csw, int m,
                              int n, float inv_r2, bool dequant, hipStream_t stream) {
    if (a.k_pad != b.k_pad) return hipErrorInvalidValue;
    const int tiles_m = (int)(a.rows_pad / BM), tiles_n = (int)(b.rows_pad / BN);
    const dim3 grid((unsigned)(tiles_m * tiles_n)), block(kThreads);
    if (dequant)
        gemm_i8_kernel<true><<<grid, block, 0, stream>>>(a.q, b.q, a.scale, b.scale, C, csh, csw, m, n, a.k_pad,
                                                         tiles_m, tiles_n, inv_r2);
    else
        gemm_i8_kernel<false><<<grid, block, 0, stream>>>(a.q, b.q, a.scale, b.scale, C, csh, csw, m, n, a.k_pad,
                                                          tiles_m, tiles_n, inv_r2);
    return hipGetLastError();
}

hipError_t launch_gemm_dequant(const PackedView &a, const PackedView &b, float *C, int64_t csh, int64_t csw, int m,
                               int n, float inv_r2, hipStream_t stream) {
    return launch_gemm(a, b, C, csh, csw, m, n, inv_r2, true, stream);
}

hipError_t launch_gemm_i32(const PackedView &a, const PackedView &b, int32_t *Acc, int m, int n, hipStream_t stream) {
    return launch_gemm(a, b, Acc, n, 1, m, n, 0.0f, false, stream);
}

}  // namespace qgemm
