// gemm_f32.hip -- the reference's UNQUANTIZED path, op_mm<float,float> (op_mm.cuh:49-65 ->
// op_matmul_kernel<float,float> :9-46), used by the harnesses for the error metric and the
// "unquantized GEMM" timing line (timing_quantize.cu:27-35).
//
// Bit-exact with the reference: every output is res = +0 then res = fmaf(a_k, b_k, res) for k
// ascending (nvcc contracts :38), followed by the zero-padded products of the last 32-wide tile,
// which only turn a -0 result into +0 (one fl(res + 0)).  Arbitrary strides (the Index() macro).
// On the f32 MFMA (v_mfma_f32_16x16x4_f32), which computes exactly that chain (see the kernel).
#include "qgemm_internal.h"

namespace qgemm {

namespace {


// FM x FN 16x16 output tiles per wave, WGM x WGN waves per block; k staged TK at a time through LDS.
// Every output is ONE v_mfma_f32_16x16x4_f32 accumulation chain over k ascending: the f32 MFMA is
// bit-for-bit the k-ordered fmaf chain D = fma(a_k3, b_k3, fma(.., fma(a_k0, b_k0, C))) with one
// rounding per product and no wider accumulation (cdna_hip_programming.md s3 'FP32-input MFMA'),
// so the chain from C = +0 is the reference's res = fmaf(a_k, b_k, res).  k past the end is staged
// as zeros: fma(0, 0, res) only turns -0 into +0, which the reference's zero-padded last 32-wide
// tile does too (k % 32 != 0 implies it; the k % 32 != 0, k % 4 == 0 case adds the +0 below).
//
// LDS holds each operand in one of two layouts, chosen per call by the operand's contiguous
// dimension so that the coalesced global loads also deposit conflict-free:
//   k-contiguous   [row][k]  stride TK + 2     (row-major A, transposed B view)
//   row-contiguous [k][row]  stride ROWS + 16  (transposed A view, row-major B)
// An MFMA operand read (lanes 0-15: rows 0-15 at k, lanes 16-31 at k+1, ...) is conflict-free in both.
template <int FM, int FN, int WGM, int WGN, int TK>
__global__ __launch_bounds__(64 * WGM * WGN) void mm_f32_mfma_kernel(
    const float *__restrict__ A, int64_t ash, int64_t asw, const float *__restrict__ B, int64_t bsh, int64_t bsw,
    float *__restrict__ C, int64_t csh, int64_t csw, int m, int n, int k, int64_t a_bs, int64_t b_bs, int64_t c_bs) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = WGM * FM * 16, TN = WGN * FN * 16;
    constexpr int KC = TK + 2;  // k-contiguous row stride (floats)
    constexpr int A_LDS = (TM * KC > TK * (TM + 16)) ? TM * KC : TK * (TM + 16);
    constexpr int B_LDS = (TN * KC > TK * (TN + 16)) ? TN * KC : TK * (TN + 16);
    constexpr int NA = TM * TK / NT, NB = TN * TK / NT;  // staged elements per thread
    static_assert(TM * TK % NT == 0 && TN * TK % NT == 0 && TK % 4 == 0, "staging shape");
    using v4f = __attribute__((__vector_size__(4 * sizeof(float)))) float;
    __shared__ float As[A_LDS];
    __shared__ float Bs[B_LDS];
    A += blockIdx.z * a_bs;
    B += blockIdx.z * b_bs;
    C += blockIdx.z * c_bs;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave / WGN, wn = wave % WGN;
    const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
    const int a_rows = m - i0, b_rows = n - j0;  // rows of this block's tiles inside the matrices
    const bool a_kc = asw == 1 || ash != 1;  // A[i][k]: k contiguous (or neither: any mapping)
    const bool b_kc = bsh == 1 && bsw != 1;  // B[k][j]: k contiguous (the B^T view of row-major K)
    // LDS strides (in floats) of the two layouts: element (row, kk) at row * rs + kk * ks
    const int a_rs = a_kc ? KC : 1, a_ks = a_kc ? 1 : TM + 16;
    const int b_rs = b_kc ? KC : 1, b_ks = b_kc ? 1 : TN + 16;
    // Thread t stages elements x = 0..NA-1 of the A tile at (row, kk) = (r0 + x * dr, k0 + x * dk):
    // NT is a multiple of TK and of TM, so one coordinate is fixed per thread and the other steps.
    static_assert(NT % TK == 0 && NT % TM == 0 && NT % TN == 0, "per-thread staging stride");
    const int ar0 = a_kc ? t / TK : t % TM, ak0 = a_kc ? t % TK : t / TM;
    const int adr = a_kc ? NT / TK : 0, adk = a_kc ? 0 : NT / TM;
    const int br0 = b_kc ? t / TK : t % TN, bk0 = b_kc ? t % TK : t / TN;
    const int bdr = b_kc ? NT / TK : 0, bdk = b_kc ? 0 : NT / TN;
    // Branch-free staging: one buffer descriptor per operand and k tile (base = the block's first row at
    // the tile's first k), fixed 32-bit lane offsets; an element outside the matrix gets an offset past
    // num_records, which the buffer unit returns as 0 without touching memory (the zero padding).
    const uint32_t a_off0 = (uint32_t)((ar0 * ash + (int64_t)ak0 * asw) * 4), a_xs = (uint32_t)((adr * ash + (int64_t)adk * asw) * 4);
    const uint32_t b_off0 = (uint32_t)((br0 * bsw + (int64_t)bk0 * bsh) * 4), b_xs = (uint32_t)((bdr * bsw + (int64_t)bdk * bsh) * 4);
    const char *a_tile = reinterpret_cast<const char *>(A + (int64_t)i0 * ash);
    const char *b_tile = reinterpret_cast<const char *>(B + (int64_t)j0 * bsw);
    const int64_t a_kstep = (int64_t)TK * asw * 4, b_kstep = (int64_t)TK * bsh * 4;
    constexpr uint32_t kOut = 0x80000000u;  // > num_records
    float ra[NA], rb[NB];
    auto fetch = [&](int k0) __attribute__((always_inline)) {
        const auto ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(a_tile), 0, 0x7fffffff, 0x00020000);
        const auto br = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(b_tile), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int x = 0; x < NA; ++x) {
            const bool ok = (ar0 + x * adr < a_rows) & (ak0 + x * adk < k - k0);  // & : no branch
            ra[x] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ar, ok ? a_off0 + x * a_xs : kOut, 0, 0));
        }
#pragma unroll
        for (int x = 0; x < NB; ++x) {
            const bool ok = (br0 + x * bdr < b_rows) & (bk0 + x * bdk < k - k0);
            rb[x] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, ok ? b_off0 + x * b_xs : kOut, 0, 0));
        }
        a_tile += a_kstep;
        b_tile += b_kstep;
    };
    auto deposit = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < NA; ++x) As[(ar0 + x * adr) * a_rs + (ak0 + x * adk) * a_ks] = ra[x];
#pragma unroll
        for (int x = 0; x < NB; ++x) Bs[(br0 + x * bdr) * b_rs + (bk0 + x * bdk) * b_ks] = rb[x];
    };
    v4f acc[FM][FN];
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
    // this lane's operand element: row (lane & 15) of each 16-row fragment, k offset lane >> 4
    const int a_base = (wm * FM * 16 + (lane & 15)) * a_rs + (lane >> 4) * a_ks;
    const int b_base = (wn * FN * 16 + (lane & 15)) * b_rs + (lane >> 4) * b_ks;
    fetch(0);
    for (int k0 = 0; k0 < k; k0 += TK) {
        deposit();
        __syncthreads();
        if (k0 + TK < k) fetch(k0 + TK);  // next tile's loads in flight during this tile's MFMAs
#pragma unroll
        for (int s = 0; s < TK / 4; ++s) {
            float av[FM], bv[FN];
#pragma unroll
            for (int a = 0; a < FM; ++a) av[a] = As[a_base + a * 16 * a_rs + 4 * s * a_ks];
#pragma unroll
            for (int b = 0; b < FN; ++b) bv[b] = Bs[b_base + b * 16 * b_rs + 4 * s * b_ks];
#pragma unroll
            for (int a = 0; a < FM; ++a)
#pragma unroll
                for (int b = 0; b < FN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    const bool padded = (k % 32) != 0;  // reference: trailing fma(0, 0, res) products of the last tile
    // D layout: lane holds rows 4 * (lane >> 4) + r, column lane & 15 of each 16 x 16 tile; stores
    // outside C get an offset past num_records and are dropped
    const auto cr = __builtin_amdgcn_make_buffer_rsrc(C + (int64_t)i0 * csh + (int64_t)j0 * csw, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int li = wm * FM * 16 + a * 16 + 4 * (lane >> 4) + r, lj = wn * FN * 16 + b * 16 + (lane & 15);
                const float v = padded ? __fadd_rn(acc[a][b][r], 0.0f) : acc[a][b][r];
                const uint32_t off = ((li < a_rows) & (lj < b_rows)) ? (uint32_t)((li * csh + lj * csw) * 4) : kOut;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), cr, off, 0, 0);
            }
}


// ---------------------------------------------------------------------------------------------
// Fast path for 16-B aligned operands (k % 4 == 0; A k-contiguous; B k-contiguous or n-contiguous
// with n % 4 == 0): the tiles stream into an NS-deep LDS ring by buffer_load_dwordx4 ... lds (no
// staging registers, NS - 1 k tiles in flight -- the attention GEMMs are load-latency-bound with
// register staging), 16-B chunks XOR-swizzled on the source side:
//   k-contiguous operand, [row][TK] : chunk c of row r at slot c ^ (r & 7)
//   n-contiguous B,       [TK][TN]  : chunk c of k-row kk at slot c ^ 4 (kk & 1)   (TN >= 32)
// Elements outside the matrix get an offset past num_records: the buffer unit writes zeros.
// s_waitcnt immediate waiting for vmcnt <= v only (gfx9 encoding: vmcnt[3:0], expcnt, lgkmcnt, vmcnt[5:4])
constexpr int vmcnt_imm(int v) { return (v & 15) | (7 << 4) | (15 << 8) | ((v >> 4) << 14); }

template <int FM, int FN, int WGM, int WGN, int TK, int NS, bool BKC>
__global__ __launch_bounds__(64 * WGM * WGN) void mm_f32_dma_kernel(
    const float *__restrict__ A, int64_t a_ld, const float *__restrict__ B, int64_t b_ld, float *__restrict__ C,
    int64_t csh, int64_t csw, int m, int n, int k, int64_t a_bs, int64_t b_bs, int64_t c_bs) {
    constexpr int NW = WGM * WGN, TM = WGM * FM * 16, TN = WGN * FN * 16;
    constexpr int A_BYTES = TM * TK * 4, B_BYTES = TN * TK * 4, STAGE = A_BYTES + B_BYTES;
    constexpr int A_INSTR = A_BYTES / 1024, B_INSTR = B_BYTES / 1024;  // 1 KiB per wave instruction
    static_assert(A_BYTES % 1024 == 0 && B_BYTES % 1024 == 0, "whole DMA instructions");
    static_assert(A_INSTR % NW == 0 && B_INSTR % NW == 0, "DMA instructions split evenly over the waves");
    constexpr int IPW = (A_INSTR + B_INSTR) / NW;  // DMA instructions per wave per stage
    constexpr int KCH = TK / 4;                    // 16-B chunks per k-contiguous row
    constexpr bool SWN = TN >= 32;                 // n-contiguous B: swizzle k-row pairs
    static_assert(KCH >= 8 && NS >= 3 && (NS - 2) * IPW <= 63, "swizzle span / ring depth / vmcnt range");
    using v4f = __attribute__((__vector_size__(4 * sizeof(float)))) float;
    __shared__ __attribute__((aligned(1024))) char lds[NS * STAGE];
    A += blockIdx.z * a_bs;
    B += blockIdx.z * b_bs;
    C += blockIdx.z * c_bs;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WGN, wn = wave % WGN;
    const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
    constexpr uint32_t kOut = 0x80000000u;
    // per-lane DMA sources: instruction q of this wave covers LDS bytes [q' * 1 KiB, +1 KiB) of the
    // operand image, q' = wave + q * NW; lane -> (row, chunk) by the inverse swizzle
    uint32_t a_src[A_INSTR / NW], b_src[B_INSTR / NW];
    int a_kc[A_INSTR / NW], b_kc[B_INSTR / NW];  // the lane's k offset within the tile (validity)
#pragma unroll
    for (int q = 0; q < A_INSTR / NW; ++q) {
        const int p = (wave + q * NW) * 1024 + lane * 16, r = p / (TK * 4), c = ((p % (TK * 4)) / 16) ^ (r & 7);
        a_kc[q] = 4 * c;
        a_src[q] = i0 + r < m ? (uint32_t)((r * a_ld + 4 * c) * 4) : kOut;
    }
#pragma unroll
    for (int q = 0; q < B_INSTR / NW; ++q) {
        const int p = (wave + q * NW) * 1024 + lane * 16;
        if (BKC) {
            const int r = p / (TK * 4), c = ((p % (TK * 4)) / 16) ^ (r & 7);
            b_kc[q] = 4 * c;
            b_src[q] = j0 + r < n ? (uint32_t)((r * b_ld + 4 * c) * 4) : kOut;
        } else {
            const int kk = p / (TN * 4), c = ((p % (TN * 4)) / 16) ^ (SWN ? 4 * (kk & 1) : 0);
            b_kc[q] = kk;
            b_src[q] = j0 + 4 * c < n ? (uint32_t)((kk * b_ld + 4 * c) * 4) : kOut;
        }
    }
    const char *a_tile = reinterpret_cast<const char *>(A + (int64_t)i0 * a_ld);
    const char *b_tile = reinterpret_cast<const char *>(BKC ? B + (int64_t)j0 * b_ld : B + j0);
    const int64_t a_kstep = (int64_t)TK * 4, b_kstep = BKC ? (int64_t)TK * 4 : (int64_t)TK * b_ld * 4;
    const int nk = (k + TK - 1) / TK;
    // (the voffset argument is cast to int explicitly: an implicit uint32_t -> int conversion there made
    // hipcc's host pass drop the kernel's launch stub without a diagnostic -- an undefined symbol at link)
#define QG_ISSUE(KT)                                                                                                   \
    do {                                                                                                               \
        const int k0_ = (KT) * TK;                                                                                     \
        char *st_ = lds + ((KT) % NS) * STAGE;                                                                         \
        const auto ar_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(a_tile + (KT) * a_kstep), 0, 0x7fffffff, \
                                                           0x00020000);                                                \
        const auto br_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(b_tile + (KT) * b_kstep), 0, 0x7fffffff, \
                                                           0x00020000);                                                \
        _Pragma("unroll") for (int q = 0; q < A_INSTR / NW; ++q) __builtin_amdgcn_raw_ptr_buffer_load_lds(             \
            ar_, (__attribute__((address_space(3))) void *)(st_ + (wave + q * NW) * 1024), 16,                         \
            (int)(a_kc[q] < k - k0_ ? a_src[q] : kOut), 0, 0, 0);                                                             \
        _Pragma("unroll") for (int q = 0; q < B_INSTR / NW; ++q) __builtin_amdgcn_raw_ptr_buffer_load_lds(             \
            br_, (__attribute__((address_space(3))) void *)(st_ + A_BYTES + (wave + q * NW) * 1024), 16,               \
            (int)(b_kc[q] < k - k0_ ? b_src[q] : kOut), 0, 0, 0);                                                             \
    } while (0)
    v4f acc[FM][FN];
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
    // MFMA operand reads: lane (row l & 15, k offset l >> 4) of each 16-row fragment
    const int sw = (lane & 7) * 16, koff = lane >> 4;
    const int a_rd = (wm * FM * 16 + (lane & 15)) * TK * 4 + koff * 4;
    int b_rd[FN];
#pragma unroll
    for (int b = 0; b < FN; ++b) {
        if (BKC) {
            b_rd[b] = (wn * FN * 16 + b * 16 + (lane & 15)) * TK * 4 + koff * 4;
        } else {
            const int c = (wn * FN * 16 + b * 16 + (lane & 15)) >> 2;  // chunk of the lane's column
            b_rd[b] = koff * TN * 4 + ((c ^ (SWN ? 4 * (koff & 1) : 0)) * 16) + (lane & 3) * 4;
        }
    }
    // Fragments are register double-buffered across k tiles: tile kt + 1's LDS reads are issued
    // before tile kt's MFMAs, so one LDS round trip per tile hides behind a tile of MFMAs.
    float av[2][KCH][FM], bv[2][KCH][FN];
#define QG_READ(KT, BUF)                                                                                             \
    do {                                                                                                             \
        const char *st_ = lds + ((KT) % NS) * STAGE;                                                                 \
        _Pragma("unroll") for (int s = 0; s < KCH; ++s) {                                                            \
            _Pragma("unroll") for (int a = 0; a < FM; ++a) av[BUF][s][a] =                                           \
                *reinterpret_cast<const float *>(st_ + a_rd + a * 16 * TK * 4 + ((s * 16) ^ sw));                    \
            _Pragma("unroll") for (int b = 0; b < FN; ++b) bv[BUF][s][b] =                                           \
                BKC ? *reinterpret_cast<const float *>(st_ + A_BYTES + b_rd[b] + ((s * 16) ^ sw))                    \
                    : *reinterpret_cast<const float *>(st_ + A_BYTES + b_rd[b] + s * 4 * TN * 4);                    \
        }                                                                                                            \
    } while (0)
    // wait until tile KT's DMA landed with up to LEFT younger tiles still in flight, in every wave: this
    // wave's counted vmcnt, then a RAW barrier (__syncthreads()' fence would wait vmcnt(0) while LDS-DMA
    // is in flight, i.e. drain the whole ring every k tile)
#define QG_LANDED(LEFT)                                                                                              \
    do {                                                                                                             \
        __builtin_amdgcn_s_waitcnt(vmcnt_imm((LEFT) * IPW));                                                         \
        if (NW > 1) {                                                                                                \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
            __builtin_amdgcn_s_barrier();                                                                            \
            asm volatile("" ::: "memory");                                                                           \
        } else {                                                                                                     \
            __builtin_amdgcn_sched_barrier(0);                                                                       \
        }                                                                                                            \
    } while (0)
#define QG_STEP(KT, CUR, NXT)                                                                                        \
    do {                                                                                                             \
        if ((KT) + 1 < nk) {                                                                                         \
            if ((KT) + NS - 2 < nk) QG_LANDED(NS - 3);                                                               \
            else QG_LANDED(0);                                                                                       \
            if ((KT) + NS - 1 < nk) QG_ISSUE((KT) + NS - 1);                                                         \
            QG_READ((KT) + 1, NXT);                                                                                  \
        }                                                                                                            \
        _Pragma("unroll") for (int s = 0; s < KCH; ++s)                                                              \
            _Pragma("unroll") for (int a = 0; a < FM; ++a)                                                           \
                _Pragma("unroll") for (int b = 0; b < FN; ++b) acc[a][b] =                                           \
                    __builtin_amdgcn_mfma_f32_16x16x4f32(av[CUR][s][a], bv[CUR][s][b], acc[a][b], 0, 0, 0);          \
    } while (0)
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
        if (p < nk) QG_ISSUE(p);
    if (NS - 2 < nk) QG_LANDED(NS - 2);
    else QG_LANDED(0);
    QG_READ(0, 0);
    for (int kt = 0; kt < nk; kt += 2) {
        QG_STEP(kt, 0, 1);
        if (kt + 1 < nk) QG_STEP(kt + 1, 1, 0);
    }
#undef QG_READ
#undef QG_LANDED
#undef QG_STEP
#undef QG_ISSUE
    const bool padded = (k % 32) != 0;
    const int a_rows = m - i0, b_rows = n - j0;
    const auto cr = __builtin_amdgcn_make_buffer_rsrc(C + (int64_t)i0 * csh + (int64_t)j0 * csw, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int li = wm * FM * 16 + a * 16 + 4 * (lane >> 4) + r, lj = wn * FN * 16 + b * 16 + (lane & 15);
                const float v = padded ? __fadd_rn(acc[a][b][r], 0.0f) : acc[a][b][r];
                const uint32_t off = ((li < a_rows) & (lj < b_rows)) ? (uint32_t)((li * csh + lj * csw) * 4) : kOut;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), cr, off, 0, 0);
            }
}

template <int FM, int FN, int WGM, int WGN, int TK, int NS>
void launch_dma(const float *A, int64_t a_ld, int64_t a_bs, const float *B, int64_t b_ld, bool bkc, int64_t b_bs,
                float *C, int64_t csh, int64_t csw, int64_t c_bs, int m, int n, int k, int batch, hipStream_t stream) {
    constexpr int TM = WGM * FM * 16, TN = WGN * FN * 16;
    const dim3 grid((unsigned)((n + TN - 1) / TN), (unsigned)((m + TM - 1) / TM), (unsigned)batch);
    if (bkc)
        mm_f32_dma_kernel<FM, FN, WGM, WGN, TK, NS, true><<<grid, 64 * WGM * WGN, 0, stream>>>(
            A, a_ld, B, b_ld, C, csh, csw, m, n, k, a_bs, b_bs, c_bs);
    else
        mm_f32_dma_kernel<FM, FN, WGM, WGN, TK, NS, false><<<grid, 64 * WGM * WGN, 0, stream>>>(
            A, a_ld, B, b_ld, C, csh, csw, m, n, k, a_bs, b_bs, c_bs);
}

template <int FM, int FN, int WGM, int WGN, int TK>
void launch_cfg(const float *A, int64_t ash, int64_t asw, int64_t a_bs, const float *B, int64_t bsh, int64_t bsw,
                int64_t b_bs, float *C, int64_t csh, int64_t csw, int64_t c_bs, int m, int n, int k, int batch,
                hipStream_t stream) {
    constexpr int TM = WGM * FM * 16, TN = WGN * FN * 16;
    const dim3 grid((unsigned)((n + TN - 1) / TN), (unsigned)((m + TM - 1) / TM), (unsigned)batch);
    mm_f32_mfma_kernel<FM, FN, WGM, WGN, TK><<<grid, 64 * WGM * WGN, 0, stream>>>(A, ash, asw, B, bsh, bsw, C, csh, csw,
                                                                                m, n, k, a_bs, b_bs, c_bs);
}

}  // namespace

hipError_t launch_mm_f32(const float *A, int64_t ash, int64_t asw, const float *B, int64_t bsh, int64_t bsw, float *C,
                         int64_t csh, int64_t csw, int m, int n, int k, hipStream_t stream) {
    return launch_mm_f32_batched(A, ash, asw, 0, B, bsh, bsw, 0, C, csh, csw, 0, m, n, k, 1, stream);
}

hipError_t launch_mm_f32_batched(const float *A, int64_t ash, int64_t asw, int64_t a_bs, const float *B, int64_t bsh,
                                 int64_t bsw, int64_t b_bs, float *C, int64_t csh, int64_t csw, int64_t c_bs, int m,
                                 int n, int k, int batch, hipStream_t stream) {
#define QG_F32(FM, FN, WGM, WGN, TK) \
    launch_cfg<FM, FN, WGM, WGN, TK>(A, ash, asw, a_bs, B, bsh, bsw, b_bs, C, csh, csw, c_bs, m, n, k, batch, stream)
#define QG_DMA(FM, FN, WGM, WGN, TK, NS) \
    launch_dma<FM, FN, WGM, WGN, TK, NS>(A, ash, a_bs, B, bkc ? bsw : bsh, bkc, b_bs, C, csh, csw, c_bs, m, n, k, batch, stream)
    // 16-B aligned operands: the LDS-DMA ring
    const bool bkc = bsh == 1 && bsw != 1;
    auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool fast = asw == 1 && ash % 4 == 0 && k % 4 == 0 && al16(A) && al16(B) && a_bs % 4 == 0 && b_bs % 4 == 0 &&
                      (bkc ? bsw % 4 == 0 : (bsw == 1 && bsh % 4 == 0 && n % 4 == 0)) && ash >= 0 && bsh >= 0 && bsw >= 0;
    // the largest tile that still gives every SIMD two waves (4 x 256 CUs x 2); k is never split:
    // every output is one sequential chain
    auto waves = [&](int tm, int tn, int wpb) {
        return (int64_t)((m + tm - 1) / tm) * ((n + tn - 1) / tn) * batch * wpb;
    };
    constexpr int64_t kWant = 2048;
    if (fast) {
        if (waves(128, 128, 4) >= kWant)
            QG_DMA(4, 4, 2, 2, 32, 3);
        else if (waves(64, 64, 4) >= kWant)
            QG_DMA(2, 2, 2, 2, 32, 3);  // attention QK^T: 12 us (was 17.9 on the f32 VALU)
        else
            QG_DMA(1, 2, 2, 2, 32, 4);  // attention PV (k = 512, 128 blocks): 10.4-11.5 us (was 34.3)
    } else if (waves(128, 128, 4) >= kWant) {
        QG_F32(4, 4, 2, 2, 32);
    } else if (waves(64, 64, 4) >= kWant) {
        QG_F32(2, 2, 2, 2, 32);
    } else if (waves(32, 32, 1) >= kWant) {
        QG_F32(2, 2, 1, 1, 32);
    } else {
        QG_F32(1, 2, 1, 1, 32);
    }
#undef QG_F32
#undef QG_DMA
    return hipGetLastError();
}

}  // namespace qgemm
