#!/usr/bin/env python3
"""Write lab/gemm_fm_epi.h: the product gemm_i8_fm (csrc/gemm_i8_kernels.h) copied as gemm_i8_fm_epi<kMap, kStore, kAux>
with epilogue store shapes / cache policies and tile-map knobs for the wide-row (FFN up, 64-KiB output rows) question of
VERDICT r05 item 1:
  kMap   0: groups of 4 tile-rows (the round-5 product); 1: groups of 8 tile-rows (the product since round 6 when
            wide_rows is set); 2: the product's patches with
            each 16-aligned run of column tiles interleaved (an XCD's first round of blocks takes the even column tiles,
            the second round the odd ones: the column offsets written at one time spread over the whole row);
            3: groups of 2 tile-rows; 4 / 5 (FFN up's 8 x 64 tiles only): a round of blocks takes all 8 tile-rows x 32
            column tiles (half of every row, contiguous) / 4 tile-rows x all 64 column tiles (whole rows)
  kStore 0: the product (paired 8-row x 128-B stores, or the LDS image when wide_rows is set);
         1: the paired stores through a buffer descriptor with cache policy kAux;
         2: no stores (the dequantize is computed and kept alive);
         3: 4 rows x 256 B per store: a 4 x 4 lane transpose (lanes c, c^4, c^8, c^12 over tiles 4g .. 4g+3, DPP);
         4: 2 rows x 512 B per store: an 8 x 8 lane transpose (lanes c ^ 1, 2, 4 over the 8 tiles, DPP)
         5: (wide rows) the LDS image shared by the two waves of a tile-row half: one full 1-KiB tile row per store
  kAux  -1: __builtin_nontemporal_store (the product's `nt`), else the buffer-store aux bits (1 sc0, 2 nt, 16 sc1)
Regenerate after changing the product kernel:  python3 lab/make_epi_fm.py"""
import os
here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, '../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h')).read()
a = src.index('// kNtC: the paired full-tile output stores')
b = src.index('// ------------------------------------------------------------------------------------------------\n// gemm_i8_small')
k = src[a:b]
reps = [
    ('template <int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>\n'
     '__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm(GemmArgs p) {',
     'template <int kMap, int kStore, int kAux, int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>\n'
     '__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm_epi(GemmArgs p) {'),
    ("    group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn, kEpi != kEpiOutlier && p.wide_rows ? 8 : 4);\n",
     """    if constexpr (kMap == 1 || kMap == 3) {  // XCD patches of 8 (2) tile-rows instead of 4
        constexpr int kG = kMap == 1 ? 8 : 2;
        const int per_group = kG * p.tiles_n, group = tile / per_group, first_m = group * kG;
        const int gsz = min(p.tiles_m - first_m, kG), w = tile - group * per_group;
        tm = first_m + w % gsz;
        tn = w / gsz;
    } else {
        group_tiles(tile, p.tiles_m, p.tiles_n, tm, tn);
        if (kMap == 2 && p.tiles_n % 16 == 0) tn = (tn & ~15) | ((tn & 7) << 1) | ((tn >> 3) & 1);
        if ((kMap == 4 || kMap == 5) && p.tiles_m == 8 && p.tiles_n == 64) {
            // FFN up only: XCD x (logical ids 64 x + w; w < 32 = its first round of blocks)
            const int x = tile >> 6, w = tile & 63;
            if (kMap == 4) {  // each round: all 8 tile-rows x 32 column tiles (a contiguous half of every row)
                tm = w & 7;
                tn = 32 * (w >> 5) + 4 * x + ((w >> 3) & 3);
            } else {          // each round: 4 tile-rows x all 64 column tiles (whole rows)
                tm = 4 * (w >> 5) + (w & 3);
                tn = 8 * x + ((w & 31) >> 2);
            }
        }
    }
"""),
    ("    const bool image = full && p.wide_rows;\n",
     "    const bool image = (kStore == 0 || kStore == 5) && full && p.wide_rows;\n"
     "    float lab_sink = 0.0f;\n"
     "    const auto rsC = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, 0x7fffffff, 0x00020000);\n"),
    ("""#pragma unroll
            for (int np = 0; np < 4; ++np) {
                const v4f o0 = tile_out(2 * np), o1 = tile_out(2 * np + 1);""",
     """            if constexpr (kStore != 0 && kStore != 5) {
                if (full) {
                    lab_v4f q[8];
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) q[ni] = tile_out(ni);
                    if constexpr (kStore == 2) {
#pragma unroll
                        for (int ni = 0; ni < 8; ++ni) lab_sink += q[ni][0] + q[ni][1] + q[ni][2] + q[ni][3];
                    } else if constexpr (kStore == 1) {
#pragma unroll
                        for (int np = 0; np < 4; ++np) {
                            lab_v4f x1 = q[2 * np], x2 = q[2 * np + 1];
                            lab_tstage_pair<8>(x1, x2, !lo);
                            const int64_t ra = gi0 + r0 + 16 * mi + (c & 7);
                            const int jc = gj0 + c0 + 32 * np + (lo ? 0 : 16) + 4 * kq;
                            lab_store<kAux>(rsC, C, ra * p.csh + jc, x1);
                            lab_store<kAux>(rsC, C, (ra + 8) * p.csh + jc, x2);
                        }
                    } else if constexpr (kStore == 3) {
                        const int a4 = c >> 2, b4 = c & 3;
#pragma unroll
                        for (int g = 0; g < 2; ++g) {
                            lab_v4f u[4] = {q[4 * g], q[4 * g + 1], q[4 * g + 2], q[4 * g + 3]};
                            lab_tstage<4, 2, 8>(u, (c & 8) != 0);
                            lab_tstage<4, 1, 4>(u, (c & 4) != 0);
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                lab_store<kAux>(rsC, C, (int64_t)(gi0 + r0 + 16 * mi + 4 * j + b4) * p.csh + gj0 + c0 + 64 * g + 16 * a4 + 4 * kq, u[j]);
                        }
                    } else if constexpr (kStore == 4) {
                        const int t8 = c & 7, h8 = c >> 3;
                        lab_tstage<8, 4, 4>(q, (c & 4) != 0);
                        lab_tstage<8, 2, 2>(q, (c & 2) != 0);
                        lab_tstage<8, 1, 1>(q, (c & 1) != 0);
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            lab_store<kAux>(rsC, C, (int64_t)(gi0 + r0 + 16 * mi + 8 * h8 + j) * p.csh + gj0 + c0 + 16 * t8 + 4 * kq, q[j]);
                    }
                    continue;
                }
            }
#pragma unroll
            for (int np = 0; np < 4; ++np) {
                const v4f o0 = tile_out(2 * np), o1 = tile_out(2 * np + 1);"""),
    # the no-store variant keeps its arithmetic alive through one conditional store at the end
    ("""                __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + c0 + c4));
            }
        }
    }
}""",
     """                __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + c0 + c4));
            }
        }
    }
    if constexpr (kStore == 2)
        if (p.reset_tickets == -12345) C[tid] = lab_sink;
}"""),
]
for x, y in reps:
    assert x in k, 'product kernel changed: update make_epi_fm.py (' + x[:50] + ')'
    k = k.replace(x, y)

reps += [
    ("    float *T = sS + 2 * BM + 4 + wave * 64 * TS;  // this wave's image (wide rows)\n",
     "    // kStore 5: the two waves of a tile-row half share one [64][TSX] image of 256 columns\n"
     "    constexpr int TSX = kStore == 5 ? 260 : TS;\n"
     "    float *T = kStore == 5 ? sS + 2 * BM + 4 + wm * 64 * TSX + wn * 128 : sS + 2 * BM + 4 + wave * 64 * TS;\n"),
    ("""                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TS + 32 * np + 4 * kq) = o0;
                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TS + 32 * np + 16 + 4 * kq) = o1;""",
     """                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TSX + 32 * np + 4 * kq) = o0;
                    *reinterpret_cast<v4f *>(T + (16 * mq + c) * TSX + 32 * np + 16 + 4 * kq) = o1;"""),
    ("""        if (image) {
            // wide rows: the half's 64 rows read back""",
     """        if (kStore == 5 && image) {
            // the pair's 64 rows x 256 columns: each wave stores 32 of them, one 1-KiB row per store, rotated order
            __syncthreads();
            const float *P = sS + 2 * BM + 4 + wm * 64 * TSX;
            const int rot = __builtin_amdgcn_readfirstlane((tn * 7 + tm * 3) & 31);
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int rr = 2 * ((it + rot) & 31) + wn;
                const v4f v = *reinterpret_cast<const v4f *>(P + rr * TSX + lane * 4);
                __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(C + (int64_t)(gi0 + r0 + 64 * s + rr) * p.csh + gj0 + lane * 4));
            }
            __syncthreads();
        } else if (image) {
            // wide rows: the half's 64 rows read back"""),
]
for x, y in reps[-3:]:
    assert x in k, 'product kernel changed: update make_epi_fm.py (' + x[:50] + ')'
    k = k.replace(x, y)

# kAux >= 100 with kStore 0 (the product's image path): the per-tile row rotation formula of the wide-row stores
#   100: none; 101: tn & 31; 102: (tm * 4 + tn) & 31; 103: (tn * 5 + tm * 9) & 31; 104: (tn * 7 + tm * 3) & 31 (rounds
#   4-5; the product takes (tn * 13 + tm * 7) since round 6)
rot_old = "            const int rot = __builtin_amdgcn_readfirstlane((tn * 13 + tm * 7) & 31);\n            const int c4 = (lane & 31) * 4;"
assert rot_old in k, 'product kernel changed: update make_epi_fm.py (rotation)'
k = k.replace(rot_old, """            const int rot = __builtin_amdgcn_readfirstlane(
                kAux == 100 ? 0 : kAux == 101 ? (tn & 31) : kAux == 102 ? ((tm * 4 + tn) & 31)
                : kAux == 103 ? ((tn * 5 + tm * 9) & 31) : kAux == 104 ? ((tn * 7 + tm * 3) & 31) : ((tn * 13 + tm * 7) & 31));
            const int c4 = (lane & 31) * 4;""")
helpers = '''typedef float lab_v4f __attribute__((ext_vector_type(4)));

// lane c reads lane c ^ X of its 16-lane row (DPP; X = 4 as two bank-masked row shifts)
template <int X>
__device__ __forceinline__ float lab_xor_lane(float v) {
    const int x = __float_as_int(v);
    if constexpr (X == 8) return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x128, 0xf, 0xf, false));  // row_ror:8
    if constexpr (X == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, false));   // quad_perm 2301
    if constexpr (X == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, false));   // quad_perm 1032
    // banks 0, 2 (c & 4 == 0) read c + 4 (row_shl:4), banks 1, 3 read c - 4 (row_shr:4)
    const int t = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xf, 0x5, false);
    return __int_as_float(__builtin_amdgcn_update_dpp(t, x, 0x114, 0xf, 0xA, false));
}

// one transpose step over lane bit X between slots s0 and s1: the low lane keeps s0 and receives the partner's s0
// into s1, the high lane receives the partner's s1 into s0 and keeps s1
template <int X>
__device__ __forceinline__ void lab_tstage_pair(lab_v4f &s0, lab_v4f &s1, bool hi) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float recv = lab_xor_lane<X>(hi ? s0[e] : s1[e]);
        s0[e] = hi ? recv : s0[e];
        s1[e] = hi ? s1[e] : recv;
    }
}

template <int NS, int SB, int X>
__device__ __forceinline__ void lab_tstage(lab_v4f (&q)[NS], bool hi) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
        if (!(s & SB)) lab_tstage_pair<X>(q[s], q[s | SB], hi);
}

template <int kAux>
__device__ __forceinline__ void lab_store(__amdgpu_buffer_rsrc_t rs, float *C, int64_t elem, lab_v4f v) {
    if constexpr (kAux < 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<lab_v4f *>(C + elem));
    } else {
        typedef int v4i_ __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_, v), rs, (int)(elem * 4), 0, kAux);
    }
}

'''
out = '''// gemm_fm_epi.h -- GENERATED by lab/make_epi_fm.py from the product gemm_i8_fm: epilogue store shapes, cache
// policies and tile maps (wide-row investigation, VERDICT r05 item 1).
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

''' + helpers + k + '''
}  // namespace gemm
}  // namespace qgemm
'''
open(os.path.join(here, 'gemm_fm_epi.h'), 'w').write(out)
print('wrote lab/gemm_fm_epi.h')
