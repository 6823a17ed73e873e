#!/usr/bin/env python3
"""Write lab/gemm_fm_ldsb.h: the product gemm_i8_fm (csrc/gemm_i8_kernels.h) copied as gemm_i8_fm_ldsb<kKnob> for the
one bounded experiment of VERDICT r05 item 2 -- fewer VMEM->VGPR load instructions per MFMA without a full LDS ring:
the B (W) half of a wave's operands arrives by LDS-DMA into a 3-stage ring shared by the two waves with the same wn
(each DMAs 4 of the half's 8 fragments per 64-deep sub-step), and is read with ds_read_b128; A stays direct-to-VGPR.
VMEM instructions per wave per sub-step 16 -> 12, LDS reads 8 per 64 MFMAs, one s_barrier per sub-step.
  kKnob 0: the product's loop with the builtin MFMA instead of the inline-asm one (the accumulators' placement)
  kKnob 1: B through the ring, DMA by __builtin_amdgcn_raw_ptr_buffer_load_lds, inline-asm MFMAs (the product's)
  kKnob 2: B through the ring, builtin MFMAs
Protocol (per sub-step u, all waves): DMA(u + 2) into slot (u + 2) % 3 at the start (its last reader finished before the
previous sub-step's barrier), the row-interleaved A loads of u + 2, and before row 4: s_waitcnt for this wave's DMA(u + 1),
s_barrier (the partner's DMA(u + 1) has landed too), ds_read of B(u + 1) -- read one phase after the wait that retires it
(cdna_hip_programming.md, LDS-DMA rings).  Only the unsplit, plain-epilogue kernel (kEpi = kEpiNone) is generated.
Regenerate after changing the product kernel:  python3 lab/make_ldsb_fm.py"""
import os
here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, '../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h')).read()
a = src.index('// kNtC: the paired full-tile output stores')
b = src.index('// ------------------------------------------------------------------------------------------------\n// gemm_i8_small')
k = src[a:b]
k = k.replace('template <int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>\n'
              '__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm(GemmArgs p) {',
              'template <int kKnob, int kEpi = kEpiNone, bool kI32 = false, int kSplit = kSplitNone, bool kNtC = !kI32, int kFirst64 = 30>\n'
              '__global__ __launch_bounds__(kFmThreads, 1) void gemm_i8_fm_ldsb(GemmArgs p) {')
loop_a = k.index('    v4i a0[8], b0[8], a1[8], b1[8], a2[8], b2[8];')
loop_b = k.index('    // the last MFMAs\' results are read by VALU below')
new_loop = r'''    v4i a0[8], b0[8], a1[8], b1[8], a2[8], b2[8];
    auto mfma = [&](v4i &acc_, const v4i &x, const v4i &y) __attribute__((always_inline)) {
        if constexpr (kKnob == 1) mfma_agpr(acc_, x, y);
        else acc_ = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, acc_, 0, 0, 0);
    };
    if constexpr (kKnob == 0) {
        // the product's loop, builtin MFMAs
        auto ld = [&](v4i (&fa)[8], v4i (&fb)[8], int j, int u) __attribute__((always_inline)) {
            const int soff = ((j & 7) * nsub + u) * 1024;
            if (j < 8) fb[j] = __builtin_amdgcn_raw_buffer_load_b128(rsB, voff, soff, 0);
            else fa[j - 8] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, soff, 0);
        };
        auto substep = [&](v4i (&ca)[8], v4i (&cb)[8], v4i (&na)[8], v4i (&nb)[8], int un, bool more)
                           __attribute__((always_inline)) {
            un = un < nloc ? un : nloc - 1;
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
                for (int ni = 0; ni < 8; ++ni) {
                    if (more && ni == 2) ld(na, nb, 2 * mi, un);
                    if (more && ni == 6) ld(na, nb, 2 * mi + 1, un);
                    mfma(acc[mi][ni], cb[ni], ca[mi]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __builtin_amdgcn_s_setprio(0);
        };
#pragma unroll
        for (int j = 0; j < 16; ++j) ld(a0, b0, j, 0);
        sS[tid] = sx;
        sS[BM + tid] = sw;
#pragma unroll
        for (int j = 0; j < 16; ++j) ld(a1, b1, j, nloc > 1 ? 1 : 0);
        int u = 0;
        for (; u + 3 <= nloc; u += 3) {
            substep(a0, b0, a2, b2, u + 2, true);
            substep(a1, b1, a0, b0, u + 3, true);
            substep(a2, b2, a1, b1, u + 4, true);
        }
        const int rest = nloc - u;
        if (rest > 0) {
            substep(a0, b0, a2, b2, 0, false);
            if (rest > 1) substep(a1, b1, a2, b2, 0, false);
        }
    } else {
        // B through the LDS ring: slot s at ring + 16 s KiB, half h at + 8 h KiB, fragment f at + f KiB (the image
        // area of sS: used by the epilogue only after the loop's final barrier)
        int8_t *ring = reinterpret_cast<int8_t *>(sS + 2 * BM + 4);
        // this wave's 4 fragments (4 wm .. 4 wm + 3) of B half wn, sub-step u, into ring slot `slot`: buffer LDS-DMA
        // on the half's descriptor (one per-lane offset, the fragment and sub-step in the scalar offset)
        auto dma = [&](int u, int slot) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int f = 4 * wm + q;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void *)(ring + ((slot * 2 + wn) * 8 + f) * 1024),
                                                     16, voff, __builtin_amdgcn_readfirstlane((f * nsub + u) * 1024), 0, 0);
            }
        };
        auto rdB = [&](v4i (&fb)[8], int slot) __attribute__((always_inline)) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                fb[ni] = *reinterpret_cast<const v4i *>(ring + ((slot * 2 + wn) * 8 + ni) * 1024 + lane * 16);
        };
        auto ldA = [&](v4i (&fa)[8], int i, int u) __attribute__((always_inline)) {
            fa[i] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voff, (i * nsub + u) * 1024, 0);
        };
        // compute sub-step u on (ca, cb); A of u + 2 into na; B of u + 1 from the ring into nb
        auto substep = [&](v4i (&ca)[8], v4i (&cb)[8], v4i (&na)[8], v4i (&nb)[8], int u, bool more)
                           __attribute__((always_inline)) {
            const int ua = u + 2 < nloc ? u + 2 : nloc - 1;
            if (more) dma(ua, (u + 2) % 3);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                if (mi == 4 && u + 1 < nloc) {
                    // this wave's DMA(u + 1): issued before A(u + 1) x 8, DMA(u + 2) x 4 and A(u + 2) rows 0..3
                    if (more) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                    rdB(nb, (u + 1) % 3);
                }
#pragma unroll
                for (int ni = 0; ni < 8; ++ni) {
                    if (more && ni == 2) ldA(na, mi, ua);
                    mfma(acc[mi][ni], cb[ni], ca[mi]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __builtin_amdgcn_s_setprio(0);
        };
        dma(0, 0);
        dma(nloc > 1 ? 1 : 0, 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) ldA(a0, i, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) ldA(a1, i, nloc > 1 ? 1 : 0);
        sS[tid] = sx;
        sS[BM + tid] = sw;
        asm volatile("s_waitcnt vmcnt(20)" ::: "memory");  // DMA(0): before DMA(1) x 4, A(0) x 8, A(1) x 8
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        rdB(b0, 0);
        int u = 0;
        for (; u + 3 <= nloc; u += 3) {
            substep(a0, b0, a2, b1, u, true);
            substep(a1, b1, a0, b2, u + 1, true);
            substep(a2, b2, a1, b0, u + 2, true);
        }
        const int rest = nloc - u;
        if (rest > 0) {
            substep(a0, b0, a2, b1, u, false);
            if (rest > 1) substep(a1, b1, a2, b2, u + 1, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA left in flight over the epilogue's image
    }
'''
k = k[:loop_a] + new_loop + k[loop_b:]
out = '''// gemm_fm_ldsb.h -- GENERATED by lab/make_ldsb_fm.py from the product gemm_i8_fm: B through an LDS-DMA ring (lab).
#pragma once

#include "../quantized-gemm-for-transformer-inference_amd/csrc/gemm_i8_kernels.h"

namespace qgemm {
namespace gemm {

''' + k + '''
}  // namespace gemm
}  // namespace qgemm
'''
open(os.path.join(here, 'gemm_fm_ldsb.h'), 'w').write(out)
print('wrote lab/gemm_fm_ldsb.h')
