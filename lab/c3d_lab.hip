// c3d_lab.hip -- LAB harness: the whole FFN-down drop-in call (BASELINE configs[2], X 2048 x 16384, W 16384 x 4096)
// as the library runs it -- pass 1 (X rows + W column maxima), pass 2 (W re-read, quantized, transposed), the int8
// GEMM -- with the sweep orders and the GEMM as variables, every output bit compared with the library's order:
//   order 0: pass 1 W-first, pass 2 forward (round 3); 1: pass 1 X-first, pass 2 bottom-up (re-reads what pass 1
//      read last); 2: pass 1 W only, pass 2 bottom-up with X's rows at its end (round 4 product); 3: order 2 with
//      non-temporal loads of W and X in pass 2; 4: order 2 with non-temporal loads of X only
//   G  gemm_i8_fm split-K 2 with both slabs (rounds 2-3) | ticket-first (one slab, uneven K split: round 4) |
//      fk (gemm_i8_fk: split-K inside the CU)
//   build/c3d_lab m n k rounds [sync|orders]   (sync: the product vs kSync, twice the product as a noise floor)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"
#include "gemm_fk.h"

using namespace qgemm;
using namespace qgemm::gemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 2048, n = argc > 2 ? atoi(argv[2]) : 4096, k = argc > 3 ? atoi(argv[3]) : 16384;
    const int rounds = argc > 4 ? atoi(argv[4]) : 7, reps = 10;
    if (k <= 4096 || m % 256 || n % 256 || k % 128) { printf("lab shape: K > 4096, whole 256-tiles\n"); return 2; }
    float *X, *W, *C, *Cref; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&C, (size_t)m * n * 4)); CK(hipMalloc(&Cref, (size_t)m * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    const int tiles_m = m / 256, tiles_n = n / 256, tiles = tiles_m * tiles_n;
    int32_t *slabs; unsigned *tickets;
    CK(hipMalloc(&slabs, (size_t)tiles * 2 * 256 * 256 * 4)); CK(hipMalloc(&tickets, 4096));
    CK(hipMemset(tickets, 0, 4096));
    CK(launch_fill_uniform(X, (int64_t)m * k, 11, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 12, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    const int col_blocks = (n + kColBlock - 1) / kColBlock, ncol = col_blocks * (int)vw.parts, nrow = (int)vx.rows_pad;
    const float range = 127.f;
    // order: 0 = W-first pass 1, forward pass 2 (round 3); 1 = X-first pass 1, pass 2 bottom-up (round 4 product);
    // 2 = W-only pass 1 (colmax_kernel), pass 2 bottom-up with X's rows at its end (pack_cols_then_rows_kernel)
    auto pass1 = [&](int order) {
        if (order >= 2) {
            colmax_kernel<true><<<dim3(col_blocks, (unsigned)vw.parts), 256, 0, s0>>>(W, n, k, n, vw.scratch, vw.rows_pad);
        } else if (order == 1) {
            pack_rows_and_colmax_kernel<-1, true><<<ncol + nrow, 256, 0, s0>>>(
                X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, n, vw.scratch, vw.rows_pad, col_blocks, ncol,
                range, reinterpret_cast<uint32_t *>(tickets), 1024);
        } else {
            pack_rows_and_colmax_kernel<-1, false><<<ncol + nrow, 256, 0, s0>>>(
                X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, n, vw.scratch, vw.rows_pad, col_blocks, ncol,
                range, reinterpret_cast<uint32_t *>(tickets), 1024);
        }
    };
    const dim3 g2((unsigned)(vw.rows_pad / kTc), (unsigned)((vw.k_pad / kTk + kTilesPerBlock - 1) / kTilesPerBlock));
    auto pass2 = [&](int order) {
        if (order == 3)
            pack_cols_then_rows_kernel<true, true><<<g2.x * g2.y + nrow, 256, 0, s0>>>(
                W, n, k, n, range, vw.scratch, vw.parts, vw.rows_pad, vw.scale, vw.q, vw.k_pad, (int)g2.x, (int)g2.y, X, k,
                m, vx.scale, vx.q, vx.rows_pad, reinterpret_cast<uint32_t *>(tickets), 1024);
        else if (order == 4)
            pack_cols_then_rows_kernel<false, true><<<g2.x * g2.y + nrow, 256, 0, s0>>>(
                W, n, k, n, range, vw.scratch, vw.parts, vw.rows_pad, vw.scale, vw.q, vw.k_pad, (int)g2.x, (int)g2.y, X, k,
                m, vx.scale, vx.q, vx.rows_pad, reinterpret_cast<uint32_t *>(tickets), 1024);
        else if (order == 2)
            pack_cols_then_rows_kernel<<<g2.x * g2.y + nrow, 256, 0, s0>>>(
                W, n, k, n, range, vw.scratch, vw.parts, vw.rows_pad, vw.scale, vw.q, vw.k_pad, (int)g2.x, (int)g2.y, X, k,
                m, vx.scale, vx.q, vx.rows_pad, reinterpret_cast<uint32_t *>(tickets), 1024);
        else if (order == 1)
            pack_cols_kernel<true, kTilesPerBlock, true><<<g2, 256, 0, s0>>>(W, n, k, n, range, vw.scratch, vw.parts,
                                                                             vw.rows_pad, vw.scale, vw.q, vw.k_pad);
        else
            pack_cols_kernel<true, kTilesPerBlock, false><<<g2, 256, 0, s0>>>(W, n, k, n, range, vw.scratch, vw.parts,
                                                                              vw.rows_pad, vw.scale, vw.q, vw.k_pad);
    };
    // g: 0 / 2 = ticket-first split-K with slice 0 = 31 of 64 k-steps (the product; the rounds 2-3 both-slabs form and the
    // XCD-pair map are lab/splitk_both_pairxcd_experiment.patch), 1 = slice 0 = 30, 3 = fk (split-K inside the CU),
    // 4 = ticket-first 31 with an s_barrier every 3 sub-steps (kSync, round 5)
    auto gemm = [&](int g, float *out) {
        GemmArgs p{};
        p.A = vx.q; p.B = vw.q; p.Cx = vx.scale; p.Cw = vw.scale; p.C = out; p.csh = n; p.csw = 1; p.m = m; p.n = n;
        p.k_pad = vx.k_pad; p.tiles_m = tiles_m; p.inv_r2 = 1.0f / (range * range); p.splits = 1;
        if (g == 3) {
            p.tiles_n = n / 128;
            gemm_i8_fk<><<<tiles * 2, 256, 0, s0>>>(p);
            return;
        }
        p.tiles_n = tiles_n; p.splits = 2; p.slabs = slabs; p.tickets = tickets; p.reset_tickets = 1;
        if (g == 0) gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 31><<<tiles * 2, 256, 0, s0>>>(p);
        if (g == 1) gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 30><<<tiles * 2, 256, 0, s0>>>(p);
        if (g == 2) gemm_i8_fm<kEpiNone, false, kSplitFirst, true, 31><<<tiles * 2, 256, 0, s0>>>(p);
        // g == 4: the product header's kSync knob (an s_barrier every 3 sub-steps), measured neutral in round 5
        // (profiles/r05_c3d_sync.log: GEMM 109.15 vs 108.93-108.95 us) and removed; lab/fm_sync_experiment.patch
    };
    struct V { std::string name; int order; int g; };
    std::vector<V> vs;
    const std::string set = argc > 5 ? argv[5] : "sync";
    if (set == "sync") vs = {{"product_nt", 3, 2}, {"product_nt_b", 3, 0}};
    else vs = {{"wonly_default", 2, 2}, {"product_nt", 3, 2}, {"nt_fk", 3, 3}};
    // reference: the library's order
    pass1(0); pass2(0); gemm(0, Cref);
    CK(hipStreamSynchronize(s0));
    std::vector<float> href((size_t)m * n), hgot(href.size());
    CK(hipMemcpy(href.data(), Cref, href.size() * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        CK(hipMemsetAsync(C, 0xff, (size_t)m * n * 4, s0));
        CK(hipMemsetAsync(vw.q, 0x5a, vw.rows_pad * vw.k_pad, s0));
        pass1(v.order); pass2(v.order); gemm(v.g, C);
        CK(hipStreamSynchronize(s0));
        CK(hipMemcpy(hgot.data(), C, hgot.size() * 4, hipMemcpyDeviceToHost));
        printf("check %-18s %s\n", v.name.c_str(), memcmp(href.data(), hgot.data(), href.size() * 4) ? "DIFF" : "same");
    }
    // timing: whole call, and each kernel by events between the launches, interleaved rounds
    hipEvent_t ev[4];
    for (auto &e : ev) CK(hipEventCreate(&e));
    std::vector<std::vector<float>> tc(vs.size()), t1(vs.size()), t2(vs.size()), tg(vs.size());
    for (int i = 0; i < 300; ++i) { pass1(3); pass2(3); gemm(2, C); }  // clocks up
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            const V &v = vs[i];
            for (int w = 0; w < 3; ++w) { pass1(v.order); pass2(v.order); gemm(v.g, C); }
            float a1 = 0, a2 = 0, ag = 0, ac = 0;
            for (int j = 0; j < reps; ++j) {
                CK(hipEventRecord(ev[0], s0)); pass1(v.order);
                CK(hipEventRecord(ev[1], s0)); pass2(v.order);
                CK(hipEventRecord(ev[2], s0)); gemm(v.g, C);
                CK(hipEventRecord(ev[3], s0)); CK(hipEventSynchronize(ev[3]));
                float x;
                CK(hipEventElapsedTime(&x, ev[0], ev[1])); a1 += x;
                CK(hipEventElapsedTime(&x, ev[1], ev[2])); a2 += x;
                CK(hipEventElapsedTime(&x, ev[2], ev[3])); ag += x;
                CK(hipEventElapsedTime(&x, ev[0], ev[3])); ac += x;
            }
            t1[i].push_back(a1 * 1000 / reps); t2[i].push_back(a2 * 1000 / reps);
            tg[i].push_back(ag * 1000 / reps); tc[i].push_back(ac * 1000 / reps);
        }
    auto med = [](std::vector<float> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
    const double b1 = 4.0 * m * k + (double)m * k + 4.0 * k * n, b2 = 4.0 * k * n + (double)k * n;
    for (size_t i = 0; i < vs.size(); ++i)
        printf("%-18s call %8.2f us (%6.0f GEMMs/s) | pass1 %7.2f (%.2f TB/s)  pass2 %7.2f (%.2f TB/s)  gemm %7.2f\n",
               vs[i].name.c_str(), med(tc[i]), 1e6 / med(tc[i]), med(t1[i]), b1 / (med(t1[i]) * 1e-6) / 1e12, med(t2[i]),
               b2 / (med(t2[i]) * 1e-6) / 1e12, med(tg[i]));
    return 0;
}
