#!/usr/bin/env python3
"""Does the packed operands' power-of-two row stride (k_pad = 4096 B) cost the GEMM?  Times the int8 GEMM +
dequantize (qgemm_mm_packed) at K = 4096 and at K = 4096 + 128*j (row strides 4224, 4352, ... B, one more
k-step each), M = N = 4096, interleaved rounds in one process.  No stride effect: time grows with the
k-steps (33/32, 34/32, ...).  Run on the GPU box."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _pkg  # noqa: E402

qg = _pkg.package(build=False)


def main():
    dev = torch.device("cuda:0")
    M = N = 4096
    cases = {}
    for K in (4096, 4224, 4352, 4608):
        X = qg.fill_uniform(torch.empty((M, K), device=dev), 1)
        W = qg.fill_uniform(torch.empty((K, N), device=dev), 2)
        cases[K] = (qg.pack_a(X), qg.pack_b(W), torch.empty((M, N), device=dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {K: [] for K in cases}
    for _ in range(7):
        for K, (pa, pb, C) in cases.items():
            for _ in range(5):
                qg.mm_packed(pa, pb, C)
            e0.record()
            for _ in range(50):
                qg.mm_packed(pa, pb, C)
            e1.record()
            e1.synchronize()
            res[K].append(e0.elapsed_time(e1) / 50 * 1e3)
    base = sorted(res[4096])[3]
    for K, v in res.items():
        v.sort()
        print(f"K={K} (row stride {K} B, {K // 128} k-steps): median {v[3]:7.2f} us  per k-step {v[3] / (K // 128):6.3f}"
              f"  ratio {v[3] / base:.3f} vs k-step ratio {(K // 128) / 32:.3f}")


if __name__ == "__main__":
    main()
