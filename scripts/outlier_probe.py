#!/usr/bin/env python3
"""Time the LLM.int8() outlier decomposition (qgemm_mm_outlier) against the plain drop-in at one shape,
with 0 / 8 / 32 outlier feature columns (|x| > 6 in 2 % of their rows); run on the GPU box, optionally
under rocprofv3 --kernel-trace --stats.  Usage: outlier_probe.py [M N K]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _pkg  # noqa: E402

qg = _pkg.package(build=False)


def main():
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 4096, 4096)
    dev = torch.device("cuda:0")
    L = qg.load()
    X = qg.fill_uniform(torch.empty((M, K), device=dev), 21)
    W = qg.fill_uniform(torch.empty((K, N), device=dev), 22)
    C = torch.empty((M, N), device=dev)
    ws = torch.empty(L.qgemm_mm_outlier_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
    s = qg._stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rng = np.random.default_rng(0)
    for ncols in (0, 8, 32):
        Xc = X.clone()
        for c in rng.choice(K, size=ncols, replace=False):
            rows = torch.from_numpy(rng.choice(M, size=max(1, M // 50), replace=False)).to(dev)
            Xc[rows, int(c)] = torch.from_numpy(rng.uniform(7, 60, rows.numel()).astype(np.float32)).to(dev)

        def call():
            rc = L.qgemm_mm_outlier(Xc.data_ptr(), W.data_ptr(), C.data_ptr(), M, N, K, 6.0, ws.data_ptr(), ws.numel(), s)
            assert rc == 0, rc

        for _ in range(5):
            call()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0.record()
            for _ in range(20):
                call()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        ts.sort()
        print(f"{M}x{N}x{K} outlier columns {ncols:3d}: qgemm_mm_outlier median {ts[2]:8.1f} us")
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(20):
            qg.op_mm_quantize(X, W, C)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    print(f"{M}x{N}x{K} plain op_mm_quantize median {ts[2]:8.1f} us")


if __name__ == "__main__":
    main()
