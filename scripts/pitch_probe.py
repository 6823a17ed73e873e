#!/usr/bin/env python3
"""Diagnostic (round 6): is FFN up's extra GEMM time the 64-KiB output pitch itself?  The drop-in
call (op_mm_quantize_ws) at FFN up (2048 x 4096 -> 16384) and at the C4 shard (8192 x 4096 -> 4096) with the output
written at its natural leading dimension and at padded ones (ldc = N + pad floats, same kernel path: wide rows stay
>= 16384 floats), the GEMM kernel timed by hipExtLaunchKernel events, interleaved rounds in one process.  A benchmark
of the caller's layout, not of the contract's (the drop-in C is M x N row-major): it only names the cause.
Run on the GPU box: python scripts/pitch_probe.py [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402  (HipEvents, load_pkg)


def main():
    import torch
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    qg = bench.load_pkg()
    L = qg.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = qg._stream(dev)
    shapes = {"ffn_up": (2048, 16384, 4096), "c4_shard": (8192, 4096, 4096)}
    pads = {"ffn_up": [0, 32, 64, 256, 1024], "c4_shard": [0, 64, 1024, 12288, 12288 + 1024]}
    bufs = {}
    for name, (M, N, K) in shapes.items():
        X = qg.fill_uniform(torch.empty((M, K), device=dev), seed=2 * 1000)
        W = qg.fill_uniform(torch.empty((K, N), device=dev), seed=2 * 1000 + 1)
        O = torch.empty((M * (N + max(pads[name])),), device=dev)
        ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
        bufs[name] = (X, W, O, ws)
    hip = bench.HipEvents(2)
    L.qgemm_set_event_mode(0)
    res = {}
    for _ in range(rounds):
        for name, (M, N, K) in shapes.items():
            X, W, O, ws = bufs[name]
            for pad in pads[name]:
                ldc = N + pad
                times = []
                for i in range(25):
                    if i >= 5:
                        L.qgemm_set_gemm_events(hip.ev[0], hip.ev[1])
                    rc = L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), N, 1, O.data_ptr(), ldc, 1, M, N, K,
                                             127.0, ws.data_ptr(), ws.numel(), s)
                    if rc:
                        raise RuntimeError(f"op_mm_quantize_ws returned {rc}")
                    if i >= 5:
                        times.append(hip.elapsed_ms(hip.ev[0], hip.ev[1]) * 1e3)
                res.setdefault((name, pad), []).append(statistics.median(times))
    hip.destroy()
    for (name, pad), v in res.items():
        print(f"{name:9s} ldc = N + {pad:5d} floats ({(shapes[name][1] + pad) * 4 / 1024:8.2f} KiB pitch): GEMM median "
              f"{statistics.median(v):7.2f} us  (rounds {', '.join(f'{x:.2f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
