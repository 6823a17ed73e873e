#!/usr/bin/env python3
"""Time the config-5 encoder forward (diagnostic; run under rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import _pkg  # noqa: E402

qg = _pkg.package(build=False)
seq, d, H, dff, blocks = 512, 1024, 16, 4096, 2
dev = torch.device("cuda", 0)
enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=1)
X = qg.fill_uniform(torch.empty((seq, d), device=dev), seed=3)
Y = torch.empty_like(X)
for _ in range(5):
    enc.forward(X, Y)
torch.cuda.synchronize()
n = 50
t0 = time.perf_counter()
for _ in range(n):
    enc.forward(X, Y)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(f"encoder forward seq={seq} d={d} H={H} dff={dff} blocks={blocks}: {dt * 1e6:.1f} us, "
      f"{1 / dt:.1f} forwards/s, {seq / dt:.0f} tokens/s")
enc.close()
