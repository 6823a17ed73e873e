#!/usr/bin/env python3
"""Config-5 encoder forward: eager launches vs the same forward captured once in a HIP graph and replayed
(diagnostic: how much of the forward is launch / inter-kernel gap).  Also checks replay is bit-identical."""
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
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    for _ in range(5):
        enc.forward(X, Y)
torch.cuda.synchronize()
ref = Y.clone()


def timed(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def eager():
    with torch.cuda.stream(s):
        enc.forward(X, Y)


g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    enc.forward(X, Y)
torch.cuda.synchronize()
Y.zero_()
g.replay()
torch.cuda.synchronize()
same = torch.equal(Y.view(torch.int32), ref.view(torch.int32))
for r in range(3):
    te = timed(eager)
    tg = timed(g.replay)
    print(f"round {r}: eager {te * 1e6:.1f} us ({1 / te:.0f}/s)  graph replay {tg * 1e6:.1f} us ({1 / tg:.0f}/s)")
print("graph replay bit-identical to eager:", same)
enc.close()
