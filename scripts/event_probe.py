#!/usr/bin/env python3
"""How do HIP-event GEMM timings compare with the kernel trace?  (diagnostic, GPU box)

Times the packed GEMM (4096^3) four ways in one process:
  burst   : events around 20 back-to-back GEMM launches (amortised, includes launch gaps)
  ext_b2b : hipExtLaunchKernel start/stop events on each of 20 back-to-back GEMMs
  ext_pk  : the same, but each GEMM preceded by the pack launch (the bench's step)
  rec_pk  : hipEventRecord around each GEMM of a pack+GEMM step
Run under rocprofv3 --kernel-trace --stats to compare with the trace's durations.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

import _pkg  # noqa: E402
from bench import HipEvents  # noqa: E402

qg = _pkg.package()
L = qg.load()
dev = torch.device("cuda", 0)
M = N = K = 4096
X = qg.fill_uniform(torch.empty((M, K), device=dev), seed=2)
W = qg.fill_uniform(torch.empty((K, N), device=dev), seed=3)
O = torch.empty((M, N), device=dev)
ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
pa, pb = qg.pack_a(X), qg.pack_b(W)
s = qg._stream(dev)
n = 20
hip = HipEvents(2 * n + 2)


def gemm(ev=None):
    if ev is not None:
        L.qgemm_set_gemm_events(hip.ev[ev], hip.ev[ev + 1])
    rc = L.qgemm_mm_packed(pa.buf.data_ptr(), pb.buf.data_ptr(), O.data_ptr(), N, 1, M, N, K, 127.0, s)
    assert rc == 0


def full(ev=None):
    if ev is not None:
        L.qgemm_set_gemm_events(hip.ev[ev], hip.ev[ev + 1])
    rc = L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                             ws.data_ptr(), ws.numel(), s)
    assert rc == 0


for _ in range(10):
    full()
torch.cuda.synchronize()
for rnd in range(3):
    # burst
    hip.hip.hipEventRecord(hip.ev[2 * n], s)
    for _ in range(n):
        gemm()
    hip.hip.hipEventRecord(hip.ev[2 * n + 1], s)
    burst = hip.elapsed_ms(hip.ev[2 * n], hip.ev[2 * n + 1]) / n
    # ext, back to back
    L.qgemm_set_event_mode(0)
    for i in range(n):
        gemm(2 * i)
    torch.cuda.synchronize()
    ext_b2b = sorted(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) for i in range(n))
    # ext after pack
    for i in range(n):
        full(2 * i)
    torch.cuda.synchronize()
    ext_pk = sorted(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) for i in range(n))
    L.qgemm_set_event_mode(1)
    for i in range(n):
        full(2 * i)
    torch.cuda.synchronize()
    rec_pk = sorted(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) for i in range(n))
    L.qgemm_set_event_mode(0)
    med = lambda v: 1e3 * v[len(v) // 2]  # noqa: E731
    print(f"round {rnd}: burst {1e3 * burst:.2f} us  ext_b2b {med(ext_b2b):.2f} (min {1e3 * ext_b2b[0]:.2f})  "
          f"ext_pk {med(ext_pk):.2f} (min {1e3 * ext_pk[0]:.2f})  rec_pk {med(rec_pk):.2f}", flush=True)
