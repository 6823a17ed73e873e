"""Does the GEMM kernel run faster when the chip has idled before it?  The drop-in call at C2 and C3-down in a loop,
with an idle gap (torch.cuda._sleep on the same stream, no memory traffic) of 0 / 50 / 200 us before each call;
the GEMM kernel timed by hipExtLaunchKernel events (qgemm_set_gemm_events).  Diagnostic only.
Run on the GPU box: python scripts/power_probe.py"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import _pkg  # noqa: E402
from bench import HipEvents  # noqa: E402

qg = _pkg.package(build=False)
L = qg.load()
dev = torch.device("cuda:0")
# cycles of torch.cuda._sleep per microsecond (it spins on the shader clock): calibrate once
def calib():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000); torch.cuda.synchronize()
    e0.record(); torch.cuda._sleep(1_000_000); e1.record(); torch.cuda.synchronize()
    return 1_000_000 / (e0.elapsed_time(e1) * 1e3)


def run(M, N, K, gap_us, cyc_per_us, calls=60):
    X = qg.fill_uniform(torch.empty((M, K), device=dev), seed=1)
    W = qg.fill_uniform(torch.empty((K, N), device=dev), seed=2)
    O = torch.empty((M, N), device=dev)
    ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    hip = HipEvents(2 * calls)
    L.qgemm_set_event_mode(0)
    for i in range(calls + 10):
        if gap_us:
            torch.cuda._sleep(int(gap_us * cyc_per_us))
        if i >= 10:
            L.qgemm_set_gemm_events(hip.ev[2 * (i - 10)], hip.ev[2 * (i - 10) + 1])
        rc = L.op_mm_quantize_ws(ctypes.c_void_p(X.data_ptr()), K, 1, ctypes.c_void_p(W.data_ptr()), N, 1,
                                 ctypes.c_void_p(O.data_ptr()), N, 1, M, N, K, ctypes.c_float(127.0),
                                 ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(s))
        assert rc == 0, rc
    torch.cuda.synchronize()
    t = sorted(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) * 1e3 for i in range(calls))
    hip.destroy()
    return t[len(t) // 2], t[0]


def main():
    cyc = calib()
    print(f"torch.cuda._sleep: {cyc:.0f} cycles per us")
    for (M, N, K, name) in [(4096, 4096, 4096, "C2"), (2048, 4096, 16384, "C3-down")]:
        for gap in (0, 50, 200, 0):
            med, mn = run(M, N, K, gap, cyc)
            print(f"{name:8s} idle gap {gap:4d} us before each call: GEMM median {med:7.2f} us  min {mn:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
