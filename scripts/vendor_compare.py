"""Same-box, same-process comparison of this build against the vendor libraries torch reaches on ROCm.

4096^3 by default (BASELINE configs[1]); interleaved rounds, median over rounds of the per-call mean.
  ours_dropin   op_mm_quantize (library workspace): quantize X and W + int8 MFMA GEMM + dequantize
  ours_gemm     qgemm_mm_packed on prepacked operands: the int8 GEMM + fused dequantize alone
  intmm         torch._int_mm (hipBLASLt int8 x int8 -> int32, B column-major), no dequantize
  llmint8_torch the same LLM.int8() vector-wise path composed from torch ops (amax, div, trunc, int8 cast,
                torch._int_mm, float dequantize) -- not bit-exact with the reference (no signed-seed absmax
                quirk), a timing point only
  bf16_mm       torch.matmul in bf16 (hipBLASLt, dense MFMA) for scale
Run on the GPU box: python scripts/vendor_compare.py [M N K]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _pkg  # noqa: E402

qg = _pkg.package(build=False)


def main():
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 4096, 4096)
    dev = torch.device("cuda:0")
    X = torch.empty((M, K), dtype=torch.float32, device=dev)
    W = torch.empty((K, N), dtype=torch.float32, device=dev)
    qg.fill_uniform(X, 11)
    qg.fill_uniform(W, 12)
    C = torch.empty((M, N), dtype=torch.float32, device=dev)
    pa, pb = qg.pack_a(X), qg.pack_b(W)
    a8 = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    b8 = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev).t()  # column-major K x N
    xb, wb = X.to(torch.bfloat16), W.to(torch.bfloat16)

    def llmint8_torch():
        cx = X.abs().amax(dim=1, keepdim=True)
        cw = W.abs().amax(dim=0, keepdim=True)
        xq = (X * (127.0 / cx)).trunc().to(torch.int8)
        wq = (W * (127.0 / cw)).trunc().to(torch.int8).t().contiguous().t()
        acc = torch._int_mm(xq, wq)
        return acc.float() * (cx * cw) * (1.0 / (127.0 * 127.0))

    variants = {
        "ours_dropin": lambda: qg.op_mm_quantize(X, W, C),
        "ours_gemm": lambda: qg.mm_packed(pa, pb, C),
        "intmm": lambda: torch._int_mm(a8, b8),
        "llmint8_torch": llmint8_torch,
        "bf16_mm": lambda: torch.matmul(xb, wb),
    }
    times = {k: [] for k in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    for f in variants.values():
        for _ in range(10):
            f()
    torch.cuda.synchronize()
    for _ in range(7):
        for name, f in variants.items():
            for _ in range(5):
                f()
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / reps * 1e3)
    ops = 2.0 * M * N * K
    print(f"M={M} N={N} K={K}  device {torch.cuda.get_device_name(0)}  torch {torch.__version__}  {qg.version()}")
    for name, ts in times.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"{name:14s} median {med:9.2f} us  min {ts[0]:9.2f} us  {ops / (med * 1e-6) / 1e12:8.1f} T(FL)OPS "
              f"{1e6 / med:9.0f} calls/s")


if __name__ == "__main__":
    main()
