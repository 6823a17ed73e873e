import os, sys, time
sys.path.insert(0, "tests")
import torch, _pkg
qg = _pkg.package()
dev = torch.device("cuda", 0)
res = []
for (M, N, K) in [(512, 3072, 1024), (512, 1024, 1024), (512, 4096, 1024), (512, 1024, 4096), (2048, 2048, 2048)]:
    X = qg.fill_uniform(torch.empty((M, K), device=dev), seed=1)
    W = qg.fill_uniform(torch.empty((K, N), device=dev), seed=2)
    pa, pb = qg.pack_a(X), qg.pack_b(W)
    O = torch.empty((M, N), device=dev)
    for _ in range(20): qg.mm_packed(pa, pb, O)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): qg.mm_packed(pa, pb, O)
    e1.record(); e1.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1000
    res.append(f"{M}x{N}x{K}: {us:.1f} us ({2*M*N*K/us/1e6:.0f} TOPS)")
print(os.environ.get("QGEMM_SPLIT_MAX"), " | ".join(res))
