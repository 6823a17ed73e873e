import torch, time
a = torch.randint(-127, 128, (4096, 4096), dtype=torch.int8, device="cuda")
b = torch.randint(-127, 128, (4096, 4096), dtype=torch.int8, device="cuda")
bt = b.t().contiguous().t()  # column-major B
for name, bb in (("row-major B", b), ("col-major B", bt)):
    try:
        for _ in range(20): c = torch._int_mm(a, bb)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        ts = []
        for r in range(5):
            e0.record()
            for _ in range(50): c = torch._int_mm(a, bb)
            e1.record(); e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 50 * 1e3)
        ts.sort()
        print(name, "median us", ts[2], "TOPS", 2 * 4096**3 / (ts[2] * 1e-6) / 1e12)
    except Exception as ex:
        print(name, "failed", ex)
