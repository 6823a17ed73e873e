"""Probe: a split-K op_mm_quantize_ws captured in a HIP graph and replayed several times.

Found: with the split-K tickets zeroed by hipMemsetAsync, the captured memset node
left a 16-byte pointer pattern in the ticket region on replay instead of zeros, so no slice became
the reducer and the output was never written; zeroing with a kernel node replays correctly.
Optional: WS_OFF=<bytes> places the workspace at an offset inside a larger allocation."""
import importlib, sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
qg = importlib.import_module("quantized-gemm-for-transformer-inference_amd")
L = qg.load()
dev = torch.device("cuda:0")
M, N, K = 512, 1024, 4096
X = torch.rand(M, K, device=dev) * 2 - 1
W = torch.rand(K, N, device=dev) * 2 - 1
need = L.op_mm_quantize_workspace_size(M, N, K)
OFF = int(os.environ.get("WS_OFF", "0"))
ws_big = torch.zeros(need + OFF, dtype=torch.uint8, device=dev)
ws = ws_big[OFF:]
O_ref = torch.empty(M, N, device=dev)
assert L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), N, 1, O_ref.data_ptr(), N, 1, M, N, K, 127.0,
                           ws.data_ptr(), ws.numel(), 0) == 0
torch.cuda.synchronize()
ws_eager = ws.clone()
O = torch.full((M, N), float("nan"), device=dev)
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rc = L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                                 ws.data_ptr(), ws.numel(), s.cuda_stream)
print("X", hex(X.data_ptr()), "W", hex(W.data_ptr()), "O_ref", hex(O_ref.data_ptr()), "ws_eager", hex(ws_eager.data_ptr()))
print("rc", rc, "ws bytes", need, "ptr", hex(ws.data_ptr()), "O", hex(O.data_ptr()))
sb = 4096 + 32 * 4 * 128 * 128 * 4
def region_diff(a, b, name):
    d = (a != b).nonzero()
    print(f"  {name}: {d.numel()} bytes differ" + (f", first at {d[0].item()} last {d[-1].item()}" if d.numel() else ""))
for r in range(3):
    O.fill_(float("nan"))
    torch.cuda.synchronize()
    TOFF = 32 * 4 * 128 * 128 * 4 if os.environ.get("QGEMM_DBG_END") else 0
    t0 = ws[TOFF:TOFF + 4096].view(torch.int32).clone()
    g.replay()
    torch.cuda.synchronize()
    t1 = ws[TOFF:TOFF + 4096].view(torch.int32).clone()
    print("replay", r, "tickets before", t0[:6].tolist(), "after", t1[:6].tolist(),
          "nonzero tickets after", int((t1 != 0).sum()), "nan frac", torch.isnan(O).float().mean().item(),
          "equal", torch.equal(O, O_ref), flush=True)
    region_diff(ws[sb:], ws_eager[sb:], "packed A/B vs eager")
    if r == 0:
        q = ws[:4096].view(torch.int64).tolist()
        print("  ticket words as u64:", [hex(v & (2**64 - 1)) for v in q[:24]])
        print("  distinct:", sorted(set(hex(v & (2**64 - 1)) for v in q)))
        full = ws[:sb + 64].view(torch.int64)
        print("  slab head u64:", [hex(v & (2**64 - 1)) for v in full[512:520].tolist()])
print("alloc head nonzero:", int((ws_big[:4096] != 0).sum()), "ticket region nonzero:", int((ws[:4096] != 0).sum()))
# no replay: do torch ops alone disturb the ticket region?
ws[:4096].zero_()
torch.cuda.synchronize()
for _ in range(3):
    O.fill_(float("nan")); torch.isnan(O).float().mean().item()
torch.cuda.synchronize()
print("torch ops only: nonzero tickets", int((ws[:4096] != 0).sum()))
