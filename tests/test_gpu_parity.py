"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit for bit.

Every test here runs the product path -- libqgemm.so's gfx950 kernels -- and compares with the
oracle (tests only) or the committed fixtures.  Bar: O, Xq, Wq, Acc bit-identical; scales Cx/Cw
value-identical (their zero sign never reaches O: fl(Cx*Cw)+0 is +0 either way).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from util import assert_bits_equal, assert_values_equal, load_cases, load_kat

pytestmark = pytest.mark.gpu


def _dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _run_full(qg, X, W, device):
    Xd, Wd = _dev(X, device), _dev(W, device)
    O = torch.full((X.shape[0], W.shape[1]), float("nan"), device=device)  # poisoned
    qg.op_quantized_mm(Xd, Wd, O, 127.0)
    torch.cuda.synchronize()
    return O.cpu().numpy()


def _check_intermediates(qg, X, W, ref, device, name):
    Xd, Wd = _dev(X, device), _dev(W, device)
    pa, pb = qg.pack_a(Xd), qg.pack_b(Wd)
    M, K = X.shape
    N = W.shape[1]
    torch.cuda.synchronize()
    assert_values_equal(pa.scale[:M].cpu().numpy(), ref["Cx"], f"{name} Cx")
    assert_values_equal(pb.scale[:N].cpu().numpy(), ref["Cw"], f"{name} Cw")
    qa, qb = pa.q.cpu().numpy(), pb.q.cpu().numpy()
    assert (qa[:M, :K] == ref["Xq"]).all(), f"{name} Xq"
    assert (qb[:N, :K] == ref["Wq"].T).all(), f"{name} Wq"
    assert not qa[M:].any() and not qa[:, K:].any(), f"{name} A padding not zero"
    assert not qb[N:].any() and not qb[:, K:].any(), f"{name} B padding not zero"
    acc = qg.mm_packed_i32(pa, pb).cpu().numpy()
    assert (acc == ref["Acc"]).all(), f"{name} Acc"


def test_kat1_reference_fixture(qg, device):
    k = load_kat()["kat1"]
    X, W = np.array(k["X"], np.float32), np.array(k["W"], np.float32)
    want = np.array([int(b, 16) for b in k["O_bits"]], np.uint32).view(np.float32).reshape(3, 2)
    assert_bits_equal(_run_full(qg, X, W, device), want, "KAT-1")
    C = qg.mm_fp32(_dev(X, device), _dev(W, device)).cpu().numpy()
    assert C.tolist() == k["unquantized"]


def test_explicit_edge_fixtures(qg, device):
    """Quirk (with/without int8 overflow), zero rows/cols, NaN/inf, K=1, M=1, N=1, extremes."""
    index, arrays = load_cases()
    for rec in index:
        if rec["kind"] != "explicit":
            continue
        n = rec["name"]
        X, W = arrays[n + "/X"], arrays[n + "/W"]
        assert_bits_equal(_run_full(qg, X, W, device), arrays[n + "/O"], n)
        ref = {key: arrays[f"{n}/{key}"] for key in ("Cx", "Cw", "Xq", "Wq", "Acc")}
        _check_intermediates(qg, X, W, ref, device, n)


def test_seeded_fixtures(qg, oracle, device):
    index, _ = load_cases()
    for rec in index:
        if rec["kind"] != "seeded":
            continue
        X, W = oracle.inputs(rec["M"], rec["N"], rec["K"], rec["seed"])
        O, ref = oracle.quantized_mm(X, W, intermediates=True)
        assert_bits_equal(_run_full(qg, X, W, device), O, rec["name"])
        _check_intermediates(qg, X, W, ref, device, rec["name"])


@pytest.mark.parametrize("M,N,K", [(512, 768, 384), (1000, 300, 1030), (64, 4096, 256), (2048, 2048, 2048),
                                   (64, 96, 5003), (33, 40, 16384), (300, 64, 8191),   # long rows: block per row
                                   (40, 72, 40000), (9, 24, 70001)])                   # past 16384: streaming rows
def test_random_shapes_full_oracle(qg, oracle, device, M, N, K):
    X, W = oracle.inputs(M, N, K, 21)
    assert_bits_equal(_run_full(qg, X, W, device), oracle.quantized_mm(X, W), f"{M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(130, 264, 1500), (70, 200, 600), (300, 4104, 4096), (96, 8192, 1025),
                                   (1, 8, 2), (33, 24, 4096), (257, 1032, 3000)])
def test_single_pass_8_column_strips(qg, oracle, device, M, N, K):
    """Shapes on the single-pass pack with 8-column W strips (n % 8 == 0 and n <= 8192 with K > 1024,
    or n % 16 != 0): buffer loads past the last row read zeros, padding strips, odd strip counts over
    the XCD map; W columns whose signed first element is the largest magnitude (absmax seed quirk)."""
    X, W = oracle.inputs(M, N, K, 61)
    W[0, ::3] = -1.75  # seed quirk in every third column (int8 saturation on the quantize)
    X[::5, 0] = -1.5
    O, ref = oracle.quantized_mm(X, W, intermediates=True)
    assert_bits_equal(_run_full(qg, X, W, device), O, f"{M}x{N}x{K}")
    _check_intermediates(qg, X, W, ref, device, f"{M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(64, 64, 128), (100, 200, 256), (512, 512, 384), (512, 1024, 1024),
                                   (512, 3072, 1024), (130, 70, 640), (512, 4096, 1024)])
def test_small_tiles_three_stage_ring(qg, oracle, device, M, N, K):
    """64-tile GEMM with the 3-stage LDS ring (<= 512 tiles): one, two and three k-steps (the prologue's
    clamped re-loads of the last k-step), ragged M/N edges, and the encoder's linear shapes."""
    X, W = oracle.inputs(M, N, K, 27)
    assert_bits_equal(_run_full(qg, X, W, device), oracle.quantized_mm(X, W), f"{M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(256, 256, 4096), (200, 300, 8192), (512, 1024, 4096), (300, 520, 1000)])
def test_split_k_shapes_repeated(qg, oracle, device, M, N, K):
    """Few-tile shapes run split-K (int32 slabs + arrival tickets, combined in-launch): exact integer
    sums, so bit-identical to the oracle; repeated calls reuse the tickets (zeroed per launch) and
    the slabs with caches warm from the previous call."""
    X, W = oracle.inputs(M, N, K, 71)
    want = oracle.quantized_mm(X, W)
    Xd, Wd = _dev(X, device), _dev(W, device)
    pa, pb = qg.pack_a(Xd), qg.pack_b(Wd)
    for i in range(3):
        O = torch.full((M, N), float("nan"), device=device)
        qg.mm_packed(pa, pb, O)
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} mm_packed call {i}")
    assert_bits_equal(_run_full(qg, X, W, device), want, f"{M}x{N}x{K} op_quantized_mm")


@pytest.mark.parametrize("M,N,K,layout", [(256, 256, 4096, "rows"), (300, 520, 4500, "rows"), (256, 512, 4096, "rows"),
                                          (256, 256, 4096, "generic")])
def test_split_k_poisoned_caller_workspace(qg, oracle, device, M, N, K, layout):
    """op_mm_quantize_ws on a workspace full of 0xFF at split-K shapes: the split-K tickets at its start
    are zeroed by the pack launch (single pass, or the row/column-absmax launch for K > 4096) or by the
    GEMM's own zeroing launch (generic strides: separate pack launches)."""
    X, W = oracle.inputs(M, N, K, 91)
    want = oracle.quantized_mm(X, W)
    L = qg.load()
    Xd, Wd = _dev(X, device), _dev(W, device)
    if layout == "generic":  # every other column of a wider buffer: the strided (fallback) pack path
        Xd = _dev(np.repeat(X, 2, axis=1), device)[:, ::2]
    a256 = lambda b: (b + 255) // 256 * 256  # noqa: E731
    assert L.op_mm_quantize_workspace_size(M, N, K) > a256(L.qgemm_packed_size(M, K)) + a256(L.qgemm_packed_size(N, K)), \
        "shape expected to run split-K"
    ws = torch.full((L.op_mm_quantize_workspace_size(M, N, K),), 255, dtype=torch.uint8, device=device)
    s = qg._stream(device)
    for i in range(2):
        O = torch.full((M, N), float("nan"), device=device)
        rc = L.op_mm_quantize_ws(Xd.data_ptr(), Xd.stride(0), Xd.stride(1), Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M,
                                 N, K, 127.0, ws.data_ptr(), ws.numel(), s)
        assert rc == 0
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} {layout} call {i}")
        ws.fill_(255)


@pytest.mark.parametrize("M,N,K", [(64, 8196, 300), (33, 12288, 4096), (128, 16384, 1000), (5, 9000, 2049),
                                   (300, 8704, 513), (300, 16384, 3001), (64, 16384, 2500), (257, 32768, 4096),
                                   (96, 16416, 3073), (1, 16384, 4096)])
def test_wide_w_pack_poisoned_workspace(qg, oracle, device, M, N, K):
    """Wide W (n > 8192, 256 < K <= 4096, the FFN-up shape class) on a workspace full of 0xFF, twice:
    16-column strips, n % 16 != 0 (8-column strips), K not a multiple of 128; n >= 16384 with K > 2048:
    the 32-column pass (rows >= 3072 through LDS; K % 4 != 0, K just past the register rows, n not a
    power of two, one row of X)."""
    X, W = oracle.inputs(M, N, K, 93)
    want = oracle.quantized_mm(X, W)
    L = qg.load()
    Xd, Wd = _dev(X, device), _dev(W, device)
    ws = torch.full((L.op_mm_quantize_workspace_size(M, N, K),), 255, dtype=torch.uint8, device=device)
    s = qg._stream(device)
    for i in range(2):
        O = torch.full((M, N), float("nan"), device=device)
        rc = L.op_mm_quantize_ws(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                                 ws.data_ptr(), ws.numel(), s)
        assert rc == 0
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} call {i}")
        ws.fill_(255)
    assert_bits_equal(_run_full(qg, X, W, device), want, f"{M}x{N}x{K} op_quantized_mm")


def test_split_k_shapes_share_library_scratch(qg, oracle, device):
    """Different split-K plans one after another on the same stream share qgemm_mm_packed's scratch
    (tickets zeroed once, re-zeroed by each launch's reducers): every call stays bit-exact."""
    shapes = [(512, 1024, 4096), (64, 512, 8192), (256, 256, 4096), (512, 3072, 1024), (512, 1024, 4096), (64, 512, 8192)]
    cache = {}
    for i, (M, N, K) in enumerate(shapes):
        if (M, N, K) not in cache:
            X, W = oracle.inputs(M, N, K, 101 + len(cache))
            cache[(M, N, K)] = (X, W, oracle.quantized_mm(X, W))
        X, W, want = cache[(M, N, K)]
        O = qg.mm_packed(qg.pack_a(_dev(X, device)), qg.pack_b(_dev(W, device)))
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"call {i}: {M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(4000, 4100, 1000), (3900, 2600, 700), (4096, 2610, 100), (3333, 4095, 800)])
def test_256_tile_kernel_ragged_shapes(qg, oracle, device, M, N, K):
    """>= 160 tiles of 256 x 256 (gemm_i8_fm, no split): ragged M and N (partial edge tiles take the guarded
    store path), and K padded to 2 / 12 / 14 / 16 sub-steps of 64 (the main loop's 3-sub-step unroll leaves
    rest 2 / 0 / 2 / 1, and at 2 sub-steps it never runs)."""
    L = qg.load()
    tile = ctypes.c_int(0)
    assert L.qgemm_gemm_plan(M, N, K, ctypes.byref(tile), None) == 1 and tile.value == 256
    X, W = oracle.inputs(M, N, K, 141)
    X[::9, 0] = -1.25
    assert_bits_equal(_run_full(qg, X, W, device), oracle.quantized_mm(X, W), f"{M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(300, 1000, 5000), (257, 4104, 8193), (64, 520, 16384), (512, 2048, 12289)])
def test_long_k_drop_in(qg, oracle, device, M, N, K):
    """4096 < K <= 16384, row-major operands (the two-pass column pack of W and the fused X-row pass) -- ragged K,
    the largest K, padding rows of the packed W (N not a multiple of 256), signed-seed quirk rows and columns;
    every output bit."""
    X, W = oracle.inputs(M, N, K, 151)
    W[0, ::5] = -1.75  # those columns' signed seed (absmax quirk)
    X[::7, 0] = -1.5
    assert_bits_equal(_run_full(qg, X, W, device), oracle.quantized_mm(X, W), f"{M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 2048), (1900, 4000, 3000), (1800, 4096, 4500)])
def test_256_tile_split_k_plans(qg, oracle, device, M, N, K):
    """128 tiles of 256 x 256 with K >= 2048: the split-K plan (S = 2) on gemm_i8_fm, ticket-first (round 4) --
    the slice that draws the ticket first stores its slab write-through from the AGPR accumulators and publishes
    it; the other adds it and runs the epilogue.  Ragged M / N / K edges, K > 4096 (two-pass pack); library
    scratch twice (the second arriver resets the ticket), then a caller workspace full of 0xFF (tickets zeroed by
    the pack launch)."""
    L = qg.load()
    assert L.qgemm_gemm_plan(M, N, K, None, None) == 2, "shape expected to run the 256-tile split-K plan"
    X, W = oracle.inputs(M, N, K, 131)
    X[::7, 0] = -1.5
    want = oracle.quantized_mm(X, W)
    Xd, Wd = _dev(X, device), _dev(W, device)
    pa, pb = qg.pack_a(Xd), qg.pack_b(Wd)
    for i in range(2):
        O = torch.full((M, N), float("nan"), device=device)
        qg.mm_packed(pa, pb, O)
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} mm_packed call {i}")
    ws = torch.full((L.op_mm_quantize_workspace_size(M, N, K),), 255, dtype=torch.uint8, device=device)
    O = torch.full((M, N), float("nan"), device=device)
    assert L.op_mm_quantize_ws(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                               ws.data_ptr(), ws.numel(), qg._stream(device)) == 0
    torch.cuda.synchronize()
    assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} caller workspace")


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 2048), (2048, 4096, 16384)])
def test_256_tile_split_k_ticket_first_repeat(qg, oracle, device, M, N, K):
    """Race screen of the ticket-first split-K hand-off (gemm_i8_fm<kSplitFirst>): 20 back-to-back calls on the
    library scratch (each second arriver polls for the first's publish, then resets the ticket for the next
    launch), every output bit of every call.  The slices of a tile finish within a few microseconds of each
    other; K = 2048 makes the two slices nearly equal (15 and 17 sub-steps).  Slice 0 usually arrives first
    here; the reverse order (slice 1 publishes while slice 0 waits) is forced by test_split_k_both_arrival_orders."""
    L = qg.load()
    assert L.qgemm_gemm_plan(M, N, K, None, None) == 2
    X, W = oracle.inputs(M, N, K, 57)
    want = oracle.quantized_mm(X, W)
    pa, pb = qg.pack_a(_dev(X, device)), qg.pack_b(_dev(W, device))
    outs = [torch.full((M, N), float("nan"), device=device) for _ in range(20)]
    for O in outs:
        qg.mm_packed(pa, pb, O)
    torch.cuda.synchronize()
    for i, O in enumerate(outs):
        assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} repeat {i}")


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 2048), (2048, 4096, 16384)])
def test_split_k_both_arrival_orders(qg, device, M, N, K):
    """The ticket-first hand-off with the K split skewed both ways (build/splitk_order_check: the product kernel
    instantiated with slice 0 = 8/64 of K -- slice 0 publishes -- 31/64 -- the product -- and 56/64 -- slice 1
    finishes first and publishes while slice 0 spins), 20 calls each on one reused scratch: every output bit
    equals the unsplit kernel's, and every ticket is back to 0."""
    import json
    import subprocess
    exe = os.path.join(qg.PKG_DIR, "build", "splitk_order_check")
    r = subprocess.run([exe, str(M), str(N), str(K), "20"], capture_output=True, text=True, timeout=120)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["ok"], out
    assert [v["first64"] for v in out["variants"]] == [8, 31, 56]


def test_device_generator_matches_oracle(qg, oracle, device):
    t = torch.empty(1 << 20, device=device)
    qg.fill_uniform(t, seed=9)
    assert_bits_equal(t.cpu().numpy(), oracle.uniform((1 << 20,), seed=9), "fill_uniform")


# BASELINE configs at full size: C2 4096^3 (one 256x256 tile per CU), C3 FFN up / down (down: K > 4096,
# the two-pass pack and split-K), the C4 shard 8192 x 4096 x 4096 (two tiles per CU) -- every output bit.
@pytest.mark.parametrize("M,N,K,cfg", [(4096, 4096, 4096, "c2"), (2048, 16384, 4096, "c3_up"),
                                       (2048, 4096, 16384, "c3_down"), (8192, 4096, 4096, "c4_shard")])
def test_full_size_every_output(qg, oracle, device, M, N, K, cfg):
    """Inputs generated on the GPU (bit-identical to the oracle's generator); the WHOLE output compared
    bit for bit with the oracle's chain on the same inputs.  C2 goes through the flat north-star entry
    point op_mm_quantize(A, B, C, M, N, K) on the null stream, the others through the Python mirror."""
    X = qg.fill_uniform(torch.empty((M, K), device=device), seed=2 * 31)
    W = qg.fill_uniform(torch.empty((K, N), device=device), seed=2 * 31 + 1)
    if cfg == "c2":
        O = torch.full((M, N), float("nan"), device=device)
        torch.cuda.synchronize()
        assert qg.load().op_mm_quantize(X.data_ptr(), W.data_ptr(), O.data_ptr(), M, N, K) == 0
    else:
        O = qg.op_mm_quantize(X, W)
    torch.cuda.synchronize()
    Xh, Wh = oracle.uniform((M, K), 2 * 31), oracle.uniform((K, N), 2 * 31 + 1)
    assert_bits_equal(X.cpu().numpy(), Xh, "X generation")
    assert_bits_equal(W.cpu().numpy(), Wh, "W generation")
    assert_bits_equal(O.cpu().numpy(), oracle.quantized_mm(Xh, Wh), f"{cfg} {M}x{N}x{K} full output")


def test_output_past_2_31_elements(qg, oracle, device):
    """A 65536 x 36864 output (2.42e9 elements, 9.7 GB: element offsets past 2^31) from K = 128: the sampled rows whose
    offsets row * N exceed 2^31, the last row and a few below it, bit for bit against the oracle's row restatement
    (its Cw over the whole W).  Exercises the 64-bit output addressing of the epilogue at a size the 288-GB HBM holds."""
    M, N, K = 65536, 36864, 128
    X = qg.fill_uniform(torch.empty((M, K), device=device), seed=2 * 53)
    W = qg.fill_uniform(torch.empty((K, N), device=device), seed=2 * 53 + 1)
    O = torch.full((M, N), float("nan"), device=device)
    torch.cuda.synchronize()
    assert qg.load().op_mm_quantize(X.data_ptr(), W.data_ptr(), O.data_ptr(), M, N, K) == 0
    torch.cuda.synchronize()
    first_past = (1 << 31) // N + 1  # the first row whose every element lies past 2^31
    rows = np.unique(np.concatenate([[0, first_past - 1, first_past, M - 1],
                                     np.linspace(first_past, M - 1, 28).astype(np.int64)]))
    got = O[torch.from_numpy(rows).to(device)].cpu().numpy()
    del O
    Xh, Wh = oracle.uniform((M, K), 2 * 53), oracle.uniform((K, N), 2 * 53 + 1)
    assert_bits_equal(got, oracle.quantized_mm_rows(Xh, Wh, rows.astype(np.int32)), f"{M}x{N}x{K} rows past 2^31")


@pytest.mark.parametrize("M,N", [(0, 64), (64, 0), (0, 0)])
def test_empty_output_is_a_no_op(qg, device, M, N):
    """M = 0 or N = 0: nothing to compute -- the call returns 0 and touches no memory (the caller's buffers keep their
    poison), through the flat entry point, the workspace form and the Python mirror."""
    K = 32
    X = torch.full((max(M, 1), K), 1.0, device=device)
    W = torch.full((K, max(N, 1)), 1.0, device=device)
    O = torch.full((8,), float("nan"), device=device)
    L = qg.load()
    torch.cuda.synchronize()
    assert L.op_mm_quantize(X.data_ptr(), W.data_ptr(), O.data_ptr(), M, N, K) == 0
    ws = torch.empty(max(1, L.op_mm_quantize_workspace_size(M, N, K)), dtype=torch.uint8, device=device)
    assert L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), max(N, 1), 1, O.data_ptr(), max(N, 1), 1, M, N, K, 127.0,
                               ws.data_ptr(), ws.numel(), None) == 0
    out = qg.op_mm_quantize(X[:M], W[:, :N])
    torch.cuda.synchronize()
    assert tuple(out.shape) == (M, N)
    assert torch.isnan(O).all()


def _uniform_rows(seed, rows, K):
    """Rows `rows` of oracle.uniform((M, K), seed) on the host without the whole matrix: the counter generator of
    oracle_uniform_at (qgemm_oracle.c), element i = row * K + col, U[-1, 1) = fl(fl(u - 0.5) * 2) (exact)."""
    c = np.uint64(0x9E3779B97F4A7C15)

    def mix64(z):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

    with np.errstate(over="ignore"):
        key = mix64(np.uint64(seed) + c)
        i = np.asarray(rows, np.uint64)[:, None] * np.uint64(K) + np.arange(K, dtype=np.uint64)[None, :]
        z = mix64(key + (i + np.uint64(1)) * c)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (u + np.float32(-0.5)) * np.float32(2.0)


def test_input_past_2_31_elements(qg, oracle, device):
    """X of 600000 x 4096 (2.46e9 elements, 9.8 GB: input offsets past 2^31; packed A 2.46 GB) times a 4096 x 256 W:
    sampled rows past the 2^31-th element of X, bit for bit against the oracle (each output row needs only its X row
    and W's column scales).  The sampled X rows are regenerated on the host and checked against the device's first."""
    M, N, K = 600000, 256, 4096
    X = qg.fill_uniform(torch.empty((M, K), device=device), seed=2 * 59)
    W = qg.fill_uniform(torch.empty((K, N), device=device), seed=2 * 59 + 1)
    O = torch.full((M, N), float("nan"), device=device)
    torch.cuda.synchronize()
    assert qg.load().op_mm_quantize(X.data_ptr(), W.data_ptr(), O.data_ptr(), M, N, K) == 0
    torch.cuda.synchronize()
    first_past = (1 << 31) // K + 1
    rows = np.unique(np.concatenate([[0, first_past - 1, first_past, M - 1],
                                     np.linspace(first_past, M - 1, 28).astype(np.int64)]))
    idx = torch.from_numpy(rows).to(device)
    got, xdev = O[idx].cpu().numpy(), X[idx].cpu().numpy()
    del O, X
    Xs = _uniform_rows(2 * 59, rows, K)
    assert_bits_equal(xdev, Xs, "X rows generation")
    Wh = oracle.uniform((K, N), 2 * 59 + 1)
    assert_bits_equal(got, oracle.quantized_mm_rows(Xs, Wh, np.arange(len(rows), dtype=np.int32)),
                      f"{M}x{N}x{K} rows past 2^31 input elements")


def test_strided_views(qg, oracle, device):
    """Transposed and sliced views, as the reference's Index() macro allows (tensor.cuh:121-149)."""
    M, N, K = 200, 150, 260
    X, W = oracle.inputs(M, N, K, 33)
    want = oracle.quantized_mm(X, W)
    Xt = _dev(np.ascontiguousarray(X.T), device).T      # X column-major  -> pack_cols path for A
    Wt = _dev(np.ascontiguousarray(W.T), device).T      # W column-major  -> pack_rows path for B
    big = torch.full((M + 7, N + 9), float("nan"), device=device)
    O = big[3:3 + M, 5:5 + N]                           # strided output
    qg.op_quantized_mm(Xt, Wt, O, 127.0)
    torch.cuda.synchronize()
    assert_bits_equal(O.cpu().numpy(), want, "transposed operands, sliced output")
    assert torch.isnan(big[:3]).all() and torch.isnan(big[:, :5]).all(), "wrote outside the view"
    # fully generic strides (every other column of a wider buffer)
    Xw = _dev(np.repeat(X, 2, axis=1), device)[:, ::2]
    Ww = _dev(np.repeat(W, 2, axis=0), device)[::2]
    O2 = torch.empty((M, N), device=device).T.contiguous().T  # column-major output
    qg.op_quantized_mm(Xw, Ww, O2, 127.0)
    torch.cuda.synchronize()
    assert_bits_equal(O2.cpu().numpy(), want, "generic strides, column-major output")


def test_c_abi_null_stream_entry_point(qg, oracle, device):
    """The flat op_mm_quantize(A,B,C,M,N,K) on the null stream, as a C caller would use it."""
    M, N, K = 300, 257, 129
    X, W = oracle.inputs(M, N, K, 41)
    Xd, Wd = _dev(X, device), _dev(W, device)
    O = torch.empty((M, N), device=device)
    torch.cuda.synchronize()
    rc = qg.load().op_mm_quantize(Xd.data_ptr(), Wd.data_ptr(), O.data_ptr(), M, N, K)
    assert rc == 0
    torch.cuda.synchronize()
    assert_bits_equal(O.cpu().numpy(), oracle.quantized_mm(X, W), "op_mm_quantize")


def test_explicit_workspace_and_prepacked_weights(qg, oracle, device):
    M, N, K = 384, 512, 640
    X, W = oracle.inputs(M, N, K, 51)
    want = oracle.quantized_mm(X, W)
    L = qg.load()
    Xd, Wd = _dev(X, device), _dev(W, device)
    ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=device)
    O = torch.empty((M, N), device=device)
    s = qg._stream(device)
    rc = L.op_mm_quantize_ws(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                             ws.data_ptr(), ws.numel(), s)
    assert rc == 0
    torch.cuda.synchronize()
    assert_bits_equal(O.cpu().numpy(), want, "explicit workspace")
    pb = qg.pack_b(Wd)  # weight packed once, reused
    for _ in range(2):
        O2 = qg.mm_packed(qg.pack_a(Xd), pb)
        torch.cuda.synchronize()
        assert_bits_equal(O2.cpu().numpy(), want, "prepacked B")


@pytest.mark.parametrize("M,N,K", [(384, 512, 640), (1000, 300, 1), (4096, 4096, 4096), (512, 1024, 4096)])
def test_op_mm_quantize_prepacked(qg, oracle, device, M, N, K):
    """op_mm_quantize_prepacked (W packed once, A quantized per call) is the drop-in bit
    for bit -- the 4096^3 headline (every output) and a split-K shape included; both C-ABI forms."""
    X, W = oracle.inputs(M, N, K, 57)
    want = oracle.quantized_mm(X, W)
    Xd, Wd = _dev(X, device), _dev(W, device)
    pb = qg.pack_b(Wd)
    for _ in range(2):
        O = qg.op_mm_quantize_prepacked(Xd, pb)
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"op_mm_quantize_prepacked_ws {M}x{N}x{K}")
    O2 = torch.full((M, N), float("nan"), device=device)
    assert qg.load().op_mm_quantize_prepacked(Xd.data_ptr(), pb.buf.data_ptr(), O2.data_ptr(), M, N, K) == 0
    torch.cuda.synchronize()
    assert_bits_equal(O2.cpu().numpy(), want, f"op_mm_quantize_prepacked {M}x{N}x{K}")


def test_unquantized_gemm_matches_reference_order(qg, oracle, device):
    """qgemm_mm_fp32 is the reference's op_mm<float,float>: sequential-k fmaf, bit-exact (on the f32
    MFMA: every tile configuration, k % 4 / k % 32 tails, K = 1)."""
    for M, N, K in [(100, 70, 96), (33, 65, 130), (512, 512, 64), (257, 300, 1000), (1, 77, 33), (64, 1, 5),
                    (5, 3, 1), (640, 640, 128), (2048, 1024, 64)]:
        X, W = oracle.inputs(M, N, K, 61)
        C = qg.mm_fp32(_dev(X, device), _dev(W, device)).cpu().numpy()
        assert_bits_equal(C, oracle.mm_fp32(X, W), f"fp32 {M}x{N}x{K}")


def test_unquantized_gemm_strided_views(qg, oracle, device):
    """Column-major / transposed operand views (the attention Q K^T form) stage through the other LDS
    layout; same bits as the contiguous oracle on the same logical matrices."""
    M, N, K = 192, 160, 200
    X, W = oracle.inputs(M, N, K, 62)
    want = oracle.mm_fp32(X, W)
    Xc = _dev(np.ascontiguousarray(X.T), device).t()  # stride (1, M)
    Wc = _dev(np.ascontiguousarray(W.T), device).t()  # stride (1, K)
    for a, b, what in [(Xc, _dev(W, device), "A col-major"), (_dev(X, device), Wc, "B col-major"), (Xc, Wc, "both")]:
        assert_bits_equal(qg.mm_fp32(a, b).cpu().numpy(), want, f"fp32 views: {what}")


def test_unquantized_gemm_special_values(qg, oracle, device):
    """Underflowing products (-0 and subnormal results), +-inf and NaN operands: the MFMA chain keeps
    the fmaf chain's bits (subnormals are not flushed; a -0 result becomes +0 only through the
    reference's zero-padded tail)."""
    rng = np.random.default_rng(63)
    for M, N, K in [(48, 40, 64), (48, 40, 36), (40, 48, 7)]:
        X = (rng.uniform(-1, 1, (M, K)) * 1e-20).astype(np.float32)
        W = (rng.uniform(-1, 1, (K, N)) * 1e-20).astype(np.float32)
        W[:, :8] *= np.float32(1e-6)   # products far below the smallest subnormal: signed zeros
        X[:4, :] *= np.float32(1e19)   # some rows land in the subnormal range
        X[5, 3] = np.inf
        X[6, 2] = -np.inf
        W[1, 9] = np.nan
        W[2, 11] = np.inf
        want = oracle.mm_fp32(X, W)
        got = qg.mm_fp32(_dev(X, device), _dev(W, device)).cpu().numpy()
        assert_bits_equal(got, want, f"fp32 special {M}x{N}x{K}")
        assert (np.signbit(want) & (want == 0)).any() or K % 32, "case should produce -0 results"


def test_device_error_stats_match_oracle(qg, oracle, device):
    """the reference's error metric on the device.  The reference-order signed mean is
    bit-identical to the sequential fp32 restatement; the fp64 statistics agree to rounding."""
    M, N, K = 300, 257, 129
    X, W = oracle.inputs(M, N, K, 81)
    C_ref, O_ref = oracle.mm_fp32(X, W), oracle.quantized_mm(X, W)
    want = oracle.error_stats(C_ref, O_ref)
    Xd, Wd = _dev(X, device), _dev(W, device)
    C = qg.mm_fp32(Xd, Wd)
    O = torch.empty((M, N), device=device)
    qg.op_quantized_mm(Xd, Wd, O, 127.0)
    got = qg.error_stats(C, O, reference_order=True)
    assert np.float32(got["signed_mean_ref"]).tobytes() == np.float32(want["signed_mean"]).tobytes()
    for key in ("mean_abs", "max_abs", "rel"):
        assert got[key] == pytest.approx(want[key], rel=1e-9, abs=0), key  # fp64 sums, different order
    # fp64 signed mean vs the fp32 sequential one: same quantity, different rounding
    assert got["signed_mean"] == pytest.approx(want["signed_mean"], rel=1e-3, abs=1e-7)
    fast = qg.error_stats(C, O)
    assert np.isnan(fast["signed_mean_ref"]) and fast["mean_abs"] == got["mean_abs"]


def test_harness_binary_reproduces_reference_output(qg):
    import os
    import subprocess
    exe = os.path.join(qg.PKG_DIR, "build", "test_quantize")
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    lines = [ln.strip() for ln in out.splitlines()]
    q = lines.index("Quantized result:")
    assert lines[q + 1].split() == ["-1.007874", "0.000000"]
    assert lines[q + 2].split() == ["-1.984252", "-2.031496"]
    assert lines[q + 3].split() == ["1.000000", "2.000000"]
    e = lines.index("Mean quantization error:")
    assert abs(float(lines[e + 1]) - 0.003937006) < 1e-8
    assert "All tests completed successfully!" in lines


def test_hip_graph_capture_replays_bit_exact(qg, oracle, device):
    """op_mm_quantize_ws with a caller workspace makes no allocation and no host sync, so it can be
    captured in a HIP graph (torch.cuda.CUDAGraph) and replayed; split-K shapes included (their ticket
    memset is a graph node)."""
    L = qg.load()
    for (M, N, K) in [(384, 512, 640), (512, 1024, 4096)]:
        X, W = oracle.inputs(M, N, K, 111)
        want = oracle.quantized_mm(X, W)
        Xd, Wd = _dev(X, device), _dev(W, device)
        ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=device)
        O = torch.full((M, N), float("nan"), device=device)
        s = torch.cuda.Stream(device)
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                rc = L.op_mm_quantize_ws(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                                         ws.data_ptr(), ws.numel(), s.cuda_stream)
                assert rc == 0
        for _ in range(3):
            O.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize()
            assert_bits_equal(O.cpu().numpy(), want, f"graph replay {M}x{N}x{K}")


def test_prepacked_graph_capture(qg, oracle, device):
    """op_mm_quantize_prepacked_ws (caller workspace, W packed once outside the graph) captured and replayed."""
    L = qg.load()
    for (M, N, K) in [(384, 512, 640), (512, 1024, 4096)]:
        X, W = oracle.inputs(M, N, K, 113)
        want = oracle.quantized_mm(X, W)
        Xd, Wd = _dev(X, device), _dev(W, device)
        pb = qg.pack_b(Wd)
        ws = torch.empty(max(1, L.op_mm_quantize_prepacked_workspace_size(M, N, K)), dtype=torch.uint8, device=device)
        O = torch.full((M, N), float("nan"), device=device)
        torch.cuda.synchronize()
        s = torch.cuda.Stream(device)
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                assert L.op_mm_quantize_prepacked_ws(Xd.data_ptr(), K, pb.buf.data_ptr(), O.data_ptr(), N, M, N, K,
                                                     ws.data_ptr(), ws.numel(), s.cuda_stream) == 0
        for _ in range(3):
            O.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize()
            assert_bits_equal(O.cpu().numpy(), want, f"prepacked graph replay {M}x{N}x{K}")


def test_concurrent_streams_with_own_workspaces(qg, oracle, device):
    L = qg.load()
    M, N, K = 512, 1024, 4096  # split-K plan on both streams
    cases = []
    for i in range(2):
        X, W = oracle.inputs(M, N, K, 120 + i)
        cases.append((_dev(X, device), _dev(W, device), oracle.quantized_mm(X, W),
                      torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=device),
                      torch.empty((M, N), device=device), torch.cuda.Stream(device)))
    torch.cuda.synchronize()
    for _ in range(5):
        for Xd, Wd, _, ws, O, s in cases:
            rc = L.op_mm_quantize_ws(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                                     ws.data_ptr(), ws.numel(), s.cuda_stream)
            assert rc == 0
    torch.cuda.synchronize()
    for i, (_, _, want, _, O, _) in enumerate(cases):
        assert_bits_equal(O.cpu().numpy(), want, f"stream {i}")


@pytest.mark.parametrize("M,N,K", [(1024, 1024, 1024), (512, 1024, 4096)])  # plain plan; split-K plan
def test_implicit_workspace_two_streams(qg, oracle, device, M, N, K):
    """op_mm_quantize_ex WITHOUT a workspace, on two streams back to back with different inputs
    of one shape -- the library's cached workspace is per (device, stream), so the two streams never share packed
    operands or split-K tickets (the reference allocates per call, op_mm.cuh:76-93).  Then the flat entry point on
    the null stream beside them."""
    L = qg.load()
    cases = []
    for i in range(2):
        X, W = oracle.inputs(M, N, K, 140 + i)
        cases.append((_dev(X, device), _dev(W, device), oracle.quantized_mm(X, W), torch.empty((M, N), device=device),
                      torch.cuda.Stream(device)))
    torch.cuda.synchronize()
    for _ in range(6):
        for Xd, Wd, _, O, s in cases:
            assert L.op_mm_quantize_ex(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, 127.0,
                                       s.cuda_stream) == 0
    torch.cuda.synchronize()
    for i, (_, _, want, O, _) in enumerate(cases):
        assert_bits_equal(O.cpu().numpy(), want, f"implicit workspace, stream {i}")
    Xd, Wd, want, _, _ = cases[0]
    O0 = torch.empty((M, N), device=device)
    assert L.op_mm_quantize(Xd.data_ptr(), Wd.data_ptr(), O0.data_ptr(), M, N, K) == 0
    torch.cuda.synchronize()
    assert_bits_equal(O0.cpu().numpy(), want, "implicit workspace, null stream")


def test_implicit_workspace_many_streams(qg, oracle, device):
    """The implicit workspace keeps at most 8 buffers per device: 12 streams, each running the implicit-workspace call
    twice (the ninth and later streams evict the least recently used buffer), then all 12 again in reverse -- every
    output bit-exact."""
    L = qg.load()
    M, N, K = 300, 520, 700
    X, W = oracle.inputs(M, N, K, 151)
    want = torch.from_numpy(oracle.quantized_mm(X, W)).to(device)
    Xd, Wd = _dev(X, device), _dev(W, device)
    streams = [torch.cuda.Stream(device) for _ in range(12)]
    outs = [torch.full((M, N), float("nan"), device=device) for _ in streams]
    torch.cuda.synchronize()
    for order in (range(12), reversed(range(12))):
        for i in order:
            for _ in range(2):
                assert L.op_mm_quantize_ex(Xd.data_ptr(), K, 1, Wd.data_ptr(), N, 1, outs[i].data_ptr(), N, 1, M, N, K,
                                           127.0, streams[i].cuda_stream) == 0
    torch.cuda.synchronize()
    for i, O in enumerate(outs):
        assert torch.equal(O.view(torch.int32), want.view(torch.int32)), f"stream {i}"


def test_lds_dma_rings_repeat_race_screen(qg, oracle, device):
    """Race screen for the LDS-DMA rings that keep stages in flight across a raw s_barrier (the 3-stage
    64-tile int8 ring, with and without split-K, and the fp32 DMA ring): many back-to-back calls of each,
    every output bit compared -- an early read of a stage shows up as rare wrong tiles, not as a fault
    (cdna_hip_programming.md s5 'Read a staged buffer one phase AFTER the wait that retires it')."""
    for M, N, K, reps in [(512, 3072, 1024, 40), (512, 1024, 4096, 40), (130, 70, 640, 40)]:
        X, W = oracle.inputs(M, N, K, 81)
        want = oracle.quantized_mm(X, W)
        pa, pb = qg.pack_a(_dev(X, device)), qg.pack_b(_dev(W, device))
        outs = [torch.empty((M, N), device=device) for _ in range(reps)]
        for O in outs:
            qg.mm_packed(pa, pb, O)
        torch.cuda.synchronize()
        for i, O in enumerate(outs):
            assert_bits_equal(O.cpu().numpy(), want, f"{M}x{N}x{K} repeat {i}")
    M, N, K = 512, 512, 1024
    X, W = oracle.inputs(M, N, K, 82)
    want = oracle.mm_fp32(X, W)
    Xd, Wd = _dev(X, device), _dev(W, device)
    outs = [qg.mm_fp32(Xd, Wd) for _ in range(30)]
    torch.cuda.synchronize()
    for i, C in enumerate(outs):
        assert_bits_equal(C.cpu().numpy(), want, f"fp32 {M}x{N}x{K} repeat {i}")


@pytest.mark.parametrize("K", [128, 256, 384, 640])
def test_fm_short_k_l2_hot_repeat(qg, oracle, device, K):
    """gemm_i8_fm (the 256-tile kernel, no split-K) at one to five 128-deep k-steps: every operand panel is tiny
    and re-read by the XCD's other tiles, so the fragment loads land as fast as they can and the epilogue's
    per-wave LDS blocks are reused right behind the k-loop; the three register sets' clamped loads past the
    last sub-step are exercised at every remainder (K / 64 = 2, 4, 6, 10); 20 back-to-back calls, every output
    bit.  (Round 2 screened the ping-pong kernel's LDS ring here; that kernel is lab-only since round 4.)"""
    M = N = 4096
    X, W = oracle.inputs(M, N, K, 131)
    want = oracle.quantized_mm(X, W)
    pa, pb = qg.pack_a(_dev(X, device)), qg.pack_b(_dev(W, device))
    outs = [torch.empty((M, N), device=device) for _ in range(20)]
    for O in outs:
        qg.mm_packed(pa, pb, O)
    torch.cuda.synchronize()
    for i, O in enumerate(outs):
        assert_bits_equal(O.cpu().numpy(), want, f"4096x4096x{K} repeat {i}")


def _fuzz_shapes(count=24, seed=20261018):
    """Seeded shapes, M, N in [1, 700], K in [1, 2100] (the oracle finishes each in well under a second): every other
    one log-uniform (small, ragged), the rest uniform over the upper range, and every sixth with K = 1, M = 1 or N = 1."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        if i % 2:  # log-uniform: mostly small, ragged sizes
            M, N, K = (int(round(np.exp(rng.uniform(0.0, np.log(hi))))) for hi in (700, 700, 2100))
        else:      # uniform in the upper three quarters: several tiles and k-steps
            M, N, K = (int(rng.integers(hi // 4, hi + 1)) for hi in (700, 700, 2100))
        if i % 6 == 1:
            K = 1
        elif i % 6 == 2:
            M = 1
        elif i % 6 == 3:
            N = 1
        out.append((max(1, M), max(1, N), max(1, K)))
    return out


@pytest.mark.parametrize("M,N,K", _fuzz_shapes())
def test_seeded_shape_fuzz(qg, oracle, device, M, N, K):
    """Shapes drawn from a fixed seed (not hand-picked), each through the drop-in call against the full oracle, with
    the absmax seed quirk planted in a few rows and columns and a NaN and an inf in X when it has room."""
    X, W = oracle.inputs(M, N, K, 71 + M + N + K)
    if K > 1:
        X[::7, 0] = -1.5   # rows whose signed first element is the largest magnitude
        W[0, ::5] = -1.25
    if M * K > 8:
        X[M // 2, K // 2] = np.nan
        X[M - 1, K - 1] = np.inf
    assert_bits_equal(_run_full(qg, X, W, device), oracle.quantized_mm(X, W), f"fuzz {M}x{N}x{K}")
