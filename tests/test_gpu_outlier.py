"""GPU parity of the LLM.int8() outlier decomposition against the oracle.

The reference holds only the unused building blocks (AbsCompareLTEConstFunc / op_outlier_extractor,
op_elemwise.cuh:293-306, 698-708), so the decomposition's definition is this build's (DESIGN.md
"Outlier decomposition", restated in oracle/qgemm_oracle.c): parity is bit-exact against that
restatement; "parity unpinned" against the reference, which never computes it.
"""
import numpy as np
import pytest
import torch

from util import assert_bits_equal

pytestmark = pytest.mark.gpu


def _dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _with_outliers(oracle, M, N, K, cols, seed):
    X, W = oracle.inputs(M, N, K, seed)
    rng = np.random.default_rng(seed)
    for c in cols:
        rows = rng.choice(M, size=max(1, M // 50), replace=False)
        X[rows, c] = rng.choice([-1.0, 1.0], size=rows.size).astype(np.float32) * rng.uniform(7, 60, rows.size)
    return X.astype(np.float32), W


# (72, 40, 33000): K > 32 768 = past the flags launch's accumulator -- its partial-word path, 64-row chunks
@pytest.mark.parametrize("M,N,K,cols", [(300, 200, 512, [3, 77, 400]), (2048, 1024, 4096, list(range(5, 4096, 257))),
                                        (64, 96, 130, [0, 129]), (72, 40, 33000, [0, 31, 32767, 32768, 32999])])
def test_outlier_decomposition_bit_exact(qg, oracle, device, M, N, K, cols):
    X, W = _with_outliers(oracle, M, N, K, cols, 5)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == len(cols)
    assert_bits_equal(C.cpu().numpy(), want, f"outlier decomposition {M}x{N}x{K}")


# shapes on the fast path (>= 160 256-tiles, row-major, K % 4 == 0, K <= 4096, N % 8 == 0): the masked
# single-pass pack and the chain in the GEMM epilogue; ragged M / N / K, mask-word edges, column 0 (the
# absmax seed) and the last column
@pytest.mark.parametrize("M,N,K,cols", [(2500, 4000, 132, [0, 1, 31, 32, 63, 131]),
                                        (2560, 4096, 1024, list(range(7, 1024, 37))),
                                        (2560, 4000, 64, list(range(64))),
                                        (512, 16384, 256, [3, 100, 255])])  # >= 64-KiB rows: the LDS-image stores
def test_outlier_fast_path_bit_exact(qg, oracle, device, M, N, K, cols):
    X, W = _with_outliers(oracle, M, N, K, cols, 9)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == len(cols)
    assert_bits_equal(C.cpu().numpy(), want, f"outlier fast path {M}x{N}x{K}")


# the fast path with many row splits of the column-mask launch (K = 128 / 256: 4 / 8 mask words, 16 splits of 512 rows
# and 13 of 640 -- M = 8257 leaves a partial last split -- so the pack ORs up to 16 partial words per mask word), counts read
# back from the workspace
@pytest.mark.parametrize("M,N,K,cols", [(8192, 1280, 128, [0, 31, 32, 127]), (8257, 1280, 256, [1, 64, 200, 255])])
def test_outlier_fast_path_many_chunks(qg, oracle, device, M, N, K, cols):
    X, W = _with_outliers(oracle, M, N, K, cols, 13)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == len(cols)
    assert_bits_equal(C.cpu().numpy(), want, f"outlier fast path {M}x{N}x{K}")


def test_outlier_fast_path_nan_and_none(qg, oracle, device):
    X, W = oracle.inputs(2560, 4096, 128, 10)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    assert cnt == 0
    assert_bits_equal(C.cpu().numpy(), oracle.quantized_mm(X, W), "fast path, no outliers")
    X[17, 0] = np.nan
    X[2000, 127] = -9.0
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == 2
    assert_bits_equal(C.cpu().numpy(), want, "fast path, NaN column")


@pytest.mark.parametrize("ncols", [0, 1, 3])
def test_outlier_chain_keeps_negative_zero(qg, oracle, device, ncols):
    """An outlier chain that underflows to -0 added to an int8 part that is -0: O = fl(-0 + -0) = -0.  The GEMM
    epilogue runs the chain on 4-column f32 MFMA steps, so a count that is not a multiple of 4 pads the last
    step -- with +0 * -0, which leaves a -0 sum alone (+0 * +0 would give +0).  O8[5, 11] is -0: acc < 0 times
    an outer product Cx * Cw that underflows to +0.  ncols = 0: no column crosses the threshold, so the fast
    path's epilogue must store O8 with no add (fl(-0 + +0) would be +0)."""
    M, N, K = 2560, 4096, 128  # the fast path: 160 256-tiles
    X, W = oracle.inputs(M, N, K, 12)
    cols = [7, 40, 90][:ncols]
    X[5, :] = 0.0
    X[5, 1] = 1e-22           # Cx[5] = 1e-22, q = 127
    W[:, 11] = 0.0
    W[1, 11] = -1e-25         # Cw[11] = 1e-25, q = -127: acc[5, 11] = -16129, fl(Cx * Cw) = +0
    for c in cols:
        X[100, c] = 50.0      # makes column c an outlier column
        X[5, c] = -1e-30
        W[c, 11] = 1e-30      # -1e-30 * 1e-30 underflows to -0
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == ncols
    assert want[5, 11] == 0.0 and np.signbit(want[5, 11]), "the oracle's value is -0"
    assert_bits_equal(C.cpu().numpy(), want, f"outlier chain -0, {ncols} columns")
    if ncols == 0:
        assert_bits_equal(want, oracle.quantized_mm(X, W), "zero outlier columns = the plain path")


def test_no_outliers_is_the_plain_path(qg, oracle, device):
    X, W = oracle.inputs(256, 300, 700, 6)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    assert cnt == 0
    assert_bits_equal(C.cpu().numpy(), oracle.quantized_mm(X, W), "no outliers")


def test_nan_column_is_an_outlier(qg, oracle, device):
    X, W = oracle.inputs(40, 50, 60, 7)
    X[3, 11] = np.nan
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == 1
    assert_bits_equal(C.cpu().numpy(), want, "NaN column")


def test_decomposition_reduces_quantization_error(qg, oracle, device):
    """The point of LLM.int8(): with outlier features, the error against the fp32 product drops."""
    X, W = _with_outliers(oracle, 256, 256, 1024, [10, 500, 900], 8)
    ref = oracle.mm_fp32(X, W)
    plain = oracle.quantized_mm(X, W)
    C, _ = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    e_plain = np.abs(ref - plain).mean()
    e_dec = np.abs(ref - C.cpu().numpy()).mean()
    assert e_dec < 0.75 * e_plain, (e_dec, e_plain)  # measured 0.117 vs 0.203


def test_outlier_graph_capture_and_repeat(qg, oracle, device):
    """qgemm_mm_outlier makes no allocation and no host sync (the outlier count stays on the device; the flags
    launch's counters and accumulator live in the workspace and a kernel zeroes them at the start of every call), so
    the four fast-path launches (zero state, flags, masked pack, GEMM with the chain) can be captured in a HIP graph
    -- here as the FIRST call on its stream -- and replayed; and 20 eager calls on one workspace give the same bits
    every time (race screen of the accumulator / count / column-list hand-offs)."""
    import torch
    M, N, K = 2560, 4096, 512
    X, W = _with_outliers(oracle, M, N, K, [0, 5, 77, 300, 511], 12)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    L = qg.load()
    Xd, Wd = _dev(X, device), _dev(W, device)
    ws = torch.empty(L.qgemm_mm_outlier_workspace_size(M, N, K), dtype=torch.uint8, device=device)
    O = torch.full((M, N), float("nan"), device=device)
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            assert L.qgemm_mm_outlier(Xd.data_ptr(), Wd.data_ptr(), O.data_ptr(), M, N, K, 6.0, ws.data_ptr(),
                                      ws.numel(), s.cuda_stream) == 0
    for _ in range(3):
        O.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, "outlier graph replay")
    for i in range(20):
        assert L.qgemm_mm_outlier(Xd.data_ptr(), Wd.data_ptr(), O.data_ptr(), M, N, K, 6.0, ws.data_ptr(), ws.numel(),
                                  s.cuda_stream) == 0
        s.synchronize()
        assert_bits_equal(O.cpu().numpy(), want, f"outlier repeat {i}")
    assert wcnt == 5


@pytest.mark.parametrize("M,N,K,t", [(2560, 4096, 256, 0.0),      # threshold 0: every column an outlier (fast path)
                                     (2560, 4004, 256, 6.0),      # N % 8 != 0: the materialising fallback
                                     (2561, 4096, 258, 6.0),      # K % 4 != 0: fallback, ragged M
                                     (2560, 4096, 256, float("inf"))])  # nothing is an outlier: the plain path
def test_outlier_edges(qg, oracle, device, M, N, K, t):
    X, W = _with_outliers(oracle, M, N, K, [1, 100, K - 1], 13)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), t)
    want, wcnt = oracle.mm_outlier(X, W, t)
    assert cnt == wcnt
    if t == 0.0:
        assert cnt == K
    if t == float("inf"):
        assert cnt == 0
        assert_bits_equal(want, oracle.quantized_mm(X, W), "oracle: no outliers = plain path")
    assert_bits_equal(C.cpu().numpy(), want, f"outlier edge {M}x{N}x{K} t={t}")


def _bench_outliers(oracle, M, N, K, ncols, seed):
    """bench.py's c2_outlier placement: ncols feature columns spread over K ((K // ncols) * c + 7c + 3 for
    its 8 columns; the 7c offset wraps within half a stride for more), |x| in 7..60 with random signs in
    every 50th row."""
    X, W = oracle.inputs(M, N, K, seed)
    rng = np.random.default_rng(seed)
    stride = K // ncols
    cols = [stride * c + (7 * c) % (stride // 2) + 3 for c in range(ncols)]
    assert len(set(cols)) == ncols and max(cols) < K
    for c in cols:
        n = X[::50, c].size
        X[::50, c] = (rng.uniform(7, 60, n) * rng.choice([-1.0, 1.0], n)).astype(np.float32)
    return X, W, cols


@pytest.mark.parametrize("ncols", [8, 32])
def test_outlier_fast_path_at_the_benched_shape(qg, oracle, device, ncols):
    """The advertised c2_outlier shape, 4096^3 with K = 4096, every output bit: 8 outlier columns take the
    LDS-staged chain in the GEMM epilogue (<= kOutlierStaged), 32 the global-memory chain."""
    M = N = K = 4096
    X, W, cols = _bench_outliers(oracle, M, N, K, ncols, 17 + ncols)
    C, cnt = qg.mm_outlier(_dev(X, device), _dev(W, device), 6.0)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert cnt == wcnt == ncols
    assert_bits_equal(C.cpu().numpy(), want, f"outlier 4096^3, {ncols} columns")


def test_outlier_unaligned_workspace_bit_exact(qg, oracle, device):
    """A caller workspace that is only 4-B aligned: the fast path keeps nothing wider than an int in it (the count,
    the column list, the flags counters and mask words), so it runs there, bit-exact."""
    M, N, K = 2560, 4096, 256
    X, W = _with_outliers(oracle, M, N, K, [1, 100, 255], 14)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    L = qg.load()
    Xd, Wd = _dev(X, device), _dev(W, device)
    need = L.qgemm_mm_outlier_workspace_size(M, N, K)
    buf = torch.empty(need + 256, dtype=torch.uint8, device=device)
    O = torch.full((M, N), float("nan"), device=device)
    s = qg._stream(device)
    assert L.qgemm_mm_outlier(Xd.data_ptr(), Wd.data_ptr(), O.data_ptr(), M, N, K, 6.0, buf.data_ptr() + 4, need,
                              s) == 0
    torch.cuda.synchronize()
    assert wcnt == 3
    assert_bits_equal(O.cpu().numpy(), want, "outlier, 4-B aligned workspace")


def _outlier_call(L, Xd, Wd, O, M, N, K, ws, stream):
    return L.qgemm_mm_outlier(Xd.data_ptr(), Wd.data_ptr(), O.data_ptr(), M, N, K, 6.0, ws.data_ptr(), ws.numel(),
                              stream)


def _outlier_case(qg, oracle, device, M, N, K, cols, seed):
    L = qg.load()
    X, W = _with_outliers(oracle, M, N, K, cols, seed)
    want, wcnt = oracle.mm_outlier(X, W, 6.0)
    assert wcnt == len(cols)
    return (_dev(X, device), _dev(W, device), want,
            torch.empty(L.qgemm_mm_outlier_workspace_size(M, N, K), dtype=torch.uint8, device=device),
            torch.full((M, N), float("nan"), device=device), torch.cuda.Stream(device))


@pytest.mark.parametrize("M,N,K", [(2560, 4096, 512), (300, 200, 516)])  # fast path; materialising fallback
def test_outlier_concurrent_streams_bit_exact(qg, oracle, device, M, N, K):
    """the flags launch's state (counters, mask accumulator) belongs to the call, in its workspace -- not
    to a library slot keyed by the stream handle.  Two streams run outlier calls at the same time, each with its own
    workspace and its own outlier columns; every output bit-exact."""
    L = qg.load()
    cases = [_outlier_case(qg, oracle, device, M, N, K, cols, 21 + i)
             for i, cols in enumerate(([0, 5, 77], [3, 300, 511, 64]))]
    torch.cuda.synchronize()
    for _ in range(8):
        for Xd, Wd, _, ws, O, s in cases:
            assert _outlier_call(L, Xd, Wd, O, M, N, K, ws, s.cuda_stream) == 0
    torch.cuda.synchronize()
    for i, (_, _, want, _, O, _) in enumerate(cases):
        assert_bits_equal(O.cpu().numpy(), want, f"outlier stream {i}, {M}x{N}x{K}")


def test_outlier_graph_replay_beside_eager_calls(qg, oracle, device):
    """a graph captured from qgemm_mm_outlier replayed while eager outlier calls (other inputs, other
    workspace) run on another stream, and on the capture stream between replays: nothing is shared between them."""
    L = qg.load()
    M, N, K = 2560, 4096, 512
    XA, WA, wantA, wsA, OA, sA = _outlier_case(qg, oracle, device, M, N, K, [0, 5, 77], 31)
    XB, WB, wantB, wsB, OB, sB = _outlier_case(qg, oracle, device, M, N, K, [3, 300, 511, 64], 32)
    torch.cuda.synchronize()
    with torch.cuda.stream(sA):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=sA):
            assert _outlier_call(L, XA, WA, OA, M, N, K, wsA, sA.cuda_stream) == 0
    for _ in range(4):
        with torch.cuda.stream(sA):
            g.replay()
        assert _outlier_call(L, XB, WB, OB, M, N, K, wsB, sB.cuda_stream) == 0
        assert _outlier_call(L, XB, WB, OB, M, N, K, wsB, sA.cuda_stream) == 0  # eager on the capture stream
    torch.cuda.synchronize()
    assert_bits_equal(OA.cpu().numpy(), wantA, "graph replay beside eager calls")
    assert_bits_equal(OB.cpu().numpy(), wantB, "eager calls beside graph replays")


def test_outlier_on_more_than_256_streams(qg, oracle, device):
    """round 5 gave each stream handle one of 256 library slots, never returned, so a process that had
    used 256 streams got hipErrorOutOfMemory from every later outlier call.  300 new streams, one call each (fast
    path and fallback shapes alternating), every result compared on the device."""
    L = qg.load()
    shapes = [(2560, 4096, 128, [1, 64]), (64, 96, 130, [0, 129])]
    cases = []
    for M, N, K, cols in shapes:
        Xd, Wd, want, ws, O, _ = _outlier_case(qg, oracle, device, M, N, K, cols, 41)
        cases.append((M, N, K, Xd, Wd, torch.from_numpy(want).to(device), ws, O))
    for i in range(300):
        M, N, K, Xd, Wd, want, ws, O = cases[i % 2]
        s = torch.cuda.Stream(device)
        O.fill_(float("nan"))
        torch.cuda.synchronize()
        assert _outlier_call(L, Xd, Wd, O, M, N, K, ws, s.cuda_stream) == 0, f"stream {i}"
        s.synchronize()
        assert torch.equal(O.view(torch.int32), want.view(torch.int32)), f"stream {i}, {M}x{N}x{K}"
