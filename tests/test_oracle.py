"""The CPU oracle (oracle/) against the reference's known answers and the committed fixtures.

Runs on CPU.  Pins: KAT-1 / KAT-2 (tests/golden/kat.json; expected values from SURVEY.md s4, not
from this oracle), an independent pure-Python literal restatement (oracle/literal.py), and the
oracle-generated regression fixtures (tests/golden/cases.*).
"""
import hashlib

import numpy as np
import pytest

from util import assert_bits_equal, load_cases, load_kat


def test_kat1_reference_fixture(oracle):
    """test_quantize.cu:38-85 fixture: every intermediate and the output bits."""
    k = load_kat()["kat1"]
    X = np.array(k["X"], np.float32)
    W = np.array(k["W"], np.float32)
    O, d = oracle.quantized_mm(X, W, k["range"], intermediates=True)
    assert d["Cx"].tolist() == k["Cx"]
    assert d["Cw"].tolist() == k["Cw"]
    assert d["Xq"].tolist() == k["Xq"]
    assert d["Acc"].tolist() == k["Acc"]
    want = np.array([int(b, 16) for b in k["O_bits"]], np.uint32).view(np.float32).reshape(3, 2)
    assert_bits_equal(O, want, "KAT-1 O")
    C = oracle.mm_fp32(X, W)
    assert C.tolist() == k["unquantized"]
    assert abs(oracle.signed_mean_error(C, O) - k["printed_signed_mean"]) < 5e-10


def test_kat2_absmax_seed_quirk(oracle):
    """op_reduction.cuh:80 seeds with the SIGNED first element: [-0.9, .5, -.3, .8] -> 0.8."""
    k = load_kat()["kat2"]
    row = np.array([k["row"]], np.float32)
    assert oracle.absmax_rows(row)[0] == np.float32(k["absmax"])
    assert oracle.absmax_cols(row.T.copy())[0] == np.float32(k["absmax"])


@pytest.mark.parametrize("M,N,K,seed", [(5, 4, 40, 1), (9, 7, 33, 2), (3, 11, 64, 3), (1, 6, 70, 4)])
def test_literal_restatement_agrees(oracle, M, N, K, seed):
    """C oracle == pure-Python literal walk of the reference kernels, bit for bit."""
    from oracle import literal
    X, W = oracle.inputs(M, N, K, seed)
    X[0, 0] = -1.5  # force the seed quirk (and an int8 overflow) into every case
    O, d = oracle.quantized_mm(X, W, intermediates=True)
    Ol, dl = literal.quantized_mm(X, W)
    assert_bits_equal(O, Ol, "O")
    for key in ("Xq", "Wq", "Acc"):
        assert (d[key] == dl[key]).all(), key
    assert_bits_equal(d["Cx"], dl["Cx"], "Cx")
    assert_bits_equal(d["Cw"], dl["Cw"], "Cw")


def test_literal_agrees_on_edge_fixtures(oracle):
    from oracle import literal
    index, arrays = load_cases()
    for rec in index:
        if rec["kind"] != "explicit" or rec["M"] * rec["N"] * rec["K"] > 30000:
            continue
        X, W = arrays[rec["name"] + "/X"], arrays[rec["name"] + "/W"]
        Ol, dl = literal.quantized_mm(X, W)
        assert_bits_equal(arrays[rec["name"] + "/O"], Ol, rec["name"])
        assert (arrays[rec["name"] + "/Acc"] == dl["Acc"]).all(), rec["name"]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_fixtures_reproduce(oracle):
    """The committed fixtures are what the oracle computes today (no silent drift)."""
    index, arrays = load_cases()
    for rec in index:
        name = rec["name"]
        if rec["kind"] == "explicit":
            O, d = oracle.quantized_mm(arrays[name + "/X"], arrays[name + "/W"], intermediates=True)
            assert_bits_equal(O, arrays[name + "/O"], name)
            for key in ("Xq", "Wq", "Acc"):
                assert (d[key] == arrays[f"{name}/{key}"]).all(), (name, key)
        else:
            X, W = oracle.inputs(rec["M"], rec["N"], rec["K"], rec["seed"])
            assert X.ravel()[:8].tolist() == rec["x_head"], "input generator drifted"
            assert W.ravel()[:8].tolist() == rec["w_head"], "input generator drifted"
            O, d = oracle.quantized_mm(X, W, intermediates=True)
            assert _sha(O) == rec["O_sha256"], name
            assert _sha(d["Acc"]) == rec["Acc_sha256"], name
            assert _sha(d["Xq"]) == rec["Xq_sha256"], name
            assert _sha(d["Wq"]) == rec["Wq_sha256"], name


def test_exact_int32_equals_reference_fp32_accumulation(oracle):
    """op_matmul_kernel<int8_t,int> accumulates through fp32 FMA (op_mm.cuh:37-39); on every input
    the tests use it equals the exact int32 sum the MFMA path computes."""
    for M, N, K, s in [(64, 64, 128, 1), (32, 48, 1024, 2), (16, 16, 4096, 3)]:
        X, W = oracle.inputs(M, N, K, s)
        _, d = oracle.quantized_mm(X, W, intermediates=True)
        assert (oracle.int8_mm_fp32emu(d["Xq"], d["Wq"]) == d["Acc"]).all()


def test_row_subset_matches_full(oracle):
    X, W = oracle.inputs(96, 80, 300, 11)
    full = oracle.quantized_mm(X, W)
    rows = np.array([0, 5, 17, 95], np.int32)
    assert_bits_equal(oracle.quantized_mm_rows(X, W, rows), full[rows], "row subset")


def test_quantize_saturates_and_zeroes_nan(oracle):
    """Defined behaviour where static_cast<int8_t> is UB: saturate; NaN -> 0."""
    X = np.array([[-1.0, 0.5, 0.25], [0.0, 0.0, 0.0]], np.float32)  # row 0: Cx = 0.5 -> -254 -> -128
    W = np.eye(3, dtype=np.float32)
    _, d = oracle.quantized_mm(X, W, intermediates=True)
    assert d["Xq"][0].tolist() == [-128, 127, 63]
    assert d["Xq"][1].tolist() == [0, 0, 0]  # 0 * (127/0 = inf) = NaN -> 0


def test_generator_is_uniform(oracle):
    u = oracle.uniform((1 << 16,), seed=3)
    assert u.min() >= -1.0 and u.max() < 1.0
    assert abs(float(u.mean())) < 0.01
    # 24 random bits: 2u-1 is exact, so every value is a multiple of 2^-23
    assert np.all(np.mod(u.astype(np.float64) * 2 ** 23, 1.0) == 0)


# ---- encoder counterpart: the C restatement against literal per-element Python loops -----------

def _literal_softmax_row(s, scale):
    import math
    f = np.float32
    mx = f(f(s[0]) * f(scale))
    for v in s[1:]:
        x = f(f(v) * f(scale))
        if x > mx:
            mx = x
    e = [f(math.exp(float(f(f(f(v) * f(scale)) - mx)))) for v in s]
    tot = f(0.0)
    for v in e:
        tot = f(tot + v)
    return np.array([f(v / tot) for v in e], np.float32)


def _literal_add_layernorm_row(a, b):
    f = np.float32
    y = [f(f(x) + f(z)) for x, z in zip(a, b)]
    mean = f(0.0)
    for v in y:
        mean = f(mean + v)
    mean = f(mean / f(len(y)))
    var = f(0.0)
    for v in y:
        d = f(v - mean)
        var = f(var + f(d * d))
    var = f(var / f(len(y)))
    return np.array([f(f(v - mean) / var) for v in y], np.float32)


def test_oracle_softmax_matches_literal(oracle):
    S = oracle.uniform((5, 37), 21) * np.float32(6.0)
    got = oracle.softmax_rows(S, 0.125)
    for r in range(S.shape[0]):
        assert np.array_equal(got[r].view(np.uint32), _literal_softmax_row(S[r], 0.125).view(np.uint32)), r


def test_oracle_add_layernorm_matches_literal(oracle):
    A, B = oracle.uniform((4, 50), 22), oracle.uniform((4, 50), 23)
    got = oracle.add_layernorm_rows(A, B)
    for r in range(A.shape[0]):
        want = _literal_add_layernorm_row(A[r], B[r])
        assert np.array_equal(got[r].view(np.uint32), want.view(np.uint32)), r


def test_oracle_linear_is_quantized_mm_plus_bias_relu(oracle):
    X, W = oracle.inputs(20, 30, 40, 24)
    b = oracle.uniform((30,), 25)
    O = oracle.quantized_mm(X, W)
    y = (O + b).astype(np.float32)
    assert np.array_equal(oracle.linear(X, W, b, False).view(np.uint32), y.view(np.uint32))
    yr = np.where(y < 0, np.float32(0), y).astype(np.float32)
    assert np.array_equal(oracle.linear(X, W, b, True).view(np.uint32), yr.view(np.uint32))


def test_oracle_encoder_heads_concatenation_equals_per_head(oracle):
    """Q/K/V for all heads from one quantized GEMM over [Wq^0 | ... | Wv^H-1] equal the per-head GEMMs
    the reference runs (attention.cuh:54-56): the scales are per row of X and per column of W."""
    d, H, seq = 16, 4, 6
    dk = d // H
    X = oracle.uniform((seq, d), 26)
    bound = np.float32(1.0 / np.sqrt(np.float64(dk)))
    heads = [oracle.uniform((d, dk), oracle.encoder_weight_seed(3, 0, 0, h), -bound, bound) for h in range(H)]
    Wcat = np.concatenate(heads, axis=1)
    full = oracle.quantized_mm(X, Wcat)
    for h in range(H):
        part = oracle.quantized_mm(X, heads[h])
        assert np.array_equal(full[:, h * dk:(h + 1) * dk].view(np.uint32), part.view(np.uint32)), h
