"""GPU parity of the encoder counterpart (BASELINE config 5) against the oracle.

The encoder's quantized linears (Q/K/V, W_O, FFN with fused bias / relu), fp32 attention GEMMs,
softmax and add + layernorm are each compared with the oracle restatement bit for bit, then the
whole stack at the reference's own shape (transformer.cu:171-178), a small shape and config 5.
"""
import numpy as np
import pytest
import torch

from util import assert_bits_equal

pytestmark = pytest.mark.gpu


def _dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


@pytest.mark.parametrize("rows,w", [(64, 7), (48, 64), (1024, 512), (5, 1000)])
def test_softmax_rows_bit_exact(qg, oracle, device, rows, w):
    S = oracle.uniform((rows, w), 3) * np.float32(8.0)
    P = qg.softmax_rows(_dev(S, device), scale=0.125)
    assert_bits_equal(P.cpu().numpy(), oracle.softmax_rows(S, 0.125), f"softmax {rows}x{w}")


def test_softmax_in_place(qg, oracle, device):
    S = oracle.uniform((256, 512), 4)
    Sd = _dev(S, device)
    qg.softmax_rows(Sd, scale=0.125, P=Sd)
    assert_bits_equal(Sd.cpu().numpy(), oracle.softmax_rows(S, 0.125), "softmax in place")


@pytest.mark.parametrize("rows,w", [(33, 8), (512, 1024), (7, 4096), (9, 100), (1, 4), (5, 2052), (3, 1028),
                                    (64, 6), (4, 1020), (2, 2044), (3, 4092), (6, 132)])
def test_add_layernorm_rows_bit_exact(qg, oracle, device, rows, w):
    """1020 / 2044 / 4092 / 132: the last lane of the register kernel's lane blocks is partly past the row (its
    elements there are -0.0, the chain's identity)."""
    A, B = oracle.uniform((rows, w), 5), oracle.uniform((rows, w), 6)
    Y = qg.add_layernorm_rows(_dev(A, device), _dev(B, device))
    assert_bits_equal(Y.cpu().numpy(), oracle.add_layernorm_rows(A, B), f"add+layernorm {rows}x{w}")


@pytest.mark.parametrize("w", [1024, 1000, 4096, 260])
def test_add_layernorm_rows_special_values(qg, oracle, device, w):
    """The register-resident kernel's lane-hop sums (DPP wave_ror) on rows holding NaN, +-inf, -0, huge and tiny
    values: the same rounding sequence as the column-order chain, bit for bit."""
    rows = 12
    A, B = oracle.uniform((rows, w), 21), oracle.uniform((rows, w), 22)
    A[1, w // 3] = np.nan
    A[2, 5] = np.inf
    A[3, 7], B[3, 9] = np.inf, -np.inf
    A[4, :] = -0.0
    B[4, :] = -0.0
    A[5, ::7] = 3.0e38
    A[6, :] = 1e-40  # subnormal inputs
    B[6, :] = 0.0
    A[7, w - 1] = -2.5e9  # the last element of the row
    A[8, 0] = 1e30  # the first
    Y = qg.add_layernorm_rows(_dev(A, device), _dev(B, device))
    assert_bits_equal(Y.cpu().numpy(), oracle.add_layernorm_rows(A, B), f"add+layernorm special values, w={w}")


def test_add_layernorm_rows_misaligned_rows(qg, oracle, device):
    """Rows 4-byte aligned only (storage offset 1): the general kernel instead of the float4 one."""
    rows, w = 40, 1024
    A, B = oracle.uniform((rows, w), 7), oracle.uniform((rows, w), 8)
    bufs = []
    for X in (A, B):
        buf = torch.zeros(rows * w + 1, dtype=torch.float32, device=device)
        buf[1:] = torch.from_numpy(X.reshape(-1)).to(device)
        bufs.append(buf[1:].view(rows, w))
    Y = qg.add_layernorm_rows(bufs[0], bufs[1])
    assert_bits_equal(Y.cpu().numpy(), oracle.add_layernorm_rows(A, B), "add+layernorm misaligned")


@pytest.mark.parametrize("M,N,K,bias,relu", [(100, 260, 300, True, True), (100, 260, 300, True, False),
                                             (100, 260, 300, False, False), (512, 1024, 1024, True, True),
                                             (512, 4096, 1024, True, False),
                                             # 32 x 32 tiles (fewer 64-tiles than CUs): K = 4096, ragged M / N
                                             (512, 1024, 4096, True, False), (300, 1000, 2048, True, True),
                                             (250, 1030, 1024, False, False)])
def test_linear_fused_bias_relu_bit_exact(qg, oracle, device, M, N, K, bias, relu):
    X, W = oracle.inputs(M, N, K, 91)
    b = oracle.uniform((N,), 92) if bias else None
    pw = qg.pack_b(_dev(W, device))
    Y = qg.linear(_dev(X, device), pw, bias=None if b is None else _dev(b, device), relu=relu)
    assert_bits_equal(Y.cpu().numpy(), oracle.linear(X, W, b, relu), f"linear {M}x{N}x{K} b={bias} relu={relu}")


@pytest.mark.parametrize("M,N,K,relu,splits", [(2048, 4096, 1024, True, 1),    # register-store pairs
                                              (2048, 4096, 2048, False, 2),   # ticket-first split-K
                                              (2048, 16384, 512, True, 1),    # >= 64-KiB rows: the LDS image
                                              (2000, 4100, 1000, True, 1)])   # partial tiles
def test_linear_fused_bias_relu_256_tiles(qg, oracle, device, M, N, K, relu, splits):
    """gemm_i8_fm's bias / bias+relu epilogues (the encoder's shapes all take the small-tile kernels), every output
    bit, on each of its store paths."""
    import ctypes
    tile = ctypes.c_int(0)
    assert qg.load().qgemm_gemm_plan(M, N, K, ctypes.byref(tile), None) == splits and tile.value == 256
    X, W = oracle.inputs(M, N, K, 93)
    b = oracle.uniform((N,), 94)
    pw = qg.pack_b(_dev(W, device))
    Y = qg.linear(_dev(X, device), pw, bias=_dev(b, device), relu=relu)
    assert_bits_equal(Y.cpu().numpy(), oracle.linear(X, W, b, relu), f"linear {M}x{N}x{K} relu={relu}")


@pytest.mark.parametrize("seq,d,H,dff,blocks", [
    (6, 8, 4, 8, 2),          # the reference's own Encoder call (transformer.cu:171-178)
    (32, 64, 4, 128, 2),
    (100, 256, 8, 512, 3),    # ragged seq, odd block count
    (257, 96, 3, 64, 1),      # fused attention: d_k 32 (no +0 step), a second 256-key chunk holding one key
    (40, 60, 5, 32, 2),       # d_k 12: k % 4 == 0, k % 32 != 0
    (480, 128, 2, 64, 1),     # seq % 64 == 32: the last P V group of 8 k-steps stands alone
    (33, 64, 1, 64, 1),       # one query row in the second tile; P V over 64 padded keys
    (300, 128, 1, 64, 1),     # d_k 128 > 64: the three-launch attention fallback
    (600, 64, 2, 64, 1),      # seq 600 > 512: fallback
])
def test_encoder_forward_bit_exact(qg, oracle, device, seq, d, H, dff, blocks):
    X = oracle.uniform((seq, d), 11)
    enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=13)
    try:
        Y = enc.forward(_dev(X, device))
        torch.cuda.synchronize()
        want = oracle.encoder_forward(X, d, H, dff, blocks, 13)
        assert_bits_equal(Y.cpu().numpy(), want, f"encoder seq={seq} d={d} H={H} dff={dff} blocks={blocks}")
        Y2 = enc.forward(_dev(X, device))   # weights cached: a second call gives the same bits
        assert_bits_equal(Y2.cpu().numpy(), want, "encoder second call")
    finally:
        enc.close()


@pytest.mark.parametrize("gain", [60.0, 1e4])
def test_encoder_forward_peaked_softmax(qg, oracle, device, gain):
    """Inputs scaled so the attention scores spread over hundreds to millions: most exps of a softmax row
    underflow to +0 and the row sums (lane-hop chains in the fused attention) run over long runs of zeros and
    a few large terms -- every output bit against the oracle."""
    seq, d, H, dff, blocks = 100, 256, 8, 512, 2
    X = oracle.uniform((seq, d), 29) * np.float32(gain)
    enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=31)
    try:
        Y = enc.forward(_dev(X, device)).cpu().numpy()
    finally:
        enc.close()
    assert_bits_equal(Y, oracle.encoder_forward(X, d, H, dff, blocks, 31), f"encoder, input x {gain}")


def test_encoder_config5_bit_exact(qg, oracle, device):
    """BASELINE config 5: d_model 1024, seq 512 (16 heads, d_ff 4096, 2 blocks)."""
    seq, d, H, dff, blocks = 512, 1024, 16, 4096, 2
    X = oracle.uniform((seq, d), 17)
    enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=19)
    try:
        Y = enc.forward(_dev(X, device)).cpu().numpy()
    finally:
        enc.close()
    assert_bits_equal(Y, oracle.encoder_forward(X, d, H, dff, blocks, 19), "encoder config 5")


def test_transformer_harness_matches_oracle(qg, oracle):
    """build/transformer (the reference main's Encoder call, transformer.cu:170-178) prints the same
    output as the oracle on its input (first op_uniform_init draw) and weight seed."""
    import os
    import subprocess
    exe = os.path.join(qg.PKG_DIR, "build", "transformer")
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    lines = [ln.strip() for ln in out.splitlines()]
    seed = int(next(ln for ln in lines if ln.startswith("weight seed:")).split()[-1])
    o = lines.index("output:")
    got = [ln.split() for ln in lines[o + 1:o + 7]]
    X = oracle.uniform((6, 8), 0)  # randgen_seed 0, first draw (op_mm_quantize.cuh op_uniform_init)
    x = lines.index("X:")
    assert [ln.split() for ln in lines[x + 1:x + 7]] == [[f"{v:.6f}" for v in row] for row in X]
    want = oracle.encoder_forward(X, 8, 4, 8, 2, seed)
    assert got == [[f"{v:.6f}" for v in row] for row in want]
    assert "All tests completed successfully!" in lines
