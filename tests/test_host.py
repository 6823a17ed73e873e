"""Host-side logic of the Python mirror (no GPU): the reference's asserts and packed geometry."""
import pytest
import torch


def test_op_quantized_mm_asserts_on_device(qg):
    X = torch.zeros(4, 3)
    W = torch.zeros(3, 2)
    O = torch.zeros(4, 2)
    with pytest.raises(AssertionError, match="on_device"):
        qg.op_quantized_mm(X, W, O, 127.0)


def test_op_quantized_mm_asserts_float32(qg):
    X = torch.zeros(4, 3, dtype=torch.float64)
    with pytest.raises(AssertionError):
        qg.op_quantized_mm(X, X.T, X, 127.0)


def test_packed_geometry(qg):
    p = qg.Packed(torch.zeros(qg.load().qgemm_packed_size(257, 129), dtype=torch.uint8), 257, 129, 127.0)
    assert (p.rows_pad, p.k_pad) == (512, 256)
    assert p.scale.numel() == 512 and p.scale.dtype == torch.float32
    assert tuple(p.q.shape) == (512, 256) and p.q.dtype == torch.int8


def _fofs(row, k, k_pad):
    """csrc/qgemm_internal.h fofs, restated: the fragment-major byte offset of packed element (row, k)."""
    return ((row >> 4) * (k_pad >> 6) + (k >> 6)) * 1024 + ((((k >> 4) & 3) << 4) + (row & 15)) * 16 + (k & 15)


def test_fragment_major_view_matches_the_kernel_layout(qg):
    """Packed.q un-permutes the fragment-major storage: element (row, k) is byte fofs(row, k) of q_raw, and
    one 1-KiB block holds one v_mfma_i32_16x16x64_i8 operand in lane order (lane l: row l & 15, k 16(l >> 4))."""
    import numpy as np
    rows, k = 257, 129
    p = qg.Packed(torch.zeros(qg.load().qgemm_packed_size(rows, k), dtype=torch.uint8), rows, k, 127.0)
    raw = p.q_raw
    pos = torch.arange(raw.numel(), dtype=torch.int64)
    raw.copy_(((pos * 7 + pos // 251) % 255 - 127).to(torch.int8))
    q = p.q.numpy()
    flat = raw.numpy()
    rng = np.random.default_rng(0)
    for r, c in zip(rng.integers(0, p.rows_pad, 500), rng.integers(0, p.k_pad, 500)):
        assert q[r, c] == flat[_fofs(int(r), int(c), p.k_pad)]
    # lane l of block (rg, kb) = row 16 rg + (l & 15), k 64 kb + 16 (l >> 4) .. +15
    rg, kb, lane = 3, 1, 37
    blk = flat[(rg * (p.k_pad // 64) + kb) * 1024 + lane * 16: (rg * (p.k_pad // 64) + kb) * 1024 + lane * 16 + 16]
    assert (blk == q[16 * rg + (lane & 15), 64 * kb + 16 * (lane >> 4): 64 * kb + 16 * (lane >> 4) + 16]).all()
