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
