"""ctypes/numpy front end of the CPU oracle (oracle/qgemm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, always as the checker or the CPU baseline.
The product path (the HIP library) never imports this module.

Every function here restates a step of the reference's ``op_quantized_mm``
(/root/reference/src/ops/op_mm.cuh:67-101); the citations live in the C source.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lock = threading.Lock()
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_u64 = ctypes.c_uint64
_c_f = ctypes.c_float


def build() -> str:
    """Compile liboracle.so (gcc, see oracle/Makefile) if it is missing or stale."""
    src = os.path.join(_HERE, "qgemm_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = ctypes.CDLL(_LIB_PATH)
            L.oracle_uniform_at.restype = _c_f
            L.oracle_uniform_at.argtypes = [_c_u64, _c_u64, _c_f, _c_f]
            L.oracle_fill_uniform.argtypes = [_f32p, _c_i64, _c_u64, _c_f, _c_f]
            L.oracle_absmax_rows.argtypes = [_f32p, _c_int, _c_int, _f32p]
            L.oracle_absmax_cols.argtypes = [_f32p, _c_int, _c_int, _f32p]
            L.oracle_inv_divide.argtypes = [_f32p, _c_int, _c_f, _f32p]
            L.oracle_quantize_rows.argtypes = [_f32p, _f32p, _c_int, _c_int, _i8p]
            L.oracle_quantize_cols.argtypes = [_f32p, _f32p, _c_int, _c_int, _i8p]
            L.oracle_int8_mm.argtypes = [_i8p, _i8p, _c_int, _c_int, _c_int, _i32p]
            L.oracle_int8_mm_fp32emu.argtypes = [_i8p, _i8p, _c_int, _c_int, _c_int, _i32p]
            L.oracle_dequantize.argtypes = [_i32p, _f32p, _f32p, _c_int, _c_int, _c_f, _f32p]
            L.oracle_quantized_mm.argtypes = [_f32p, _f32p, _f32p, _c_int, _c_int, _c_int, _c_f]
            L.oracle_quantized_mm_ex.argtypes = [_f32p, _f32p, _f32p, _c_int, _c_int, _c_int, _c_f,
                                                 _f32p, _f32p, _i8p, _i8p, _i32p]
            L.oracle_quantized_mm_rows.argtypes = [_f32p, _f32p, _f32p, _c_int, _c_int, _c_int, _c_f,
                                                   np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS"),
                                                   _c_int]
            L.oracle_mm_fp32.argtypes = [_f32p, _f32p, _f32p, _c_int, _c_int, _c_int]
            L.oracle_signed_mean_error.restype = _c_f
            L.oracle_signed_mean_error.argtypes = [_f32p, _f32p, _c_i64]
            L.oracle_error_stats.argtypes = [_f32p, _f32p, _c_i64, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
            L.oracle_softmax_rows.argtypes = [_f32p, _f32p, _c_i64, _c_int, _c_f]
            L.oracle_add_layernorm_rows.argtypes = [_f32p, _f32p, _f32p, _c_i64, _c_int]
            L.oracle_linear.argtypes = [_f32p, _f32p, ctypes.c_void_p, _c_int, _f32p, _c_int, _c_int, _c_int]
            L.oracle_encoder_weight_seed.restype = _c_u64
            L.oracle_encoder_weight_seed.argtypes = [_c_u64, _c_int, _c_int, _c_int]
            L.oracle_encoder_forward.argtypes = [_f32p, _f32p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_u64]
            L.oracle_set_threads.argtypes = [_c_int]
            L.oracle_mm_outlier.restype = _c_int
            L.oracle_mm_outlier.argtypes = [_f32p, _f32p, _f32p, _c_int, _c_int, _c_int, _c_f]
            _lib = L
    return _lib


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ----------------------------------------------------------------------------- inputs
def set_threads(n: int) -> None:
    """OpenMP thread count of the restatement's parallel loops (bench.py cpu_baseline)."""
    lib().oracle_set_threads(int(n))


def uniform(shape, seed: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """Seeded U[lo,hi) fp32 matrix, bit-identical to the HIP fill kernel (qgemm_fill_uniform)."""
    n = int(np.prod(shape))
    out = np.empty(n, dtype=np.float32)
    lib().oracle_fill_uniform(out, n, seed, lo, hi)
    return out.reshape(shape)


def inputs(M: int, N: int, K: int, seed: int):
    """X[M,K] from seed 2s, W[K,N] from seed 2s+1."""
    return uniform((M, K), 2 * seed), uniform((K, N), 2 * seed + 1)


# ------------------------------------------------------------------------- the chain
def absmax_rows(X):
    X = _c(X, np.float32)
    M, K = X.shape
    out = np.empty(M, dtype=np.float32)
    lib().oracle_absmax_rows(X, M, K, out)
    return out


def absmax_cols(W):
    W = _c(W, np.float32)
    K, N = W.shape
    out = np.empty(N, dtype=np.float32)
    lib().oracle_absmax_cols(W, K, N, out)
    return out


def quantized_mm(X, W, range_: float = 127.0, intermediates: bool = False):
    """O = op_quantized_mm(X, W, range) -- fp32 in, fp32 out.  With ``intermediates``
    also returns dict(Cx, Cw, Xq, Wq, Acc) (Wq in the reference's K x N layout)."""
    X = _c(X, np.float32)
    W = _c(W, np.float32)
    M, K = X.shape
    K2, N = W.shape
    assert K == K2, "X.w == W.h (op_mm.cuh:71)"
    O = np.empty((M, N), dtype=np.float32)
    if not intermediates:
        lib().oracle_quantized_mm(X, W, O, M, N, K, range_)
        return O
    Cx = np.empty(M, np.float32)
    Cw = np.empty(N, np.float32)
    Xq = np.empty((M, K), np.int8)
    Wq = np.empty((K, N), np.int8)
    Acc = np.empty((M, N), np.int32)
    lib().oracle_quantized_mm_ex(X, W, O, M, N, K, range_, Cx, Cw, Xq, Wq, Acc)
    return O, dict(Cx=Cx, Cw=Cw, Xq=Xq, Wq=Wq, Acc=Acc)


def quantized_mm_rows(X, W, rows, range_: float = 127.0):
    """Rows ``rows`` of op_quantized_mm(X, W) only (rows are independent given Cw)."""
    X = _c(X, np.float32)
    W = _c(W, np.float32)
    M, K = X.shape
    _, N = W.shape
    rows = _c(rows, np.int32)
    out = np.empty((len(rows), N), dtype=np.float32)
    lib().oracle_quantized_mm_rows(X, W, out, M, N, K, range_, rows, len(rows))
    return out


def int8_mm(Xq, Wq):
    Xq = _c(Xq, np.int8)
    Wq = _c(Wq, np.int8)
    M, K = Xq.shape
    _, N = Wq.shape
    out = np.empty((M, N), np.int32)
    lib().oracle_int8_mm(Xq, Wq, M, N, K, out)
    return out


def int8_mm_fp32emu(Xq, Wq):
    """The reference's literal fp32-FMA integer accumulation (op_mm.cuh:37-39)."""
    Xq = _c(Xq, np.int8)
    Wq = _c(Wq, np.int8)
    M, K = Xq.shape
    _, N = Wq.shape
    out = np.empty((M, N), np.int32)
    lib().oracle_int8_mm_fp32emu(Xq, Wq, M, N, K, out)
    return out


def mm_fp32(X, W):
    """Unquantized op_mm<float,float> (sequential-k fmaf)."""
    X = _c(X, np.float32)
    W = _c(W, np.float32)
    M, K = X.shape
    _, N = W.shape
    C = np.empty((M, N), np.float32)
    lib().oracle_mm_fp32(X, W, C, M, N, K)
    return C


def signed_mean_error(C, O) -> float:
    """The reference's printed "Mean quantization error" (timing_quantize.cu:67-70)."""
    C = _c(C, np.float32).ravel()
    O = _c(O, np.float32).ravel()
    return float(lib().oracle_signed_mean_error(C, O, C.size))


def error_stats(C, O) -> dict:
    C = _c(C, np.float32).ravel()
    O = _c(O, np.float32).ravel()
    a, m, r = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    lib().oracle_error_stats(C, O, C.size, ctypes.byref(a), ctypes.byref(m), ctypes.byref(r))
    return dict(signed_mean=signed_mean_error(C, O), mean_abs=a.value, max_abs=m.value,
                rel=a.value / r.value if r.value else float("nan"))


# ---- encoder counterpart (qgemm_oracle.c "Encoder counterpart") ----------------

def softmax_rows(S, scale: float = 1.0):
    """op_multiply(S, scale) + op_softmax per row (op_softmax.cuh:6-29), correctly rounded exp."""
    S = _c(S, np.float32)
    P = np.empty_like(S)
    lib().oracle_softmax_rows(S, P, S.size // S.shape[-1], S.shape[-1], float(scale))
    return P


def add_layernorm_rows(A, B):
    """op_add + op_layernorm as written (op_layernorm.cuh:6-33: (y - mean) / var)."""
    A, B = _c(A, np.float32), _c(B, np.float32)
    Y = np.empty_like(A)
    lib().oracle_add_layernorm_rows(A, B, Y, A.size // A.shape[-1], A.shape[-1])
    return Y


def linear(X, W, b=None, relu=False):
    """LinearLayer.forward with the quantized GEMM (linear.cuh:50-54) [+ op_relu]."""
    X, W = _c(X, np.float32), _c(W, np.float32)
    M, K = X.shape
    N = W.shape[1]
    Y = np.empty((M, N), np.float32)
    bb = None if b is None else _c(b, np.float32)
    lib().oracle_linear(X, W, None if bb is None else bb.ctypes.data, 1 if relu else 0, Y, M, N, K)
    return Y


def encoder_weight_seed(base: int, block: int, kind: int, head: int) -> int:
    return int(lib().oracle_encoder_weight_seed(base, block, kind, head))


def encoder_forward(X, d_model: int, n_heads: int, d_ff: int, n_blocks: int, seed: int):
    """transformer.cu:14-77's Encoder with quantized linears (decisions: DESIGN.md "Encoder")."""
    X = _c(X, np.float32)
    seq = X.shape[0]
    assert X.shape[1] == d_model
    Y = np.empty_like(X)
    lib().oracle_encoder_forward(X, Y, seq, d_model, n_heads, d_ff, n_blocks, seed)
    return Y


def mm_outlier(X, W, threshold: float = 6.0):
    """LLM.int8() decomposition: returns (O, number of outlier columns)."""
    X, W = _c(X, np.float32), _c(W, np.float32)
    M, K = X.shape
    N = W.shape[1]
    O = np.empty((M, N), np.float32)
    cnt = lib().oracle_mm_outlier(X, W, O, M, N, K, float(threshold))
    return O, int(cnt)
