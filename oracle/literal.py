"""Pure-Python literal restatement of the reference kernels (small cases only).

TEST INFRASTRUCTURE ONLY.  A second, independent restatement used to cross-check
the C oracle: it walks the reference's kernels loop by loop with numpy float32
scalars (IEEE single, one rounding per operation), so a transcription slip in one
restatement shows up as a disagreement with the other.

  absmax     op_reduction.cuh:71-117 (colwise/rowwise kernels) + AbsMaxFunc :7-25
  scale      op_elemwise.cuh:131-143 InvDivideConstFunc, op_inv_divide :657-667
  quantize   op_elemwise.cuh:106-114 MultiplyWithTypecastFunc, bcast kernel :404-424
  int8 mm    op_mm.cuh:9-46 op_matmul_kernel<int8_t,int> (tile loop, fp32 staging, fma)
  outer      op_mm.cuh:96-97 op_mm<float,float> with K = 1
  dequant    op_elemwise.cuh:93-103 DequantizeFunc, op_mm.cuh:99 MultiplyConstFunc
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
TILE = 32  # TILE_WIDTH, op_mm.cuh:6


def _fma32(a, b, c):
    """fmaf(a, b, c): exact a*b+c, rounded once to float32 (finite operands)."""
    from fractions import Fraction
    if not (math.isfinite(float(a)) and math.isfinite(float(b)) and math.isfinite(float(c))):
        with np.errstate(all="ignore"):
            return f32(float(a) * float(b) + float(c))  # inf/NaN propagate identically
    r = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    if r == 0:
        # IEEE: an exact zero sum is +0 in round-to-nearest unless both addends are -0
        prod_neg = (math.copysign(1.0, float(a)) * math.copysign(1.0, float(b))) < 0
        if prod_neg and math.copysign(1.0, float(c)) < 0:
            return f32(-0.0)
        return f32(0.0)
    return _round_to_f32(r)


def _round_to_f32(r):
    """Round a Fraction to the nearest float32, ties to even (no double rounding)."""
    from fractions import Fraction
    x = f32(float(r))
    cands = [x, np.nextafter(x, f32(np.inf)), np.nextafter(x, f32(-np.inf))]
    best = min(cands, key=lambda c: (abs(Fraction(float(c)) - r),
                                     int(np.frombuffer(f32(c).tobytes(), np.uint32)[0]) & 1))
    return f32(best)


def absmax_functor(x, acc):
    """AbsMaxFunc::operator() (op_reduction.cuh:11-24)."""
    if x > 0:
        if x > acc:
            acc = x
    else:
        if -x > acc:
            acc = f32(-x)
    return acc


def absmax_rows(X):
    M, K = X.shape
    out = np.empty(M, f32)
    for idx in range(M):              # op_reduction_kernel_colwise, one thread per row
        acc = f32(X[idx, 0])          # :80 Index(out, idx, 0) = Index(in, idx, 0)
        for i in range(1, K):         # :81-83
            acc = absmax_functor(f32(X[idx, i]), acc)
        out[idx] = acc
    return out


def absmax_cols(W):
    K, N = W.shape
    out = np.empty(N, f32)
    for idx in range(N):              # op_reduction_kernel_rowwise, one thread per column
        acc = f32(W[0, idx])          # :105
        for i in range(1, K):         # :106-108
            acc = absmax_functor(f32(W[i, idx]), acc)
        out[idx] = acc
    return out


def to_int8(v):
    """static_cast<int8_t>(float): truncation; saturation / NaN->0 where C++ leaves it undefined."""
    v = float(v)
    if v != v:
        return 0
    t = math.trunc(v) if math.isfinite(v) else (127 if v > 0 else -128)
    return max(-128, min(127, t))


def quantized_mm(X, W, range_=127.0):
    X = np.asarray(X, f32)
    W = np.asarray(W, f32)
    M, K = X.shape
    _, N = W.shape
    r = f32(range_)
    with np.errstate(all="ignore"):
        Cx = absmax_rows(X)
        Cw = absmax_cols(W)
        sx = np.array([r / c for c in Cx], f32)          # InvDivideConstFunc: b / x
        sw = np.array([r / c for c in Cw], f32)
        Xq = np.array([[to_int8(f32(X[i, k] * sx[i])) for k in range(K)] for i in range(M)], np.int8)
        Wq = np.array([[to_int8(f32(W[k, j] * sw[j])) for j in range(N)] for k in range(K)], np.int8)
        # op_matmul_kernel<int8_t,int>: int res; res += (float)a*(float)b per tile element
        ntiles = (K - 1) // TILE + 1
        Acc = np.zeros((M, N), np.int32)
        for i in range(M):
            for j in range(N):
                res = 0
                for t in range(ntiles * TILE):
                    a = f32(Xq[i, t]) if t < K else f32(0)
                    b = f32(Wq[t, j]) if t < K else f32(0)
                    res = int(math.trunc(float(_fma32(a, b, f32(res)))))
                Acc[i, j] = res
        # Outer = op_mm(Cx, Cw): res = 0; res += Cx*Cw (+ 31 zero products)
        Outer = np.empty((M, N), f32)
        for i in range(M):
            for j in range(N):
                res = _fma32(Cx[i], Cw[j], f32(0.0))
                for _ in range(TILE - 1):
                    res = _fma32(f32(0.0), f32(0.0), res)
                Outer[i, j] = res
        O = np.empty((M, N), f32)
        inv = f32(f32(1.0) / f32(r * r))
        for i in range(M):
            for j in range(N):
                o = f32(f32(Acc[i, j]) * Outer[i, j])   # DequantizeFunc
                O[i, j] = f32(o * inv)                   # MultiplyConstFunc
    return O, dict(Cx=Cx, Cw=Cw, Xq=Xq, Wq=Wq, Acc=Acc)
