// op_mm_quantize.cuh -- the Tensor-level operator API of the hot path, as a thin adaptor over the
// C-ABI (include/qgemm.h).  A translation unit written against the reference's
//     template<typename T> void op_quantized_mm(const Tensor<T>&, const Tensor<T>&, Tensor<T>&, T range)
//     (/root/reference/src/ops/op_mm.cuh:67-101)
// compiles unchanged against this header and links libqgemm.so instead of instantiating the
// reference's ten-launch chain.  Also provides the two neighbours the reference harnesses call
// beside it: op_mm<float,float> (op_mm.cuh:49-65, the unquantized path) and op_uniform_init
// (op_elemwise.cuh:728-744, seeded from the global randgen_seed like the reference's).
#pragma once

#include <type_traits>

#include "qgemm.h"
#include "utils/tensor.h"

extern unsigned long long randgen_seed;  // defined by each harness, as in the reference (test_quantize.cu:11)

// op_mm.cuh:67-101.  Asserts exactly as the reference does (:71-72); strided views are passed through.
template <typename T>
void op_quantized_mm(const Tensor<T> &X, const Tensor<T> &W, Tensor<T> &O, T range) {
    static_assert(std::is_same<T, float>::value, "op_quantized_mm is instantiated at T=float only");
    assert(X.h == O.h && W.w == O.w && X.w == W.h);
    assert(X.on_device && W.on_device && O.on_device);
    hipAssert(static_cast<hipError_t>(op_mm_quantize_ex(X.data(), X.stride_h, X.stride_w, W.data(), W.stride_h,
                                                        W.stride_w, O.data(), O.stride_h, O.stride_w, X.h, W.w, X.w,
                                                        range, nullptr)));
}

// op_mm.cuh:49-65 at T = OutT = float: the unquantized reference GEMM (bit-exact, sequential-k fma).
inline void op_mm(const Tensor<float> &A, const Tensor<float> &B, Tensor<float> &C) {
    assert(A.h == C.h && B.w == C.w && A.w == B.h);
    assert(A.on_device && B.on_device && C.on_device);
    hipAssert(static_cast<hipError_t>(qgemm_mm_fp32(A.data(), A.stride_h, A.stride_w, B.data(), B.stride_h,
                                                    B.stride_w, C.data(), C.stride_h, C.stride_w, A.h, B.w, A.w,
                                                    nullptr)));
}

// op_elemwise.cuh:728-744: U[min,max) fill.  The reference draws from a function-static cuRAND
// generator; here every call advances a per-process call counter mixed into the seed, so
// successive calls give different (reproducible) matrices, as successive cuRAND draws do.
template <typename T>
void op_uniform_init(Tensor<T> &t, T min = 0, T max = 1) {
    static_assert(std::is_same<T, float>::value, "float tensors only");
    assert(t.offset == 0 && t.stride_w == 1);
    assert(t.on_device);
    static unsigned long long draws = 0;
    const unsigned long long seed = randgen_seed * 0x100000001B3ULL + draws++;
    hipAssert(static_cast<hipError_t>(
        qgemm_fill_uniform(t.rawp, (int64_t)t.h * t.w, seed, (float)min, (float)max, nullptr)));
}
