// encoder.h -- the reference's Encoder (transformer.cu:14-77) on the quantized path, over the C-ABI
// (qgemm_encoder_*, include/qgemm.h).  Two forms:
//   QuantizedEncoder  -- weights drawn once and packed (the LLM.int8() weight cache), forward per call
//   Encoder(X, output, n_heads, n_blocks, d_ff) -- the reference's free-function signature: draws the
//                        weights (seeded from randgen_seed, like op_uniform_init) and runs one forward
// Decisions where the reference cannot run as written (arity, d_ff sizing, per-call weights, host
// round trip): DESIGN.md "Encoder".
#pragma once

#include <cassert>
#include <cstdint>

#include "qgemm.h"
#include "utils/tensor.h"

extern unsigned long long randgen_seed;  // defined by each harness (transformer.cu:12 = 0)

class QuantizedEncoder {
public:
    QuantizedEncoder(int d_model, int n_heads, int d_ff, int n_blocks, int max_seq, uint64_t seed)
        : d_model_(d_model) {
        hipAssert(static_cast<hipError_t>(
            qgemm_encoder_create(d_model, n_heads, d_ff, n_blocks, max_seq, seed, &handle_)));
    }
    QuantizedEncoder(const QuantizedEncoder &) = delete;
    QuantizedEncoder &operator=(const QuantizedEncoder &) = delete;
    ~QuantizedEncoder() { qgemm_encoder_destroy(handle_); }

    // X, output: seq x d_model, contiguous, on the device (the reference asserts on_device)
    void forward(const Tensor<float> &X, Tensor<float> &output) {
        assert(X.on_device && output.on_device && X.w == d_model_ && output.h == X.h && output.w == X.w);
        assert(X.offset == 0 && X.stride_w == 1 && X.stride_h == X.w);
        assert(output.offset == 0 && output.stride_w == 1 && output.stride_h == output.w);
        hipAssert(static_cast<hipError_t>(qgemm_encoder_forward(handle_, X.rawp, output.rawp, X.h, nullptr)));
    }

private:
    void *handle_ = nullptr;
    int d_model_;
};

// transformer.cu:14 signature.  Seed of the weights: the next op_uniform_init-style draw.
inline uint64_t encoder_draw_seed() {
    static unsigned long long draws = 0;
    return randgen_seed * 0x9E3779B97F4A7C15ULL + 0x5EEDULL + draws++;
}

inline void Encoder(const Tensor<float> &X, Tensor<float> &output, int n_heads, int n_blocks, int d_ff) {
    QuantizedEncoder enc{X.w, n_heads, d_ff, n_blocks, X.h, encoder_draw_seed()};
    enc.forward(X, output);
}
