// transformer.cpp -- counterpart of the reference's /root/reference/src/transformer.cu main
// (:170-185): X{6,8} U(-1,1), Encoder(X, enc_output, n_heads = 4, n_blocks = 2, d_ff = 8), with the
// encoder's linears on the int8 quantized path.  The reference's main also runs a Decoder (out of
// scope) and does not compile (arity bug, transformer.cu:37).  Prints the input,
// the weight seed and the output in the reference's tensor text format.
#include <iostream>

#include "modules/encoder.h"
#include "ops/op_mm_quantize.cuh"

unsigned long long randgen_seed = 0;  // transformer.cu:12

int main() {
    Tensor<float> X{6, 8, true};
    op_uniform_init(X, -1.0f, 1.0f);
    Tensor<float> enc_output{X.h, X.w, true};
    const int n_heads = 4, n_blocks = 2, d_ff = 8;

    std::cout << "ENCODER\n=======\n";
    std::cout << "X: \n" << X.str() << std::endl;
    const uint64_t seed = encoder_draw_seed();
    {
        QuantizedEncoder enc{X.w, n_heads, d_ff, n_blocks, X.h, seed};
        enc.forward(X, enc_output);
    }
    std::cout << "weight seed: " << seed << std::endl;
    std::cout << "output: \n" << enc_output.str() << std::endl;
    hipAssert(hipDeviceSynchronize());
    std::cout << "All tests completed successfully!" << std::endl;
    return 0;
}
