// exp_cr_experiment.h -- lab only, NOT used by the library: fl32(exp((double)x)) for fp32 x (the
// softmax's exp definition), bit-identical to converting the library's double exp, with
// about 2/3 of its double-precision instructions.  Measured slower anyway: 921 vs 1251 G exps/s
// (lab/exp_lab.hip) and 29.6 vs 28.4 us per fused attention launch (the LDS table read and the
// midpoint test cost more than the FMAs saved), so the kernels keep (float)exp((double)x).
//
//   x = k ln2/64 + r, |r| <= ln2/128 (Cody-Waite with FMAs), e^r - 1 by its degree-7 Taylor polynomial
//   (truncation < r^8/8! < 2^-75), times 2^(j/64) from a 64-entry table, times 2^(k>>6): the double
//   result y is within ~2 ulp of e^x.  Its float rounding then equals the exact value's -- and the
//   library path's, itself within 1 ulp -- unless the 29 bits of y below float precision lie within 64
//   of the rounding midpoint; those inputs (about 1 in 4 million), results outside the normal float
//   range (x < -87 or x > 88), NaN and infinities take the library path.
// Checked exhaustively against (float)exp((double)x) on the GPU over every fp32 bit pattern
// (lab/exp_lab.hip: 0 mismatches in 2^32).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace qgemm {

// 2^(j/64), j = 0..63, correctly rounded (generated with 60-digit decimal arithmetic)
__device__ constexpr double kExp2Tab64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0,
};

// tab: kExp2Tab64 staged in LDS by the caller (64 doubles)
__device__ __forceinline__ float exp_cr(float xf, const double *tab) {
    if (!(xf >= -87.0f && xf <= 88.0f)) return (float)exp((double)xf);  // NaN, +-inf, non-normal results
    const double x = (double)xf;
    const double kd = __builtin_rint(x * 0x1.71547652b82fep+6);  // x * 64/ln2
    const int k = (int)kd;
    double r = __builtin_fma(kd, -0x1.62e42fefa4000p-7, x);       // - k * (ln2/64)_hi
    r = __builtin_fma(kd, 0x1.8432a1b0e2634p-49, r);              // - k * (ln2/64)_lo
    double q = __builtin_fma(r, 0x1.a01a01a01a01ap-13, 0x1.6c16c16c16c17p-10);
    q = __builtin_fma(r, q, 0x1.1111111111111p-7);
    q = __builtin_fma(r, q, 0x1.5555555555555p-5);
    q = __builtin_fma(r, q, 0x1.5555555555555p-3);
    q = __builtin_fma(r, q, 0.5);
    const double p = __builtin_fma(r * r, q, r);                  // e^r - 1
    const double t = tab[k & 63];
    const double y = __builtin_ldexp(__builtin_fma(t, p, t), k >> 6);
    const uint32_t low = (uint32_t)__double_as_longlong(y) & 0x1fffffffu;  // the 29 bits below float precision
    if (low - 0x0fffffc0u < 0x80u) return (float)exp(x);        // within 64 of the midpoint 0x10000000
    return (float)y;
}

}  // namespace qgemm
