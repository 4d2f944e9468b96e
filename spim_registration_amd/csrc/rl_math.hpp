// rl_math.hpp -- the per-voxel RL rules shared by the rocFFT-backend kernels
// (rl_kernels.hip) and the fused spectral engine (fftconv.hip): one definition, so
// the two update paths cannot drift apart.  Device code; float op order of the Java
// reference (compile with -ffp-contract=off).
#pragma once

#include "rl_kernels.hpp"

namespace spimdecon {

// extendMirrorSingle index (numpy 'reflect'), periodic for far coordinates
__device__ __forceinline__ int64_t mirror_idx(int64_t s, int64_t n) {
    if (n == 1) return 0;
    const int64_t p = 2 * (n - 1);
    int64_t j = s % p;
    if (j < 0) j += p;
    return j >= n ? p - j : j;
}

// d / lambda rounded to nearest, as Java's double division, from inv = RN(1 / lambda):
// q = d * inv lies within 1.5 ulp of d / lambda; the first fma correction makes it
// faithful, the second (Markstein: r = d - lambda q is exact, inv within half an
// ulp of 1 / lambda) correctly rounded.  5 double ops instead of the scaled division
// sequence (2 div_scale, a quarter-rate rcp, 7 fma, div_fmas, div_fixup).  Operands
// here: d = sqrt(1 + 2 lambda v) - 1 is 0 or in [2^-52, 2^512], lambda > 0 normal;
// an infinite d keeps the quotient (the corrections would turn it into NaN).
// (tests/test_oracle.py::test_tikhonov_division_correctly_rounded checks the sequence
// against exact rational division)
__device__ __forceinline__ double div_rn_by(double d, double lambda, double inv) {
    const double q0 = d * inv;
    const double r0 = __builtin_fma(-lambda, q0, d);
    const double q1 = __builtin_fma(r0, inv, q0);
    const double r1 = __builtin_fma(-lambda, q1, d);
    const double q2 = __builtin_fma(r1, inv, q1);
    return __builtin_isfinite(q0) ? q2 : q0;
}

// sqrt(x) for finite x >= 1: the instruction sequence LLVM emits for a correctly
// rounded double sqrt (v_rsq_f64 + Goldschmidt refinement, two fma corrections),
// without its scaling of inputs below 2^-767 and its zero / infinity select, which
// never apply to x = 1 + 2 lambda v with a finite float v > 0 -- so the same bits
// as sqrt() here, in 10 double ops instead of 18.
__device__ __forceinline__ double sqrt_ge1(double x) {
    double h = __builtin_amdgcn_rsq(x);
    double g = x * h;
    h = h * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}

// MVDeconvolution.computeNextValue (:671-703) with lambda's sign known at compile
// time: the Tikhonov branch (double sqrt / divide) is not even if-converted into the
// lambda = 0 kernels.  inv_lambda = 1.0 / lambda (hoisted by the caller).
template <bool TIK>
__device__ __forceinline__ float next_value_t(float last, float integral, float weight, double lambda,
                                              double inv_lambda) {
    const float value = __fmul_rn(last, integral);
    float adjusted;
    if (value > 0.0f) {
        if constexpr (TIK) {
            const double x = 1.0 + 2.0 * lambda * (double)value;
            // (x = +inf, from v = +inf or a huge lambda: Java's sqrt stays infinite)
            adjusted = (float)div_rn_by((x < __builtin_inf() ? sqrt_ge1(x) : x) - 1.0, lambda, inv_lambda);
        } else {
            adjusted = value;
        }
    } else {
        adjusted = kMinValue;
    }
    const float next = isnan(adjusted) ? kMinValue : fmaxf(kMinValue, adjusted);
    return __fadd_rn(last, __fmul_rn(__fsub_rn(next, last), weight));
}

// Same, lambda tested at run time (lambda > 0: Tikhonov, MVDeconvolution.java:681-690)
__device__ __forceinline__ float next_value(float last, float integral, float weight, double lambda) {
    return lambda > 0.0 ? next_value_t<true>(last, integral, weight, lambda, 1.0 / lambda)
                        : next_value_t<false>(last, integral, weight, lambda, 0.0);
}

}  // namespace spimdecon
