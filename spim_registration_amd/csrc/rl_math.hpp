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

// MVDeconvolution.computeNextValue (:671-703) with lambda's sign known at compile
// time: the Tikhonov branch (double sqrt / divide) is not even if-converted into the
// lambda = 0 kernels.
template <bool TIK>
__device__ __forceinline__ float next_value_t(float last, float integral, float weight, double lambda) {
    const float value = __fmul_rn(last, integral);
    float adjusted;
    if (value > 0.0f) {
        if constexpr (TIK) adjusted = (float)((sqrt(1.0 + 2.0 * lambda * (double)value) - 1.0) / lambda);
        else adjusted = value;
    } else {
        adjusted = kMinValue;
    }
    const float next = isnan(adjusted) ? kMinValue : fmaxf(kMinValue, adjusted);
    return __fadd_rn(last, __fmul_rn(__fsub_rn(next, last), weight));
}

// Same, lambda tested at run time (lambda > 0: Tikhonov, MVDeconvolution.java:681-690)
__device__ __forceinline__ float next_value(float last, float integral, float weight, double lambda) {
    return lambda > 0.0 ? next_value_t<true>(last, integral, weight, lambda)
                        : next_value_t<false>(last, integral, weight, lambda);
}

}  // namespace spimdecon
