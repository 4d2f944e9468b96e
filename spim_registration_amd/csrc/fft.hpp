// fft.hpp -- rocFFT in-place 3D real transforms on the padded-row layout.
//
// Layout of one padded volume (lengths Mx, My, Mz; x fastest):
//   real view:    Sx = 2*(Mx/2+1) floats per row, rows My, planes Mz
//   complex view: Hx = Mx/2+1 complex per row (same bytes)
// Both directions are unnormalised; the 1/(Mx*My*Mz) factor is folded into
// the kernel spectra.
#pragma once

#include <rocfft/rocfft.h>

#include <cstdint>

#include "common.hpp"

namespace spimdecon {

struct PadDims {
    int64_t M[3] = {0, 0, 0};  // FFT lengths {Mx, My, Mz}
    int64_t Sx() const { return 2 * (M[0] / 2 + 1); }
    int64_t Hx() const { return M[0] / 2 + 1; }
    int64_t real_floats() const { return Sx() * M[1] * M[2]; }
    int64_t complex_count() const { return Hx() * M[1] * M[2]; }
    int64_t logical() const { return M[0] * M[1] * M[2]; }
};

// smallest m >= need of the form 2^a 3^b 5^c 7^d (even when `even`)
int64_t fft_fast_size(int64_t need, bool even);

void rocfft_init_once();

class FftPlan3D {
public:
    FftPlan3D() = default;
    ~FftPlan3D();
    FftPlan3D(const FftPlan3D&) = delete;
    FftPlan3D& operator=(const FftPlan3D&) = delete;

    // plans both directions for `pd` on the current device, bound to `stream`
    void create(const PadDims& pd, hipStream_t stream);
    void forward(float* buf);   // in-place R2C
    void inverse(float* buf);   // in-place C2R
    const PadDims& dims() const { return pd_; }
    size_t work_bytes() const { return work_bytes_; }

private:
    void destroy();
    PadDims pd_;
    rocfft_plan fwd_ = nullptr, inv_ = nullptr;
    rocfft_execution_info info_ = nullptr;
    void* work_ = nullptr;
    size_t work_bytes_ = 0;
};

}  // namespace spimdecon
