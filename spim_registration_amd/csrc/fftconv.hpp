// fftconv.hpp -- fused spectral-convolution engine for the RL iteration (MI355X).
//
// rocFFT runs a 540^3 R2C at ~8x the cost of one HBM pass (profiles/r01_*); this
// engine instead streams the padded volume through five HBM passes per
// convolution and fuses every pointwise step of the RL update into them:
//
//   X pass (rows, contiguous)      inverse real FFT of the previous convolution
//                                  -> pointwise (quotient | Tikhonov update)
//                                  -> forward real FFT of the next operand
//   Y pass (columns, stride Hp)    complex FFT along y          (fwd / inv)
//   Z pass (columns, stride My*Hp) FFT along z * kernel spectrum * inverse FFT
//
// Spectrum layout C[qz][qy][kx] (float2, row pitch Hp = Hx rounded to 16,
// Hx = Mx/2 + 1).  Two real rows are transformed as one complex row (real /
// imaginary parts) and split into their half spectra.  All 1D FFTs are
// mixed-radix Stockham (radix 2, 3, 4, 5, 7) in LDS with a float twiddle
// table computed in double.  Both directions are unnormalised; 1/(Mx*My*Mz) is
// folded into the kernel spectra.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "common.hpp"
#include "rl_kernels.hpp"

namespace spimdecon {

constexpr int kFftMaxStages = 16;

struct Fft1D {
    int L = 0;
    int ns = 0;
    uint64_t radix_packed = 0;   // radix of stage s in bits [4s, 4s+4) (no indexed array:
                                 // a dynamically indexed kernel-argument array goes to scratch)
    const float2* tw = nullptr;  // device table exp(-2*pi*i*m/L), m < L
    int n1 = 0, n2 = 0;          // two-factor fast path (L = n1 * n2), 0 = Stockham
    __host__ __device__ int radix(int s) const { return int((radix_packed >> (4 * s)) & 15u); }
};

// Engine knobs, read from the environment once per plan (SpectralPlan::create), so the
// hot loop reads no environment and tests can toggle them per session:
//   SPIMDECON_YPF=0      y passes at one block per CU without the register prefetch
//   SPIMDECON_ZKD=0      no compile-time trim of the zero outer taps in the direct z pass
//   SPIMDECON_ZDIRECT=0  the fused FFT z pass (k_col2f MODE 5) instead of the direct one
struct EngineKnobs {
    bool ypf = true, zkd = true, zdirect = true;
    static EngineKnobs from_env();
};

// per-slab engine state (twiddles, row maps)
struct SpectralPlan {
    SlabGeom g{};
    int64_t Hx = 0, Hp = 0;
    Fft1D fx, fy, fz;
    DBuf<float2> twx, twy, twz;
    DBuf<int> row_mirror;  // [My*Mz] local source row (lz*ny+ly) of the mirror extension; -1 skip
    DBuf<int> row_one;     // [My*Mz] own local row if interior; -2 constant 1; -1 skip
    // x pass the last update launch ran: 2 = two-factor tiles (k_xtile), 1 = per-wave
    // rows (k_xrows), 0 = Stockham rows (k_xpass); -1 = none yet (mvd_xpass_mode)
    mutable int xmode_update = -1;
    EngineKnobs knobs;
    int64_t spectrum_elems() const { return Hp * g.My * g.Mz; }
    // allow_2f: use the two-factor register kernels for lengths in the fast-path table
    // z_fft = false: no z transform plan (the direct z convolution needs none, and then
    // Mz = nz + 2 cz need not be an FFT length)
    // knobs: the session's EngineKnobs, read once when its slabs are sized
    void create(const SlabGeom& geom, bool allow_2f, bool z_fft, const EngineKnobs& knobs);
};

// FFT length for `need` samples (even when `even`).  policy 0: the two-factor
// fast-path size when it is within 25% of the smallest 2,3,5,7-smooth size,
// else that smooth size (Stockham path); 1: always the fast-path table;
// 2: always the smooth size.
int64_t engine_fast_size(int64_t need, bool even, int policy = 0);

// true when a slab of nx * ny * nzs voxels with kernel half sizes <= halo keeps every
// buffer the fast passes address (psi, views, spectra) inside their 32-bit offset
// range; the session splits a device's share into more slabs until it does
bool engine_slab_fits(int64_t nx, int64_t ny, int64_t nzs, const int halo[3], int policy);

// ---- passes (all asynchronous on `s`) ----
// psi -> C (x-spectra of the mirror-extended psi rows)
void engine_forward_psi(const SpectralPlan& p, const float* psi, float2* C, hipStream_t s);
// small kernel (kx,ky,kz) -> full 3D spectrum in Kspec (scaled), uses `work` as scratch-free in place
void engine_kernel_spectrum(const SpectralPlan& p, const float* d_kernel, int kx, int ky, int kz,
                            float scale, float2* Kspec, hipStream_t s);
// compact kernel spectra (two-factor z length only): the x and y transforms of the
// placed kernel on its 2*cz+1 non-zero z-planes, [2cz+1][My][Hp]; the z pass
// (engine_zpass_compact) computes the z transform in its tiles.  `work` is a
// full spectrum_elems() scratch buffer.
bool engine_kernel_compact_ok(const SpectralPlan& p);
// the direct z convolution (fftconv_zd.inc) applies: compact kernels then run it
bool engine_zdirect_ok(const SpectralPlan& p);
// the same decision from the padded dims, before a plan exists (the session then
// sizes Mz = nz + 2 cz exactly)
bool engine_zdirect_dims_ok(int64_t Mx, int64_t My, int64_t Mz, int cz, bool zdirect_knob);
// z pass of a slab: 0 = fused FFT with full kernel spectra, 1 = fused FFT with
// compact kernels, 3 = direct convolution with compact kernels (z chunks, k_zdmc)
int engine_zpass_mode(const SpectralPlan& p, bool compact);
int64_t engine_kernel_compact_elems(const SpectralPlan& p);
void engine_kernel_compact(const SpectralPlan& p, const float* d_kernel, int kx, int ky, int kz, float scale,
                           float2* work, float2* Kc, hipStream_t s);
void engine_zpass_compact(const SpectralPlan& p, float2* C, const float2* Kc, hipStream_t s);
// Y pass: in-place complex FFT along y (inverse when inv)
void engine_ypass(const SpectralPlan& p, float2* C, bool inv, hipStream_t s);
// Forward y pass of the z planes [z0, z1) only (false: not available for this plan,
// run engine_ypass instead)
bool engine_ypass_planes(const SpectralPlan& p, float2* C, int z0, int z1, hipStream_t s);
// the same over [z0, z1) and [z2, z3) as one launch
bool engine_ypass_planes2(const SpectralPlan& p, float2* C, int z0, int z1, int z2, int z3, hipStream_t s);
// Z pass: forward z FFT, multiply by K (when K != nullptr) and inverse z FFT
void engine_zpass(const SpectralPlan& p, float2* C, const float2* K, hipStream_t s);
// packed row pairs (rows 2i, 2i+1 of the My*Mz padded rows) an x pass covers:
// [b0, b0 + n0) then [b1, b1 + n1)
struct PairRanges {
    int b0 = 0, n0 = 0, b1 = 0, n1 = 0;
};
// all packed row pairs of a slab
PairRanges all_pairs(const SpectralPlan& p);

// X pass A: conv1 result (Cin) -> quotient with img -> forward spectrum into Cout
void engine_quotient(const SpectralPlan& p, Store st, const float2* Cin, const void* img,
                     float2* Cout, const PairRanges& pr, hipStream_t s);
// X pass B: conv2 result (Cin) -> update psi_in -> psi_out, forward spectrum of the
// mirror-extended psi_out into Cout (when Cout != nullptr); stats partials (2 doubles / block).
// returns the number of partials written
int64_t engine_update(const SpectralPlan& p, Store st, const float2* Cin, const float* psi_in,
                      const void* w, double lambda, float* psi_out, float2* Cout, double* partials,
                      const PairRanges& pr, hipStream_t s);

}  // namespace spimdecon
