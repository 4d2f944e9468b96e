// rl_kernels.hpp -- launchers of the RL pointwise/pad kernels (rl_kernels.hip).
#pragma once

#include <cstdint>

#include "common.hpp"

namespace spimdecon {

// Geometry of one z-slab and its padded FFT volume.
struct SlabGeom {
    int64_t nx, ny, nz;   // local slab dims (nx, ny global; nz local)
    int64_t z0, nzg;      // first global plane, global nz
    int64_t Mx, My, Mz;   // FFT lengths
    int64_t Sx;           // padded real row stride (2*(Mx/2+1))
    int cx, cy, cz;       // halo = max kernel half size per axis
};

enum class Store { F32 = 0, F16 = 1 };

constexpr float kMinValue = 0.0001f;  // MVDeconvolution.java:49

// Ra[q] = E_mirror(psi)[s(q)] for every padded position except internal z halos.
void launch_pad_mirror(const SlabGeom& g, const float* psi, float* Ra, hipStream_t s);

// Rb[q] = img>0 ? img/Ra : 1 inside, 1 outside the global volume (internal z
// halos skipped).  Ra holds the convolve1 result at padded interior slots.
void launch_quotient_pad(const SlabGeom& g, Store st, const void* img, const float* Ra, float* Rb,
                         hipStream_t s);

// psi_out = update(psi_in, Rb, w) at interior; Ra[q] = E_mirror(psi_out)[s(q)];
// per-block {sum |change|, max |change|} partials into `partials` (2 doubles / block).
// Returns the number of blocks (partials written).
int64_t launch_update_pad(const SlabGeom& g, Store st, const float* psi_in, const float* Rb,
                          const void* w, double lambda, float* psi_out, float* Ra,
                          double* partials, bool write_pad, hipStream_t s);

// out[i] = the RL update rule (MVDeconvolution.computeNextValue) of voxel i, device arrays
void launch_next_value(const float* last, const float* integral, const float* weight, int64_t n, double lambda,
                       float* out, hipStream_t s);

// out[0] += sum(partials[2i]), out[1] = max(out[1], max(partials[2i+1])) -- single block,
// deterministic order.  `accumulate` = 0 overwrites out.
void launch_reduce_partials(const double* partials, int64_t nblocks, double* out, int accumulate,
                            hipStream_t s);

// complex multiply C[i] *= K[i] over n complex values
void launch_spec_mul(float* C, const float* K, int64_t n, hipStream_t s);

// zero `R` then place kernel k (dims kx,ky,kz x-fastest) circularly shifted so
// its centre k/2 sits at the origin, scaled by `scale`.
void launch_place_kernel(const SlabGeom& g, const float* k, int kx, int ky, int kz, float scale,
                         float* R, hipStream_t s);

// first iteration: per-block partials {sum of mean, count of voxels with data}
int64_t launch_first_iteration(int64_t n, int nviews, Store st, const void* const* d_imgs,
                               double* partials, hipStream_t s);
void launch_fill(float* p, int64_t n, float v, hipStream_t s);
// psi = v <= 0 ? minValue : v   (checkNumbers clamp, MVDeconvolution.java:295-305)
void launch_clamp_min(float* p, int64_t n, hipStream_t s);
// psi = 0 where every view has img <= 0 (MVDeconvolution.java:180-187)
void launch_mask(float* psi, int64_t n, int nviews, Store st, const void* const* d_imgs,
                 hipStream_t s);
// float32 -> fp16 conversion (storage mode)
void launch_to_half(const float* in, void* out, int64_t n, hipStream_t s);
// bytes from src to dst by a copy kernel on s (src may live on a peer device)
void launch_pull_copy(float* dst, const float* src, size_t bytes, hipStream_t s);
// Swaps the two outer axes of an x-fastest volume, whole x rows at a time (the
// y-slab layout of the session): a [nz][ny][nx] -> b[ny][nz][nx], b(y,z) = a(z,y).
// Coalesced row copies (one block per row pair of 4 rows), nx % 4 == 0 not needed.
void launch_swap_outer(const float* a, float* b, int64_t nx, int64_t ny, int64_t nz, hipStream_t s);

}  // namespace spimdecon
