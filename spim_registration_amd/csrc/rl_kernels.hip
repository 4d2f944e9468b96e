// rl_kernels.hip -- HBM-bound pointwise / halo-pad kernels of the RL iteration.
//
// Padded volume layout (fft.hpp): circular placement -- padded coordinate q
// maps to image coordinate s(q) = q < n + c ? q : q - M, so the image interior
// sits at q = s (row-aligned with the unpadded arrays) and the halo of width c
// wraps around the end of each axis.  Every kernel walks the padded volume
// one wave per padded row (wave-uniform z/y decode, lanes over x).
//
// Float semantics follow the Java reference exactly (no contraction):
//   quotient  img > 0 ? img / blurred : 1             MVDeconvolution.java:473-525
//   update    computeNextValue + Tikhonov (f64 sqrt)   MVDeconvolution.java:671-705
#include "rl_kernels.hpp"
#include "rl_math.hpp"

#include <algorithm>

namespace spimdecon {

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ int64_t s_of_q(int64_t q, int64_t n, int c, int64_t M) {
    return q < n + c ? q : q - M;
}

template <int S>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
    if constexpr (S == 0) {
        return static_cast<const float*>(p)[i];
    } else {
        return __half2float(static_cast<const __half*>(p)[i]);
    }
}

struct RowMap {
    bool skip;       // internal z halo (filled by the exchange) or out-of-range row
    bool zout;       // outside the global volume in z
    bool yout;
    int64_t lz, ly;  // mirror-mapped local source row
    bool zin, yin;   // row is an interior row (s == mirror(s))
    int64_t sy;
};

__device__ __forceinline__ RowMap map_row(const SlabGeom& g, int64_t row) {
    RowMap r;
    const int64_t qz = row / g.My;
    const int64_t qy = row - qz * g.My;
    const int64_t sz = s_of_q(qz, g.nz, g.cz, g.Mz);
    const int64_t gz = g.z0 + sz;
    const bool global_in = gz >= 0 && gz < g.nzg;
    r.skip = global_in && (sz < 0 || sz >= g.nz);
    r.zout = !global_in;
    r.lz = mirror_idx(gz, g.nzg) - g.z0;
    r.zin = (sz >= 0 && sz < g.nz);
    if (!r.skip && (r.lz < 0 || r.lz >= g.nz)) r.skip = true;  // host guarantees this never happens
    r.sy = s_of_q(qy, g.ny, g.cy, g.My);
    r.yout = r.sy < 0 || r.sy >= g.ny;
    r.ly = mirror_idx(r.sy, g.ny);
    r.yin = !r.yout;
    return r;
}

__global__ __launch_bounds__(kBlock) void k_pad_mirror(SlabGeom g, const float* __restrict__ psi,
                                                        float* __restrict__ Ra) {
    const int lane = threadIdx.x & 63;
    const int64_t rows = g.My * g.Mz;
    for (int64_t row = int64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6); row < rows;
         row += int64_t(gridDim.x) * kWaves) {
        const RowMap r = map_row(g, row);
        if (r.skip) continue;
        const float* src = psi + (r.lz * g.ny + r.ly) * g.nx;
        float* dst = Ra + row * g.Sx;
        for (int64_t qx = lane; qx < g.Mx; qx += 64) {
            const int64_t lx = mirror_idx(s_of_q(qx, g.nx, g.cx, g.Mx), g.nx);
            dst[qx] = src[lx];
        }
    }
}

template <int S>
__global__ __launch_bounds__(kBlock) void k_quotient_pad(SlabGeom g, const void* __restrict__ img,
                                                          const float* __restrict__ Ra,
                                                          float* __restrict__ Rb) {
    const int lane = threadIdx.x & 63;
    const int64_t rows = g.My * g.Mz;
    for (int64_t row = int64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6); row < rows;
         row += int64_t(gridDim.x) * kWaves) {
        const RowMap r = map_row(g, row);
        if (r.skip) continue;
        float* dst = Rb + row * g.Sx;
        if (r.zout || r.yout) {
            for (int64_t qx = lane; qx < g.Mx; qx += 64) dst[qx] = 1.0f;
            continue;
        }
        // interior row: q == s, Ra row == this row
        const float* blurred = Ra + row * g.Sx;
        const int64_t base = (r.lz * g.ny + r.ly) * g.nx;
        for (int64_t qx = lane; qx < g.Mx; qx += 64) {
            float out = 1.0f;
            if (qx < g.nx) {
                const float iv = ld<S>(img, base + qx);
                if (iv > 0.0f) out = __fdiv_rn(iv, blurred[qx]);
            }
            dst[qx] = out;
        }
    }
}

__device__ __forceinline__ void block_reduce_sum_max(double& sum, float& mx, double* sh_sum,
                                                     float* sh_max) {
    for (int off = 32; off > 0; off >>= 1) {
        sum += __shfl_xor(sum, off, 64);
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh_sum[wid] = sum;
        sh_max[wid] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWaves; ++w) {
            sum += sh_sum[w];
            mx = fmaxf(mx, sh_max[w]);
        }
    }
}

template <int S>
__global__ __launch_bounds__(kBlock) void k_update_pad(SlabGeom g, const float* __restrict__ psi_in,
                                                        const float* __restrict__ Rb,
                                                        const void* __restrict__ w, double lambda,
                                                        float* __restrict__ psi_out,
                                                        float* __restrict__ Ra,
                                                        double* __restrict__ partials,
                                                        int write_pad) {
    __shared__ double sh_sum[kWaves];
    __shared__ float sh_max[kWaves];
    const int lane = threadIdx.x & 63;
    const int64_t rows = g.My * g.Mz;
    double sum = 0.0;
    float mx = -1.0f;
    for (int64_t row = int64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6); row < rows;
         row += int64_t(gridDim.x) * kWaves) {
        const RowMap r = map_row(g, row);
        if (r.skip) continue;
        const bool interior_row = r.zin && r.yin;
        if (!write_pad && !interior_row) continue;
        const int64_t vbase = (r.lz * g.ny + r.ly) * g.nx;
        const float* integ = Rb + (r.lz * g.My + r.ly) * g.Sx;  // interior slot of the source row
        float* dst = Ra + row * g.Sx;
        for (int64_t qx = lane; qx < g.Mx; qx += 64) {
            const int64_t sx = s_of_q(qx, g.nx, g.cx, g.Mx);
            const bool xin = sx >= 0 && sx < g.nx;
            if (!write_pad && !xin) continue;
            const int64_t lx = mirror_idx(sx, g.nx);
            const float last = psi_in[vbase + lx];
            const float nv = next_value(last, integ[lx], ld<S>(w, vbase + lx), lambda);
            if (write_pad) dst[qx] = nv;
            if (interior_row && xin) {
                psi_out[vbase + lx] = nv;
                const float ch = fabsf(__fsub_rn(nv, last));
                sum += (double)ch;
                mx = fmaxf(mx, ch);
            }
        }
    }
    block_reduce_sum_max(sum, mx, sh_sum, sh_max);
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = sum;
        partials[2 * blockIdx.x + 1] = (double)mx;
    }
}

// one block of kRedThreads: the update pass leaves one {sum, max} per block (one
// tile per block: ~18 k partials at 540^3), summed in a fixed order (deterministic)
constexpr int kRedThreads = 1024;
__global__ __launch_bounds__(kRedThreads) void k_reduce_partials(const double* __restrict__ partials,
                                                                 int64_t n, double* out, int accumulate) {
    __shared__ double sh_sum[kRedThreads / 64];
    __shared__ double sh_max[kRedThreads / 64];
    double sum = 0.0, mx = -1.0;
    for (int64_t i = threadIdx.x; i < n; i += kRedThreads) {
        sum += partials[2 * i];
        mx = fmax(mx, partials[2 * i + 1]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        sum += __shfl_xor(sum, off, 64);
        mx = fmax(mx, __shfl_xor(mx, off, 64));
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh_sum[wid] = sum;
        sh_max[wid] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w2 = 1; w2 < kRedThreads / 64; ++w2) {
            sum += sh_sum[w2];
            mx = fmax(mx, sh_max[w2]);
        }
        if (accumulate) {
            out[0] += sum;
            out[1] = fmax(out[1], mx);
        } else {
            out[0] = sum;
            out[1] = mx;
        }
    }
}

// ComplexFloatType.mul: (a*c - b*d, a*d + b*c)
__global__ __launch_bounds__(kBlock) void k_spec_mul(float4* __restrict__ C,
                                                      const float4* __restrict__ K, int64_t n2,
                                                      float2* __restrict__ Ct,
                                                      const float2* __restrict__ Kt, int tail) {
    const int64_t stride = int64_t(gridDim.x) * kBlock;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n2; i += stride) {
        const float4 a = C[i];
        const float4 k = K[i];
        float4 r;
        r.x = a.x * k.x - a.y * k.y;
        r.y = a.x * k.y + a.y * k.x;
        r.z = a.z * k.z - a.w * k.w;
        r.w = a.z * k.w + a.w * k.z;
        C[i] = r;
    }
    if (tail && blockIdx.x == 0 && threadIdx.x == 0) {
        const float2 a = *Ct;
        const float2 k = *Kt;
        *Ct = make_float2(a.x * k.x - a.y * k.y, a.x * k.y + a.y * k.x);
    }
}

__global__ void k_place_kernel(SlabGeom g, const float* __restrict__ k, int kx, int ky, int kz,
                               float scale, float* __restrict__ R) {
    const int64_t n = int64_t(kx) * ky * kz;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t jx = i % kx;
        const int64_t jy = (i / kx) % ky;
        const int64_t jz = i / (int64_t(kx) * ky);
        int64_t qx = (jx - kx / 2) % g.Mx; if (qx < 0) qx += g.Mx;
        int64_t qy = (jy - ky / 2) % g.My; if (qy < 0) qy += g.My;
        int64_t qz = (jz - kz / 2) % g.Mz; if (qz < 0) qz += g.Mz;
        // kernels larger than the FFT volume wrap (accumulate): atomic keeps it exact for overlaps
        atomicAdd(&R[(qz * g.My + qy) * g.Sx + qx], k[i] * scale);
    }
}

template <int S>
__global__ __launch_bounds__(kBlock) void k_first_iteration(int64_t n, int nviews,
                                                             const void* const* __restrict__ imgs,
                                                             double* __restrict__ partials) {
    __shared__ double sh_a[kWaves];
    __shared__ double sh_b[kWaves];
    double msum = 0.0, cnt = 0.0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * kBlock) {
        double s = 0.0;
        int c = 0;
        for (int v = 0; v < nviews; ++v) {
            const double x = (double)ld<S>(imgs[v], i);
            if (x > 0.0) {
                s += x;
                ++c;
            }
        }
        if (c > 0) {
            msum += s / (double)c;
            cnt += 1.0;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        msum += __shfl_xor(msum, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh_a[wid] = msum;
        sh_b[wid] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWaves; ++w) {
            msum += sh_a[w];
            cnt += sh_b[w];
        }
        partials[2 * blockIdx.x] = msum;
        partials[2 * blockIdx.x + 1] = cnt;
    }
}

__global__ void k_fill(float* p, int64_t n, float v) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        p[i] = v;
}

__global__ void k_clamp_min(float* p, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        if (p[i] <= 0.0f) p[i] = kMinValue;
}

template <int S>
__global__ void k_mask(float* psi, int64_t n, int nviews, const void* const* __restrict__ imgs) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        bool any = false;
        for (int v = 0; v < nviews; ++v) any |= ld<S>(imgs[v], i) > 0.0f;
        if (!any) psi[i] = 0.0f;
    }
}

__global__ void k_to_half(const float* __restrict__ in, __half* __restrict__ out, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        out[i] = __float2half(in[i]);
}

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap = 256 * 16) {
    int64_t b = ceil_div(work, per_block);
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return unsigned(b);
}

}  // namespace

void launch_pad_mirror(const SlabGeom& g, const float* psi, float* Ra, hipStream_t s) {
    const unsigned grid = grid_for(g.My * g.Mz, kWaves);
    hipLaunchKernelGGL(k_pad_mirror, dim3(grid), dim3(kBlock), 0, s, g, psi, Ra);
    SD_HIP(hipGetLastError());
}

void launch_quotient_pad(const SlabGeom& g, Store st, const void* img, const float* Ra, float* Rb,
                         hipStream_t s) {
    const unsigned grid = grid_for(g.My * g.Mz, kWaves);
    if (st == Store::F32)
        hipLaunchKernelGGL(k_quotient_pad<0>, dim3(grid), dim3(kBlock), 0, s, g, img, Ra, Rb);
    else
        hipLaunchKernelGGL(k_quotient_pad<1>, dim3(grid), dim3(kBlock), 0, s, g, img, Ra, Rb);
    SD_HIP(hipGetLastError());
}

int64_t launch_update_pad(const SlabGeom& g, Store st, const float* psi_in, const float* Rb,
                          const void* w, double lambda, float* psi_out, float* Ra,
                          double* partials, bool write_pad, hipStream_t s) {
    const unsigned grid = grid_for(g.My * g.Mz, kWaves);
    if (st == Store::F32)
        hipLaunchKernelGGL(k_update_pad<0>, dim3(grid), dim3(kBlock), 0, s, g, psi_in, Rb, w,
                           lambda, psi_out, Ra, partials, int(write_pad));
    else
        hipLaunchKernelGGL(k_update_pad<1>, dim3(grid), dim3(kBlock), 0, s, g, psi_in, Rb, w,
                           lambda, psi_out, Ra, partials, int(write_pad));
    SD_HIP(hipGetLastError());
    return grid;
}

void launch_reduce_partials(const double* partials, int64_t nblocks, double* out, int accumulate,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kRedThreads), 0, s, partials, nblocks, out,
                       accumulate);
    SD_HIP(hipGetLastError());
}

void launch_spec_mul(float* C, const float* K, int64_t n, hipStream_t s) {
    const int64_t n2 = n / 2;
    const int tail = int(n & 1);
    const unsigned grid = grid_for(n2, kBlock, 256 * 32);
    hipLaunchKernelGGL(k_spec_mul, dim3(grid), dim3(kBlock), 0, s, reinterpret_cast<float4*>(C),
                       reinterpret_cast<const float4*>(K), n2,
                       reinterpret_cast<float2*>(C) + (n - 1),
                       reinterpret_cast<const float2*>(K) + (n - 1), tail);
    SD_HIP(hipGetLastError());
}

void launch_place_kernel(const SlabGeom& g, const float* k, int kx, int ky, int kz, float scale,
                         float* R, hipStream_t s) {
    SD_HIP(hipMemsetAsync(R, 0, size_t(g.Sx * g.My * g.Mz) * sizeof(float), s));
    const int64_t n = int64_t(kx) * ky * kz;
    hipLaunchKernelGGL(k_place_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, g, k, kx, ky, kz,
                       scale, R);
    SD_HIP(hipGetLastError());
}

int64_t launch_first_iteration(int64_t n, int nviews, Store st, const void* const* d_imgs,
                               double* partials, hipStream_t s) {
    const unsigned grid = grid_for(n, kBlock, 2048);
    if (st == Store::F32)
        hipLaunchKernelGGL(k_first_iteration<0>, dim3(grid), dim3(kBlock), 0, s, n, nviews, d_imgs,
                           partials);
    else
        hipLaunchKernelGGL(k_first_iteration<1>, dim3(grid), dim3(kBlock), 0, s, n, nviews, d_imgs,
                           partials);
    SD_HIP(hipGetLastError());
    return grid;
}

void launch_fill(float* p, int64_t n, float v, hipStream_t s) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n, v);
    SD_HIP(hipGetLastError());
}

void launch_clamp_min(float* p, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_clamp_min, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n);
    SD_HIP(hipGetLastError());
}

void launch_mask(float* psi, int64_t n, int nviews, Store st, const void* const* d_imgs,
                 hipStream_t s) {
    if (st == Store::F32)
        hipLaunchKernelGGL(k_mask<0>, dim3(grid_for(n, 256)), dim3(256), 0, s, psi, n, nviews,
                           d_imgs);
    else
        hipLaunchKernelGGL(k_mask<1>, dim3(grid_for(n, 256)), dim3(256), 0, s, psi, n, nviews,
                           d_imgs);
    SD_HIP(hipGetLastError());
}

// b[y][z][:] = a[z][y][:]; block = 256 threads over one row (grid-stride over rows)
__global__ __launch_bounds__(256) void k_swap_outer(const float* __restrict__ a, float* __restrict__ b, int64_t nx,
                                                    int64_t ny, int64_t nz) {
    const int64_t rows = ny * nz;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        const int64_t y = r / nz, z = r % nz;   // destination row r = y * nz + z
        const float* src = a + (z * ny + y) * nx;
        float* dst = b + r * nx;
        for (int64_t x = threadIdx.x; x < nx; x += 256) dst[x] = src[x];
    }
}

void launch_swap_outer(const float* a, float* b, int64_t nx, int64_t ny, int64_t nz, hipStream_t s) {
    const int64_t rows = ny * nz;
    if (rows == 0 || nx == 0) return;
    hipLaunchKernelGGL(k_swap_outer, dim3(unsigned(std::min<int64_t>(rows, 256 * 64))), dim3(256), 0, s, a, b, nx,
                       ny, nz);
    SD_HIP(hipGetLastError());
}

// out[i] = computeNextValue(last[i], integral[i], weight[i]) -- the per-voxel rule of
// both update paths, exposed for bit-exact checks against the reference rule
__global__ __launch_bounds__(kBlock) void k_next_value(const float* __restrict__ last,
                                                       const float* __restrict__ integ,
                                                       const float* __restrict__ w, int64_t n, double lambda,
                                                       float* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (i < n) out[i] = next_value(last[i], integ[i], w[i], lambda);
}

void launch_next_value(const float* last, const float* integral, const float* weight, int64_t n, double lambda,
                       float* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_next_value, dim3(unsigned((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, last, integral,
                       weight, n, lambda, out);
    SD_HIP(hipGetLastError());
}

// halo planes pulled by a kernel (SPIMDECON_PULL=kernel) instead of hipMemcpyAsync: the
// loads read the source's HBM directly (a peer device's over xGMI when src lives there,
// peer access enabled), 16-B accesses, four in flight per lane, a few blocks only
__global__ __launch_bounds__(256) void k_pull_copy(const float4* __restrict__ src, float4* __restrict__ dst,
                                                   int64_t n4) {
    const int64_t stride = int64_t(gridDim.x) * 256;
    int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n4; i += stride) dst[i] = src[i];
}

void launch_pull_copy(float* dst, const float* src, size_t bytes, hipStream_t s) {
    SD_CHECK(bytes % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0,
             SPIMDECON_ERR_ARG, "pull copy needs 16-B aligned whole float4");
    const int64_t n4 = int64_t(bytes / 16);
    if (n4 == 0) return;
    const unsigned grid = unsigned(std::min<int64_t>(64, (n4 + 1023) / 1024));
    hipLaunchKernelGGL(k_pull_copy, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                       reinterpret_cast<float4*>(dst), n4);
    SD_HIP(hipGetLastError());
}

void launch_to_half(const float* in, void* out, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_to_half, dim3(grid_for(n, 256)), dim3(256), 0, s, in,
                       static_cast<__half*>(out), n);
    SD_HIP(hipGetLastError());
}

}  // namespace spimdecon
