// kernel_prep.hip -- MVDeconFFT.init on the GPU: normImg quirk, inverted /
// exponential / compound kernels (spim/process/fusion/deconvolution/MVDeconFFT.java:162-333,
// AdjustInput.java:29-100, Mirror.java:31-108).  Kernels are tiny (<= ~51^3);
// these are single-launch, latency-bound setup kernels.
#include "kernel_prep.hpp"

namespace spimdecon {

namespace {

constexpr int kBlock = 256;

// AdjustInput.normImg with the sumImg double count: total = sums[0] + sum_p sums[p]
// over 2*T flat portions (FusionHelper.divideIntoPortions), then
// t = (float)((double)t / total).  One block, deterministic order.
__global__ __launch_bounds__(kBlock) void k_norm_img(float* __restrict__ k, int64_t n, int nportions,
                                                      double* __restrict__ scratch) {
    __shared__ double sh[kBlock / 64];
    const int64_t chunk = n / nportions;
    const int64_t mod = n % nportions;
    for (int p = 0; p < nportions; ++p) {
        const int64_t start = int64_t(p) * chunk;
        const int64_t len = (p == nportions - 1) ? chunk + mod : chunk;
        double s = 0.0;
        for (int64_t i = threadIdx.x; i < len; i += kBlock) s += (double)k[start + i];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int w = 0; w < kBlock / 64; ++w) t += sh[w];
            scratch[p] = t;
        }
        __syncthreads();
    }
    __shared__ double total;
    if (threadIdx.x == 0) {
        double t = scratch[0];
        for (int p = 0; p < nportions; ++p) t += scratch[p];
        total = t;
    }
    __syncthreads();
    const double tot = total;
    for (int64_t i = threadIdx.x; i < n; i += kBlock) k[i] = (float)((double)k[i] / tot);
}

// Mirror.mirror along every axis (sequential-order semantics: for an even
// axis the middle pair is swapped twice and stays in place).
__device__ __forceinline__ int mirror_pos(int p, int s) {
    if ((s & 1) == 0 && (p == s / 2 - 1 || p == s / 2)) return p;
    return s - 1 - p;
}

__global__ void k_invert(const float* __restrict__ in, float* __restrict__ out, int kx, int ky,
                         int kz) {
    const int64_t n = int64_t(kx) * ky * kz;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int x = int(i % kx), y = int((i / kx) % ky), z = int(i / (int64_t(kx) * ky));
        const int64_t j = (int64_t(mirror_pos(z, kz)) * ky + mirror_pos(y, ky)) * kx + mirror_pos(x, kx);
        out[i] = in[j];
    }
}

// FFTConvolution(extendZero(a), a, extendZero(b), b, out): 'same' size as a,
// true convolution with b's centre b/2 at the origin; float64 accumulation.
// The same sum with the taps of one output voxel split over a block (double partial
// sums reduced in the block): a thread per output left all but ~72 blocks idle for
// the 31x19x31 kernels of 45-degree views (1.2 ms per compound-kernel convolution).
__global__ __launch_bounds__(kBlock) void k_conv_same_zero_blk(const float* __restrict__ a, int ax, int ay, int az,
                                                                const float* __restrict__ b, int bx, int by, int bz,
                                                                float* __restrict__ out) {
    __shared__ double part[kBlock / 64];
    const int64_t i = blockIdx.x;
    const int x = int(i % ax), y = int((i / ax) % ay), z = int(i / (int64_t(ax) * ay));
    const int cx = bx / 2, cy = by / 2, cz = bz / 2;
    const int nb = bx * by * bz;
    double acc = 0.0;
    // (jx, jy, jz) of t advanced by kBlock per step with carries instead of three runtime
    // divisions per product (same products in the same order)
    const int dx = kBlock % bx, dyq = kBlock / bx;
    const int dy = dyq % by, dz = dyq / by;
    int t = threadIdx.x;
    int jx = t % bx, jy = (t / bx) % by, jz = t / (bx * by);
    for (; t < nb; t += kBlock) {
        const int sx = x + cx - jx, sy = y + cy - jy, sz = z + cz - jz;
        if (!(sx < 0 || sx >= ax || sy < 0 || sy >= ay || sz < 0 || sz >= az))
            acc += double(a[(int64_t(sz) * ay + sy) * ax + sx]) * double(b[t]);
        jx += dx;
        int cy1 = dy, cz1 = dz;
        if (jx >= bx) { jx -= bx; ++cy1; }
        jy += cy1;
        if (jy >= by) { jy -= by; ++cz1; }
        jz += cz1;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double sum = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) sum += part[w];
        out[i] = float(sum);
    }
}

__global__ __launch_bounds__(kBlock) void k_conv_same_zero(const float* __restrict__ a, int ax,
                                                            int ay, int az,
                                                            const float* __restrict__ b, int bx,
                                                            int by, int bz,
                                                            float* __restrict__ out) {
    const int64_t n = int64_t(ax) * ay * az;
    const int cx = bx / 2, cy = by / 2, cz = bz / 2;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int x = int(i % ax), y = int((i / ax) % ay), z = int(i / (int64_t(ax) * ay));
        double acc = 0.0;
        for (int jz = 0; jz < bz; ++jz) {
            const int sz = z + cz - jz;
            if (sz < 0 || sz >= az) continue;
            for (int jy = 0; jy < by; ++jy) {
                const int sy = y + cy - jy;
                if (sy < 0 || sy >= ay) continue;
                const float* arow = a + (int64_t(sz) * ay + sy) * ax;
                const float* brow = b + (int64_t(jz) * by + jy) * bx;
                for (int jx = 0; jx < bx; ++jx) {
                    const int sx = x + cx - jx;
                    if (sx < 0 || sx >= ax) continue;
                    acc += (double)arow[sx] * (double)brow[jx];
                }
            }
        }
        out[i] = (float)acc;
    }
}

// out = a * b (float; MVDeconFFT.java:230-235,277-282 `output * tmp`)
__global__ void k_mul(const float* __restrict__ a, float* __restrict__ b, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        b[i] = __fmul_rn(a[i], b[i]);
}

// MVDeconFFT.pow (:325-333): result = v; repeat (power-1) times result *= v
__global__ void k_pow(const float* __restrict__ in, float* __restrict__ out, int64_t n, int power) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const float v = in[i];
        float r = v;
        for (int p = 1; p < power; ++p) r = __fmul_rn(r, v);
        out[i] = r;
    }
}

unsigned grid_of(int64_t n) {
    int64_t b = ceil_div(n, kBlock);
    return unsigned(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

struct DevKernel {
    DBuf<float> d;
    int k[3];
    int64_t n() const { return int64_t(k[0]) * k[1] * k[2]; }
};

void norm_img(DevKernel& K, int T, double* scratch, hipStream_t s) {
    hipLaunchKernelGGL(k_norm_img, dim3(1), dim3(kBlock), 0, s, K.d.p, K.n(), 2 * T, scratch);
    SD_HIP(hipGetLastError());
}

void invert(const DevKernel& in, DevKernel& out, hipStream_t s) {
    out.k[0] = in.k[0]; out.k[1] = in.k[1]; out.k[2] = in.k[2];
    if (out.d.n != size_t(in.n())) out.d.alloc(in.n());
    hipLaunchKernelGGL(k_invert, dim3(grid_of(in.n())), dim3(kBlock), 0, s, in.d.p, out.d.p, in.k[0],
                       in.k[1], in.k[2]);
    SD_HIP(hipGetLastError());
}

void conv_same_zero(const DevKernel& a, const DevKernel& b, DevKernel& out, hipStream_t s) {
    out.k[0] = a.k[0]; out.k[1] = a.k[1]; out.k[2] = a.k[2];
    if (out.d.n != size_t(a.n())) out.d.alloc(a.n());
    if (a.n() * b.n() >= (int64_t(1) << 22)) {   // large kernels: one block per output voxel
        hipLaunchKernelGGL(k_conv_same_zero_blk, dim3(unsigned(a.n())), dim3(kBlock), 0, s, a.d.p, a.k[0], a.k[1],
                           a.k[2], b.d.p, b.k[0], b.k[1], b.k[2], out.d.p);
    } else {
        hipLaunchKernelGGL(k_conv_same_zero, dim3(grid_of(a.n())), dim3(kBlock), 0, s, a.d.p, a.k[0],
                           a.k[1], a.k[2], b.d.p, b.k[0], b.k[1], b.k[2], out.d.p);
    }
    SD_HIP(hipGetLastError());
}

void mul_into(const DevKernel& a, DevKernel& b, hipStream_t s) {
    hipLaunchKernelGGL(k_mul, dim3(grid_of(a.n())), dim3(kBlock), 0, s, a.d.p, b.d.p, a.n());
    SD_HIP(hipGetLastError());
}

void copy(const DevKernel& in, DevKernel& out, hipStream_t s) {
    out.k[0] = in.k[0]; out.k[1] = in.k[1]; out.k[2] = in.k[2];
    if (out.d.n != size_t(in.n())) out.d.alloc(in.n());
    SD_HIP(hipMemcpyAsync(out.d.p, in.d.p, in.d.bytes(), hipMemcpyDeviceToDevice, s));
}

}  // namespace

void prepare_kernels_gpu(std::vector<HostKernel>& k1, std::vector<HostKernel>& k2, int psftype,
                         int ij_threads, int dev) {
    check_device(dev);
    DeviceGuard guard(dev);
    SD_CHECK(ij_threads >= 1, SPIMDECON_ERR_ARG, "ij_threads must be >= 1");
    SD_CHECK(psftype >= 0 && psftype <= 3, SPIMDECON_ERR_ARG, "unknown psftype");
    const int V = int(k1.size());
    SD_CHECK(V >= 1, SPIMDECON_ERR_ARG, "no views");
    hipStream_t s;
    SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{s};

    std::vector<DevKernel> K1(V);
    for (int v = 0; v < V; ++v) {
        for (int d = 0; d < 3; ++d) {
            SD_CHECK(k1[v].dims[d] >= 1 && (k1[v].dims[d] & 1), SPIMDECON_ERR_ARG,
                     "kernel dims must be odd (EfficientBayesianBased.java:792-799)");
            K1[v].k[d] = k1[v].dims[d];
        }
        SD_CHECK(k1[v].data.size() == size_t(K1[v].n()), SPIMDECON_ERR_ARG, "kernel size mismatch");
        K1[v].d.alloc(K1[v].n());
        SD_HIP(hipMemcpyAsync(K1[v].d.p, k1[v].data.data(), K1[v].d.bytes(), hipMemcpyHostToDevice, s));
    }
    DBuf<double> scratch(2 * size_t(ij_threads));
    std::vector<DevKernel> K2(V);
    DevKernel tmp, in, ker, out, out2;
    for (int v = 0; v < V; ++v) {
        norm_img(K1[v], ij_threads, scratch.p, s);                          // :165
        if (V == 1 || psftype == MVD_PSF_INDEPENDENT) {                     // :176-180
            invert(K1[v], K2[v], s);
        } else if (psftype == MVD_PSF_EFFICIENT_BAYESIAN) {                 // :181-244
            invert(K1[v], tmp, s);
            for (int w = 0; w < V; ++w) {
                if (w == v) continue;
                invert(K1[v], in, s);
                conv_same_zero(in, K1[w], out, s);
                invert(K1[w], ker, s);
                conv_same_zero(out, ker, out2, s);
                mul_into(out2, tmp, s);
            }
            norm_img(tmp, ij_threads, scratch.p, s);
            copy(tmp, K2[v], s);
        } else if (psftype == MVD_PSF_OPTIMIZATION_I) {                     // :245-291
            copy(K1[v], tmp, s);
            for (int w = 0; w < V; ++w) {
                if (w == v) continue;
                invert(K1[w], ker, s);
                conv_same_zero(K1[v], ker, out, s);
                mul_into(out, tmp, s);
            }
            norm_img(tmp, ij_threads, scratch.p, s);
            invert(tmp, K2[v], s);
        } else {                                                            // OPTIMIZATION_II :292-302
            DevKernel e;
            e.k[0] = K1[v].k[0]; e.k[1] = K1[v].k[1]; e.k[2] = K1[v].k[2];
            e.d.alloc(K1[v].n());
            hipLaunchKernelGGL(k_pow, dim3(grid_of(K1[v].n())), dim3(kBlock), 0, s, K1[v].d.p, e.d.p,
                               K1[v].n(), V);
            SD_HIP(hipGetLastError());
            norm_img(e, ij_threads, scratch.p, s);
            invert(e, K2[v], s);
        }
    }
    k2.resize(V);
    for (int v = 0; v < V; ++v) {
        k1[v].data.resize(K1[v].n());
        SD_HIP(hipMemcpyAsync(k1[v].data.data(), K1[v].d.p, K1[v].d.bytes(), hipMemcpyDeviceToHost, s));
        k2[v].dims[0] = K2[v].k[0]; k2[v].dims[1] = K2[v].k[1]; k2[v].dims[2] = K2[v].k[2];
        k2[v].data.resize(K2[v].n());
        SD_HIP(hipMemcpyAsync(k2[v].data.data(), K2[v].d.p, K2[v].d.bytes(), hipMemcpyDeviceToHost, s));
    }
    SD_HIP(hipStreamSynchronize(s));
}

}  // namespace spimdecon
