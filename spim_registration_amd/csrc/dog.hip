// dog.hip -- separable Gaussian convolution (SeparableConvolutionCUDALib ABI) and the
// Difference-of-Gaussian bead-detection pass on MI355X.
//
// References (under /root/reference/src/main/java/):
//   spim/process/cuda/CUDASeparableConvolution.java:13-21        convolve_N ABI
//   spim/process/cuda/CUDASeparableConvolutionFunctions.java:127-245 kernels, sizes
//   spim/process/interestpointdetection/ProcessDOG.java:40-178   pipeline, sigmas
//   spim/process/interestpointdetection/DifferenceOfGaussianCUDA.java:116-181 (accurate = mirror-single)
//   spim/process/interestpointdetection/DifferenceOfGaussianNewPeakFinder.java:54-136
//   mpicbg/spim/segmentation/InteractiveIntegral.java:360-468     findPeaks / isSpecialPoint
//   spim/process/fusion/FusionHelper.java:176-234                 normalizeImage
//
// Data flow of one DoG (all HBM-resident, 5 streaming passes):
//   x-pass  img --(normalise on the fly)--> G1x, G2x      (both sigmas from one read)
//   y-pass  G1x -> G1xy, G2x -> G2xy
//   z-pass  G1xy, G2xy -> dog = (G2 - G1) * 1/(k-1)       (subtraction fused)
//   peaks   26-neighbour extremum test + order-preserving compaction
// Accumulation order per pass = tap order in float32 (matches the oracle bit for bit).
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace spimdecon {

namespace {

constexpr int kBlock = 256;
enum Oob { OOB_ZERO = 0, OOB_VALUE = 1, OOB_BORDER = 2, OOB_MIRROR = 3 };

struct Dims3 {
    int64_t nx, ny, nz;
};

__device__ __forceinline__ int64_t ext_index(int64_t i, int64_t n, int mode, bool& outside) {
    outside = false;
    if (i >= 0 && i < n) return i;
    if (mode == OOB_BORDER) return i < 0 ? 0 : n - 1;
    if (mode == OOB_MIRROR) {
        if (n == 1) return 0;
        const int64_t p = 2 * (n - 1);
        int64_t j = i % p;
        if (j < 0) j += p;
        return j >= n ? p - j : j;
    }
    outside = true;
    return 0;
}

struct NormParams {
    const float* minmax;  // device {min, max} or nullptr (no normalisation)
};

// FusionHelper.normalizeImage: (t - min) / (max - min) in float; skipped when
// the range is NaN / inf / 0 (the reference then keeps the raw image).
__device__ __forceinline__ float normalize(float v, const float* mm) {
    if (!mm) return v;
    const float mn = mm[0];
    const float diff = __fsub_rn(mm[1], mn);
    if (isnan(diff) || isinf(diff) || diff == 0.0f) return v;
    return __fdiv_rn(__fsub_rn(v, mn), diff);
}

// One separable pass along `axis` (0 = x, 1 = y, 2 = z) for NK (1 or 2) kernels
// of equal length K; MODE_OUT: 0 = write each result, 1 = write (o1 - o0) * scale.
template <int NK>
__global__ __launch_bounds__(kBlock) void k_sep_pass(Dims3 d, int axis, const float* __restrict__ in0,
                                                      const float* __restrict__ in1,
                                                      const float* __restrict__ k0,
                                                      const float* __restrict__ k1, int K, int mode,
                                                      float value, float* __restrict__ out0,
                                                      float* __restrict__ out1, int dog_out,
                                                      float dog_scale, const float* mm) {
    const int64_t n = d.nx * d.ny * d.nz;
    const int r = K / 2;
    const int64_t len = axis == 0 ? d.nx : (axis == 1 ? d.ny : d.nz);
    const int64_t stride = axis == 0 ? 1 : (axis == 1 ? d.nx : d.nx * d.ny);
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * kBlock) {
        int64_t pos;
        if (axis == 0) pos = i % d.nx;
        else if (axis == 1) pos = (i / d.nx) % d.ny;
        else pos = i / (d.nx * d.ny);
        const int64_t base = i - pos * stride;
        float a0 = 0.0f, a1 = 0.0f;
        for (int j = 0; j < K; ++j) {
            bool outside;
            const int64_t src = ext_index(pos + j - r, len, mode, outside);
            float v0, v1 = 0.0f;
            if (outside) {
                v0 = mode == OOB_VALUE ? value : 0.0f;
                v1 = v0;
            } else {
                v0 = normalize(in0[base + src * stride], mm);
                if (NK == 2) v1 = in1 ? normalize(in1[base + src * stride], mm) : v0;
            }
            a0 = __fadd_rn(a0, __fmul_rn(v0, k0[j]));
            if (NK == 2) a1 = __fadd_rn(a1, __fmul_rn(v1, k1[j]));
        }
        if (dog_out) {
            out0[i] = __fmul_rn(__fsub_rn(a1, a0), dog_scale);
        } else {
            out0[i] = a0;
            if (NK == 2) out1[i] = a1;
        }
    }
}

// Tiled separable passes (the bench path): 32-bit indices, the line segment of a
// block staged in LDS once (extension and normalisation applied while loading),
// taps from LDS, the same float32 tap order per output as k_sep_pass.  x pass: a
// block = 256 consecutive outputs of one row; y / z passes: 64 x-columns x 64
// positions along the axis (lanes run along x: coalesced, conflict-free).
typedef float dg_v2 __attribute__((ext_vector_type(2)));
constexpr int kSepX = 256;
constexpr int kSepRows = 8;  // rows per x-pass block (one 256-thread block per row segment was launch-bound)
constexpr int kSepTX = 64;
constexpr int kSepTY = 4;
constexpr int kSepTL = 64;

__device__ __forceinline__ int ext_index32(int i, int n, int mode, bool& outside) {
    outside = false;
    if (i >= 0 && i < n) return i;
    if (mode == OOB_BORDER) return i < 0 ? 0 : n - 1;
    if (mode == OOB_MIRROR) {
        if (n == 1) return 0;
        const int p = 2 * (n - 1);
        int j = i % p;
        if (j < 0) j += p;
        return j >= n ? p - j : j;
    }
    outside = true;
    return 0;
}

template <int NK>
__global__ __launch_bounds__(kSepX) void k_sep_x(Dims3 d, const float* __restrict__ in0,
                                                  const float* __restrict__ in1, const float* __restrict__ k0,
                                                  const float* __restrict__ k1, int K, int mode, float value,
                                                  float* __restrict__ out0, float* __restrict__ out1, int dog_out,
                                                  float dog_scale, const float* mm) {
    // NK == 2: both kernels' operands interleaved (float2), so one packed v_pk_mul /
    // v_pk_add (IEEE round-to-nearest per component, no FMA: bit-exact) serves both
    extern __shared__ __attribute__((aligned(8))) float sm[];
    const int r = K / 2;
    const int W = kSepX + K - 1;
    float* s0 = sm;                 // NK == 1: [W]; NK == 2: float2 [W]
    float* t0 = sm + NK * W;        // NK == 1: [K]; NK == 2: float2 [K]
    float2* s01 = reinterpret_cast<float2*>(sm);
    float2* t01 = reinterpret_cast<float2*>(t0);
    const int nx = int(d.nx);
    const int x0 = int(blockIdx.x) * kSepX;
    const int t = threadIdx.x;
    for (int i = t; i < K; i += kSepX) {
        if (NK == 2) t01[i] = make_float2(k0[i], k1[i]);
        else t0[i] = k0[i];
    }
    const bool same = in1 == nullptr || in1 == in0;
    const int y0 = int(blockIdx.y) * kSepRows;
    const int y1 = min(int(d.ny), y0 + kSepRows);
    for (int y = y0; y < y1; ++y) {
    const uint32_t row = (uint32_t(blockIdx.z) * uint32_t(d.ny) + uint32_t(y)) * uint32_t(nx);
    __syncthreads();  // the previous row's LDS reads are done
    for (int i = t; i < W; i += kSepX) {
        bool outside;
        const int src = ext_index32(x0 - r + i, nx, mode, outside);
        float v0, v1;
        if (outside) {
            v0 = mode == OOB_VALUE ? value : 0.0f;
            v1 = v0;
        } else {
            v0 = normalize(in0[row + src], mm);
            v1 = same ? v0 : normalize(in1[row + src], mm);
        }
        if (NK == 2) s01[i] = make_float2(v0, v1);
        else s0[i] = v0;
    }
    __syncthreads();
    const int x = x0 + t;
    if (x < nx) {
        float a0 = 0.0f, a1 = 0.0f;
        if constexpr (NK == 2) {
            dg_v2 acc = {0.0f, 0.0f};
            for (int j = 0; j < K; ++j) {
                const float2 v = s01[t + j], k = t01[j];
                acc = acc + dg_v2{v.x, v.y} * dg_v2{k.x, k.y};  // tap order kept, no contraction
            }
            a0 = acc.x;
            a1 = acc.y;
        } else {
            for (int j = 0; j < K; ++j) a0 = __fadd_rn(a0, __fmul_rn(s0[t + j], t0[j]));
        }
        if (dog_out) {
            out0[row + x] = __fmul_rn(__fsub_rn(a1, a0), dog_scale);
        } else {
            out0[row + x] = a0;
            if (NK == 2) out1[row + x] = a1;
        }
    }
    }
}

// AX 1 (y) or 2 (z): grid (x tiles, axis tiles, other coordinate)
// KW > 0: the tap count K == KW is known at compile time and a thread computes 16
// consecutive outputs from a register window of 16 + KW - 1 staged values (KW + 15
// LDS reads instead of 16 * KW); same per-output tap order.
template <int NK, int AX, int KW = 0>
__global__ __launch_bounds__(kSepTX * kSepTY) void k_sep_yz(Dims3 d, const float* __restrict__ in0,
                                                            const float* __restrict__ in1,
                                                            const float* __restrict__ k0,
                                                            const float* __restrict__ k1, int K, int mode,
                                                            float value, float* __restrict__ out0,
                                                            float* __restrict__ out1, int dog_out,
                                                            float dog_scale, const float* mm) {
    extern __shared__ __attribute__((aligned(8))) float sm[];
    const int r = K / 2;
    const int H = kSepTL + K - 1;  // staged positions along the axis
    float* s0 = sm;                       // NK == 1: [H][64]; NK == 2: float2 [H][64]
    float* t0 = sm + NK * H * kSepTX;     // NK == 1: [K]; NK == 2: float2 [K]
    float2* s01 = reinterpret_cast<float2*>(sm);
    float2* t01 = reinterpret_cast<float2*>(t0);
    const int nx = int(d.nx), ny = int(d.ny), nz = int(d.nz);
    const int len = AX == 1 ? ny : nz;
    const uint32_t astride = AX == 1 ? uint32_t(nx) : uint32_t(nx) * uint32_t(ny);
    const int tx = threadIdx.x % kSepTX, ty = threadIdx.x / kSepTX;
    const int x = int(blockIdx.x) * kSepTX + tx;
    const int a0p = int(blockIdx.y) * kSepTL;
    const int other = int(blockIdx.z);  // z for the y pass, y for the z pass
    const uint32_t base = AX == 1 ? uint32_t(other) * uint32_t(nx) * uint32_t(ny) + uint32_t(x)
                                  : uint32_t(other) * uint32_t(nx) + uint32_t(x);
    for (int i = threadIdx.x; i < K; i += kSepTX * kSepTY) {
        if (NK == 2) t01[i] = make_float2(k0[i], k1[i]);
        else t0[i] = k0[i];
    }
    const bool xin = x < nx;
    const bool same = in1 == nullptr || in1 == in0;
    for (int i = ty; i < H; i += kSepTY) {
        bool outside;
        const int src = ext_index32(a0p - r + i, len, mode, outside);
        float v0 = 0.0f, v1 = 0.0f;
        if (outside) {
            v0 = mode == OOB_VALUE ? value : 0.0f;
            v1 = v0;
        } else if (xin) {
            v0 = normalize(in0[base + uint32_t(src) * astride], mm);
            v1 = same ? v0 : normalize(in1[base + uint32_t(src) * astride], mm);
        }
        if (NK == 2) s01[i * kSepTX + tx] = make_float2(v0, v1);
        else s0[i * kSepTX + tx] = v0;
    }
    __syncthreads();
    if (!xin) return;
    if constexpr (KW > 0) {
        constexpr int OW = kSepTL / kSepTY;  // 16 consecutive outputs per thread
        constexpr int WN = OW + KW - 1;
        const int ob = ty * OW;
        if constexpr (NK == 2) {
            dg_v2 acc[OW], w[WN];
#pragma unroll
            for (int i = 0; i < WN; ++i) {
                const float2 v = s01[(ob + i) * kSepTX + tx];
                w[i] = dg_v2{v.x, v.y};
            }
#pragma unroll
            for (int o = 0; o < OW; ++o) acc[o] = dg_v2{0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const float2 kk = t01[j];
                const dg_v2 k = dg_v2{kk.x, kk.y};
#pragma unroll
                for (int o = 0; o < OW; ++o) acc[o] = acc[o] + w[o + j] * k;  // tap order kept
            }
#pragma unroll
            for (int o = 0; o < OW; ++o) {
                const int p = a0p + ob + o;
                if (p < len) {
                    const uint32_t idx = base + uint32_t(p) * astride;
                    if (dog_out) {
                        out0[idx] = __fmul_rn(__fsub_rn(acc[o].y, acc[o].x), dog_scale);
                    } else {
                        out0[idx] = acc[o].x;
                        out1[idx] = acc[o].y;
                    }
                }
            }
        } else {
            float acc[OW], w[WN];
#pragma unroll
            for (int i = 0; i < WN; ++i) w[i] = s0[(ob + i) * kSepTX + tx];
#pragma unroll
            for (int o = 0; o < OW; ++o) acc[o] = 0.0f;
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const float k = t0[j];
#pragma unroll
                for (int o = 0; o < OW; ++o) acc[o] = __fadd_rn(acc[o], __fmul_rn(w[o + j], k));
            }
#pragma unroll
            for (int o = 0; o < OW; ++o) {
                const int p = a0p + ob + o;
                if (p < len) out0[base + uint32_t(p) * astride] = acc[o];
            }
        }
        return;
    }
    for (int o = ty; o < kSepTL; o += kSepTY) {
        const int p = a0p + o;
        if (p >= len) break;
        float a0 = 0.0f, a1 = 0.0f;
        if constexpr (NK == 2) {
            dg_v2 acc = {0.0f, 0.0f};
            for (int j = 0; j < K; ++j) {
                const float2 v = s01[(o + j) * kSepTX + tx], k = t01[j];
                acc = acc + dg_v2{v.x, v.y} * dg_v2{k.x, k.y};
            }
            a0 = acc.x;
            a1 = acc.y;
        } else {
            for (int j = 0; j < K; ++j) a0 = __fadd_rn(a0, __fmul_rn(s0[(o + j) * kSepTX + tx], t0[j]));
        }
        const uint32_t idx = base + uint32_t(p) * astride;
        if (dog_out) {
            out0[idx] = __fmul_rn(__fsub_rn(a1, a0), dog_scale);
        } else {
            out0[idx] = a0;
            if (NK == 2) out1[idx] = a1;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_minmax(const float* __restrict__ in, int64_t n,
                                                    float* __restrict__ partial) {
    __shared__ float smn[kBlock / 64], smx[kBlock / 64];
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * kBlock) {
        const float v = in[i];
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, 64));
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) {
            mn = fminf(mn, smn[w]);
            mx = fmaxf(mx, smx[w]);
        }
        partial[2 * blockIdx.x] = mn;
        partial[2 * blockIdx.x + 1] = mx;
    }
}

// min / max over the per-block partials: one wave, lane-strided then shuffles
// (min and max are order-independent, so the result equals a sequential scan)
__global__ __launch_bounds__(64) void k_minmax_final(float* partial, int nb) {
    float mn = INFINITY, mx = -INFINITY;
    for (int b = threadIdx.x; b < nb; b += 64) {
        mn = fminf(mn, partial[2 * b]);
        mx = fmaxf(mx, partial[2 * b + 1]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, 64));
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    }
    if (threadIdx.x == 0) {
        partial[0] = mn;
        partial[1] = mx;
    }
}

// InteractiveIntegral.isSpecialPoint: 0 invalid, 1 MIN, 2 MAX
__device__ __forceinline__ int special_point(const float* __restrict__ dog, Dims3 d, int64_t i,
                                             int64_t x, int64_t y, int64_t z, float minv, float& val) {
    if (x < 1 || y < 1 || z < 1 || x > d.nx - 2 || y > d.ny - 2 || z > d.nz - 2) return 0;
    const float c = dog[i];
    val = c;
    if (fabsf(c) < minv) return 0;
    bool is_min = true, is_max = true;
    const int64_t sy = d.nx, sz = d.nx * d.ny;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                if (dz == 0 && dy == 0 && dx == 0) continue;
                const float v = dog[i + dz * sz + dy * sy + dx];
                is_min &= (v >= c);
                is_max &= (v <= c);
            }
    // "this mixup is intended": all neighbours >= centre => MAX (bright bead)
    if (is_min) return 2;
    if (is_max) return 1;
    return 0;
}

constexpr int kItems = 16;  // voxels per thread per chunk; chunk = kBlock * kItems

// (x, y, z) of flat index i: 32-bit divisions when the volume allows (a 64-bit
// division is a ~100-instruction software routine on the GPU)
__device__ __forceinline__ void flat_coords(int64_t i, const Dims3& d, int64_t& x, int64_t& y, int64_t& z) {
    if (d.nx * d.ny * d.nz < (int64_t(1) << 32)) {
        const uint32_t ii = uint32_t(i), nx = uint32_t(d.nx), ny = uint32_t(d.ny);
        const uint32_t q = ii / nx;
        x = ii - q * nx;
        z = q / ny;
        y = q - uint32_t(z) * ny;
    } else {
        x = i % d.nx;
        y = (i / d.nx) % d.ny;
        z = i / (d.nx * d.ny);
    }
}

__global__ __launch_bounds__(kBlock) void k_peaks_count(const float* __restrict__ dog, Dims3 d,
                                                         float minv, int want_min, int want_max,
                                                         int* __restrict__ counts) {
    __shared__ int sh[kBlock / 64];
    const int64_t n = d.nx * d.ny * d.nz;
    const int64_t chunk0 = int64_t(blockIdx.x) * kBlock * kItems;
    int cnt = 0;
    for (int it = 0; it < kItems; ++it) {
        const int64_t i = chunk0 + int64_t(it) * kBlock + threadIdx.x;
        if (i >= n) break;
        int64_t x, y, z;
        flat_coords(i, d, x, y, z);
        float v;
        const int sp = special_point(dog, d, i, x, y, z, minv, v);
        cnt += (sp == 2 && want_max) || (sp == 1 && want_min);
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += sh[w];
        counts[blockIdx.x] = t;
    }
}

// exclusive scan of counts: one block of kScanThreads, each thread scans a contiguous
// run of counts sequentially after a block-wide scan of the run totals
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_scan(const int* __restrict__ counts, int64_t nb,
                                                       int64_t* __restrict__ offsets) {
    __shared__ int64_t tot[kScanThreads];
    const int t = threadIdx.x;
    const int64_t per = (nb + kScanThreads - 1) / kScanThreads;
    const int64_t b0 = min(nb, int64_t(t) * per), b1 = min(nb, b0 + per);
    int64_t sum = 0;
    for (int64_t b = b0; b < b1; ++b) sum += counts[b];
    tot[t] = sum;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t v = t >= off ? tot[t - off] : 0;
        __syncthreads();
        tot[t] += v;
        __syncthreads();
    }
    int64_t run = tot[t] - sum;  // exclusive prefix of this run
    for (int64_t b = b0; b < b1; ++b) {
        offsets[b] = run;
        run += counts[b];
    }
    if (t == kScanThreads - 1) offsets[nb] = tot[t];
}

struct PeakOut {
    int32_t x, y, z;
    float intensity;
    int32_t is_min, is_max;
};

__global__ __launch_bounds__(kBlock) void k_peaks_write(const float* __restrict__ dog, Dims3 d,
                                                         float minv, int want_min, int want_max,
                                                         const int64_t* __restrict__ offsets,
                                                         PeakOut* __restrict__ out, int64_t cap) {
    __shared__ int wave_cnt[kBlock / 64];
    __shared__ int64_t base_sh;
    const int64_t n = d.nx * d.ny * d.nz;
    const int64_t chunk0 = int64_t(blockIdx.x) * kBlock * kItems;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) base_sh = offsets[blockIdx.x];
    __syncthreads();
    for (int it = 0; it < kItems; ++it) {
        const int64_t i = chunk0 + int64_t(it) * kBlock + threadIdx.x;
        int sp = 0;
        float v = 0.0f;
        int64_t x = 0, y = 0, z = 0;
        if (i < n) {
            flat_coords(i, d, x, y, z);
            sp = special_point(dog, d, i, x, y, z, minv, v);
        }
        const bool flag = (sp == 2 && want_max) || (sp == 1 && want_min);
        const unsigned long long m = __ballot(flag);
        if (lane == 0) wave_cnt[wid] = __popcll(m);
        __syncthreads();
        int prefix = 0;
        for (int w = 0; w < wid; ++w) prefix += wave_cnt[w];
        const int64_t pos = base_sh + prefix + __popcll(m & ((1ull << lane) - 1ull));
        if (flag && pos < cap) {
            PeakOut p;
            p.x = int32_t(x); p.y = int32_t(y); p.z = int32_t(z);
            p.intensity = fabsf(v);
            p.is_min = sp == 1;
            p.is_max = sp == 2;
            out[pos] = p;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int w = 0; w < kBlock / 64; ++w) t += wave_cnt[w];
            base_sh += t;
        }
        __syncthreads();
    }
}

unsigned grid_of(int64_t n, int64_t cap = 4096) {
    int64_t b = ceil_div(n, kBlock);
    return unsigned(b < 1 ? 1 : (b > cap ? cap : b));
}

void sep_pass(const Dims3& d, int axis, const float* in0, const float* in1, const float* k0,
              const float* k1, int K, int mode, float value, float* out0, float* out1, bool dog,
              float dog_scale, const float* mm, hipStream_t s) {
    const int64_t n = d.nx * d.ny * d.nz;
    const bool two = in1 || k1;
    const int nk = two ? 2 : 1;
    // tiled passes: 32-bit indices, grid y/z extents within 65535
    const int64_t tl = axis == 0 ? 1 : ceil_div(axis == 1 ? d.ny : d.nz, int64_t(kSepTL));
    const int64_t oth = axis == 0 ? d.nz : (axis == 1 ? d.nz : d.ny);
    if (n < (int64_t(1) << 31) && (axis == 0 ? d.ny : tl) <= 65535 && oth <= 65535) {
        if (axis == 0) {
            const size_t lds = size_t(nk * (kSepX + K - 1) + nk * K) * sizeof(float);
            const dim3 grid(unsigned(ceil_div(d.nx, int64_t(kSepX))), unsigned(ceil_div(d.ny, int64_t(kSepRows))),
                            unsigned(d.nz));
            if (two)
                hipLaunchKernelGGL(k_sep_x<2>, grid, dim3(kSepX), lds, s, d, in0, in1, k0, k1, K, mode, value,
                                   out0, out1, int(dog), dog_scale, mm);
            else
                hipLaunchKernelGGL(k_sep_x<1>, grid, dim3(kSepX), lds, s, d, in0, in1, k0, k1, K, mode, value,
                                   out0, out1, int(dog), dog_scale, mm);
        } else {
            const size_t lds = size_t(nk * (kSepTL + K - 1) * kSepTX + nk * K) * sizeof(float);
            const dim3 grid(unsigned(ceil_div(d.nx, int64_t(kSepTX))), unsigned(tl), unsigned(oth));
#define SD_SEPYZ1(NKV, AXV, KWV)                                                                          \
            SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep_yz<NKV, AXV, KWV>),           \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));            \
            hipLaunchKernelGGL((k_sep_yz<NKV, AXV, KWV>), grid, dim3(kSepTX * kSepTY), lds, s, d, in0, in1, k0, \
                               k1, K, mode, value, out0, out1, int(dog), dog_scale, mm);
#define SD_SEPYZ(NKV, AXV)                                    \
            if (K == 7) { SD_SEPYZ1(NKV, AXV, 7) }            \
            else if (K == 15) { SD_SEPYZ1(NKV, AXV, 15) }     \
            else { SD_SEPYZ1(NKV, AXV, 0) }
            if (two && axis == 1) { SD_SEPYZ(2, 1) }
            else if (two) { SD_SEPYZ(2, 2) }
            else if (axis == 1) { SD_SEPYZ(1, 1) }
            else { SD_SEPYZ(1, 2) }
#undef SD_SEPYZ
#undef SD_SEPYZ1
        }
        SD_HIP(hipGetLastError());
        return;
    }
    if (in1 || k1)
        hipLaunchKernelGGL(k_sep_pass<2>, dim3(grid_of(n)), dim3(kBlock), 0, s, d, axis, in0, in1, k0,
                           k1, K, mode, value, out0, out1, int(dog), dog_scale, mm);
    else
        hipLaunchKernelGGL(k_sep_pass<1>, dim3(grid_of(n)), dim3(kBlock), 0, s, d, axis, in0, in1, k0,
                           k1, K, mode, value, out0, out1, int(dog), dog_scale, mm);
    SD_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- host-side kernel math
float f32(double x) { return float(x); }

// LaPlaceFunctions.computeK / computeKWeight / computeSigma / computeSigmaDiff
void dog_sigmas(float sigma, const double image_sigma[3], double s1[3], double s2[3], float* kinv) {
    const float k = float(std::pow(2.0, double(1.0f / 4.0f)));
    *kinv = 1.0f / (k - 1.0f);
    float steps[4];
    steps[0] = sigma;
    for (int i = 1; i <= 3; ++i) steps[i] = steps[i - 1] * k;
    for (int d = 0; d < 3; ++d) {
        const float isg = std::min(float(image_sigma[d]), sigma);
        auto diff = [&](float b) {
            const float dd = b * b - isg * isg;
            return float(std::sqrt(double(dd)));
        };
        s1[d] = diff(steps[0]);
        s2[d] = diff(steps[1]);
    }
}

// imglib1 Util.createGaussianKernel1DDouble(sigma, true)
std::vector<double> gaussian_kernel(double sigma) {
    std::vector<double> g;
    if (sigma <= 0) {
        g.assign(3, 0.0);
        g[1] = 1.0;
    } else {
        const int size = std::max(3, 2 * int(3 * sigma + 0.5) + 1);
        const double two_sq = 2 * sigma * sigma;
        g.assign(size, 0.0);
        const int c = size / 2;
        for (int x = c; x >= 0; --x) {
            const double val = std::exp(-(double(x) * x) / two_sq);
            g[c - x] = val;
            g[c + x] = val;
        }
    }
    double sum = 0;
    for (double v : g) sum += v;
    for (double& v : g) v /= sum;
    return g;
}

// CUDASeparableConvolutionFunctions.getCUDAKernels: pad to the smallest supported size
int cuda_kernels(const double sig[3], std::vector<float> out[3]) {
    static const int sizes[5] = {7, 15, 31, 63, 127};
    std::vector<double> k[3];
    size_t longest = 0;
    for (int d = 0; d < 3; ++d) {
        k[d] = gaussian_kernel(sig[d]);
        longest = std::max(longest, k[d].size());
    }
    int size = -1;
    for (int s : sizes)
        if (longest <= size_t(s)) { size = s; break; }
    SD_CHECK(size > 0, SPIMDECON_ERR_ARG, "Gaussian kernel bigger than maximally supported size (127)");
    for (int d = 0; d < 3; ++d) {
        out[d].assign(size, 0.0f);
        const int s = (size - int(k[d].size())) / 2;
        for (size_t i = 0; i < k[d].size(); ++i) out[d][s + i] = float(k[d][i]);
    }
    return size;
}

}  // namespace

// ---------------------------------------------------------------- convolve_N
void separable_convolve(float* image, const float* kx, const float* ky, const float* kz, int w,
                        int h, int dd, bool cx, bool cy, bool cz, int oob, float oobv, int dev, int K) {
    SD_CHECK(image, SPIMDECON_ERR_ARG, "null image");
    SD_CHECK(w >= 1 && h >= 1 && dd >= 1, SPIMDECON_ERR_ARG, "bad dims");
    SD_CHECK(oob >= 0 && oob <= 3, SPIMDECON_ERR_ARG, "bad outofbounds mode");
    SD_CHECK((!cx || kx) && (!cy || ky) && (!cz || kz), SPIMDECON_ERR_ARG, "null kernel");
    check_device(dev);
    DeviceGuard guard(dev);
    hipStream_t s;
    SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct SG { hipStream_t s; ~SG() { (void)hipStreamDestroy(s); } } sg{s};
    const Dims3 d{w, h, dd};
    const int64_t n = int64_t(w) * h * dd;
    DBuf<float> a(n), b(n), dk(3 * size_t(K));
    SD_HIP(hipMemcpyAsync(a.p, image, n * 4, hipMemcpyHostToDevice, s));
    const float* ks[3] = {kx, ky, kz};
    const bool on[3] = {cx, cy, cz};
    float* cur = a.p;
    float* nxt = b.p;
    for (int ax = 0; ax < 3; ++ax) {
        if (!on[ax]) continue;
        SD_HIP(hipMemcpyAsync(dk.p + ax * K, ks[ax], K * 4, hipMemcpyHostToDevice, s));
        sep_pass(d, ax, cur, nullptr, dk.p + ax * K, nullptr, K, oob, oobv, nxt, nullptr, false, 0.f,
                 nullptr, s);
        std::swap(cur, nxt);
    }
    SD_HIP(hipMemcpyAsync(image, cur, n * 4, hipMemcpyDeviceToHost, s));
    SD_HIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- DoG
// ---------------------------------------------------------------- quadratic localization
// IPD/Localization.java:47-88 (imglib1 SubpixelLocalization, maxNumMoves 10,
// allowMaximaTolerance); finite differences and 3x3 inverse as in the reference's
// own fit, mpicbg/spim/registration/bead/laplace/LaPlaceFunctions.java:30-170,243-466.
// One thread per peak; all fit arithmetic in double, -ffp-contract=off.
struct LocOut {
    float pos[3];
    float value;
};

constexpr int kLocMaxMoves = 10;
constexpr double kLocTolerance = 0.01;

__global__ void k_localize(const float* __restrict__ dog, Dims3 d, const PeakOut* __restrict__ pk,
                           int64_t np, LocOut* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const PeakOut q = pk[i];
    int p[3] = {q.x, q.y, q.z};
    const int64_t dim[3] = {d.nx, d.ny, d.nz};
    auto v = [&](int dx, int dy, int dz) -> float {
        return dog[(int64_t(p[2] + dz) * d.ny + (p[1] + dy)) * d.nx + (p[0] + dx)];
    };
    double X[3] = {0, 0, 0}, g[3] = {0, 0, 0};
    bool stable = false, valid = true;
    int moves = 0;
    for (;;) {
        ++moves;
        const float temp = 2.0f * v(0, 0, 0);
        double H[9];
        H[0] = double(v(1, 0, 0) - temp) + double(v(-1, 0, 0));
        H[4] = double(v(0, 1, 0) - temp) + double(v(0, -1, 0));
        H[8] = double(v(0, 0, 1) - temp) + double(v(0, 0, -1));
        auto cross = [](float a, float b, float c, float e) {
            return double(((a - b) / 2.0f - (c - e) / 2.0f) / 2.0f);
        };
        H[5] = H[7] = cross(v(0, 1, 1), v(0, -1, 1), v(0, 1, -1), v(0, -1, -1));
        H[2] = H[6] = cross(v(1, 0, 1), v(-1, 0, 1), v(1, 0, -1), v(-1, 0, -1));
        H[1] = H[3] = cross(v(1, 1, 0), v(-1, 1, 0), v(1, -1, 0), v(-1, -1, 0));
        g[0] = (double(v(1, 0, 0)) - double(v(-1, 0, 0))) / 2.0;
        g[1] = (double(v(0, 1, 0)) - double(v(0, -1, 0))) / 2.0;
        g[2] = (double(v(0, 0, 1)) - double(v(0, 0, -1))) / 2.0;
        const double det = H[0] * H[4] * H[8] + H[3] * H[7] * H[2] + H[6] * H[1] * H[5] -
                            H[2] * H[4] * H[6] - H[5] * H[7] * H[0] - H[8] * H[1] * H[3];
        if (det == 0.0) {
            valid = false;
            break;
        }
        const double A[9] = {(H[4] * H[8] - H[5] * H[7]) / det, (H[2] * H[7] - H[1] * H[8]) / det,
                             (H[1] * H[5] - H[2] * H[4]) / det, (H[5] * H[6] - H[3] * H[8]) / det,
                             (H[0] * H[8] - H[2] * H[6]) / det, (H[2] * H[3] - H[0] * H[5]) / det,
                             (H[3] * H[7] - H[4] * H[6]) / det, (H[1] * H[6] - H[0] * H[7]) / det,
                             (H[0] * H[4] - H[1] * H[3]) / det};
        for (int r = 0; r < 3; ++r) X[r] = -(A[3 * r] * g[0] + A[3 * r + 1] * g[1] + A[3 * r + 2] * g[2]);
        stable = true;
        const double thr = 0.5 + moves * kLocTolerance;
        for (int a = 0; a < 3; ++a)
            if (fabs(X[a]) > thr) {
                p[a] += X[a] > 0 ? 1 : -1;
                stable = false;
            }
        if (!stable)
            for (int a = 0; a < 3; ++a)
                if (p[a] <= 0 || p[a] >= dim[a] - 1) valid = false;
        if (!valid || stable || moves > kLocMaxMoves) break;
    }
    LocOut o;
    if (valid && stable) {
        const double fit = (X[0] * g[0] + X[1] * g[1] + X[2] * g[2]) / 2.0;
        for (int a = 0; a < 3; ++a) o.pos[a] = float(p[a]) + float(X[a]);
        o.value = v(0, 0, 0) + float(fit);
    } else {  // no stable fit: the peak stays as detected
        o.pos[0] = float(q.x);
        o.pos[1] = float(q.y);
        o.pos[2] = float(q.z);
        o.value = q.intensity;
    }
    out[i] = o;
}

// the DoG image (kept on the device) and the reference-ordered peak list
struct DogRun {
    Dims3 d{};
    DBuf<float> dog;
    std::vector<PeakOut> peaks;
};

void dog_run(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out,
             hipStream_t s, DogRun& r) {
    SD_CHECK(img && dims && p, SPIMDECON_ERR_ARG, "null argument");
    SD_CHECK(dims[0] >= 1 && dims[1] >= 1 && dims[2] >= 1, SPIMDECON_ERR_ARG, "bad dims");
    SD_CHECK(p->localization == 0 || p->localization == 1, SPIMDECON_ERR_ARG,
             "localization must be 0 (none) or 1 (quadratic); the Gaussian fit is not implemented in "
             "the reference either (Localization.java:90-96)");
    SD_CHECK(p->ij_threads >= 1, SPIMDECON_ERR_ARG, "ij_threads must be >= 1");
    const Dims3 d{dims[0], dims[1], dims[2]};
    r.d = d;
    const int64_t n = d.nx * d.ny * d.nz;

    // ProcessDOG.java:61-105
    const float min_peak = p->localization == 0 ? p->threshold : p->threshold / 10.0f;
    double s1[3], s2[3];
    float kinv;
    dog_sigmas(p->sigma, p->image_sigma, s1, s2, &kinv);
    std::vector<float> k1[3], k2[3];
    const int K1 = cuda_kernels(s1, k1);
    const int K2 = cuda_kernels(s2, k2);
    const int K = std::max(K1, K2);
    auto pad_to = [](std::vector<float>& k, int K) {
        if (int(k.size()) == K) return;
        std::vector<float> o(K, 0.0f);
        const int off = (K - int(k.size())) / 2;
        std::copy(k.begin(), k.end(), o.begin() + off);
        k.swap(o);
    };
    std::vector<float> kall;
    for (int a = 0; a < 3; ++a) {
        pad_to(k1[a], K);
        pad_to(k2[a], K);
        kall.insert(kall.end(), k1[a].begin(), k1[a].end());
        kall.insert(kall.end(), k2[a].begin(), k2[a].end());
    }
    DBuf<float> dk(kall.size());
    SD_HIP(hipMemcpyAsync(dk.p, kall.data(), kall.size() * 4, hipMemcpyHostToDevice, s));
    auto kp = [&](int axis, int which) { return dk.p + (2 * axis + which) * K; };

    DBuf<float> b0(n), b1(n), b2(n), b3(n);
    // img / dog_out may be host or device pointers (unified addressing infers the copy)
    SD_HIP(hipMemcpyAsync(b0.p, img, n * 4, hipMemcpyDefault, s));
    DBuf<float> mm(2 * 4096);
    const bool use_given = !(std::isnan(p->min_intensity) || std::isnan(p->max_intensity) ||
                             std::isinf(p->min_intensity) || std::isinf(p->max_intensity) ||
                             p->min_intensity == p->max_intensity);
    if (use_given) {
        const float h2[2] = {float(p->min_intensity), float(p->max_intensity)};
        SD_HIP(hipMemcpyAsync(mm.p, h2, 8, hipMemcpyHostToDevice, s));
    } else {
        const unsigned nb = grid_of(n);
        hipLaunchKernelGGL(k_minmax, dim3(nb), dim3(kBlock), 0, s, b0.p, n, mm.p);
        hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(64), 0, s, mm.p, int(nb));
        SD_HIP(hipGetLastError());
    }
    // x-pass (normalise fused) -> b1 (sigma1), b2 (sigma2)
    sep_pass(d, 0, b0.p, b0.p, kp(0, 0), kp(0, 1), K, OOB_MIRROR, 0.f, b1.p, b2.p, false, 0.f, mm.p, s);
    // y-pass: b1 -> b3, b2 -> b0
    sep_pass(d, 1, b1.p, b2.p, kp(1, 0), kp(1, 1), K, OOB_MIRROR, 0.f, b3.p, b0.p, false, 0.f, nullptr, s);
    // z-pass + DoG: (b3, b0) -> b1 = (G2 - G1) * kinv
    sep_pass(d, 2, b3.p, b0.p, kp(2, 0), kp(2, 1), K, OOB_MIRROR, 0.f, b1.p, nullptr, true, kinv,
             nullptr, s);
    const float* dog = b1.p;
    if (dog_out) SD_HIP(hipMemcpyAsync(dog_out, dog, n * 4, hipMemcpyDefault, s));

    // peaks: order-preserving compaction in flat order
    const int64_t chunk = int64_t(kBlock) * kItems;
    const int64_t nb = ceil_div(n, chunk);
    DBuf<int> counts(nb);
    DBuf<int64_t> offsets(nb + 1);
    const int wmin = p->find_min ? 1 : 0, wmax = p->find_max ? 1 : 0;
    hipLaunchKernelGGL(k_peaks_count, dim3(unsigned(nb)), dim3(kBlock), 0, s, dog, d, min_peak, wmin,
                       wmax, counts.p);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(kScanThreads), 0, s, counts.p, nb, offsets.p);
    SD_HIP(hipGetLastError());
    int64_t total = 0;
    SD_HIP(hipMemcpyAsync(&total, offsets.p + nb, 8, hipMemcpyDeviceToHost, s));
    SD_HIP(hipStreamSynchronize(s));
    DBuf<PeakOut> dpk(std::max<int64_t>(total, 1));
    hipLaunchKernelGGL(k_peaks_write, dim3(unsigned(nb)), dim3(kBlock), 0, s, dog, d, min_peak, wmin,
                       wmax, offsets.p, dpk.p, total);
    SD_HIP(hipGetLastError());
    r.peaks.resize(total);
    if (total)
        SD_HIP(hipMemcpyAsync(r.peaks.data(), dpk.p, total * sizeof(PeakOut), hipMemcpyDeviceToHost, s));
    SD_HIP(hipStreamSynchronize(s));
    // reference order: per-thread lists by x % T, each in flat order (InteractiveIntegral.java:394,437-438)
    const int T = p->ij_threads;
    std::stable_sort(r.peaks.begin(), r.peaks.end(),
                     [T](const PeakOut& a, const PeakOut& b) { return (a.x % T) < (b.x % T); });
    r.dog = std::move(b1);
}

struct StreamHolder {
    hipStream_t s = nullptr;
    StreamHolder() { SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
    ~StreamHolder() { (void)hipStreamDestroy(s); }
};

// DifferenceOfGaussianNewPeakFinder.getSimplePeaks level: candidates with
// |v| >= threshold (localization 0) or threshold / 10 (localization 1)
void dog_compute(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out,
                 spim_peak* peaks, int64_t max_peaks, int64_t* npeaks) {
    SD_CHECK(npeaks && p, SPIMDECON_ERR_ARG, "null argument");
    check_device(p->device);
    DeviceGuard guard(p->device);
    StreamHolder sh;
    DogRun r;
    dog_run(img, dims, p, dog_out, sh.s, r);
    const int64_t total = int64_t(r.peaks.size());
    *npeaks = total;
    if (peaks) {
        const int64_t m = std::min(total, max_peaks);
        for (int64_t i = 0; i < m; ++i) {
            peaks[i].x = r.peaks[i].x;
            peaks[i].y = r.peaks[i].y;
            peaks[i].z = r.peaks[i].z;
            peaks[i].intensity = r.peaks[i].intensity;
            peaks[i].is_min = r.peaks[i].is_min;
            peaks[i].is_max = r.peaks[i].is_max;
        }
    }
}

// ProcessDOG.compute's result: interest points after Localization (:150-168)
void dog_interest_points(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out,
                         spim_interest_point* out, int64_t max_out, int64_t* nout) {
    SD_CHECK(nout && p, SPIMDECON_ERR_ARG, "null argument");
    check_device(p->device);
    DeviceGuard guard(p->device);
    StreamHolder sh;
    DogRun r;
    dog_run(img, dims, p, dog_out, sh.s, r);
    std::vector<spim_interest_point> pts;
    const int64_t np = int64_t(r.peaks.size());
    if (p->localization == 0) {  // Localization.noLocalization (:19-45)
        pts.resize(np);
        for (int64_t i = 0; i < np; ++i) {
            pts[i].pos[0] = r.peaks[i].x;
            pts[i].pos[1] = r.peaks[i].y;
            pts[i].pos[2] = r.peaks[i].z;
            pts[i].intensity = r.peaks[i].intensity;
            pts[i].is_max = r.peaks[i].is_max;
        }
    } else if (np > 0) {  // Localization.computeQuadraticLocalization (:47-88)
        DBuf<PeakOut> dpk(np);
        DBuf<LocOut> dloc(np);
        SD_HIP(hipMemcpyAsync(dpk.p, r.peaks.data(), np * sizeof(PeakOut), hipMemcpyHostToDevice, sh.s));
        hipLaunchKernelGGL(k_localize, dim3(unsigned(ceil_div(np, 256))), dim3(256), 0, sh.s, r.dog.p, r.d,
                           dpk.p, np, dloc.p);
        SD_HIP(hipGetLastError());
        std::vector<LocOut> loc(np);
        SD_HIP(hipMemcpyAsync(loc.data(), dloc.p, np * sizeof(LocOut), hipMemcpyDeviceToHost, sh.s));
        SD_HIP(hipStreamSynchronize(sh.s));
        for (int64_t i = 0; i < np; ++i) {
            if (!(std::fabs(loc[i].value) > p->threshold)) continue;
            spim_interest_point ip{};
            for (int a = 0; a < 3; ++a) ip.pos[a] = loc[i].pos[a];
            ip.intensity = loc[i].value;
            ip.is_max = r.peaks[i].is_max;
            pts.push_back(ip);
        }
    }
    *nout = int64_t(pts.size());
    if (out) std::copy(pts.begin(), pts.begin() + std::min<int64_t>(max_out, int64_t(pts.size())), out);
}

}  // namespace spimdecon

// ---------------------------------------------------------------- extern "C"
using namespace spimdecon;

#define CONVOLVE_N(N)                                                                            \
    extern "C" int32_t convolve_##N(float* image, const float* kernelX, const float* kernelY,  \
                                    const float* kernelZ, int imageW, int imageH, int imageD,   \
                                    int32_t convolveX, int32_t convolveY, int32_t convolveZ,    \
                                    int outofbounds, float outofboundsvalue, int devCUDA) {     \
        const int st = guarded([&] {                                                            \
            separable_convolve(image, kernelX, kernelY, kernelZ, imageW, imageH, imageD,         \
                               convolveX != 0, convolveY != 0, convolveZ != 0, outofbounds,     \
                               outofboundsvalue, devCUDA, N);                                   \
        });                                                                                     \
        return st == SPIMDECON_OK ? 1 : 0;                                                      \
    }

CONVOLVE_N(7)
CONVOLVE_N(15)
CONVOLVE_N(31)
CONVOLVE_N(63)
CONVOLVE_N(127)

extern "C" void spim_dog_params_default(spim_dog_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->sigma = 1.8f;
    p->threshold = 0.008f;
    p->localization = 0;
    p->image_sigma[0] = p->image_sigma[1] = p->image_sigma[2] = 0.5;
    p->find_min = 0;
    p->find_max = 1;
    p->min_intensity = std::nan("");
    p->max_intensity = std::nan("");
    p->ij_threads = 8;
    p->device = 0;
}

extern "C" int spim_dog_interest_points(const float* img, const int64_t* dims, const spim_dog_params* p,
                                        float* dog_out, spim_interest_point* out, int64_t max_out,
                                        int64_t* nout) {
    return guarded([&] { dog_interest_points(img, dims, p, dog_out, out, max_out, nout); });
}

extern "C" int spim_dog_compute(const float* img, const int64_t* dims, const spim_dog_params* p,
                                float* dog_out, spim_peak* peaks, int64_t max_peaks,
                                int64_t* npeaks) {
    return guarded([&] { dog_compute(img, dims, p, dog_out, peaks, max_peaks, npeaks); });
}
