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
// Data flow of one DoG (all HBM-resident, two streaming passes for Gaussians of 7 / 15 /
// 31 taps -- the ProcessDOG sigmas):
//   k_dog_xy  img --(normalise on the fly)--> x then y Gaussians of both sigmas -> G12
//   k_dog_z   G12 -> z Gaussians -> dog = (G2 - G1) * 1/(k-1) -> 26-neighbour test ->
//             candidate append; device radix sort into the reference's order
// (63 / 127 taps: the separate x / y / z passes, then a candidate pass over the DoG.)
// Accumulation order = tap order in float32 (matches the oracle bit for bit).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace spimdecon {

// dog_sort.hip
size_t peak_sort_temp_bytes(int64_t n, int end_bit);
void peak_sort(void* tmp, size_t tmp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
               uint32_t* vout, int64_t n, int end_bit, hipStream_t s);
size_t point_select_temp_bytes(int64_t n);
void point_select(void* tmp, size_t tmp_bytes, const spim_interest_point* in, const unsigned char* flags,
                  spim_interest_point* out, int* nsel, int64_t n, hipStream_t s);

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

// ---------------------------------------------------------------- fused DoG (the ProcessDOG path)
// Two streaming kernels replace the three separable passes and the two peak passes:
//   k_dog_xy  img --normalise--> x, then y Gaussians of both sigmas -> G12 (float2 per voxel)
//   k_dog_z   G12 -> z Gaussians -> DoG (stored only when asked) -> 26-neighbour test ->
//             candidates appended as (key, record); a device radix sort on the key
//             (x % T) << 40 | flat restores the reference order (dog_sort.hip).
// Every output keeps the float32 tap order of k_sep_x / k_sep_yz (packed mul, then
// packed add, no contraction): the DoG image is bit-identical to the separate passes.
// HBM per voxel: 4 B read + 8 B write (xy), 8 B read (+ 4 B DoG write) (z) -- 20-24 B
// against 48 B for the separate passes plus two re-reads of the DoG by the peak passes.
constexpr int kDxyTX = 64;   // xy tile: outputs along x (TY along y: template)
constexpr int kDxySeg = 8;   // x outputs per thread in the x phase (register window)
constexpr int kDzBX = 64;    // z kernel: a box of 64 x BY columns = one wave per row, the
                             // outer ring is the peak test's halo (62 x (BY - 2) tested columns)
// planes loaded ahead of use (3 left the HBM latency exposed; 12 or 16 no better, 16
// costs a wave per SIMD); KW + kDzPD must be a multiple of 4 (the ring slots)
#ifndef SPIMDECON_DZ_PD
#define SPIMDECON_DZ_PD 9
#endif
constexpr int kDzPD = SPIMDECON_DZ_PD;
                             // (a step computes in ~350 cycles; a load takes thousands)
constexpr int kDzChunk = 128; // DoG planes per block (the window adds KW - 1 + 2 loads; 64: 2.46 vs 2.35 ms)
constexpr int kDzMaxLen = 512;
constexpr int kDpkY = 4;
#ifndef SPIMDECON_DZC_PD
#define SPIMDECON_DZC_PD 9
#endif
#ifndef SPIMDECON_DZC_ILV
#define SPIMDECON_DZC_ILV 0
#endif
constexpr int kDzcPD = SPIMDECON_DZC_PD;   // k_dog_zconv: planes loaded ahead    // k_dog_peaks: rows per lane
constexpr int kDpkPD = 2;   // k_dog_peaks: planes loaded ahead   // k_dog_z plane-offset table: chunk + 2 + KW - 1 + PD entries

__device__ __forceinline__ int mirror32(int i, int n) {
    bool o;
    return ext_index32(i, n, OOB_MIRROR, o);
}

// LDS writes visible to the block, without the release fence of __syncthreads (which
// would also wait for the planes loaded ahead)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS pitch (floats) of the staged input rows of k_dog_xy: >= iw, a multiple of 4 (16-B
// aligned rows for the b128 window reads) and 4 * odd modulo 64, so that the 16 lanes of a
// ds_read_b128 group -- 16 consecutive rows of one segment, rows mod 16 all distinct --
// start on 16 distinct 4-bank groups (MI355X_MICROARCH.md LDS table): conflict-free
__host__ __device__ constexpr int dxy_in_pitch(int iw) {
    int p = (iw + 3) / 4 * 4;
    while ((p / 4) % 2 == 0) p += 4;
    return p;
}
// row pitch (float2) of the x-phase results: 64 + 2, so the 8 consecutive rows of a
// ds_write_b128 group land on 8 distinct 4-bank groups mod 32
constexpr int kDxySxP = kDxyTX + 2;

// (v - mn) / diff correctly rounded (__fdiv_rn's result) from the reciprocal rd = RN(1/diff):
// q = v * rd, then two Markstein corrections q += (a - q * diff) * rd with exact fma
// residuals -- the second starts from a faithful quotient, so it rounds correctly
// (Markstein's theorem; the Tikhonov step, rl_math.hpp, uses the same scheme in double).
// Outside the range where the residuals are exact (0, tiny, huge or non-finite a) the
// IEEE division itself.  5 VALU instead of the ~10 of the scaled division sequence.
// (caller: |a| in [2^-48, 2^48] or a == +0, and diff in [2^-48, 2^48]: q and the
// residuals stay normal; -0 would come out +0, so it takes the division)
__device__ __forceinline__ float div_rn_rcp_core(float a, float diff, float rd) {
    float q = __fmul_rn(a, rd);
    q = __fmaf_rn(__fmaf_rn(-q, diff, a), rd, q);
    return __fmaf_rn(__fmaf_rn(-q, diff, a), rd, q);
}

// The box of a k_dog_z block.  With `xcd` the dispatch order is remapped so that each
// XCD (blocks go round-robin to the 8 XCDs, each with its own L2) walks a contiguous
// range of boxes with y fastest: the boxes it holds at once are y-neighbours, whose
// overlapping halo rows (2 of every BY) then come from that L2 instead of HBM.
// (k_dog_xy: x fastest, so each XCD's resident tiles share their x and y halo columns.)
struct DzBox { int bx, by, bz; };
template <bool YFAST>
__device__ __forceinline__ DzBox xcd_box(bool xcd) {
    if (!xcd) return {int(blockIdx.x), int(blockIdx.y), int(blockIdx.z)};
    const unsigned gx = gridDim.x, gy = gridDim.y;
    const unsigned n = gx * gy * gridDim.z;
    const unsigned lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const unsigned k = lin & 7u, j = lin >> 3, q = n >> 3, r = n & 7u;
    const unsigned l = k * q + min(k, r) + j;           // XCD k: logical boxes [k q + min(k, r), ...)
    if (YFAST) return {int((l / gy) % gx), int(l % gy), int(l / (gy * gx))};
    return {int(l % gx), int((l / gx) % gy), int(l / (gx * gy))};
}

// Strips: a block walks one 64-column strip of one plane down y in steps of TY output rows.
// Each step stages, normalises and x-convolves only its TY new input rows; the KW - 1 rows
// above them are the previous step's last x results, carried (the y phase's last run holds
// them in registers and writes them to the first LDS rows after a barrier), and a strip
// starts with the KW - 1 rows above its first step.  Tiles of TY rows (round 4) recomputed
// the KW - 1 halo rows of every tile: (TY + KW - 1) / TY = 1.29 times the x phase and the
// normalisation at TY = 48, against (ny + KW - 1) / ny = 1.02 here.  TY = 32: a step's x
// phase is 32 rows x 8 segments = one item per thread (48 rows left two of the four waves
// a second item, and the blocks of a CU run their phases in step, so the SIMDs of those
// waves set the pace: no gain at 48), 4 blocks per CU; 768^3: k_dog_xy 1.63 -> 1.47 ms,
// DoG 3.67 -> 3.52 ms (profiles/r05_dog_strips_ab.txt).
template <int KW, int TY, bool BUF = true, int JT = 0>
__global__ __launch_bounds__(256, 4) void k_dog_xy(Dims3 d, const float* __restrict__ in, const float2* __restrict__ kx,
                                                const float2* __restrict__ ky, float2* __restrict__ g12,
                                                const float* __restrict__ mm, int xcd, int mm_exact) {
    constexpr int R = KW / 2;
    constexpr int IW = kDxyTX + KW - 1;          // staged input columns
    constexpr int IP = dxy_in_pitch(IW);         // pitch (see dxy_in_pitch)
    constexpr int IH = TY + KW - 1;              // x-result rows of a step's window
    constexpr int NSEG = kDxyTX / kDxySeg;
    constexpr int WX = kDxySeg + KW - 1;
    constexpr int OY = TY / 4;                   // y outputs per thread (4 runs per column)
    constexpr int WY = OY + KW - 1;
    static_assert(TY % 4 == 0 && OY + 2 * R == WY, "4 runs per column");
    __shared__ __attribute__((aligned(16))) float sin_[TY * IP];
    __shared__ __attribute__((aligned(16))) float2 sx[IH * kDxySxP];
    const int nx = int(d.nx), ny = int(d.ny);
    const int gx = (nx + kDxyTX - 1) / kDxyTX, gy = (ny + TY - 1) / TY;
    const int nstrips = gx * int(d.nz);
    const int t = threadIdx.x;
    // FusionHelper.normalizeImage constants (skipped for a NaN / inf / zero range)
    bool norm = false;
    float mn = 0.0f, diff = 1.0f, rd = 1.0f;
    if (mm) {
        mn = mm[0];
        diff = __fsub_rn(mm[1], mn);
        norm = !(isnan(diff) || isinf(diff) || diff == 0.0f);
        rd = __frcp_rn(diff);
        if (!(fabsf(diff) >= 0x1p-48f && fabsf(diff) <= 0x1p48f)) rd = 0.0f;   // (division only)
    }
    // mm_exact: mn / mx are the image's own min / max (k_minmax, not caller-given), so
    // every finite value has mn <= v <= mx and a = v - mn lies in [0, diff]; with
    // |mn| >= 2^-20 a non-zero a is at least the float spacing just below 2^-20 (2^-44), and
    // a = 0 is +0: every a is in the reciprocal path's exact range (NaN stays NaN either
    // way), so the per-value range check is skipped for the whole launch
    const bool allfast = norm && mm_exact != 0 && rd != 0.0f && fabsf(mn) >= 0x1p-20f;
    // Tap trim: the JT leading (and trailing) taps of the x and y kernels are zero for both
    // sigmas (padded to KW; the host instantiates JT).  When k_minmax found every value
    // finite (mm[2] == 0) and the image is normalised by its own range, every staged value
    // lies in [0, 1] and every partial sum is finite and never -0 (it starts at +0; the
    // taps are >= 0), so such a tap's +-0 product leaves the sum's bits unchanged: skipped.
    // Otherwise (NaN / inf in the image, a caller-given range) every padded tap is applied,
    // as before (one uniform branch per item between the two unrolled tap loops).
    const bool trim = JT > 0 && mm && norm && mm_exact != 0 && mm[2] == 0.0f;
    // thread t stages column t % IPC (IPC = IP rounded up so three rows fit 256 threads)
    // of rows t / IPC, t / IPC + RPT, ...: the column's mirror index once, the row's per
    // load.  Steps whose staged box lies inside the volume index without the mirror
    // arithmetic.
    constexpr int RPT = 256 / IW;                // rows staged per pass
    constexpr int IPC = 256 / RPT;               // threads per row (>= IW)
    constexpr int NE = (TY + RPT - 1) / RPT;     // rows per thread and step
    const int col = t % IPC, r0 = t / IPC;
    const bool cact = col < IW && r0 < RPT;
    // BUF (image below 4 GiB): buffer loads, the lane's row offset in a VGPR and the
    // pass offset RPT * e * nx in the scalar offset (no per-load address arithmetic; rows
    // past the step load in range or return 0 and are never staged); y mirror indices by
    // one reflection when ny > R (the modulo of mirror32 cost ~15 VALU per staged value
    // on the border strips)
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(in), 0, int(uint32_t(BUF ? uint64_t(d.nx * d.ny * d.nz) * 4u : 0u)), 0x00020000);
    const bool yrefl = ny > R;
    // input rows [ys, ys + NR) of strip s -> v (row r0 + RPT e of the unit; NR = 2R for the
    // rows above a strip, TY for a step)
    auto stage_loads = [&](int s, int ys, auto nrc, float* v) {
        constexpr int NR = decltype(nrc)::value;
        constexpr int NEc = (NR + RPT - 1) / RPT;
        const int x0 = (s % gx) * kDxyTX;
        const uint32_t plane = uint32_t(s / gx) * uint32_t(ny) * uint32_t(nx);
        const bool inside = x0 - R >= 0 && x0 - R + IW <= nx && ys >= 0 && ys + NR <= ny;
        if (inside) {
            const uint32_t base = plane + uint32_t(ys) * uint32_t(nx) + uint32_t(x0 - R + min(col, IW - 1));
            if constexpr (BUF) {
                const uint32_t vo = (base + uint32_t(r0) * uint32_t(nx)) * 4u;
#pragma unroll
                for (int e = 0; e < NEc; ++e)
                    v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         rin, int(vo), int(uint32_t(RPT * e) * uint32_t(nx) * 4u), 0));
            } else {
#pragma unroll
                for (int e = 0; e < NEc; ++e) v[e] = in[base + uint32_t(min(r0 + RPT * e, NR - 1)) * uint32_t(nx)];
            }
        } else {
            const uint32_t gxo = plane + uint32_t(mirror32(x0 - R + min(col, IW - 1), nx));
#pragma unroll
            for (int e = 0; e < NEc; ++e) {
                const int yy = ys + min(r0 + RPT * e, NR - 1);
                const int my = yrefl ? (ny - 1) - abs((ny - 1) - abs(yy)) : mirror32(yy, ny);
                if constexpr (BUF)
                    v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         rin, int((gxo + uint32_t(my) * uint32_t(nx)) * 4u), 0, 0));
                else
                    v[e] = in[gxo + uint32_t(my) * uint32_t(nx)];
            }
        }
    };
    // normalise the staged values of a step and store them to the LDS rows
    auto norm_store = [&](auto nrc, float* v) {
        constexpr int NR = decltype(nrc)::value;
        constexpr int NEc = (NR + RPT - 1) / RPT;
        if (norm) {
            // one wave-uniform decision for all values: the reciprocal path unless a value
            // of the wave leaves its exact range (then the IEEE division for all)
            bool bad = rd == 0.0f;
#pragma unroll
            for (int e = 0; e < NEc; ++e) {
                v[e] = __fsub_rn(v[e], mn);
                if (!allfast) {
                    const float aa = fabsf(v[e]);
                    bad |= !((aa >= 0x1p-48f && aa <= 0x1p48f) || __float_as_uint(v[e]) == 0u);   // (+0 only)
                }
            }
            if (allfast || !__any(bad)) {
#pragma unroll
                for (int e = 0; e < NEc; ++e) v[e] = div_rn_rcp_core(v[e], diff, rd);
            } else {
#pragma unroll
                for (int e = 0; e < NEc; ++e) v[e] = __fdiv_rn(v[e], diff);
            }
        }
        if (cact) {   // (the previous step's x phase finished at its mid-step barrier)
#pragma unroll
            for (int e = 0; e < NEc; ++e) {
                const int row = r0 + RPT * e;
                if (row >= NR) break;
                sin_[row * IP + col] = v[e];
            }
        }
    };
    // x phase over the step's NR staged rows into sx rows xrow0 + row: lane = staged row,
    // a segment of kDxySeg outputs from a window of WX values (b128 reads through the pitch IP)
    auto x_phase = [&](auto nrc, int xrow0) {
        constexpr int NR = decltype(nrc)::value;
#pragma unroll 1
        for (int it = t; it < NR * NSEG; it += 256) {
            const int row = it % NR, seg = it / NR;
            const float* src = sin_ + row * IP + seg * kDxySeg;
            float w[WX];
#pragma unroll
            for (int i = 0; i < WX; ++i) w[i] = src[i];
            dg_v2 acc[kDxySeg];
#pragma unroll
            for (int o = 0; o < kDxySeg; ++o) acc[o] = dg_v2{0.0f, 0.0f};
            auto taps = [&](auto j0c) {
                constexpr int J0 = decltype(j0c)::value;
#pragma unroll
                for (int j = J0; j < KW - J0; ++j) {
                    const dg_v2 k = dg_v2{kx[j].x, kx[j].y};
#pragma unroll
                    for (int o = 0; o < kDxySeg; ++o) acc[o] = acc[o] + dg_v2{w[o + j], w[o + j]} * k;  // tap order kept
                }
            };
            if (trim) taps(std::integral_constant<int, JT>{});
            else taps(std::integral_constant<int, 0>{});
            float2* dst = sx + (xrow0 + row) * kDxySxP + seg * kDxySeg;
#pragma unroll
            for (int o = 0; o < kDxySeg; ++o) dst[o] = make_float2(acc[o].x, acc[o].y);
        }
    };
    using PREc = std::integral_constant<int, 2 * R>;
    using TYc = std::integral_constant<int, TY>;
    // persistent blocks over the strips; the next step's input values are loaded into
    // registers while this step is transformed
    // xcd: blocks go round-robin to the 8 XCDs (each its own L2); the logical block index
    // makes XCD k's blocks a contiguous range, so the strips one XCD holds at a time are x
    // neighbours whose halo columns its L2 serves (else they come from HBM twice)
    float v[NE];
    int strip = int(blockIdx.x);
    if (xcd) {
        const unsigned b = blockIdx.x, k = b & 7u, j = b >> 3, q = gridDim.x >> 3, r = gridDim.x & 7u;
        strip = int(k * q + min(k, r) + j);
    }
    // units of a strip: step -1 stages and x-convolves the 2R rows above the strip into sx
    // rows 0 .. 2R - 1; step k >= 0 its TY new rows [k TY + R, k TY + TY + R) into sx rows
    // 2R .., then the y phase of output rows [k TY, k TY + TY)
    int step = -1;
    if (strip < nstrips) stage_loads(strip, -R, PREc{}, v);
    const int c = t & (kDxyTX - 1), run = t / kDxyTX;
    while (strip < nstrips) {
        const int x0 = (strip % gx) * kDxyTX;
        const uint32_t plane = uint32_t(strip / gx) * uint32_t(ny) * uint32_t(nx);
        const int y0 = step * TY;
        const bool pre = step < 0;
        if (pre) norm_store(PREc{}, v);
        else norm_store(TYc{}, v);
        // the next unit's values are in flight during this unit's phases
        int nstrip = strip, nstep = step + 1;
        if (nstep == gy) {
            nstrip = strip + int(gridDim.x);
            nstep = -1;
        }
        if (nstrip < nstrips) {
            if (nstep < 0) stage_loads(nstrip, -R, PREc{}, v);
            else stage_loads(nstrip, nstep * TY + R, TYc{}, v);
        }
        __syncthreads();   // (also: the previous step's y phase no longer reads sx)
        if (pre) x_phase(PREc{}, 0);
        else x_phase(TYc{}, 2 * R);
        __syncthreads();
        if (pre) {   // (block-uniform)
            strip = nstrip;
            step = nstep;
            continue;
        }
        // y phase: column c, OY consecutive outputs
        const int x = x0 + c;
        dg_v2 w[WY];
        if (x < nx) {
#pragma unroll
            for (int i = 0; i < WY; ++i) {
                const float2 vv = sx[(run * OY + i) * kDxySxP + c];
                w[i] = dg_v2{vv.x, vv.y};
            }
            dg_v2 acc[OY];
#pragma unroll
            for (int o = 0; o < OY; ++o) acc[o] = dg_v2{0.0f, 0.0f};
            auto taps = [&](auto j0c) {
                constexpr int J0 = decltype(j0c)::value;
#pragma unroll
                for (int j = J0; j < KW - J0; ++j) {
                    const dg_v2 k = dg_v2{ky[j].x, ky[j].y};
#pragma unroll
                    for (int o = 0; o < OY; ++o) acc[o] = acc[o] + w[o + j] * k;
                }
            };
            if (trim) taps(std::integral_constant<int, JT>{});
            else taps(std::integral_constant<int, 0>{});
#pragma unroll
            for (int o = 0; o < OY; ++o) {
                const int y = y0 + run * OY + o;
                if (y < ny) g12[plane + uint32_t(y) * uint32_t(nx) + uint32_t(x)] = make_float2(acc[o].x, acc[o].y);
            }
        }
        // the last run holds the x results of the next step's first 2R rows: to sx rows
        // 0 .. 2R - 1 once every run has read its window (block-uniform branch)
        if (nstep >= 0) {
            __syncthreads();
            if (run == 3 && x < nx) {
#pragma unroll
                for (int i = 0; i < 2 * R; ++i) sx[i * kDxySxP + c] = make_float2(w[OY + i].x, w[OY + i].y);
            }
        }
        strip = nstrip;
        step = nstep;
    }
}

struct PeakOut {   // (k_dog_z's cand_flush writes it as three int pairs)
    int32_t x, y, z;
    float intensity;
    int32_t is_min, is_max;
};

// candidate sink: unordered append of (key, record); count may exceed cap (the host reruns)
struct PeakSink {
    float minv;
    int want_min, want_max, T;
    uint64_t* keys;
    uint32_t* vals;
    PeakOut* recs;
    unsigned* count;
    unsigned cap;
};

// one wave-wide append; every lane of the wave must call it
__device__ __forceinline__ void sink_append(const PeakSink& pk, bool flag, int x, int y, int z, uint64_t flat,
                                            float c, int sp) {
    const unsigned long long bal = __ballot(flag);
    if (bal == 0ull) return;
    const int lane = int(threadIdx.x & 63);
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(pk.count, unsigned(__popcll(bal)));
    base = unsigned(__shfl(int(base), 0, 64));
    const unsigned pos = base + unsigned(__popcll(bal & ((1ull << lane) - 1ull)));
    if (flag && pos < pk.cap) {
        pk.keys[pos] = (uint64_t(x % pk.T) << 40) | flat;
        pk.vals[pos] = pos;
        PeakOut o;
        o.x = x;
        o.y = y;
        o.z = z;
        o.intensity = fabsf(c);
        o.is_min = sp == 1;
        o.is_max = sp == 2;
        pk.recs[pos] = o;
    }
}

// Per-wave candidate buffer of k_dog_z: entries {x, y | sp << 30, z, bits(|c|)} collect in
// LDS and go to the sink 64 at a time (one global atomic per flush instead of one per
// wave-step with a candidate; its returned value is the only vmcnt(0) in the loop)
constexpr int kCandBuf = 64;
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (the sink is read through a pointer: its fields are loaded here, at a flush, instead of
// holding 10 SGPRs for the whole z loop)
// (global-address-space stores and atomic: flat ones count in both vmcnt and lgkmcnt,
// and a flat operation pending at a join made every later load wait in k_dog_z's
// loop a vmcnt(0) -- the plane prefetch drained three times per unrolled rotation)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ void cand_flush(const PeakSink* __restrict__ sink, const int4* buf, int n, int nx,
                                           uint32_t pstride) {
    if (n == 0) return;
    wave_lds_sync();
    const PeakSink pk = *sink;
    const int lane = int(threadIdx.x & 63);
    unsigned base = 0;
    if (lane == 0)
        base = __hip_atomic_fetch_add(gbl(pk.count), unsigned(n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = unsigned(__shfl(int(base), 0, 64));
    if (lane < n) {
        const int4 e = buf[lane];
        const unsigned pos = base + unsigned(lane);
        if (pos < pk.cap) {
            const int x = e.x, y = e.y & 0x3fffffff, sp = int(unsigned(e.y) >> 30), z = e.z;
            *gbl(pk.keys + pos) = (uint64_t(x % pk.T) << 40) | (uint64_t(z) * pstride + uint64_t(y) * uint32_t(nx) + x);
            *gbl(pk.vals + pos) = pos;
            // the PeakOut record {x, y, z, intensity, is_min, is_max} as three 8-B stores
            typedef int v2i __attribute__((ext_vector_type(2)));
            v2i* r = reinterpret_cast<v2i*>(pk.recs + pos);
            *gbl(r) = v2i{x, y};
            *gbl(r + 1) = v2i{z, e.w};
            *gbl(r + 2) = v2i{sp == 1 ? 1 : 0, sp == 2 ? 1 : 0};
        }
    }
    wave_lds_sync();   // the buffer is rewritten after the flush
}

// z Gaussians + DoG + peak test over one column box and one chunk of planes.  Each
// thread keeps its column's window of KW planes (+ kDzPD loaded ahead) of (G1, G2) in
// registers, rotating by unrolling; the DoG planes go through a 4-plane LDS ring.  The
// 26-neighbour test is min / max of the 3x3x3 box (the box includes the centre, so
// "all neighbours >= c" <=> box min >= c); a plane holding a NaN takes the
// reference's comparison loop instead (NaN compares false).
//
// The ring: slot = (plane - qa) & 3, a compile-time constant of the unrolled step (NW is
// a multiple of 4), rows padded by one above and below and one element before and after,
// so the 3x3 neighbourhood is ONE per-thread address plus eight immediate offsets (edge
// lanes read a neighbouring row's element or a pad -- they are never tested).  The
// step's VALU work is the convolution's 2 KW packed ops plus ~20 for the test: the test
// had cost as much VALU as the convolution (r3t cost split).
template <int BY, int BX>
struct DzRing {
    static constexpr int kRow = BX, kSlot = (BY + 2) * BX, kSize = 4 * kSlot + 2;
    // element (slot, row r in [-1, BY], column c in [-1, BX])
    static __device__ __forceinline__ int at(int slot, int r, int c) { return 1 + slot * kSlot + (r + 1) * kRow + c; }
};

// InteractiveIntegral.isSpecialPoint (:443-468) over the ring (centre plane slot sc,
// row ty, column tx): 2 = every neighbour >= c ("MAX"), 1 = every neighbour <= c, 0 =
// neither.  Only for boxes holding a NaN (compares false), out of line.
template <int BY, int BX>
__device__ __noinline__ int dz_special_nan(const float* Dr, int sc, int ty, int tx, float c) {
    bool ge = true, le = true;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                if (dz == 0 && dy == 0 && dx == 0) continue;
                const float v = Dr[DzRing<BY, BX>::at((sc + dz) & 3, ty + dy, tx + dx)];
                ge &= v >= c;
                le &= v <= c;
            }
    return ge ? 2 : (le ? 1 : 0);
}

// min / max of three, one instruction (NaN-free inputs: planes holding a NaN take
// dz_special_nan; minnum / maxnum would add canonicalising maxes of the LDS values)
__device__ __forceinline__ float dz_min3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float dz_max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// BX x BY columns per block (64 x 8: one wave per row; 62 x 6 of them tested).
// ONE: the DoG image is below 2 GiB, one buffer resource covers it (the plane goes in
// the scalar offset); else a resource per plane.  want: bit 0 minima, bit 1 maxima.
// The z taps are symmetric (gaussian_kernel builds them so): taps j and KW - 1 - j are
// the same value and only R + 1 of them are held in SGPRs.
// SL: the source plane of each load from scalar mirror arithmetic (needs nz > KW / 2: one
// reflection) and a buffer resource per plane, so the load's address is the column's
// constant byte offset; else the LDS plane table and a 64-bit address per load.
// FROMDOG: the split z stage's test pass -- the DoG planes are read from the image
// k_dog_zconv stored (`dsrc`, PD planes ahead) instead of being convolved here; the test,
// the ring and the candidate records are the same code, so the same candidates.
template <int KW, int BY, int PD, int BX, bool ONE, bool SL, bool FROMDOG = false>
__global__ __launch_bounds__(BX * BY) void k_dog_z(Dims3 d, const float2* __restrict__ g12,
                                                         const float2* __restrict__ kz, float scale, int zc_len,
                                                         float* __restrict__ dog, float minv, int want,
                                                         const PeakSink* __restrict__ sink, int xcd,
                                                         const float* __restrict__ dsrc = nullptr) {
    constexpr int R = KW / 2;
    constexpr int NW = FROMDOG ? 12 : KW + PD;
    static_assert(NW % 4 == 0, "ring slots are compile-time: the unrolled rotation is whole ring turns");
    using Ring = DzRing<BY, BX>;
    __shared__ float Dr[Ring::kSize];
    __shared__ int nanq[4];
    __shared__ int4 cbuf[BX * BY / 64][kCandBuf];   // one candidate buffer per wave
    int ccount = 0;                       // wave-uniform fill of this wave's buffer
    const int t = threadIdx.x, tx = t & (BX - 1), ty = t / BX;
    const int wv = t >> 6, lane = t & 63;
    const int nx = int(d.nx), ny = int(d.ny), nz = int(d.nz);
    const DzBox bb = xcd_box<true>(xcd != 0);
    const int X0 = bb.bx * (BX - 2), Y0 = bb.by * (BY - 2);
    const int x = X0 + tx, y = Y0 + ty;
    const bool valid = x < nx && y < ny;
    const int z0 = bb.bz * zc_len, z1 = min(nz, z0 + zc_len);
    const int qa = max(z0 - 1, 0), qb = min(z1 + 1, nz);   // DoG planes computed
    const int len = qb - qa + KW - 1;                       // source planes loaded
    const int tlo = max(z0, 1), thi = min(z1, nz - 1);      // centre planes tested
    const uint32_t ntest = uint32_t(max(thi - tlo, 0));
    const uint32_t pstride = uint32_t(nx) * uint32_t(ny);
    const uint32_t col = valid ? uint32_t(y) * uint32_t(nx) + uint32_t(x) : 0u;
    // DoG store ownership: the tile's tested columns, plus the volume's outer ring
    const bool lastx = bb.bx == int(gridDim.x) - 1, lasty = bb.by == int(gridDim.y) - 1;
    const bool own = valid && tx >= (bb.bx == 0 ? 0 : 1) && (lastx || tx < BX - 1) &&
                     ty >= (bb.by == 0 ? 0 : 1) && (lasty || ty < BY - 1);
    const bool inner = valid && tx >= 1 && tx < BX - 1 && ty >= 1 && ty < BY - 1 && x <= nx - 2 &&
                       y <= ny - 2;
    // element offset of the source plane of every window index (mirror-single
    // extension, the tail repeating the last plane), for volumes the scalar path cannot take
    __shared__ uint32_t zoff[SL || FROMDOG ? 1 : kDzMaxLen];
    if constexpr (!SL && !FROMDOG)
        for (int i = t; i < kDzMaxLen; i += BX * BY)
            zoff[i] = uint32_t(mirror32(qa - R + min(i, len - 1), nz)) * pstride;
    if (t < 4) nanq[t] = INT_MIN;   // (no plane)
    __syncthreads();
    // unconditional loads (columns outside the volume read column 0): no branch merge,
    // so they stay in flight PD planes ahead
    const uint32_t plane_bytes = pstride * 8u;
    // FROMDOG: DoG plane qa + i (the tail repeating the last plane)
    const uint32_t dsrc_bytes = FROMDOG ? pstride * 4u : 0u;
    auto ldd = [&](int i) -> float {
        const int q = qa + min(i, qb - qa - 1);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(dsrc) + size_t(uint32_t(q)) * pstride, 0, int(dsrc_bytes), 0x00020000);
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, int(col * 4u), 0, 0));
    };
    auto ld = [&](int i) -> float2 {
        if constexpr (SL) {
            const int tz = qa - R + min(i, len - 1);
            const int m = (nz - 1) - abs((nz - 1) - abs(tz));   // mirror-single, one reflection
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float2*>(g12) + size_t(uint32_t(m)) * pstride, 0, int(plane_bytes), 0x00020000);
            return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, int(col * 8u), 0, 0));
        } else {
            return g12[zoff[min(i, kDzMaxLen - 1)] + col];
        }
    };
    // step s: window = source planes s .. s + KW - 1 in slots (s + j) % NW, DoG plane
    // q = qa + s; the step count is padded to whole NW rotations (padded steps test and
    // store nothing), so the unrolled body has no exits
    float2 w[FROMDOG ? 1 : NW];
    float wd[FROMDOG ? NW : 1];
#pragma unroll
    for (int p = 0; p < NW - 1; ++p) {
        if constexpr (FROMDOG) wd[p] = ldd(p);
        else w[p] = ld(p);
    }
    const int nsteps = (qb - qa + NW - 1) / NW * NW;
    float mnA = 0.f, mxA = 0.f, mnB = 0.f, mxB = 0.f, mnC = 0.f, mxC = 0.f, dB = 0.f, dC = 0.f;
    int nanhist = 0;   // bit k: the block's DoG plane q - k holds a NaN
    // DoG stores: one buffer resource over the whole image with the plane in the scalar
    // offset when the image is below 2 GiB (else one resource per plane)
    const uint64_t dog_total = dog ? uint64_t(pstride) * uint64_t(nz) * 4u : 0u;
    const __amdgpu_buffer_rsrc_t rall = __builtin_amdgcn_make_buffer_rsrc(dog, 0, ONE ? int(dog_total) : 0,
                                                                          0x00020000);
    const uint32_t dog_bytes = dog ? pstride * 4u : 0u;
    const bool want_min = (want & 1) != 0, want_max = (want & 2) != 0;
    float* const rbase = Dr + Ring::at(0, ty - 1, tx - 1);   // this thread's neighbourhood corner
    for (int sb = 0; sb < nsteps; sb += NW) {
#pragma unroll
        for (int ph = 0; ph < NW; ++ph) {
            const int st = sb + ph;
            float dv;
            if constexpr (FROMDOG) {
                wd[(ph + NW - 1) % NW] = ldd(st + NW - 1);
                dv = valid ? wd[ph % NW] : 0.0f;
            } else {
            w[(ph + NW - 1) % NW] = ld(st + NW - 1);
            dg_v2 acc = {0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < KW; ++j) {   // tap order kept
                const float2 v = w[(ph + j) % NW];
                const float2 k = kz[j <= R ? j : KW - 1 - j];
                acc = acc + dg_v2{v.x, v.y} * dg_v2{k.x, k.y};
            }
            dv = valid ? __fmul_rn(__fsub_rn(acc.y, acc.x), scale) : 0.0f;
            }
            const int q = qa + st;
            if constexpr (!FROMDOG) {   // the DoG store: a buffer store, dropped (out of range) unless owned
                const bool st_ok = own && uint32_t(q - z0) < uint32_t(z1 - z0);
                const int vo = int(st_ok ? col * 4u : 0x80000000u);
                if constexpr (ONE) {
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dv), rall, vo,
                                                          int(uint32_t(min(q, nz - 1)) * pstride * 4u), 0);
                } else {
                    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                        dog + (dog ? size_t(min(q, nz - 1)) * pstride : 0), 0, int(dog_bytes), 0x00020000);
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dv), rd, vo, 0, 0);
                }
            }
            const int slot = ph & 3;   // == (q - qa) & 3 (sb is a multiple of NW, so of 4): a constant once unrolled
            float* const P = rbase + slot * Ring::kSlot;
            P[Ring::kRow + 1] = dv;        // (row ty, column tx)
            if (__ballot(dv != dv) != 0ull && tx == 0) nanq[slot] = q;
            lds_barrier();
            const int nq = __builtin_amdgcn_readfirstlane(nanq[slot]);
            nanhist = ((nanhist << 1) | (nq == q ? 1 : 0)) & 7;
            mnA = mnB; mxA = mxB; mnB = mnC; mxB = mxC;
            dB = dC;
            dC = dv;
            {   // 3x3 box of this plane (the centre included), every lane
                const float a0 = P[0], a1 = P[1], a2 = P[2];
                const float b0 = P[Ring::kRow], b2 = P[Ring::kRow + 2];
                const float c0 = P[2 * Ring::kRow], c1 = P[2 * Ring::kRow + 1], c2 = P[2 * Ring::kRow + 2];
                mnC = dz_min3(dz_min3(a0, a1, a2), dz_min3(b0, b2, c0), dz_min3(c1, c2, dv));
                mxC = dz_max3(dz_max3(a0, a1, a2), dz_max3(b0, b2, c0), dz_max3(c1, c2, dv));
            }
            const int zc = q - 1;   // centre plane of the test
            if (uint32_t(zc - tlo) < ntest) {   // zc in [tlo, thi)
                const float c = dB;
                const bool cand = inner && !(fabsf(c) < minv);
                // "this mixup is intended" (InteractiveIntegral.isSpecialPoint): every
                // neighbour >= c is a MAX (sp 2), every neighbour <= c a MIN (sp 1); lane
                // masks, no per-lane branches
                // (the min / max path for every lane, then -- a uniform branch, rare -- the
                // comparison loop when a plane of the box held a NaN: no exec-mask merges)
                const bool ge = dz_min3(mnA, mnB, mnC) >= c;
                const bool le = dz_max3(mxA, mxB, mxC) <= c;
                bool is_max = cand && ge;
                bool is_min = cand && !ge && le;
                if (nanhist != 0) {   // a NaN in the box: the reference's comparison loop
                    const int spn = cand ? dz_special_nan<BY, BX>(Dr, (slot + 3) & 3, ty, tx, c) : 0;
                    is_max = spn == 2;
                    is_min = spn == 1;
                }
                const int sp = is_max ? 2 : 1;
                const bool flag = (is_max && want_max) || (is_min && want_min);
                const unsigned long long bal = __ballot(flag);
                if (bal != 0ull) {
                    const int nb = __popcll(bal);
                    if (ccount + nb > kCandBuf) {
                        cand_flush(sink, cbuf[wv], ccount, nx, pstride);
                        ccount = 0;
                    }
                    if (flag)
                        cbuf[wv][ccount + __popcll(bal & ((1ull << lane) - 1ull))] =
                            make_int4(x, y | (sp << 30), zc, __float_as_int(fabsf(c)));
                    ccount += nb;
                }
            }
        }
    }
    cand_flush(sink, cbuf[wv], ccount, nx, pstride);
}

// The split z stage, part 1: z Gaussians + DoG for every voxel, one thread per (x, y)
// column of a chunk of zc_len planes (a wave = 64 consecutive x of one row), a register
// window of KW planes + PD loaded ahead, rotating by unrolling; the DoG is stored for
// every voxel and the 26-neighbour test runs afterwards over the stored image
// (k_dog_z<..., FROMDOG>).  Columns are independent: no halo ring (the fused k_dog_z
// convolved its box's ring too, 1.38x the loads and convolutions), no LDS, no barrier.
// Same tap order and DoG expression as k_dog_z: the same bits.
// (plane bytes nx * ny * 8 < 2^31: one buffer resource per source plane; ONE: the DoG
// image below 2 GiB, one resource with the plane in the scalar offset)
template <int KW, int PD, bool ONE, bool ONEG>
__global__ __launch_bounds__(256) void k_dog_zconv(Dims3 d, const float2* __restrict__ g12,
                                                   const float2* __restrict__ kz, float scale, int zc_len,
                                                   float* __restrict__ dog) {
    constexpr int R = KW / 2;
    constexpr int NW = KW + PD;
    const int nx = int(d.nx), ny = int(d.ny), nz = int(d.nz);
    const int lane = int(threadIdx.x & 63);
    const int gxw = (nx + 63) / 64;                                          // waves per row
    const int wid = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + int(threadIdx.x >> 6));
    const int y = wid / gxw;
    if (y >= ny) return;   // (wave-uniform; no barriers in this kernel)
    const int x = (wid % gxw) * 64 + lane;
    const bool valid = x < nx;
    const int z0 = int(blockIdx.y) * zc_len, z1 = min(nz, z0 + zc_len);
    const int len = z1 - z0 + KW - 1;   // source planes
    const uint32_t pstride = uint32_t(nx) * uint32_t(ny);
    const uint32_t col = uint32_t(y) * uint32_t(nx) + uint32_t(valid ? x : nx - 1);
    // G12 below 4 GiB (every 768^3-class view): one resource, the source plane's byte
    // offset in the scalar offset (a resource per plane held 4 SGPRs per window slot)
    const uint64_t g12_bytes = uint64_t(pstride) * uint64_t(nz) * 8u;
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(g12), 0, int(uint32_t(g12_bytes < 0xffffffffull ? g12_bytes : 0xffffffffull)), 0x00020000);
    auto ld = [&](int i) -> float2 {
        // mirror-single extension, one reflection (the host takes this kernel for nz > KW / 2)
        const int tz = z0 - R + min(i, len - 1);
        const int m = (nz - 1) - abs((nz - 1) - abs(tz));
        if constexpr (ONEG)
            return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rg, int(col * 8u),
                                                                                   int(uint32_t(m) * pstride * 8u), 0));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float2*>(g12) + size_t(uint32_t(m)) * pstride, 0, int(pstride * 8u), 0x00020000);
        return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, int(col * 8u), 0, 0));
    };
    float2 w[NW];
#pragma unroll
    for (int p = 0; p < NW - 1; ++p) w[p] = ld(p);
    const int nsteps = (z1 - z0 + NW - 1) / NW * NW;   // padded to whole rotations (stores dropped)
    const uint64_t dog_total = uint64_t(pstride) * uint64_t(nz) * 4u;
    const __amdgpu_buffer_rsrc_t rall = __builtin_amdgcn_make_buffer_rsrc(dog, 0, ONE ? int(dog_total) : 0, 0x00020000);
    for (int sb = 0; sb < nsteps; sb += NW) {
#pragma unroll
        for (int ph = 0; ph < NW; ++ph) {
            const int st = sb + ph;
            w[(ph + NW - 1) % NW] = ld(st + NW - 1);
            dg_v2 acc = {0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < KW; ++j) {   // tap order kept
                const float2 v = w[(ph + j) % NW];
                const float2 k = kz[j <= R ? j : KW - 1 - j];
                acc = acc + dg_v2{v.x, v.y} * dg_v2{k.x, k.y};
                if (SPIMDECON_DZC_ILV) __builtin_amdgcn_sched_barrier(0);
            }
            const float dv = __fmul_rn(__fsub_rn(acc.y, acc.x), scale);
            const int q = z0 + st;
            const int vo = int(valid && q < z1 ? col * 4u : 0x80000000u);
            if constexpr (ONE) {
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dv), rall, vo,
                                                      int(uint32_t(min(q, nz - 1)) * pstride * 4u), 0);
            } else {
                const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                    dog + size_t(min(q, nz - 1)) * pstride, 0, int(pstride * 4u), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dv), rd, vo, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);   // one load per step (hoisting them all held a rotation of VGPRs)
        }
    }
}

// The split z stage, part 2: the 26-neighbour test over the stored DoG image.  A wave =
// 64 consecutive x (lanes 1..62 tested, lanes 0 and 63 their halo) x DPY rows per lane,
// walking a chunk of zc_len centre planes: per plane each lane loads its column's DPY + 2
// rows (PD planes ahead), the x neighbours come from DPP lane shifts, the y neighbours
// from the lane's own rows, and the 3x3 min / max of the last two planes stay in
// registers -- no LDS ring, no barrier (k_dog_z<FROMDOG> over the same image: 1.19 ms per
// 768^3, this structure's serial step).  A centre plane next to a plane holding a NaN
// (any loaded value of the wave) takes the reference's comparison loop over the image
// for the wave (NaN compares false; min3 / max3 would drop it).
__device__ __forceinline__ float dpp_from_left(float v) {    // lane i <- lane i - 1 (wave_shr:1)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_from_right(float v) {   // lane i <- lane i + 1 (wave_shl:1)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

template <int DPY, int PD>
__global__ __launch_bounds__(256) void k_dog_peaks(Dims3 d, const float* __restrict__ dog, int zc_len, float minv,
                                                   int want, const PeakSink* __restrict__ sink, int xcd) {
    constexpr int NR = DPY + 2;    // rows loaded per plane
    constexpr int NW = PD + 1;     // planes in the load ring
    __shared__ int4 cbuf[4][kCandBuf];
    const int lane = int(threadIdx.x & 63), wv = int(threadIdx.x >> 6);
    const int nx = int(d.nx), ny = int(d.ny), nz = int(d.nz);
    const int nsx = (nx - 2 + 61) / 62, nyb = (ny - 2 + DPY - 1) / DPY;
    const int nzc = (nz - 2 + zc_len - 1) / zc_len;
    // xcd: blocks go round-robin to the 8 XCDs; the logical block index gives each XCD a
    // contiguous range, so the y-neighbour waves sharing a halo row run on one L2
    int lb = int(blockIdx.x);
    if (xcd) {
        const unsigned b = blockIdx.x, k = b & 7u, j = b >> 3, q = gridDim.x >> 3, r = gridDim.x & 7u;
        lb = int(k * q + min(k, r) + j);
    }
    const int wid = __builtin_amdgcn_readfirstlane(lb * 4 + wv);
    if (wid >= nsx * nyb * nzc) return;   // (wave-uniform; no block barriers below)
    const int sx = wid % nsx, yb = (wid / nsx) % nyb, zb = wid / (nsx * nyb);
    const int x = sx * 62 + lane;                       // lane 0: the halo column x0 - 1
    const bool xt = lane >= 1 && lane <= 62 && x <= nx - 2;
    const int xl = min(x, nx - 1);
    const int ybase = yb * DPY;                         // row r of the lane: y = ybase + r (r = 0: halo)
    const int tlo = 1 + zb * zc_len, thi = min(nz - 1, tlo + zc_len);   // centre planes tested
    const int qa = tlo - 1, qb = thi + 1;               // planes loaded
    const uint32_t pstride = uint32_t(nx) * uint32_t(ny);
    const uint64_t total = uint64_t(pstride) * uint64_t(nz) * 4u;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(dog), 0, int(uint32_t(total < 0xffffffffull ? total : 0xffffffffull)), 0x00020000);
    const uint32_t xoff = uint32_t(xl) * 4u;   // the only per-lane offset: rows and planes are scalar
    auto ldp = [&](int i, float* v) {   // plane qa + i (the tail repeating the last plane)
        const uint32_t po = uint32_t(qa + min(i, qb - qa - 1)) * pstride * 4u;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t so = po + uint32_t(min(ybase + r, ny - 1)) * uint32_t(nx) * 4u;
            v[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rd, int(xoff), int(so), 0));
        }
    };
    float ring[NW][NR];
#pragma unroll
    for (int p = 0; p < NW - 1; ++p) ldp(p, ring[p]);
    float mnA[DPY], mxA[DPY], mnB[DPY], mxB[DPY], cB[DPY];
#pragma unroll
    for (int r = 0; r < DPY; ++r) mnA[r] = mxA[r] = mnB[r] = mxB[r] = cB[r] = 0.0f;
    int nanhist = 0;   // bit k: plane q - k held a NaN (any loaded value of the wave)
    int ccount = 0;
    const bool want_min = (want & 1) != 0, want_max = (want & 2) != 0;
    const int nsteps = (qb - qa + NW - 1) / NW * NW;
    for (int sb = 0; sb < nsteps; sb += NW) {
#pragma unroll
        for (int ph = 0; ph < NW; ++ph) {
            const int st = sb + ph;
            ldp(st + NW - 1, ring[(ph + NW - 1) % NW]);
            const float* v = ring[ph % NW];   // plane q = qa + st
            const int q = qa + st;
            bool hasnan = false;
            float xmn[NR], xmx[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                hasnan |= v[r] != v[r];
                const float l = dpp_from_left(v[r]), rr = dpp_from_right(v[r]);
                xmn[r] = dz_min3(l, v[r], rr);
                xmx[r] = dz_max3(l, v[r], rr);
            }
            nanhist = ((nanhist << 1) | (__ballot(hasnan) != 0ull ? 1 : 0)) & 7;
            float mnC[DPY], mxC[DPY];
#pragma unroll
            for (int r = 0; r < DPY; ++r) {
                mnC[r] = dz_min3(xmn[r], xmn[r + 1], xmn[r + 2]);
                mxC[r] = dz_max3(xmx[r], xmx[r + 1], xmx[r + 2]);
            }
            const int zc = q - 1;   // centre plane of the test
            if (q < qb && zc >= tlo) {
                // per row: bit r of fl = candidate, of mx = a MAX ("this mixup is intended",
                // InteractiveIntegral.isSpecialPoint: every neighbour >= c is a MAX)
                unsigned fl = 0u, mxb = 0u;
#pragma unroll
                for (int r = 0; r < DPY; ++r) {
                    const float c = cB[r];
                    const bool cand = xt && ybase + 1 + r <= ny - 2 && !(fabsf(c) < minv);
                    const bool ge = dz_min3(mnA[r], mnB[r], mnC[r]) >= c;
                    const bool le = dz_max3(mxA[r], mxB[r], mxC[r]) <= c;
                    const bool is_max = cand && ge, is_min = cand && !ge && le;
                    fl |= unsigned((is_max && want_max) || (is_min && want_min)) << r;
                    mxb |= unsigned(is_max) << r;
                }
                if (nanhist != 0) {   // a NaN next to this plane: the comparison loop (rare)
                    fl = 0u;
                    mxb = 0u;
#pragma unroll 1
                    for (int r = 0; r < DPY; ++r) {
                        const int y = ybase + 1 + r;
                        const float c = dog[size_t(zc) * pstride + size_t(min(y, ny - 1)) * size_t(nx) + size_t(xl)];
                        const bool cand = xt && y <= ny - 2 && !(fabsf(c) < minv);
                        bool ge = true, le = true;
                        if (cand) {
#pragma unroll 1
                            for (int k = 0; k < 27; ++k) {
                                if (k == 13) continue;   // (the centre)
                                const float u = dog[size_t(zc + k / 9 - 1) * pstride + size_t(y + (k / 3) % 3 - 1) * size_t(nx) +
                                                    size_t(x + k % 3 - 1)];
                                ge &= u >= c;
                                le &= u <= c;
                            }
                        }
                        const int spn = !cand ? 0 : ge ? 2 : le ? 1 : 0;
                        fl |= unsigned((spn == 2 && want_max) || (spn == 1 && want_min)) << r;
                        mxb |= unsigned(spn == 2) << r;
                    }
                }
                if (__ballot(fl != 0u) != 0ull) {   // (rare: a few candidates per million voxels)
#pragma unroll
                    for (int r = 0; r < DPY; ++r) {
                        const bool flag = ((fl >> r) & 1u) != 0u;
                        const unsigned long long bal = __ballot(flag);
                        if (bal == 0ull) continue;
                        const int nb = __popcll(bal);
                        if (ccount + nb > kCandBuf) {
                            cand_flush(sink, cbuf[wv], ccount, nx, pstride);
                            ccount = 0;
                        }
                        const int sp = ((mxb >> r) & 1u) ? 2 : 1;
                        if (flag)
                            cbuf[wv][ccount + __popcll(bal & ((1ull << lane) - 1ull))] =
                                make_int4(x, (ybase + 1 + r) | (sp << 30), zc, __float_as_int(fabsf(cB[r])));
                        ccount += nb;
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < DPY; ++r) {
                mnA[r] = mnB[r]; mxA[r] = mxB[r];
                mnB[r] = mnC[r]; mxB[r] = mxC[r];
                cB[r] = v[r + 1];
            }
        }
    }
    cand_flush(sink, cbuf[wv], ccount, nx, pstride);
}

__global__ __launch_bounds__(kBlock) void k_minmax(const float* __restrict__ in, int64_t n,
                                                    float* __restrict__ partial) {
    __shared__ float smn[kBlock / 64], smx[kBlock / 64];
    __shared__ int sbad[kBlock / 64];
    float mn = INFINITY, mx = -INFINITY;
    float z = 0.0f;   // v * 0 summed: NaN once any value is NaN or infinite (finite: +-0)
    const int64_t stride = int64_t(gridDim.x) * kBlock;
    const int64_t t0 = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(in) & 15u) == 0) {   // 16-B loads, then the tail
        const float4* in4 = reinterpret_cast<const float4*>(in);
        const int64_t n4 = n / 4;
        for (int64_t i = t0; i < n4; i += stride) {
            const float4 v = in4[i];
            mn = fminf(fminf(mn, v.x), fminf(v.y, fminf(v.z, v.w)));
            mx = fmaxf(fmaxf(mx, v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
            z += (v.x * 0.0f + v.y * 0.0f) + (v.z * 0.0f + v.w * 0.0f);
        }
        for (int64_t i = 4 * n4 + t0; i < n; i += stride) {
            mn = fminf(mn, in[i]);
            mx = fmaxf(mx, in[i]);
            z += in[i] * 0.0f;
        }
    } else {
        for (int64_t i = t0; i < n; i += stride) {
            const float v = in[i];
            mn = fminf(mn, v);
            mx = fmaxf(mx, v);
            z += v * 0.0f;
        }
    }
    int bad = isnan(z) ? 1 : 0;
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, 64));
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        bad |= __shfl_xor(bad, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
        sbad[threadIdx.x >> 6] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) {
            mn = fminf(mn, smn[w]);
            mx = fmaxf(mx, smx[w]);
            bad |= sbad[w];
        }
        partial[2 * blockIdx.x] = mn;
        partial[2 * blockIdx.x + 1] = mx;
        partial[2 * gridDim.x + blockIdx.x] = bad ? 1.0f : 0.0f;
    }
}

// min / max over the per-block partials: one wave, lane-strided then shuffles
// (min and max are order-independent, so the result equals a sequential scan)
// partial[2] = 1 when any value is NaN or infinite, else 0 (k_dog_xy's tap trim)
__global__ __launch_bounds__(64) void k_minmax_final(float* partial, int nb) {
    float mn = INFINITY, mx = -INFINITY, bad = 0.0f;
    for (int b = threadIdx.x; b < nb; b += 64) {
        mn = fminf(mn, partial[2 * b]);
        mx = fmaxf(mx, partial[2 * b + 1]);
        bad = fmaxf(bad, partial[2 * nb + b]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, 64));
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        bad = fmaxf(bad, __shfl_xor(bad, off, 64));
    }
    if (threadIdx.x == 0) {
        partial[0] = mn;
        partial[1] = mx;
        partial[2] = bad;
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

// candidates of a DoG volume already in HBM (the fallback for Gaussians of 63 / 127 taps)
__global__ __launch_bounds__(kBlock) void k_peaks_append(const float* __restrict__ dog, Dims3 d, PeakSink pk) {
    const int64_t n = d.nx * d.ny * d.nz;
    for (int64_t i0 = int64_t(blockIdx.x) * kBlock; i0 < n; i0 += int64_t(gridDim.x) * kBlock) {
        const int64_t i = i0 + threadIdx.x;
        int sp = 0;
        float v = 0.0f;
        int64_t x = 0, y = 0, z = 0;
        if (i < n) {
            flat_coords(i, d, x, y, z);
            sp = special_point(dog, d, i, x, y, z, pk.minv, v);
        }
        const bool flag = (sp == 2 && pk.want_max) || (sp == 1 && pk.want_min);
        sink_append(pk, flag, int(x), int(y), int(z), uint64_t(i), v, sp);
    }
}

__global__ void k_gather_peaks(const PeakOut* __restrict__ recs, const uint32_t* __restrict__ order, int64_t n,
                               PeakOut* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = recs[order[i]];
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

// tuning knobs for A/B runs (tools/dog_bench.py); defaults are the measured best
int dog_env(const char* name, int def) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : def;
}

// true when p is device memory of `dev` itself (read / written in place by its kernels);
// host memory and other devices' buffers are staged through the workspace instead (a
// kernel on dev would fault on another device's memory without peer access)
bool is_device_ptr(const void* p, int dev) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable host memory: not registered with HIP
        return false;
    }
    return at.type == hipMemoryTypeDevice && at.device == dev;
}

// Per-device DoG workspace, grown on demand and kept between calls (a 768^3 view needs
// ~3.6 GB of G12 plus the candidate lists; hipMalloc / hipFree of that per call cost
// more than the DoG itself).  One call at a time per device holds its mutex;
// spim_dog_release_workspace frees it.
struct DogWork {
    std::mutex mu;
    DBuf<float> in, dog, taps, mm, tmp_a, tmp_b, tmp_c, tmp_d;
    DBuf<float2> g12;
    DBuf<uint64_t> keys, keys_sorted;
    DBuf<uint32_t> vals, vals_sorted;
    DBuf<PeakOut> recs, peaks;
    DBuf<unsigned> count;
    DBuf<unsigned char> sort_tmp;
    DBuf<LocOut> loc;                      // localisation results
    DBuf<spim_interest_point> ips, ips_sel;  // interest points before / after the threshold
    DBuf<unsigned char> flags, sel_tmp;
    DBuf<int> nsel;
    DBuf<PeakSink> sink;                   // k_dog_z's sink, read at its flushes
    // the calls' stream, created once (a stream per call cost ~1 ms of host time per
    // 768^3 call: r3l trace, 1.17 ms before the first copy)
    hipStream_t stream = nullptr;
    hipStream_t get_stream() {
        if (!stream) SD_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        return stream;
    }
    void release() {
        if (stream) {
            (void)hipStreamDestroy(stream);
            stream = nullptr;
        }
        for (DBuf<float>* b : {&in, &dog, &taps, &mm, &tmp_a, &tmp_b, &tmp_c, &tmp_d}) b->release();
        g12.release();
        keys.release(); keys_sorted.release(); vals.release(); vals_sorted.release();
        recs.release(); peaks.release(); count.release(); sort_tmp.release();
        loc.release(); ips.release(); ips_sel.release(); flags.release(); sel_tmp.release(); nsel.release();
        sink.release();
    }
};

std::mutex g_dogwork_mu;
// never destroyed (as legacy.cpp's g_ctx): no hipFree / hipStreamDestroy from a static
// destructor racing the HIP runtime's own teardown at process exit
std::map<int, std::unique_ptr<DogWork>>& g_dogwork = *new std::map<int, std::unique_ptr<DogWork>>();

DogWork& dog_work(int dev) {
    std::lock_guard<std::mutex> lk(g_dogwork_mu);
    auto& w = g_dogwork[dev];
    if (!w) w.reset(new DogWork());
    return *w;
}

template <typename T>
void grow(DBuf<T>& b, size_t n) {
    if (b.n < n) b.alloc(n);
}

// the DoG image (on the device) and the reference-ordered candidate list (on the device)
struct DogRun {
    Dims3 d{};
    const float* dog = nullptr;   // nullptr when neither localisation nor the image was asked for
    int64_t np = 0;
    const PeakOut* dpeaks = nullptr;
};

int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

void dog_run(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out, bool need_dog,
             hipStream_t s, DogWork& w, DogRun& r) {
    SD_CHECK(img && dims && p, SPIMDECON_ERR_ARG, "null argument");
    SD_CHECK(dims[0] >= 1 && dims[1] >= 1 && dims[2] >= 1, SPIMDECON_ERR_ARG, "bad dims");
    SD_CHECK(p->localization == 0 || p->localization == 1, SPIMDECON_ERR_ARG,
             "localization must be 0 (none) or 1 (quadratic); the Gaussian fit is not implemented in "
             "the reference either (Localization.java:90-96)");
    SD_CHECK(p->ij_threads >= 1 && p->ij_threads < (1 << 20), SPIMDECON_ERR_ARG, "ij_threads must be >= 1");
    const Dims3 d{dims[0], dims[1], dims[2]};
    r.d = d;
    const int64_t n = d.nx * d.ny * d.nz;
    SD_CHECK(n < (int64_t(1) << 40), SPIMDECON_ERR_ARG, "volume too large");

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
    // the same taps interleaved per axis, (sigma1[j], sigma2[j]) pairs, for the fused kernels
    // (k_dog_z reads the z taps as a symmetric half)
    for (int j = 0; j < K; ++j)
        SD_CHECK(k1[2][j] == k1[2][K - 1 - j] && k2[2][j] == k2[2][K - 1 - j], SPIMDECON_ERR_STATE,
                 "asymmetric z taps");
    for (int a = 0; a < 3; ++a)
        for (int j = 0; j < K; ++j) {
            kall.push_back(k1[a][j]);
            kall.push_back(k2[a][j]);
        }
    grow(w.taps, kall.size());
    SD_HIP(hipMemcpyAsync(w.taps.p, kall.data(), kall.size() * 4, hipMemcpyHostToDevice, s));
    auto kp = [&](int axis, int which) { return w.taps.p + (2 * axis + which) * K; };
    auto kp2 = [&](int axis) { return reinterpret_cast<const float2*>(w.taps.p + 6 * K + 2 * axis * K); };
    // leading taps zero for both sigmas along an axis (k_dog_xy may skip them, see there)
    auto zero_lead = [&](int a) {
        int t = 0;
        while (t < K / 2 && k1[a][t] == 0.0f && k2[a][t] == 0.0f && k1[a][K - 1 - t] == 0.0f &&
               k2[a][K - 1 - t] == 0.0f)
            ++t;
        return t;
    };
    // (instantiated for 0 and 1 trimmed taps -- 1 at the default sigma 1.8; 2 spilled VGPRs)
    // (SPIMDECON_DOG_TRIM=0: every padded tap always)
    const int jt = dog_env("SPIMDECON_DOG_TRIM", 1) ? std::min(1, std::min(zero_lead(0), zero_lead(1))) : 0;

    // the view: read in place when it already lives in HBM, else one upload
    const float* in = img;
    if (!is_device_ptr(img, p->device)) {
        grow(w.in, size_t(n));
        SD_HIP(hipMemcpyAsync(w.in.p, img, n * 4, hipMemcpyDefault, s));   // host or another device
        in = w.in.p;
    }
    grow(w.mm, 3 * 4096);
    const bool use_given = !(std::isnan(p->min_intensity) || std::isnan(p->max_intensity) ||
                             std::isinf(p->min_intensity) || std::isinf(p->max_intensity) ||
                             p->min_intensity == p->max_intensity);
    if (use_given) {
        // (mm[2] = 1: values not scanned, k_dog_xy keeps every padded tap)
        const float h2[3] = {float(p->min_intensity), float(p->max_intensity), 1.0f};
        SD_HIP(hipMemcpyAsync(w.mm.p, h2, 12, hipMemcpyHostToDevice, s));
    } else {
        const unsigned nb = grid_of(n);
        hipLaunchKernelGGL(k_minmax, dim3(nb), dim3(kBlock), 0, s, in, n, w.mm.p);
        hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(64), 0, s, w.mm.p, int(nb));
        SD_HIP(hipGetLastError());
    }
    // DoG destination: the caller's device buffer, else the workspace (copied out at the end)
    float* dogp = nullptr;
    const bool dog_dev = dog_out && is_device_ptr(dog_out, p->device);
    if (need_dog) {
        if (dog_dev) {
            dogp = dog_out;
        } else {
            grow(w.dog, size_t(n));
            dogp = w.dog.p;
        }
    }
    grow(w.count, 1);
    unsigned cap = unsigned(std::min<int64_t>(std::max<int64_t>(int64_t(1) << 16, n / 256), int64_t(1) << 30));
    cap = std::max<unsigned>(cap, unsigned(std::min<size_t>(w.recs.n, size_t(1) << 30)));
    const int T = p->ij_threads;
    const int wmin = p->find_min ? 1 : 0, wmax = p->find_max ? 1 : 0;
    const bool fused = (K == 7 || K == 15 || K == 31) && n < (int64_t(1) << 32) && d.ny <= 65535 * 32 &&
                       d.nz <= 65535;
    // (chunk + 2 + KW - 1 source planes must fit k_dog_z's kDzMaxLen plane table)
    const int zc = std::min(kDzMaxLen - 128, kDzChunk);
    constexpr int ty = 32;     // strip steps (48-row tiles: 32 measured slower; strips: 32 beat 48, r05_dog_strips_ab.txt)
    constexpr int xcd = 1;     // XCD-contiguous y-fastest boxes of k_dog_z
    constexpr int xcd_xy = 1;  // XCD-contiguous tile ranges of k_dog_xy
    // k_dog_xy: persistent blocks (4 per CU at 32-row steps: 34.5 KB of LDS each), strips x
    // fastest
    const int64_t xy_strips = ceil_div(d.nx, kDxyTX) * d.nz;
    const dim3 gxy(unsigned(std::min<int64_t>(xy_strips, int64_t(256) * 4)));
    // k_dog_z box: 64 x 8 (512 threads); 64 x 16 and 32 x 16 measured slower (r3i)
    constexpr int bx = 64, bz_y = 8;
    // scalar plane indices (one mirror reflection: nz > K / 2; plane bytes in 31 bits)
    const bool zsl = d.nz > K / 2 && d.nx * d.ny * 8 < (int64_t(1) << 31);
    const dim3 gz(unsigned(std::max<int64_t>(1, ceil_div(d.nx - 2, bx - 2))),
                  unsigned(std::max<int64_t>(1, ceil_div(d.ny - 2, bz_y - 2))), unsigned(ceil_div(d.nz, zc)));
    bool store_dog = need_dog;
    // the split z stage (default): k_dog_zconv stores the DoG of every voxel, then k_dog_z
    // tests over the stored image (SPIMDECON_DOG_SPLIT=0: the fused k_dog_z); a candidate
    // overflow reruns the test pass only
    // (k_dog_zconv's one-reflection plane index needs nz > K / 2; k_dog_peaks addresses the
    // DoG image through one buffer resource with 32-bit plane offsets: below 4 GiB)
    const bool split = fused && dog_env("SPIMDECON_DOG_SPLIT", 1) != 0 && d.nx * d.ny * 8 < (int64_t(1) << 31) &&
                       d.nz > K / 2 && uint64_t(n) * 4u < 0xffffffffull;
    const int zc1 = std::max(1, dog_env("SPIMDECON_DOG_ZC_CHUNK", 256));
    if (split && !dogp) {
        grow(w.dog, size_t(n));
        dogp = w.dog.p;
    }
    if (fused) {
        grow(w.g12, size_t(n));
        const bool xbuf = uint64_t(n) * 4u < 0xffffffffull;
        // (k_minmax's own range: the per-value range check is skipped; SPIMDECON_DOG_MM_EXACT=0
        // keeps it -- 1.52-1.62 vs 1.66 ms per 768^3, bit-exact, gpu_r3z11.sh)
        const int mmx = !use_given && dog_env("SPIMDECON_DOG_MM_EXACT", 1) != 0 ? 1 : 0;
#define SD_DOGXY3(KV, JV)                                                                                   \
        if (xbuf) hipLaunchKernelGGL((k_dog_xy<KV, ty, true, JV>), gxy, dim3(256), 0, s, d, in, kp2(0), kp2(1), w.g12.p, w.mm.p, xcd_xy, mmx); \
        else hipLaunchKernelGGL((k_dog_xy<KV, ty, false, JV>), gxy, dim3(256), 0, s, d, in, kp2(0), kp2(1), w.g12.p, w.mm.p, xcd_xy, mmx);
#define SD_DOGXY(KV) if (jt == 1) { SD_DOGXY3(KV, 1) } else { SD_DOGXY3(KV, 0) }
        if (K == 7) { SD_DOGXY(7) } else if (K == 15) { SD_DOGXY(15) } else { SD_DOGXY(31) }
#undef SD_DOGXY
#undef SD_DOGXY3
        SD_HIP(hipGetLastError());
        if (split) {
            const int64_t waves = ceil_div(d.nx, int64_t(64)) * d.ny;
            const dim3 gc(unsigned(ceil_div(waves, int64_t(4))), unsigned(ceil_div(d.nz, int64_t(zc1))));
            const bool one1 = uint64_t(n) * 4u < 0x80000000ull, oneg = uint64_t(n) * 8u < 0xffffffffull;
#define SD_DOGZC(KV) if (one1 && oneg) hipLaunchKernelGGL((k_dog_zconv<KV, kDzcPD, true, true>), gc, dim3(256), 0, s, d, w.g12.p, kp2(2), kinv, zc1, dogp); \
            else if (oneg) hipLaunchKernelGGL((k_dog_zconv<KV, kDzcPD, false, true>), gc, dim3(256), 0, s, d, w.g12.p, kp2(2), kinv, zc1, dogp); \
            else hipLaunchKernelGGL((k_dog_zconv<KV, kDzcPD, false, false>), gc, dim3(256), 0, s, d, w.g12.p, kp2(2), kinv, zc1, dogp);
            if (K == 7) { SD_DOGZC(7) } else if (K == 15) { SD_DOGZC(15) } else { SD_DOGZC(31) }
#undef SD_DOGZC
            SD_HIP(hipGetLastError());
        }
    } else {
        // Gaussians of 63 / 127 taps: the separate passes, then a candidate pass over the DoG
        grow(w.tmp_a, size_t(n));
        grow(w.tmp_b, size_t(n));
        grow(w.tmp_c, size_t(n));
        grow(w.tmp_d, size_t(n));
        if (!dogp) {
            grow(w.dog, size_t(n));
            dogp = w.dog.p;
        }
        sep_pass(d, 0, in, in, kp(0, 0), kp(0, 1), K, OOB_MIRROR, 0.f, w.tmp_a.p, w.tmp_b.p, false, 0.f, w.mm.p, s);
        sep_pass(d, 1, w.tmp_a.p, w.tmp_b.p, kp(1, 0), kp(1, 1), K, OOB_MIRROR, 0.f, w.tmp_c.p, w.tmp_d.p, false,
                 0.f, nullptr, s);
        sep_pass(d, 2, w.tmp_c.p, w.tmp_d.p, kp(2, 0), kp(2, 1), K, OOB_MIRROR, 0.f, dogp, nullptr, true, kinv,
                 nullptr, s);
    }
    unsigned total = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        grow(w.keys, cap);
        grow(w.vals, cap);
        grow(w.recs, cap);
        SD_HIP(hipMemsetAsync(w.count.p, 0, sizeof(unsigned), s));
        const PeakSink pk{min_peak, wmin, wmax, T, w.keys.p, w.vals.p, w.recs.p, w.count.p, cap};
        if (split) {
            grow(w.sink, 1);
            SD_HIP(hipMemcpyAsync(w.sink.p, &pk, sizeof(pk), hipMemcpyHostToDevice, s));   // (synchronised below)
            const int want = wmin | (wmax << 1);
            // (the ring test of k_dog_z over the stored image measured 1.19 vs 0.42 ms)
            if (d.nx >= 3 && d.ny >= 3 && d.nz >= 3) {   // (else no voxel has 26 neighbours)
                constexpr int zcp = 64;
                const int64_t nwave = ceil_div(d.nx - 2, int64_t(62)) * ceil_div(d.ny - 2, int64_t(kDpkY)) *
                                      ceil_div(d.nz - 2, int64_t(zcp));
                const dim3 gp(unsigned(ceil_div(nwave, int64_t(4))));
                hipLaunchKernelGGL((k_dog_peaks<kDpkY, kDpkPD>), gp, dim3(256), 0, s, d, dogp, zcp, min_peak, want, w.sink.p, 1);
            }
        } else if (fused) {
            float* dst = store_dog ? dogp : nullptr;
            grow(w.sink, 1);
            SD_HIP(hipMemcpyAsync(w.sink.p, &pk, sizeof(pk), hipMemcpyHostToDevice, s));   // (synchronised below)
            const bool one = uint64_t(n) * 4u < 0x80000000ull;
            const int want = wmin | (wmax << 1);
#define SD_DOGZ4(KV, BYV, ONEV, SLV) hipLaunchKernelGGL((k_dog_z<KV, BYV, kDzPD, 64, ONEV, SLV>), gz, dim3(64 * BYV), 0, s, d, w.g12.p, kp2(2), kinv, zc, dst, min_peak, want, w.sink.p, xcd);
#define SD_DOGZ3(KV, ONEV, SLV) SD_DOGZ4(KV, bz_y, ONEV, SLV)
#define SD_DOGZ2(KV, ONEV) if (zsl) { SD_DOGZ3(KV, ONEV, true) } else { SD_DOGZ3(KV, ONEV, false) }
#define SD_DOGZ(KV) if (one) { SD_DOGZ2(KV, true) } else { SD_DOGZ2(KV, false) }
            if (K == 7) { SD_DOGZ(7) } else if (K == 15) { SD_DOGZ(15) } else { SD_DOGZ(31) }
#undef SD_DOGZ
#undef SD_DOGZ2
#undef SD_DOGZ3
#undef SD_DOGZ4
        } else {
            hipLaunchKernelGGL(k_peaks_append, dim3(grid_of(n)), dim3(kBlock), 0, s, dogp, d, pk);
        }
        SD_HIP(hipGetLastError());
        SD_HIP(hipMemcpyAsync(&total, w.count.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
        SD_HIP(hipStreamSynchronize(s));
        if (total <= cap) break;
        cap = total;          // rerun with room for every candidate (the DoG is already stored)
        store_dog = false;
    }
    // reference order: ascending (x % T) << 40 | flat
    r.np = total;
    r.dog = dogp;
    if (total > 0) {
        grow(w.keys_sorted, total);
        grow(w.vals_sorted, total);
        grow(w.peaks, total);
        const int end_bit = 40 + bits_for(uint64_t(T - 1));
        const size_t tb = peak_sort_temp_bytes(total, end_bit);
        grow(w.sort_tmp, std::max<size_t>(tb, 1));
        peak_sort(w.sort_tmp.p, tb, w.keys.p, w.keys_sorted.p, w.vals.p, w.vals_sorted.p, total, end_bit, s);
        hipLaunchKernelGGL(k_gather_peaks, dim3(unsigned(ceil_div(total, 256))), dim3(256), 0, s, w.recs.p,
                           w.vals_sorted.p, int64_t(total), w.peaks.p);
        SD_HIP(hipGetLastError());
        r.dpeaks = w.peaks.p;
    }
    if (dog_out && !dog_dev) SD_HIP(hipMemcpyAsync(dog_out, dogp, n * 4, hipMemcpyDefault, s));
}

struct StreamHolder {   // the workspace's stream (held under its mutex)
    hipStream_t s = nullptr;
    explicit StreamHolder(DogWork& w) : s(w.get_stream()) {}
};

// DifferenceOfGaussianNewPeakFinder.getSimplePeaks level: candidates with
// |v| >= threshold (localization 0) or threshold / 10 (localization 1)
void dog_compute(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out,
                 spim_peak* peaks, int64_t max_peaks, int64_t* npeaks) {
    SD_CHECK(npeaks && p, SPIMDECON_ERR_ARG, "null argument");
    check_device(p->device);
    DeviceGuard guard(p->device);
    DogWork& w = dog_work(p->device);
    std::lock_guard<std::mutex> lk(w.mu);
    StreamHolder sh(w);
    DogRun r;
    dog_run(img, dims, p, dog_out, dog_out != nullptr, sh.s, w, r);
    *npeaks = r.np;
    const int64_t m = peaks ? std::min(r.np, max_peaks) : 0;
    std::vector<PeakOut> hp(std::max<int64_t>(m, 0));
    if (m > 0) SD_HIP(hipMemcpyAsync(hp.data(), r.dpeaks, m * sizeof(PeakOut), hipMemcpyDeviceToHost, sh.s));
    SD_HIP(hipStreamSynchronize(sh.s));
    for (int64_t i = 0; i < m; ++i) {
        peaks[i].x = hp[i].x;
        peaks[i].y = hp[i].y;
        peaks[i].z = hp[i].z;
        peaks[i].intensity = hp[i].intensity;
        peaks[i].is_min = hp[i].is_min;
        peaks[i].is_max = hp[i].is_max;
    }
}

// candidates -> interest points on the device: Localization.noLocalization (:19-45)
// copies them; with quadratic localisation (:47-88) the caller keeps those whose fitted
// |value| > threshold (flag), in candidate order
template <bool LOC>
__global__ void k_to_points(const PeakOut* __restrict__ pk, const LocOut* __restrict__ loc, int64_t np, float thr,
                            spim_interest_point* __restrict__ ips, unsigned char* __restrict__ flags) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= np) return;
    spim_interest_point ip{};
    if constexpr (LOC) {
        const LocOut l = loc[i];
        for (int a = 0; a < 3; ++a) ip.pos[a] = l.pos[a];
        ip.intensity = l.value;
        flags[i] = fabsf(l.value) > thr ? 1 : 0;   // float against float (Localization.java:74)
    } else {
        ip.pos[0] = pk[i].x;
        ip.pos[1] = pk[i].y;
        ip.pos[2] = pk[i].z;
        ip.intensity = pk[i].intensity;
    }
    ip.is_max = pk[i].is_max;
    ips[i] = ip;
}

// ProcessDOG.compute's result: interest points after Localization (:150-168).  The
// candidates (threshold / 10 with quadratic localisation: millions on a noisy 768^3
// view) stay on the device; only the interest points are copied out.
void dog_interest_points(const float* img, const int64_t* dims, const spim_dog_params* p, float* dog_out,
                         spim_interest_point* out, int64_t max_out, int64_t* nout) {
    SD_CHECK(nout && p, SPIMDECON_ERR_ARG, "null argument");
    check_device(p->device);
    DeviceGuard guard(p->device);
    DogWork& w = dog_work(p->device);
    std::lock_guard<std::mutex> lk(w.mu);
    StreamHolder sh(w);
    DogRun r;
    dog_run(img, dims, p, dog_out, p->localization == 1 || dog_out != nullptr, sh.s, w, r);
    const int64_t np = r.np;
    int64_t n = 0;
    const spim_interest_point* res = nullptr;
    if (np > 0) {
        grow(w.ips, size_t(np));
        const unsigned grid = unsigned(ceil_div(np, int64_t(256)));
        if (p->localization == 0) {
            hipLaunchKernelGGL(k_to_points<false>, dim3(grid), dim3(256), 0, sh.s, r.dpeaks, nullptr, np, 0.0f,
                               w.ips.p, nullptr);
            SD_HIP(hipGetLastError());
            res = w.ips.p;
            n = np;
        } else {
            grow(w.loc, size_t(np));
            grow(w.flags, size_t(np));
            grow(w.ips_sel, size_t(np));
            grow(w.nsel, 1);
            hipLaunchKernelGGL(k_localize, dim3(grid), dim3(256), 0, sh.s, r.dog, r.d, r.dpeaks, np, w.loc.p);
            SD_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_to_points<true>, dim3(grid), dim3(256), 0, sh.s, r.dpeaks, w.loc.p, np,
                               float(p->threshold), w.ips.p, w.flags.p);
            SD_HIP(hipGetLastError());
            const size_t tb = point_select_temp_bytes(np);
            grow(w.sel_tmp, std::max<size_t>(tb, 1));
            point_select(w.sel_tmp.p, tb, w.ips.p, w.flags.p, w.ips_sel.p, w.nsel.p, np, sh.s);
            int hn = 0;
            SD_HIP(hipMemcpyAsync(&hn, w.nsel.p, sizeof(int), hipMemcpyDeviceToHost, sh.s));
            SD_HIP(hipStreamSynchronize(sh.s));
            res = w.ips_sel.p;
            n = hn;
        }
    }
    const int64_t m = out ? std::min<int64_t>(max_out, n) : 0;
    if (m > 0) SD_HIP(hipMemcpyAsync(out, res, size_t(m) * sizeof(spim_interest_point), hipMemcpyDefault, sh.s));
    SD_HIP(hipStreamSynchronize(sh.s));
    *nout = n;
}

void dog_release_workspace(int dev) {
    check_device(dev);
    DeviceGuard guard(dev);
    DogWork& w = dog_work(dev);
    std::lock_guard<std::mutex> lk(w.mu);
    SD_HIP(hipDeviceSynchronize());
    w.release();
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

extern "C" int spim_dog_release_workspace(int device) {
    return guarded([&] { dog_release_workspace(device); });
}

extern "C" int spim_dog_compute(const float* img, const int64_t* dims, const spim_dog_params* p,
                                float* dog_out, spim_peak* peaks, int64_t max_peaks,
                                int64_t* npeaks) {
    return guarded([&] { dog_compute(img, dims, p, dog_out, peaks, max_peaks, npeaks); });
}
