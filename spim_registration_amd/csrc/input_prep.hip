// input_prep.hip -- deconvolution input preparation on the GPU.
//
// Restates (paths under /root/reference/src/main/java/, DECON =
// spim/process/fusion/deconvolution/):
//   resampling       DECON/TransformInput.java:74-95, TransformInputAndWeights.java:86-121
//   virtual weights  spim/process/fusion/weights/TransformedInterpolatedRealRandomAccess.java:96-118
//   blending         spim/process/fusion/weights/BlendingRealRandomAccess.java:25-104
//   normalisation    DECON/WeightNormalizer.java:52-205, weights/NormalizingRandomAccess.java:36-45
//   OSEM             DECON/ProcessForDeconvolution.java:318-384
// The imglib2 pieces absent from the container (affine inverse, applyInverse,
// NLinearInterpolator3D) follow the restatement in oracle/input_ref.py.
// One thread per output voxel; HBM-bound gathers (the source stack is read
// through L2 with trilinear locality).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "resample.hpp"
#include "spimdecon.h"

namespace spimdecon {
void check_device(int dev);

namespace {

constexpr int kIpBlock = 256;

struct ViewArgs {
    const float* src;
    int sx, sy, sz;
    AffineInv a;
    float border[3], range[3];
};

// BlendingRealRandomAccess.computeWeight (:78-104), float arithmetic
__device__ float blend_weight(const float t[3], const int dims[3], const float* border, const float* range,
                              const double* lut) {
    float w = 1.0f;
    for (int d = 0; d < 3; ++d) {
        const float l = t[d];
        const float a = l - border[d];
        const float b = (float(dims[d] - 1) - l) - border[d];
        const float dist = fmaxf(0.0f, fminf(a, b));
        if (dist == 0.0f) return 0.0f;
        const float rel = dist / range[d];
        if (rel < 1.0f) {
            int idx = int(floor(double(rel) * 1000.0 + 0.5));
            idx = idx < 0 ? 0 : (idx > 1000 ? 1000 : idx);
            w = float(double(w) * lut[idx]);
        }
    }
    return w;
}

__device__ __forceinline__ float nlinear(const float* src, int sx, int sy, int sz, const float t[3]) {
    return nlinear_at<kExtMirror>(src, sx, sy, sz, t[0], t[1], t[2]);
}

__global__ __launch_bounds__(kIpBlock) void k_transform_view(ViewArgs v, int64_t bx, int64_t by, int64_t bz,
                                                             int64_t nx, int64_t ny, int64_t n, int weight_type,
                                                             const double* __restrict__ lut,
                                                             float* __restrict__ img_out,
                                                             float* __restrict__ w_out) {
    int64_t x, y, z;
    if (!tiled_xyz(nx, ny, n / (nx * ny), x, y, z)) return;
    const int64_t i = (z * ny + y) * nx + x;
    // TransformInput: s = (float) position + offset; t = inv3 (s - translation)
    const float s0 = float(x) + float(bx), s1 = float(y) + float(by), s2 = float(z) + float(bz);
    const double d0 = double(s0) - v.a.tr[0], d1 = double(s1) - v.a.tr[1], d2 = double(s2) - v.a.tr[2];
    float t[3];
    for (int r = 0; r < 3; ++r)
        t[r] = float(v.a.inv[3 * r] * d0 + v.a.inv[3 * r + 1] * d1 + v.a.inv[3 * r + 2] * d2);
    float val = 0.0f;
    if (t[0] >= 0.0f && t[1] >= 0.0f && t[2] >= 0.0f && t[0] < float(v.sx) && t[1] < float(v.sy) &&
        t[2] < float(v.sz))  // FusionHelper.intersects (double compares of float values)
        val = fmaxf(1e-4f, nlinear(v.src, v.sx, v.sy, v.sz, t));
    img_out[i] = val;
    const int dims[3] = {v.sx, v.sy, v.sz};
    float w = 1.0f;
    if (weight_type == SPIM_WEIGHTS_PRECOMPUTED) {
        w = blend_weight(t, dims, v.border, v.range, lut);
    } else if (weight_type == SPIM_WEIGHTS_VIRTUAL) {
        const double q0 = double(x + bx), q1 = double(y + by), q2 = double(z + bz);
        float u[3];
        for (int r = 0; r < 3; ++r)
            u[r] = float(q0 * v.a.full[4 * r] + q1 * v.a.full[4 * r + 1] + q2 * v.a.full[4 * r + 2] +
                         v.a.full[4 * r + 3]);
        w = blend_weight(u, dims, v.border, v.range, lut);
    }
    w_out[i] = w;
}

// WeightNormalizer: sum over views (double, view order), count of views with w > 0;
// PRECOMPUTED: w /= sum in place; VIRTUAL: S = sum > 1 ? (float) sum : 1.
// Overlap statistics per reference portion (grid.y = portion, grid.x = blocks striding
// over it): per-thread min / sum of the counts, one atomic pair per block.
__global__ __launch_bounds__(kIpBlock) void k_weight_sum(float* const* __restrict__ ws, int nviews, int64_t n,
                                                         int weight_type, float* __restrict__ S,
                                                         int64_t chunk, int nportions,
                                                         int* __restrict__ pmin,
                                                         unsigned long long* __restrict__ psum) {
    __shared__ int smin[kIpBlock / 64];
    __shared__ unsigned long long ssum[kIpBlock / 64];
    const int port = int(blockIdx.y);
    // the last portion takes the remainder (all of it when size < portions)
    const int64_t lo = chunk > 0 ? int64_t(port) * chunk : (port == nportions - 1 ? 0 : n);
    const int64_t hi = port == nportions - 1 ? n : lo + chunk;
    int m = nviews;
    unsigned long long sm = 0ull;
    for (int64_t i = lo + int64_t(blockIdx.x) * kIpBlock + threadIdx.x; i < hi;
         i += int64_t(gridDim.x) * kIpBlock) {
        double sum = 0.0;
        int cnt = 0;
        for (int v = 0; v < nviews; ++v) {
            const float w = ws[v][i];
            sum += w;
            if (w > 0.0f) ++cnt;
        }
        if (weight_type == SPIM_WEIGHTS_PRECOMPUTED) {
            for (int v = 0; v < nviews; ++v) ws[v][i] = float(double(ws[v][i]) / sum);
        } else {
            S[i] = sum > 1.0 ? float(sum) : 1.0f;
        }
        m = min(m, cnt);
        sm += (unsigned long long)cnt;
    }
    for (int off = 32; off > 0; off >>= 1) {
        m = min(m, __shfl_xor(m, off, 64));
        sm += __shfl_xor(sm, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        smin[threadIdx.x >> 6] = m;
        ssum[threadIdx.x >> 6] = sm;
    }
    __syncthreads();
    if (threadIdx.x == 0 && lo < hi) {
        for (int w = 1; w < kIpBlock / 64; ++w) {
            m = min(m, smin[w]);
            sm += ssum[w];
        }
        atomicMin(&pmin[port], m);
        atomicAdd(&psum[port], sm);
    }
}

__global__ __launch_bounds__(kIpBlock) void k_final_weight(float* __restrict__ w, const float* __restrict__ S,
                                                           int64_t n, int weight_type, double osem) {
    const int64_t i = int64_t(blockIdx.x) * kIpBlock + threadIdx.x;
    if (i >= n) return;
    // Java Math.min propagates NaN (PRECOMPUTED weights are NaN where no view has data)
    if (weight_type == SPIM_WEIGHTS_VIRTUAL) {
        const double v = (double(w[i]) / double(S[i])) * osem;
        w[i] = float(isnan(v) ? v : fmin(1.0, v));
    } else if (weight_type == SPIM_WEIGHTS_PRECOMPUTED && osem != 1.0) {
        const float v = w[i] * float(osem);
        w[i] = isnan(v) ? v : fminf(1.0f, v);
    }
}

// ---------------------------------------------------------------- weighted-average fusion
// spim/process/fusion/weightedavg/ProcessParalellPortionWeight.java:86-127 (blending)
// and ProcessParalellPortion.java:86-120 (plain mean); SURVEY 8f #3.
struct FuseView {
    const float* src;
    int sx, sy, sz;
    double inv[9], tr[3];
    float border[3], range[3];
};

__device__ float nearest1(const float* src, int sx, int sy, int sz, const float t[3]) {
    const int x = mirror1(int(floor(double(t[0]) + 0.5)), sx);
    const int y = mirror1(int(floor(double(t[1]) + 0.5)), sy);
    const int z = mirror1(int(floor(double(t[2]) + 0.5)), sz);
    return src[(int64_t(z) * sy + y) * sx + x];
}

__global__ __launch_bounds__(kIpBlock) void k_fuse(const FuseView* __restrict__ views, int nviews, int64_t bx,
                                                   int64_t by, int64_t bz, int64_t nx, int64_t ny, int64_t n,
                                                   float ds, int interp, int blend, const double* __restrict__ lut,
                                                   float* __restrict__ out) {
    int64_t x, y, z;
    if (!tiled_xyz(nx, ny, n / (nx * ny), x, y, z)) return;
    const int64_t i = (z * ny + y) * nx + x;
    float f0 = float(x), f1 = float(y), f2 = float(z);
    if (ds != 1.0f) {
        f0 = f0 * ds;
        f1 = f1 * ds;
        f2 = f2 * ds;
    }
    const float s0 = f0 + float(bx), s1 = f1 + float(by), s2 = f2 + float(bz);
    double sum = 0.0, sumw = 0.0;
    int cnt = 0;
    for (int v = 0; v < nviews; ++v) {
        const FuseView& fv = views[v];
        const double d0 = double(s0) - fv.tr[0], d1 = double(s1) - fv.tr[1], d2 = double(s2) - fv.tr[2];
        float t[3];
        for (int r = 0; r < 3; ++r)
            t[r] = float(fv.inv[3 * r] * d0 + fv.inv[3 * r + 1] * d1 + fv.inv[3 * r + 2] * d2);
        if (!(t[0] >= 0.0f && t[1] >= 0.0f && t[2] >= 0.0f && t[0] < float(fv.sx) && t[1] < float(fv.sy) &&
              t[2] < float(fv.sz)))
            continue;
        const double val = interp ? double(nlinear(fv.src, fv.sx, fv.sy, fv.sz, t))
                                  : double(nearest1(fv.src, fv.sx, fv.sy, fv.sz, t));
        if (blend) {
            const int dims[3] = {fv.sx, fv.sy, fv.sz};
            const double w = blend_weight(t, dims, fv.border, fv.range, lut);
            sum += val * w;
            sumw += w;
        } else {
            sum += val;
            ++cnt;
        }
    }
    out[i] = blend ? (sumw > 0.0 ? float(sum / sumw) : 0.0f) : (cnt > 0 ? float(sum / cnt) : 0.0f);
}

std::vector<double> blending_lut() {
    std::vector<double> lut(1001, 0.0);
    for (double d = 0; d <= 1.0001; d = d + 0.001)
        lut[size_t(std::floor(d * 1000.0 + 0.5))] = (std::cos((1 - d) * M_PI) + 1) / 2;
    return lut;
}

}  // namespace

void prepare_inputs(int nviews, const spim_view_source* views, const spim_input_params* p, float* const* img_out,
                    float* const* w_out, double* osem_used, int* min_overlap, double* avg_overlap) {
    SD_CHECK(nviews >= 1 && views && p && img_out && w_out, SPIMDECON_ERR_ARG, "null argument");
    SD_CHECK(p->weight_type == SPIM_WEIGHTS_NONE || p->weight_type == SPIM_WEIGHTS_PRECOMPUTED ||
                 p->weight_type == SPIM_WEIGHTS_VIRTUAL,
             SPIMDECON_ERR_ARG, "unknown weight type");
    SD_CHECK(p->bb_dims[0] >= 1 && p->bb_dims[1] >= 1 && p->bb_dims[2] >= 1, SPIMDECON_ERR_ARG, "bad bounding box");
    SD_CHECK(p->ij_threads >= 1, SPIMDECON_ERR_ARG, "ij_threads must be >= 1");
    check_device(p->device);
    DeviceGuard guard(p->device);
    hipStream_t s;
    SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct SG {
        hipStream_t s;
        ~SG() { (void)hipStreamDestroy(s); }
    } sg{s};
    const int64_t nx = p->bb_dims[0], ny = p->bb_dims[1], nz = p->bb_dims[2];
    const int64_t n = nx * ny * nz;
    const unsigned grid = unsigned(ceil_div(n, int64_t(kIpBlock)));
    const std::vector<double> lut = blending_lut();
    DBuf<double> dlut(lut.size());
    SD_HIP(hipMemcpyAsync(dlut.p, lut.data(), lut.size() * 8, hipMemcpyHostToDevice, s));

    // per-view outputs on the device (the caller's buffers when out_on_device)
    std::vector<DBuf<float>> own_img(nviews), own_w(nviews);
    std::vector<float*> dimg(nviews), dw(nviews);
    for (int v = 0; v < nviews; ++v) {
        if (p->out_on_device) {
            dimg[v] = img_out[v];
            dw[v] = w_out[v];
        } else {
            own_img[v].alloc(n);
            own_w[v].alloc(n);
            dimg[v] = own_img[v].p;
            dw[v] = own_w[v].p;
        }
    }
    for (int v = 0; v < nviews; ++v) {
        const spim_view_source& vs = views[v];
        SD_CHECK(vs.img && vs.dims[0] >= 1 && vs.dims[1] >= 1 && vs.dims[2] >= 1, SPIMDECON_ERR_ARG,
                 "bad view source");
        SD_CHECK(vs.dims[0] < (1 << 30) && vs.dims[1] < (1 << 30) && vs.dims[2] < (1 << 30), SPIMDECON_ERR_ARG,
                 "view too large");
        ViewArgs a{};
        const int64_t sn = vs.dims[0] * vs.dims[1] * vs.dims[2];
        DBuf<float> dsrc;
        if (p->src_on_device) {
            a.src = vs.img;
        } else {
            dsrc.alloc(sn);
            SD_HIP(hipMemcpyAsync(dsrc.p, vs.img, sn * 4, hipMemcpyHostToDevice, s));
            a.src = dsrc.p;
        }
        a.sx = int(vs.dims[0]);
        a.sy = int(vs.dims[1]);
        a.sz = int(vs.dims[2]);
        a.a = invert_model(vs.model);
        for (int d = 0; d < 3; ++d) {
            a.border[d] = p->blending_border[d];
            a.range[d] = p->blending_range[d];
        }
        SD_CHECK(tiled_blocks(nx, ny, nz) < (int64_t(1) << 31), SPIMDECON_ERR_ARG, "bounding box too large");
        hipLaunchKernelGGL(k_transform_view, dim3(unsigned(tiled_blocks(nx, ny, n / (nx * ny)))), dim3(kIpBlock), 0,
                           s, a, p->bb_min[0], p->bb_min[1],
                           p->bb_min[2], nx, ny, n, p->weight_type, dlut.p, dimg[v], dw[v]);
        SD_HIP(hipGetLastError());
        SD_HIP(hipStreamSynchronize(s));  // the source buffer is released at the end of the iteration
    }
    double osem = 1.0;
    int mn = -1;
    double av = std::nan("");
    if (p->weight_type != SPIM_WEIGHTS_NONE) {
        const int np = 2 * p->ij_threads;  // FusionHelper.divideIntoPortions(size, 2T)
        DBuf<float*> dws(nviews);
        SD_HIP(hipMemcpyAsync(dws.p, dw.data(), nviews * sizeof(float*), hipMemcpyHostToDevice, s));
        DBuf<float> S(p->weight_type == SPIM_WEIGHTS_VIRTUAL ? n : 1);
        DBuf<int> pmin(np);
        DBuf<unsigned long long> psum(np);
        std::vector<int> hmin(np, nviews);
        SD_HIP(hipMemcpyAsync(pmin.p, hmin.data(), np * 4, hipMemcpyHostToDevice, s));
        SD_HIP(hipMemsetAsync(psum.p, 0, np * 8, s));
        const int64_t span = std::max<int64_t>(n / np, n - (n / np) * (np - 1));   // the largest portion
        const unsigned bx = unsigned(std::max<int64_t>(1, std::min<int64_t>(ceil_div(span, kIpBlock), 8192 / np)));
        hipLaunchKernelGGL(k_weight_sum, dim3(bx, unsigned(np)), dim3(kIpBlock), 0, s, dws.p, nviews, n,
                           p->weight_type, S.p, n / np, np, pmin.p, psum.p);
        SD_HIP(hipGetLastError());
        std::vector<unsigned long long> hsum(np);
        SD_HIP(hipMemcpyAsync(hmin.data(), pmin.p, np * 4, hipMemcpyDeviceToHost, s));
        SD_HIP(hipMemcpyAsync(hsum.data(), psum.p, np * 8, hipMemcpyDeviceToHost, s));
        SD_HIP(hipStreamSynchronize(s));
        // WeightNormalizer.process (:74-86): min over portions, mean of per-portion means
        mn = nviews;
        double acc = 0.0;
        for (int q = 0; q < np; ++q) {
            const int64_t loop = q == np - 1 ? n - (n / np) * (np - 1) : n / np;
            mn = std::min(mn, hmin[q]);
            acc += loop > 0 ? double(hsum[q]) / double(loop) : std::nan("");
        }
        av = acc / np;
        // ProcessForDeconvolution.java:318-336
        osem = p->osem_index == 1 ? double(std::max(1, mn))
               : p->osem_index == 2 ? std::max(1.0, av)
                                    : p->osem_speedup;
        for (int v = 0; v < nviews; ++v)
            hipLaunchKernelGGL(k_final_weight, dim3(grid), dim3(kIpBlock), 0, s, dw[v], S.p, n, p->weight_type,
                               osem);
        SD_HIP(hipGetLastError());
    }
    if (!p->out_on_device) {
        for (int v = 0; v < nviews; ++v) {
            SD_HIP(hipMemcpyAsync(img_out[v], dimg[v], n * 4, hipMemcpyDeviceToHost, s));
            SD_HIP(hipMemcpyAsync(w_out[v], dw[v], n * 4, hipMemcpyDeviceToHost, s));
        }
    }
    SD_HIP(hipStreamSynchronize(s));
    if (osem_used) *osem_used = osem;
    if (min_overlap) *min_overlap = mn;
    if (avg_overlap) *avg_overlap = av;
}

void fuse_weighted_average(int nviews, const spim_view_source* views, const spim_fusion_params* p,
                           const float* borders, const float* ranges, float* out) {
    SD_CHECK(nviews >= 1 && views && p && out, SPIMDECON_ERR_ARG, "null argument");
    SD_CHECK(!p->use_blending || (borders && ranges), SPIMDECON_ERR_ARG, "blending needs borders and ranges");
    SD_CHECK(p->bb_dims[0] >= 1 && p->bb_dims[1] >= 1 && p->bb_dims[2] >= 1, SPIMDECON_ERR_ARG, "bad bounding box");
    SD_CHECK(p->interpolation == 0 || p->interpolation == 1, SPIMDECON_ERR_ARG, "interpolation must be 0 or 1");
    check_device(p->device);
    DeviceGuard guard(p->device);
    hipStream_t s;
    SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct SG {
        hipStream_t s;
        ~SG() { (void)hipStreamDestroy(s); }
    } sg{s};
    const int64_t nx = p->bb_dims[0], ny = p->bb_dims[1], nz = p->bb_dims[2];
    const int64_t n = nx * ny * nz;
    const std::vector<double> lut = blending_lut();
    DBuf<double> dlut(lut.size());
    SD_HIP(hipMemcpyAsync(dlut.p, lut.data(), lut.size() * 8, hipMemcpyHostToDevice, s));
    std::vector<DBuf<float>> srcs(nviews);
    std::vector<FuseView> fv(nviews);
    for (int v = 0; v < nviews; ++v) {
        const spim_view_source& vs = views[v];
        SD_CHECK(vs.img && vs.dims[0] >= 1 && vs.dims[1] >= 1 && vs.dims[2] >= 1 && vs.dims[0] < (1 << 30) &&
                     vs.dims[1] < (1 << 30) && vs.dims[2] < (1 << 30),
                 SPIMDECON_ERR_ARG, "bad view source");
        const int64_t sn = vs.dims[0] * vs.dims[1] * vs.dims[2];
        if (p->src_on_device) {
            fv[v].src = vs.img;
        } else {
            srcs[v].alloc(sn);
            SD_HIP(hipMemcpyAsync(srcs[v].p, vs.img, sn * 4, hipMemcpyHostToDevice, s));
            fv[v].src = srcs[v].p;
        }
        fv[v].sx = int(vs.dims[0]);
        fv[v].sy = int(vs.dims[1]);
        fv[v].sz = int(vs.dims[2]);
        const AffineInv a = invert_model(vs.model);
        std::memcpy(fv[v].inv, a.inv, sizeof(a.inv));
        std::memcpy(fv[v].tr, a.tr, sizeof(a.tr));
        for (int d = 0; d < 3; ++d) {
            fv[v].border[d] = borders ? borders[3 * v + d] : 0.0f;
            fv[v].range[d] = ranges ? ranges[3 * v + d] : 1.0f;
        }
    }
    DBuf<FuseView> dfv(nviews);
    SD_HIP(hipMemcpyAsync(dfv.p, fv.data(), nviews * sizeof(FuseView), hipMemcpyHostToDevice, s));
    DBuf<float> dout;
    float* o = out;
    if (!p->out_on_device) {
        dout.alloc(n);
        o = dout.p;
    }
    static_assert(kIpBlock == kTileX * kTileZ, "one tile per block");
    SD_CHECK(tiled_blocks(nx, ny, nz) < (int64_t(1) << 31), SPIMDECON_ERR_ARG, "bounding box too large");
    hipLaunchKernelGGL(k_fuse, dim3(unsigned(tiled_blocks(nx, ny, n / (nx * ny)))), dim3(kIpBlock), 0, s, dfv.p,
                       nviews, p->bb_min[0], p->bb_min[1], p->bb_min[2], nx, ny, n, p->downsampling,
                       p->interpolation, p->use_blending ? 1 : 0, dlut.p, o);
    SD_HIP(hipGetLastError());
    if (!p->out_on_device) SD_HIP(hipMemcpyAsync(out, o, n * 4, hipMemcpyDeviceToHost, s));
    SD_HIP(hipStreamSynchronize(s));
}

}  // namespace spimdecon

using namespace spimdecon;

extern "C" void spim_fusion_params_default(spim_fusion_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->downsampling = 1.0f;
    p->interpolation = 1;  // Fusion.defaultInterpolation (linear)
    p->use_blending = 1;   // Fusion.defaultUseBlending
    p->device = 0;
}

extern "C" int spim_fuse_weighted_average(int nviews, const spim_view_source* views, const spim_fusion_params* p,
                                          const float* blending_borders, const float* blending_ranges,
                                          float* out) {
    return guarded([&] { fuse_weighted_average(nviews, views, p, blending_borders, blending_ranges, out); });
}

extern "C" void spim_input_params_default(spim_input_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    for (int d = 0; d < 3; ++d) {
        p->blending_border[d] = -8.0f;  // EfficientBayesianBased.java:75-76 (range 12, border -8)
        p->blending_range[d] = 12.0f;
    }
    p->weight_type = SPIM_WEIGHTS_VIRTUAL;
    p->osem_index = 0;
    p->osem_speedup = 1.0;
    p->ij_threads = 8;
    p->device = 0;
}

extern "C" int spim_prepare_inputs(int nviews, const spim_view_source* views, const spim_input_params* p,
                                   float* const* img_out, float* const* weight_out, double* osem_used,
                                   int* min_overlap, double* avg_overlap) {
    return guarded([&] {
        prepare_inputs(nviews, views, p, img_out, weight_out, osem_used, min_overlap, avg_overlap);
    });
}
