// psf.hip -- PSF extraction and transformation on the GPU.
//
// Restates spim/process/fusion/deconvolution/ExtractPSF.java (paths under
// /root/reference/src/main/java/):
//   extractPSFLocal              :383-422  (n-linear over extendPeriodic, summed per bead)
//   normalize                    :281-299  ((v - min) / (max - min) in double)
//   transformPSF + transform     :309-346, :424-460 (odd size, centre kept, extendZero)
//   computeAverageTransformedPSF :164-208  (point-mirrored sum into the max size)
//   computeMaxProjection         :110-162
// One thread per output voxel; PSFs are small (10^4-10^6 voxels), the source
// stack is read through L2 by the bead loop.  The oracle is oracle/psf_ref.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include <memory>

#include "common.hpp"
#include "resample.hpp"
#include "spimdecon.h"

namespace spimdecon {

namespace {

constexpr int kPsfBlock = 256;

struct Dim3 {
    int x, y, z;
    __host__ __device__ int64_t n() const { return int64_t(x) * y * z; }
};

// Two-phase extractPSFLocal for many beads: every (bead, voxel) sample of a bead
// chunk in parallel, then each voxel's float sum over the chunk in bead order (the
// reference's order, so the result is bit-identical to the one-thread-per-voxel loop,
// which left all but a few dozen CUs idle: 57 ms for 67k beads of a 768^3 view).
// grid (voxel blocks of kPsfSpt * kPsfBlock, beads): the bead from blockIdx.y, 32-bit voxel
// coordinates (the flat 64-bit index's divisions were ~100-instruction software routines).
// The sample at integer offset k from a bead at position c is the trilinear interpolation at
// p = k + c (double).  Whenever that sum is exact -- always, unless |p| rises into the next
// binade of |c| -- floor(p) = floor(c) + k and p - floor(p) = c - floor(c): the eight corner
// weights are the bead's, computed once per thread for its kPsfSpt voxels; an inexact sum
// (checked: (p - k) != c) takes nlinear_at itself.  The same operations on the same values
// either way: bit-identical to nlinear_at per voxel.
constexpr int kPsfSpt = 8;   // voxels per thread
__global__ __launch_bounds__(kPsfBlock) void k_psf_samples(const float* __restrict__ img, Dim3 s,
                                                           const double* __restrict__ locs, int64_t nb, Dim3 p,
                                                           float* __restrict__ samp) {
    const uint32_t np = uint32_t(p.n());
    const uint32_t l = blockIdx.y;
    if (int64_t(l) >= nb) return;
    const double c0 = locs[3 * l], c1 = locs[3 * l + 1], c2 = locs[3 * l + 2];
    const double f0 = floor(c0), f1 = floor(c1), f2 = floor(c2);
    const double w0 = c0 - f0, w1 = c1 - f1, w2 = c2 - f2;
    const double i0 = 1.0 - w0, i1 = 1.0 - w1, i2 = 1.0 - w2;
    // corner order of nlinear_at: 000, 100, 110, 010, 011, 111, 101, 001
    const double W[8] = {i0 * i1 * i2, w0 * i1 * i2, w0 * w1 * i2, i0 * w1 * i2,
                         i0 * w1 * w2, w0 * w1 * w2, w0 * i1 * w2, i0 * i1 * w2};
    const int b0 = int(f0), b1 = int(f1), b2 = int(f2);
    const uint32_t px = uint32_t(p.x), pxy = uint32_t(p.x) * uint32_t(p.y);
    const int64_t py = s.x, pz = int64_t(s.x) * s.y;
    for (int v = 0; v < kPsfSpt; ++v) {
        const uint32_t i = (blockIdx.x * kPsfSpt + uint32_t(v)) * kPsfBlock + threadIdx.x;
        if (i >= np) break;
        const int z = int(i / pxy), r = int(i - uint32_t(z) * pxy);
        const int y = r / int(px), x = r - y * int(px);
        const double k0 = double(x - p.x / 2), k1 = double(y - p.y / 2), k2 = double(z - p.z / 2);
        const double q0 = k0 + c0, q1 = k1 + c1, q2 = k2 + c2;
        const int xa = b0 + (x - p.x / 2), ya = b1 + (y - p.y / 2), za = b2 + (z - p.z / 2);
        float out;
        if (q0 - k0 == c0 && q1 - k1 == c1 && q2 - k2 == c2 && xa >= 0 && ya >= 0 && za >= 0 && xa + 1 < s.x &&
            ya + 1 < s.y && za + 1 < s.z) {
            const float* bp = img + (int64_t(za) * s.y + ya) * s.x + xa;
            float acc = float(double(bp[0]) * W[0]);
            acc = acc + float(double(bp[1]) * W[1]);
            acc = acc + float(double(bp[py + 1]) * W[2]);
            acc = acc + float(double(bp[py]) * W[3]);
            acc = acc + float(double(bp[pz + py]) * W[4]);
            acc = acc + float(double(bp[pz + py + 1]) * W[5]);
            acc = acc + float(double(bp[pz + 1]) * W[6]);
            acc = acc + float(double(bp[pz]) * W[7]);
            out = acc;
        } else {
            out = nlinear_at<kExtPeriodic>(img, s.x, s.y, s.z, q0, q1, q2);
        }
        samp[int64_t(l) * np + i] = out;
    }
}

__global__ __launch_bounds__(kPsfBlock) void k_psf_accumulate(const float* __restrict__ samp, int64_t nb,
                                                              int64_t np, float* __restrict__ acc) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    if (i >= np) return;
    float a = acc[i];
    int64_t l = 0;
    // 32 loads ahead, adds in bead order (with 8 the ~9k chains of a view waited on one HBM
    // round trip per 8 beads)
    constexpr int U = 32;
    for (; l + U <= nb; l += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = samp[(l + u) * np + i];
#pragma unroll
        for (int u = 0; u < U; ++u) a = a + v[u];
    }
    for (; l < nb; ++l) a = a + samp[l * np + i];
    acc[i] = a;
}

__global__ __launch_bounds__(kPsfBlock) void k_psf_extract(const float* __restrict__ img, Dim3 s,
                                                           const double* __restrict__ locs, int64_t nloc, Dim3 p,
                                                           float* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    if (i >= p.n()) return;
    const int x = int(i % p.x), y = int((i / p.x) % p.y), z = int(i / (int64_t(p.x) * p.y));
    const double r0 = double(x - p.x / 2), r1 = double(y - p.y / 2), r2 = double(z - p.z / 2);
    float acc = 0.0f;
    for (int64_t l = 0; l < nloc; ++l)
        acc = acc + nlinear_at<kExtPeriodic>(img, s.x, s.y, s.z, r0 + locs[3 * l], r1 + locs[3 * l + 1],
                                             r2 + locs[3 * l + 2]);
    out[i] = acc;
}

// single-block min/max (the PSF is small); NaN never wins a comparison, as in Java
__global__ __launch_bounds__(1024) void k_psf_minmax(const float* __restrict__ v, int64_t n,
                                                     double* __restrict__ mm) {
    __shared__ double smin[1024], smax[1024];
    double lo = DBL_MAX, hi = -DBL_MAX;
    for (int64_t i = threadIdx.x; i < n; i += 1024) {
        const double a = v[i];
        if (a < lo) lo = a;
        if (a > hi) hi = a;
    }
    smin[threadIdx.x] = lo;
    smax[threadIdx.x] = hi;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (int(threadIdx.x) < w) {
            smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + w]);
            smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        mm[0] = smin[0];
        mm[1] = smax[0];
    }
}

__global__ __launch_bounds__(kPsfBlock) void k_psf_normalize(float* __restrict__ v, int64_t n,
                                                             const double* __restrict__ mm) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    if (i >= n) return;
    v[i] = float((double(v[i]) - mm[0]) / (mm[1] - mm[0]));
}

struct Inv12 {
    double m[12];
};

__global__ __launch_bounds__(kPsfBlock) void k_psf_transform(const float* __restrict__ psf, Dim3 s, Inv12 f,
                                                             double o0, double o1, double o2, Dim3 t,
                                                             float* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    if (i >= t.n()) return;
    const int x = int(i % t.x), y = int((i / t.x) % t.y), z = int(i / (int64_t(t.x) * t.y));
    const double a = x + o0, b = y + o1, c = z + o2;
    const double q0 = a * f.m[0] + b * f.m[1] + c * f.m[2] + f.m[3];
    const double q1 = a * f.m[4] + b * f.m[5] + c * f.m[6] + f.m[7];
    const double q2 = a * f.m[8] + b * f.m[9] + c * f.m[10] + f.m[11];
    out[i] = nlinear_at<kExtZero>(psf, s.x, s.y, s.z, q0, q1, q2);
}

struct PsfRef {
    const float* p;
    Dim3 d;
};

__global__ __launch_bounds__(kPsfBlock) void k_psf_average(const PsfRef* __restrict__ psfs, int npsf, Dim3 m,
                                                           float* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    if (i >= m.n()) return;
    const int x = int(i % m.x), y = int((i / m.x) % m.y), z = int(i / (int64_t(m.x) * m.y));
    float acc = 0.0f;
    for (int k = 0; k < npsf; ++k) {
        const Dim3 d = psfs[k].d;
        // avg(psfCenter - loc + avgCenter) += psf(loc)
        const int lx = d.x / 2 + m.x / 2 - x, ly = d.y / 2 + m.y / 2 - y, lz = d.z / 2 + m.z / 2 - z;
        if (lx < 0 || ly < 0 || lz < 0 || lx >= d.x || ly >= d.y || lz >= d.z) continue;
        acc = acc + psfs[k].p[(int64_t(lz) * d.y + ly) * d.x + lx];
    }
    out[i] = acc;
}

__global__ __launch_bounds__(kPsfBlock) void k_max_projection(const float* __restrict__ img, Dim3 s, int dim,
                                                              float* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * kPsfBlock + threadIdx.x;
    const int n0 = dim == 0 ? s.y : s.x, n1 = dim == 2 ? s.y : s.z;
    if (i >= int64_t(n0) * n1) return;
    const int a = int(i % n0), b = int(i / n0);
    int x, y, z, len;
    int64_t stride;
    if (dim == 0) { x = 0; y = a; z = b; len = s.x; stride = 1; }
    else if (dim == 1) { x = a; y = 0; z = b; len = s.y; stride = s.x; }
    else { x = a; y = b; z = 0; len = s.z; stride = int64_t(s.x) * s.y; }
    const float* q = img + (int64_t(z) * s.y + y) * s.x + x;
    double mx = -DBL_MAX;
    for (int k = 0; k < len; ++k) {
        const double v = q[k * stride];
        if (v > mx) mx = v;
    }
    out[i] = float(mx);
}

Dim3 dim3_of(const int64_t* d, const char* what) {
    SD_CHECK(d, SPIMDECON_ERR_ARG, std::string(what) + ": null dims");
    for (int k = 0; k < 3; ++k)
        SD_CHECK(d[k] >= 1 && d[k] < (int64_t(1) << 30), SPIMDECON_ERR_ARG, std::string(what) + ": bad dims");
    return Dim3{int(d[0]), int(d[1]), int(d[2])};
}

unsigned grid_for(int64_t n) { return unsigned(ceil_div(n, int64_t(kPsfBlock))); }

struct Stream {
    hipStream_t s{};
    Stream() { SD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
    ~Stream() { (void)hipStreamDestroy(s); }
};

// transformPSF (:309-346): odd size that holds the transformed box, and the
// offset keeping model(dim / 2) at the centre voxel
void transformed_size(const int64_t size[3], const double* m, int64_t out[3], double off[3]) {
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int c = 0; c < 8; ++c) {
        const double p[3] = {(c & 1) ? double(size[0] - 1) : 0.0, (c & 2) ? double(size[1] - 1) : 0.0,
                             (c & 4) ? double(size[2] - 1) : 0.0};
        for (int r = 0; r < 3; ++r) {
            const double t = p[0] * m[4 * r] + p[1] * m[4 * r + 1] + p[2] * m[4 * r + 2] + m[4 * r + 3];
            lo[r] = std::min(lo[r], t);
            hi[r] = std::max(hi[r], t);
        }
    }
    const double c[3] = {double(size[0] / 2), double(size[1] / 2), double(size[2] / 2)};
    for (int r = 0; r < 3; ++r) {
        int64_t n = int64_t(hi[r] - lo[r]) + 1;
        if (n % 2 == 0) ++n;
        out[r] = n;
        const double t = c[0] * m[4 * r] + c[1] * m[4 * r + 1] + c[2] * m[4 * r + 2] + m[4 * r + 3];
        off[r] = t - double(n / 2);
    }
}

void launch_transform(const float* dpsf, Dim3 s, const double* model, float* dout, Dim3& t, hipStream_t st) {
    int64_t size[3] = {s.x, s.y, s.z}, ts[3];
    double off[3];
    transformed_size(size, model, ts, off);
    t = dim3_of(ts, "transformed psf");
    const AffineInv a = invert_model(model);
    Inv12 f;
    std::memcpy(f.m, a.full, sizeof(f.m));
    hipLaunchKernelGGL(k_psf_transform, dim3(grid_for(t.n())), dim3(kPsfBlock), 0, st, dpsf, s, f, off[0], off[1],
                       off[2], t, dout);
    SD_HIP(hipGetLastError());
}

}  // namespace

void psf_transformed_size(const int64_t* psf_size, const double* model, int64_t* out_size, double* offset) {
    SD_CHECK(model && out_size, SPIMDECON_ERR_ARG, "null argument");
    dim3_of(psf_size, "psf");
    double off[3];
    transformed_size(psf_size, model, out_size, off);
    (void)invert_model(model);
    if (offset) std::memcpy(offset, off, sizeof(off));
}

void transform_psf(const float* psf, const int64_t* psf_size, const double* model, float* out, int device) {
    SD_CHECK(psf && model && out, SPIMDECON_ERR_ARG, "null argument");
    const Dim3 s = dim3_of(psf_size, "psf");
    check_device(device);
    DeviceGuard guard(device);
    Stream st;
    DBuf<float> dp(s.n());
    SD_HIP(hipMemcpyAsync(dp.p, psf, s.n() * 4, hipMemcpyHostToDevice, st.s));
    int64_t ts[3];
    double off[3];
    transformed_size(psf_size, model, ts, off);
    DBuf<float> dt(dim3_of(ts, "transformed psf").n());
    Dim3 t;
    launch_transform(dp.p, s, model, dt.p, t, st.s);
    SD_HIP(hipMemcpyAsync(out, dt.p, t.n() * 4, hipMemcpyDeviceToHost, st.s));
    SD_HIP(hipStreamSynchronize(st.s));
}

namespace {
// One view's device buffers and stream, kept across calls (per device; the pool is never
// destroyed: no destructor racing the HIP runtime's teardown at exit).  Fresh buffers and
// streams per call cost a hipMalloc / hipFree (which synchronises the device) per buffer
// and view: the C4 pipeline's PSF stage spent most of its time there.
struct PsfWork {
    Stream st;
    DBuf<float> dimg, dpsf, samp, dt;
    DBuf<double> dloc, mm;
};
template <typename T>
void ensure(DBuf<T>& b, size_t n) {
    if (b.n < n) b.alloc(n);
}
struct PsfPool {
    std::mutex mu;   // one extract call at a time per device
    std::vector<std::unique_ptr<PsfWork>> w;
};
std::mutex g_psf_pool_mu;
std::map<int, std::unique_ptr<PsfPool>>& g_psf_pool = *new std::map<int, std::unique_ptr<PsfPool>>();
PsfPool& psf_pool(int dev) {
    std::lock_guard<std::mutex> lk(g_psf_pool_mu);
    auto& p = g_psf_pool[dev];
    if (!p) p.reset(new PsfPool());
    return *p;
}
}  // namespace

// One view's ExtractPSF.extract (:281-299) + transformPSF, in three steps so several
// views can run concurrently (extract_psfs): the per-voxel sum over the beads is a
// serial float chain in bead order (bit-exact with the reference), so one view offers
// only psf_size (~9k) parallel chains; eight views on eight streams fill 8x more.
struct PsfJob {
    const float* img = nullptr;
    Dim3 s{}, p{};
    const double* model = nullptr;
    int64_t nloc = 0;
    float* psf_original = nullptr;
    float* psf_transformed = nullptr;
    int64_t psf_size[3] = {0, 0, 0};
    PsfWork& w;
    const float* src = nullptr;
    int64_t chunk = 0;
    int64_t tn = 0;   // transformed PSF voxels

    PsfJob(PsfWork& w_, const float* img_, const int64_t* dims, int img_on_device, const double* locations,
           int64_t nloc_, const int64_t* psf_size_, const double* model_, float* orig, float* trans)
        : img(img_), model(model_), nloc(nloc_), psf_original(orig), psf_transformed(trans), w(w_) {
        SD_CHECK(img && psf_original && nloc >= 0 && (nloc == 0 || locations), SPIMDECON_ERR_ARG, "null argument");
        SD_CHECK(!psf_transformed || model, SPIMDECON_ERR_ARG, "a transformed PSF needs the view model");
        s = dim3_of(dims, "image");
        p = dim3_of(psf_size_, "psf");
        std::memcpy(psf_size, psf_size_, sizeof(psf_size));
        // buffers (grown, reused) and uploads (asynchronous on this job's stream)
        src = img;
        if (!img_on_device) {
            ensure(w.dimg, s.n());
            SD_HIP(hipMemcpyAsync(w.dimg.p, img, s.n() * 4, hipMemcpyHostToDevice, w.st.s));
            src = w.dimg.p;
        }
        ensure(w.dloc, size_t(std::max<int64_t>(nloc, 1)) * 3);
        if (nloc) SD_HIP(hipMemcpyAsync(w.dloc.p, locations, nloc * 24, hipMemcpyHostToDevice, w.st.s));
        ensure(w.dpsf, p.n());
        ensure(w.mm, 2);
        if (nloc > 64) {   // bead chunks of <= 2^26 samples (256 MB), <= 65535 beads (grid.y)
            SD_CHECK(p.n() < (int64_t(1) << 31), SPIMDECON_ERR_ARG, "psf too large");
            chunk = std::max<int64_t>(1, std::min<int64_t>({nloc, (int64_t(1) << 26) / p.n(), int64_t(65535)}));
            ensure(w.samp, size_t(chunk * p.n()));
        }
        if (psf_transformed) {
            int64_t ts[3];
            double off[3];
            transformed_size(psf_size, model, ts, off);
            tn = dim3_of(ts, "transformed psf").n();
            ensure(w.dt, size_t(tn));
        }
    }

    void launch() {
        const hipStream_t st = w.st.s;
        if (nloc <= 64) {
            hipLaunchKernelGGL(k_psf_extract, dim3(grid_for(p.n())), dim3(kPsfBlock), 0, st, src, s, w.dloc.p, nloc,
                               p, w.dpsf.p);
        } else {
            SD_HIP(hipMemsetAsync(w.dpsf.p, 0, p.n() * 4, st));
            for (int64_t l0 = 0; l0 < nloc; l0 += chunk) {
                const int64_t nb = std::min(chunk, nloc - l0);
                hipLaunchKernelGGL(k_psf_samples, dim3(unsigned(ceil_div(p.n(), int64_t(kPsfBlock) * kPsfSpt)),
                                                       unsigned(nb)),
                                   dim3(kPsfBlock), 0, st, src, s, w.dloc.p + 3 * l0, nb, p, w.samp.p);
                hipLaunchKernelGGL(k_psf_accumulate, dim3(grid_for(p.n())), dim3(kPsfBlock), 0, st, w.samp.p, nb,
                                   p.n(), w.dpsf.p);
            }
        }
        SD_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_psf_minmax, dim3(1), dim3(1024), 0, st, w.dpsf.p, p.n(), w.mm.p);
        SD_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_psf_normalize, dim3(grid_for(p.n())), dim3(kPsfBlock), 0, st, w.dpsf.p, p.n(), w.mm.p);
        SD_HIP(hipGetLastError());
        if (psf_transformed) {
            Dim3 t;
            launch_transform(w.dpsf.p, p, model, w.dt.p, t, st);
        }
    }

    // the copies out only now: a copy into pageable host memory blocks the host until
    // the stream has drained, which would serialise the views' launches
    void finish() {
        SD_HIP(hipMemcpyAsync(psf_original, w.dpsf.p, p.n() * 4, hipMemcpyDefault, w.st.s));
        if (psf_transformed) SD_HIP(hipMemcpyAsync(psf_transformed, w.dt.p, size_t(tn) * 4, hipMemcpyDefault, w.st.s));
        SD_HIP(hipStreamSynchronize(w.st.s));
    }
};

void extract_psf(const float* img, const int64_t* dims, int img_on_device, const double* locations, int64_t nloc,
                 const int64_t* psf_size, const double* model, float* psf_original, float* psf_transformed,
                 int device) {
    check_device(device);
    DeviceGuard guard(device);
    PsfPool& pool = psf_pool(device);
    std::lock_guard<std::mutex> lk(pool.mu);
    if (pool.w.empty()) pool.w.emplace_back(new PsfWork());
    PsfJob job(*pool.w[0], img, dims, img_on_device, locations, nloc, psf_size, model, psf_original, psf_transformed);
    job.launch();
    job.finish();
}

void extract_psfs(int nviews, const float* const* imgs, const int64_t* dims, int img_on_device,
                  const double* const* locations, const int64_t* nlocations, const int64_t* psf_size,
                  const double* models, float* const* psf_original, float* const* psf_transformed, int device) {
    SD_CHECK(nviews >= 0 && (nviews == 0 || (imgs && dims && locations && nlocations && psf_original)),
             SPIMDECON_ERR_ARG, "null argument");
    check_device(device);
    DeviceGuard guard(device);
    PsfPool& pool = psf_pool(device);
    std::lock_guard<std::mutex> lk(pool.mu);
    while (int(pool.w.size()) < nviews) pool.w.emplace_back(new PsfWork());
    std::vector<std::unique_ptr<PsfJob>> jobs;
    jobs.reserve(size_t(nviews));
    for (int v = 0; v < nviews; ++v)
        jobs.emplace_back(new PsfJob(*pool.w[size_t(v)], imgs[v], dims + 3 * v, img_on_device, locations[v],
                                     nlocations[v], psf_size, models ? models + 12 * v : nullptr, psf_original[v],
                                     psf_transformed ? psf_transformed[v] : nullptr));
    for (auto& j : jobs) j->launch();
    for (auto& j : jobs) j->finish();
}

void average_transformed_psf(int npsf, const float* const* psfs, const int64_t* psf_dims, float* avg,
                             int64_t* avg_dims, int device) {
    SD_CHECK(npsf >= 1 && psfs && psf_dims && avg_dims, SPIMDECON_ERR_ARG, "null argument");
    std::vector<Dim3> d(npsf);
    int64_t m[3] = {0, 0, 0};
    for (int k = 0; k < npsf; ++k) {
        d[k] = dim3_of(psf_dims + 3 * k, "psf");
        m[0] = std::max<int64_t>(m[0], d[k].x);
        m[1] = std::max<int64_t>(m[1], d[k].y);
        m[2] = std::max<int64_t>(m[2], d[k].z);
    }
    std::memcpy(avg_dims, m, sizeof(m));
    if (!avg) return;
    const Dim3 md = dim3_of(m, "average psf");
    check_device(device);
    DeviceGuard guard(device);
    Stream st;
    std::vector<DBuf<float>> dp(npsf);
    std::vector<PsfRef> refs(npsf);
    for (int k = 0; k < npsf; ++k) {
        SD_CHECK(psfs[k], SPIMDECON_ERR_ARG, "null psf");
        dp[k].alloc(d[k].n());
        SD_HIP(hipMemcpyAsync(dp[k].p, psfs[k], d[k].n() * 4, hipMemcpyHostToDevice, st.s));
        refs[k] = PsfRef{dp[k].p, d[k]};
    }
    DBuf<PsfRef> drefs(npsf);
    SD_HIP(hipMemcpyAsync(drefs.p, refs.data(), npsf * sizeof(PsfRef), hipMemcpyHostToDevice, st.s));
    DBuf<float> dout(md.n());
    hipLaunchKernelGGL(k_psf_average, dim3(grid_for(md.n())), dim3(kPsfBlock), 0, st.s, drefs.p, npsf, md, dout.p);
    SD_HIP(hipGetLastError());
    SD_HIP(hipMemcpyAsync(avg, dout.p, md.n() * 4, hipMemcpyDeviceToHost, st.s));
    SD_HIP(hipStreamSynchronize(st.s));
}

void max_projection(const float* img, const int64_t* dims, int min_dim, float* out, int64_t* out_dims, int* used_dim,
                    int device) {
    SD_CHECK(out_dims, SPIMDECON_ERR_ARG, "null argument");
    const Dim3 s = dim3_of(dims, "image");
    SD_CHECK(min_dim < 3, SPIMDECON_ERR_ARG, "min_dim must be < 3");
    if (min_dim < 0) {  // the first smallest dimension (:116-128)
        min_dim = 0;
        for (int k = 0; k < 3; ++k)
            if (dims[k] < dims[min_dim]) min_dim = k;
    }
    int j = 0;
    for (int k = 0; k < 3; ++k)
        if (k != min_dim) out_dims[j++] = dims[k];
    if (used_dim) *used_dim = min_dim;
    if (!out) return;
    SD_CHECK(img, SPIMDECON_ERR_ARG, "null image");
    check_device(device);
    DeviceGuard guard(device);
    Stream st;
    DBuf<float> di(s.n());
    SD_HIP(hipMemcpyAsync(di.p, img, s.n() * 4, hipMemcpyHostToDevice, st.s));
    const int64_t no = out_dims[0] * out_dims[1];
    DBuf<float> dout(no);
    hipLaunchKernelGGL(k_max_projection, dim3(grid_for(no)), dim3(kPsfBlock), 0, st.s, di.p, s, min_dim, dout.p);
    SD_HIP(hipGetLastError());
    SD_HIP(hipMemcpyAsync(out, dout.p, no * 4, hipMemcpyDeviceToHost, st.s));
    SD_HIP(hipStreamSynchronize(st.s));
}

}  // namespace spimdecon

using namespace spimdecon;

extern "C" int spim_psf_transformed_size(const int64_t psf_size[3], const double model[12], int64_t out_size[3],
                                         double offset[3]) {
    return guarded([&] { psf_transformed_size(psf_size, model, out_size, offset); });
}

extern "C" int spim_transform_psf(const float* psf, const int64_t psf_size[3], const double model[12], float* out,
                                  int device) {
    return guarded([&] { transform_psf(psf, psf_size, model, out, device); });
}

extern "C" int spim_extract_psf(const float* img, const int64_t dims[3], int img_on_device, const double* locations,
                                int64_t nlocations, const int64_t psf_size[3], const double model[12],
                                float* psf_original, float* psf_transformed, int device) {
    return guarded([&] {
        extract_psf(img, dims, img_on_device, locations, nlocations, psf_size, model, psf_original, psf_transformed,
                    device);
    });
}

extern "C" int spim_extract_psfs(int nviews, const float* const* imgs, const int64_t* dims, int img_on_device,
                                 const double* const* locations, const int64_t* nlocations,
                                 const int64_t psf_size[3], const double* models, float* const* psf_original,
                                 float* const* psf_transformed, int device) {
    return guarded([&] {
        extract_psfs(nviews, imgs, dims, img_on_device, locations, nlocations, psf_size, models, psf_original,
                     psf_transformed, device);
    });
}

// frees the per-view buffers and streams extract_psf(s) keep on a device (-1: every device)
void psf_release_workspace(int device) {
    std::lock_guard<std::mutex> lk(g_psf_pool_mu);
    for (auto& kv : g_psf_pool) {
        if (device >= 0 && kv.first != device) continue;
        if (!kv.second) continue;
        std::lock_guard<std::mutex> lp(kv.second->mu);   // (no extract call in flight)
        DeviceGuard guard(kv.first);
        for (auto& w : kv.second->w) SD_HIP(hipStreamSynchronize(w->st.s));
        kv.second->w.clear();
    }
}

extern "C" int spim_psf_release_workspace(int device) {
    return guarded([&] { psf_release_workspace(device); });
}

extern "C" int spim_average_transformed_psf(int npsfs, const float* const* psfs, const int64_t* psf_dims,
                                            float* avg, int64_t avg_dims[3], int device) {
    return guarded([&] { average_transformed_psf(npsfs, psfs, psf_dims, avg, avg_dims, device); });
}

extern "C" int spim_max_projection(const float* img, const int64_t dims[3], int min_dim, float* out,
                                   int64_t out_dims[2], int* used_dim, int device) {
    return guarded([&] { max_projection(img, dims, min_dim, out, out_dims, used_dim, device); });
}
