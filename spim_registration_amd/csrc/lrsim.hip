// lrsim.hip -- the legacy simultaneous-update multiview Lucy-Richardson rule (opt-in),
// with the views sharded over RCCL ranks and one all-reduce of the compound correction
// per iteration (the north star's "RCCL all-reduce over xGMI of the
// compound correction image").
//
// Reference (paths under /root/reference/src/main/java/):
//   mpicbg/spim/postprocessing/deconvolution/LucyRichardsonMultiViewDeconvolution.java
//     :24-60   normImage of every kernel        (LRMV below)
//     :62-85   psi = (float) normAllImages(...)  (:360-457)
//     :98-178  per view: blurred = conv(psi, K); q = img / blurred; contribution = conv(q, K)
//              -- the views of one iteration all read the same psi, and the reference
//              hands them to threads by view % numThreads == myNumber (:127-128); here to
//              ranks by view % nranks == rank
//     :201-270 per voxel: value = prod pow(c, w) or sum c * w over views with w > 0, num =
//              sum w; psi * pow(value, 1 / num) or psi * value / num; minValue if num == 0
//     :290-330 Tikhonov, the NaN / minValue clamp, sum and max of |change|
// Not MVDeconvolution's sequential rule (session.cpp): each view's correction here is
// computed from the same psi, so the per-voxel merge is associative over ranks -- a sum
// (additive) or a product (multiplicative) all-reduce of one double per voxel.
//
// Per rank and iteration (full psi replica on every rank; n voxels, M padded reals):
//   pad psi (mirror) -> R2C, once for all views of the rank
//   per owned view: spectrum * K -> C2R -> img / blurred, mirror-padded -> R2C -> * K -> C2R
//                   -> value (double per voxel) *= pow(c, w)  or  += c * w
//   ncclAllReduce(value, prod | sum)  (num, the sum of the weights, is reduced once at init)
//   psi = rule(psi, value, num), Tikhonov, clamp; {sum, max} |change| (identical on all ranks)
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "fft.hpp"
#include "rl_kernels.hpp"
#include "rl_math.hpp"

namespace spimdecon {

#define SD_NCCL_LR(expr)                                                                         \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess)                                                                   \
            ::spimdecon::fail(SPIMDECON_ERR_COMM, std::string(#expr " failed: ") + ncclGetErrorString(_r)); \
    } while (0)

namespace {

constexpr int kB = 256;
constexpr int kW = kB / 64;
constexpr double kLrMin = 0.0001;   // LRMV:30 (double)

inline unsigned grid_of(int64_t work, int64_t per_block, int64_t cap = 256 * 16) {
    int64_t b = ceil_div(work, per_block);
    return unsigned(std::max<int64_t>(1, std::min(b, cap)));
}

// The exact sum of the values rounded once to double: BigDecimal.add over (double) t,
// then doubleValue() (LRMV:460-475).  Shewchuk's non-overlapping partials with the
// half-way correction of the final rounding (the algorithm of Python's math.fsum).
double exact_sum(const float* v, int64_t n) {
    std::vector<double> p;
    for (int64_t k = 0; k < n; ++k) {
        double x = double(v[k]);
        size_t i = 0;
        for (double y : p) {
            if (std::fabs(x) < std::fabs(y)) std::swap(x, y);
            const double hi = x + y;
            const double lo = y - (hi - x);
            if (lo != 0.0) p[i++] = lo;
            x = hi;
        }
        p.resize(i);
        p.push_back(x);
    }
    if (p.empty()) return 0.0;
    size_t m = p.size();
    double hi = p[--m], lo = 0.0;
    while (m > 0) {
        const double x = hi, y = p[--m];
        hi = x + y;
        lo = y - (hi - x);
        if (lo != 0.0) break;
    }
    if (m > 0 && ((lo < 0.0 && p[m - 1] < 0.0) || (lo > 0.0 && p[m - 1] > 0.0))) {
        const double y = lo * 2.0, x = hi + y;
        if (y == x - hi) hi = x;
    }
    return hi;
}

// ---------------------------------------------------------------- kernels

// normAllImages, this rank's views (LRMV:382-407): s = sum of img over views with weight
// != 0 (double, view order), c = their count
__global__ __launch_bounds__(kB) void k_lr_overlap(int64_t n, int nv, const float* const* __restrict__ imgs,
                                                   const float* const* __restrict__ ws, double* __restrict__ s,
                                                   double* __restrict__ c) {
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB) {
        double a = 0.0, b = 0.0;
        for (int v = 0; v < nv; ++v)
            if (ws[v][i] != 0.0f) {
                a += (double)imgs[v][i];
                b += 1.0;
            }
        s[i] = a;
        c[i] = b;
    }
}

// block partials of {sum of s where c > 1, sum of c there} (LRMV:409-413)
__global__ __launch_bounds__(kB) void k_lr_avg_partials(int64_t n, const double* __restrict__ s,
                                                        const double* __restrict__ c, double* __restrict__ part) {
    __shared__ double sa[kW], sb[kW];
    double a = 0.0, b = 0.0;
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB)
        if (c[i] > 1.0) {
            a += s[i];
            b += c[i];
        }
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        sa[threadIdx.x >> 6] = a;
        sb[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kW; ++w) {
            a += sa[w];
            b += sb[w];
        }
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

// num = sum of the weights > 0 of this rank's views (LRMV:228-235), double
__global__ __launch_bounds__(kB) void k_lr_num(int64_t n, int nv, const float* const* __restrict__ ws,
                                               double* __restrict__ num) {
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB) {
        double a = 0.0;
        for (int v = 0; v < nv; ++v) {
            const float w = ws[v][i];
            if (w > 0.0f) a += (double)w;
        }
        num[i] = a;
    }
}

__global__ __launch_bounds__(kB) void k_lr_fill(double* __restrict__ p, int64_t n, double v) {
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB) p[i] = v;
}

// C = A * K over n2 complex pairs (+ one tail value): the psi spectrum stays intact for
// the rank's next view
__global__ __launch_bounds__(kB) void k_lr_cmul(const float4* __restrict__ A, const float4* __restrict__ K,
                                                float4* __restrict__ Cc, int64_t n2, const float2* __restrict__ At,
                                                const float2* __restrict__ Kt, float2* __restrict__ Ct, int tail) {
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n2; i += int64_t(gridDim.x) * kB) {
        const float4 a = A[i], k = K[i];
        float4 r;
        r.x = a.x * k.x - a.y * k.y;
        r.y = a.x * k.y + a.y * k.x;
        r.z = a.z * k.z - a.w * k.w;
        r.w = a.z * k.w + a.w * k.z;
        Cc[i] = r;
    }
    if (tail && blockIdx.x == 0 && threadIdx.x == 0) {
        const float2 a = *At, k = *Kt;
        *Ct = make_float2(a.x * k.x - a.y * k.y, a.x * k.y + a.y * k.x);
    }
}

__device__ __forceinline__ int64_t lr_src(int64_t q, int64_t n, int c, int64_t M) {
    return mirror_idx(q < n + c ? q : q - M, n);
}

// Rc = the mirror-extended quotient img / blurred over the whole padded volume (LRMV:146-154:
// a plain float division; FourierConvolution extends the quotient image like any other)
__global__ __launch_bounds__(kB) void k_lr_quot_pad(SlabGeom g, const float* __restrict__ img,
                                                    const float* __restrict__ Rb, float* __restrict__ Rc) {
    const int lane = threadIdx.x & 63;
    const int64_t rows = g.My * g.Mz;
    for (int64_t row = int64_t(blockIdx.x) * kW + (threadIdx.x >> 6); row < rows; row += int64_t(gridDim.x) * kW) {
        const int64_t qz = row / g.My, qy = row - qz * g.My;
        const int64_t lz = lr_src(qz, g.nz, g.cz, g.Mz), ly = lr_src(qy, g.ny, g.cy, g.My);
        const float* irow = img + (lz * g.ny + ly) * g.nx;
        const float* brow = Rb + (lz * g.My + ly) * g.Sx;   // interior slot of the source row
        float* dst = Rc + row * g.Sx;
        for (int64_t qx = lane; qx < g.Mx; qx += 64) {
            const int64_t lx = lr_src(qx, g.nx, g.cx, g.Mx);
            dst[qx] = __fdiv_rn(irow[lx], brow[lx]);
        }
    }
}

// value (double per voxel) merged with this view's contribution c (interior slots of Rc)
// where its weight is > 0: value *= pow(c, w) (multiplicative) or value += c * w (a float
// product, LRMV:227-235)
template <bool MULT>
__global__ __launch_bounds__(kB) void k_lr_accum(SlabGeom g, const float* __restrict__ Rc,
                                                 const float* __restrict__ w, double* __restrict__ value) {
    const int lane = threadIdx.x & 63;
    const int64_t rows = g.ny * g.nz;
    for (int64_t row = int64_t(blockIdx.x) * kW + (threadIdx.x >> 6); row < rows; row += int64_t(gridDim.x) * kW) {
        const int64_t z = row / g.ny, y = row - z * g.ny;
        const float* crow = Rc + (z * g.My + y) * g.Sx;
        const int64_t base = row * g.nx;
        for (int64_t x = lane; x < g.nx; x += 64) {
            const float wv = w[base + x];
            if (wv > 0.0f) {
                if constexpr (MULT)
                    value[base + x] *= pow((double)crow[x], (double)wv);
                else
                    value[base + x] += (double)__fmul_rn(crow[x], wv);
            }
        }
    }
}

// the new psi (LRMV:254-330) and block partials {sum |change|, max |change|}
template <bool MULT, bool TIK>
__global__ __launch_bounds__(kB) void k_lr_update(int64_t n, float* __restrict__ psi, const double* __restrict__ value,
                                                  const double* __restrict__ num, double lambda,
                                                  double* __restrict__ part) {
    __shared__ double ss[kW];
    __shared__ float sm[kW];
    double sum = 0.0;
    float mx = -1.0f;
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB) {
        const float last = psi[i];
        const double nm = num[i];
        double v;
        if (nm > 0.0) {
            if constexpr (MULT)
                v = (double)last * pow(value[i], 1.0 / nm);
            else
                v = (double)last * 1.0 * value[i] / nm;   // psi * nextPsi(= 1) * value / num
        } else {
            v = kLrMin;
        }
        float f = (float)v;
        if constexpr (TIK) f = (float)((sqrt(1.0 + 2.0 * lambda * (double)f) - 1.0) / lambda);
        const float next = isnan(f) ? (float)kLrMin : (float)fmax(kLrMin, (double)f);
        psi[i] = next;
        const float ch = fabsf(__fsub_rn(last, next));
        sum += (double)ch;
        mx = fmaxf(mx, ch);
    }
    for (int off = 32; off > 0; off >>= 1) {
        sum += __shfl_xor(sum, off, 64);
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        ss[threadIdx.x >> 6] = sum;
        sm[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kW; ++w) {
            sum += ss[w];
            mx = fmaxf(mx, sm[w]);
        }
        part[2 * blockIdx.x] = sum;
        part[2 * blockIdx.x + 1] = (double)mx;
    }
}

// sums of both halves of the block partials (fixed order: deterministic)
__global__ __launch_bounds__(1024) void k_lr_sum2(const double* __restrict__ part, int64_t nb, double* out) {
    __shared__ double sa[16], sb[16];
    double a = 0.0, b = 0.0;
    for (int64_t i = threadIdx.x; i < nb; i += 1024) {
        a += part[2 * i];
        b += part[2 * i + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        sa[threadIdx.x >> 6] = a;
        sb[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) {
            a += sa[w];
            b += sb[w];
        }
        out[0] = a;
        out[1] = b;
    }
}

// a = a + b, or a * b (mult): one device group's partial merged into group 0's
__global__ __launch_bounds__(kB) void k_lr_merge(double* __restrict__ a, const double* __restrict__ b, int64_t n,
                                                 int mult) {
    for (int64_t i = int64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += int64_t(gridDim.x) * kB)
        a[i] = mult ? a[i] * b[i] : a[i] + b[i];
}

}  // namespace

// ---------------------------------------------------------------- the session

struct LrView {
    int kd[3] = {0, 0, 0};         // {kx, ky, kz}
    int grp = -1;                  // device group holding the view (-1: another rank's view)
    std::vector<float> kernel;     // normalised at init (LRMV:45-58)
    DBuf<float> img, w, spec;      // held views only
};

// One device's replica: psi, the padded buffers, its views' partial value.  Group 0 also
// merges the other groups' partials, applies the rule and hands psi back to them.
struct LrGroup {
    int dev = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    FftPlan3D plan;
    DBuf<float> psi, Ra, Rb, Rc;
    DBuf<double> value, num, tmp;  // tmp (group 0): another group's partial, merged from there
    DBuf<const float*> ptrs;       // the group's img pointers, then its weight pointers
    int nown = 0;
};

class LrSim {
public:
    // devs: the device of each group (repeats allowed: several groups on one GPU run the
    // same code path); views go to groups round robin, as the reference's threads take them
    LrSim(const int64_t* dims, const std::vector<int>& devs, int nranks, int rank, const char* comm_id) {
        SD_CHECK(dims && dims[0] >= 1 && dims[1] >= 1 && dims[2] >= 1, SPIMDECON_ERR_ARG, "bad dims");
        SD_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, SPIMDECON_ERR_ARG, "bad rank");
        SD_CHECK(nranks == 1 || comm_id != nullptr, SPIMDECON_ERR_ARG, "nranks > 1 needs comm_id");
        SD_CHECK(!devs.empty(), SPIMDECON_ERR_ARG, "no devices");
        SD_CHECK(devs.size() == 1 || (nranks == 1 && comm_id == nullptr), SPIMDECON_ERR_ARG,
                 "several devices per process and RCCL ranks cannot be combined");
        for (int d : devs) check_device(d);
        for (int d = 0; d < 3; ++d) dims_[d] = dims[d];
        n_ = dims[0] * dims[1] * dims[2];
        nranks_ = nranks;
        rank_ = rank;
        grp_ = std::vector<LrGroup>(devs.size());   // (LrGroup is not movable: sized once)
        for (size_t g = 0; g < devs.size(); ++g) {
            LrGroup& G = grp_[g];
            G.dev = devs[g];
            DeviceGuard guard(G.dev);
            SD_HIP(hipStreamCreateWithFlags(&G.st, hipStreamNonBlocking));
            SD_HIP(hipEventCreateWithFlags(&G.ev, hipEventDisableTiming));
            if (g > 0 && G.dev != devs[0]) {   // partials and psi move between group 0 and g over xGMI
                for (auto pr : {std::make_pair(G.dev, devs[0]), std::make_pair(devs[0], G.dev)}) {
                    int can = 0;
                    SD_HIP(hipDeviceCanAccessPeer(&can, pr.first, pr.second));
                    if (!can) continue;
                    DeviceGuard g2(pr.first);
                    const hipError_t e = hipDeviceEnablePeerAccess(pr.second, 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) SD_HIP(e);
                    (void)hipGetLastError();
                }
            }
        }
        if (comm_id) {
            if (const char* e = std::getenv("SPIMDECON_RCCL_TIMEOUT")) timeout_s_ = std::max(1.0, std::atof(e));
            DeviceGuard guard(grp_[0].dev);
            ncclUniqueId id;
            std::memcpy(&id, comm_id, sizeof(id));
            SD_NCCL_LR(ncclCommInitRank(&comm_, nranks, id, rank));
        }
    }

    ~LrSim() {
        if (comm_) {
            DeviceGuard guard(grp_[0].dev);
            ncclCommDestroy(comm_);
        }
        if (dead_) {   // an aborted communicator: do not block in hipFree behind dead work
            new std::vector<LrView>(std::move(views_));
            new std::vector<LrGroup>(std::move(grp_));
            return;
        }
        for (auto& G : grp_) {
            DeviceGuard guard(G.dev);
            if (G.st) (void)hipStreamSynchronize(G.st);
        }
        for (auto& v : views_) {
            if (v.grp < 0) continue;
            DeviceGuard guard(grp_[v.grp].dev);
            v.img.release(); v.w.release(); v.spec.release();
        }
        for (auto& G : grp_) {
            DeviceGuard guard(G.dev);
            G.psi.release(); G.Ra.release(); G.Rb.release(); G.Rc.release();
            G.value.release(); G.num.release(); G.tmp.release(); G.ptrs.release();
            if (G.ev) (void)hipEventDestroy(G.ev);
            if (G.st) (void)hipStreamDestroy(G.st);
        }
        part_.release();
        red_.release();
    }

    void add_view(const float* img, const float* w, const float* kernel, const int* kd) {
        SD_CHECK(!inited_, SPIMDECON_ERR_STATE, "views must be added before lrsim_init");
        SD_CHECK(kd && kd[0] >= 1 && kd[1] >= 1 && kd[2] >= 1, SPIMDECON_ERR_ARG, "bad kernel dims");
        for (int d = 0; d < 3; ++d)
            SD_CHECK(kd[d] % 2 == 1, SPIMDECON_ERR_ARG, "kernel dims must be odd");
        LrView v;
        for (int d = 0; d < 3; ++d) v.kd[d] = kd[d];
        const int idx = int(views_.size());
        if (idx % nranks_ == rank_)   // LRMV:127-128, threads -> ranks, then -> this rank's groups
            v.grp = (idx / nranks_) % int(grp_.size());
        if (v.grp >= 0) {
            SD_CHECK(img && w && kernel, SPIMDECON_ERR_ARG,
                     "img, weight and kernel are required for a view this rank owns (LRMV:401 reads every weight)");
            LrGroup& G = grp_[v.grp];
            DeviceGuard guard(G.dev);
            v.img.alloc(size_t(n_));
            v.w.alloc(size_t(n_));
            SD_HIP(hipMemcpyAsync(v.img.p, img, size_t(n_) * 4, hipMemcpyDefault, G.st));
            SD_HIP(hipMemcpyAsync(v.w.p, w, size_t(n_) * 4, hipMemcpyDefault, G.st));
            SD_HIP(hipStreamSynchronize(G.st));
            const int64_t kn = int64_t(kd[0]) * kd[1] * kd[2];
            v.kernel.assign(kernel, kernel + kn);
        }
        views_.push_back(std::move(v));
    }

    // normImage of the kernels, their spectra, normAllImages -> psi (LRMV:24-85)
    double init() {
        SD_CHECK(!inited_, SPIMDECON_ERR_STATE, "lrsim_init called twice");
        SD_CHECK(!views_.empty(), SPIMDECON_ERR_STATE, "no views");
        int c[3] = {0, 0, 0};
        int64_t khash = 0;
        for (auto& v : views_)
            for (int d = 0; d < 3; ++d) {
                c[d] = std::max(c[d], v.kd[d] / 2);
                khash = khash * 131 + v.kd[d];
            }
        {
            const int64_t mine[7] = {0x4c52534d31LL, nranks_, dims_[0], dims_[1], dims_[2], int64_t(views_.size()),
                                     khash};
            agree(mine, 7, "lrsim_init");
        }
        g_.nx = dims_[0]; g_.ny = dims_[1]; g_.nz = dims_[2];
        g_.z0 = 0; g_.nzg = dims_[2];
        g_.cx = c[0]; g_.cy = c[1]; g_.cz = c[2];
        for (int d = 0; d < 3; ++d) pd_.M[d] = fft_fast_size(dims_[d] + 2 * c[d], d == 0);
        g_.Mx = pd_.M[0]; g_.My = pd_.M[1]; g_.Mz = pd_.M[2];
        g_.Sx = pd_.Sx();
        const size_t R = size_t(pd_.real_floats());
        const float scale = float(1.0 / double(pd_.logical()));
        const unsigned gb = grid_of(n_, kB, 4096);
        for (size_t gi = 0; gi < grp_.size(); ++gi) {
            LrGroup& G = grp_[gi];
            DeviceGuard guard(G.dev);
            G.plan.create(pd_, G.st);
            G.psi.alloc(size_t(n_));
            G.Ra.alloc(R);
            G.Rb.alloc(R);
            G.Rc.alloc(R);
            G.value.alloc(size_t(n_));
            G.num.alloc(size_t(n_));
            if (gi == 0 && grp_.size() > 1) G.tmp.alloc(size_t(n_));
            std::vector<const float*> hp;
            for (auto& v : views_)
                if (v.grp == int(gi)) hp.push_back(v.img.p);
            for (auto& v : views_)
                if (v.grp == int(gi)) hp.push_back(v.w.p);
            G.nown = int(hp.size() / 2);
            G.ptrs.alloc(std::max<size_t>(hp.size(), 1));
            if (!hp.empty())
                SD_HIP(hipMemcpyAsync(G.ptrs.p, hp.data(), hp.size() * sizeof(void*), hipMemcpyHostToDevice, G.st));
            // kernels: exact-sum normalisation (host), spectra scaled by 1 / (Mx My Mz)
            DBuf<float> dk;
            for (auto& v : views_) {
                if (v.grp != int(gi)) continue;
                const double s = exact_sum(v.kernel.data(), int64_t(v.kernel.size()));
                for (auto& t : v.kernel) t = (float)((double)t / s);
                dk.alloc(v.kernel.size());
                SD_HIP(hipMemcpyAsync(dk.p, v.kernel.data(), v.kernel.size() * 4, hipMemcpyHostToDevice, G.st));
                v.spec.alloc(R);
                launch_place_kernel(g_, dk.p, v.kd[0], v.kd[1], v.kd[2], scale, v.spec.p, G.st);
                G.plan.forward(v.spec.p);
                SD_HIP(hipStreamSynchronize(G.st));
            }
            // normAllImages: the group's per-voxel partials {sum of img where w != 0, count}
            hipLaunchKernelGGL(k_lr_overlap, dim3(gb), dim3(kB), 0, G.st, n_, G.nown, imgs_of(G), ws_of(G),
                               G.value.p, G.num.p);
            SD_HIP(hipGetLastError());
        }
        LrGroup& G0 = grp_[0];
        DeviceGuard guard(G0.dev);
        part_.alloc(size_t(2) * gb);
        red_.alloc(2);
        merge_groups(&LrGroup::value, false);
        merge_groups(&LrGroup::num, false);
        allreduce(G0.value.p, n_, ncclSum);
        allreduce(G0.num.p, n_, ncclSum);
        hipLaunchKernelGGL(k_lr_avg_partials, dim3(gb), dim3(kB), 0, G0.st, n_, G0.value.p, G0.num.p, part_.p);
        hipLaunchKernelGGL(k_lr_sum2, dim3(1), dim3(1024), 0, G0.st, part_.p, int64_t(gb), red_.p);
        SD_HIP(hipGetLastError());
        double r[2];
        SD_HIP(hipMemcpyAsync(r, red_.p, sizeof(r), hipMemcpyDeviceToHost, G0.st));
        wait();
        avg_ = r[1] == 0.0 ? 1.0 : r[0] / r[1];
        // num = sum of the weights > 0 (constant over the iterations): merged and reduced once
        for (auto& G : grp_) {
            DeviceGuard g2(G.dev);
            launch_fill(G.psi.p, n_, (float)avg_, G.st);
            hipLaunchKernelGGL(k_lr_num, dim3(gb), dim3(kB), 0, G.st, n_, G.nown, ws_of(G), G.num.p);
            SD_HIP(hipGetLastError());
        }
        merge_groups(&LrGroup::num, false);
        allreduce(G0.num.p, n_, ncclSum);
        for (auto& G : grp_) {
            DeviceGuard g2(G.dev);
            SD_HIP(hipStreamSynchronize(G.st));
        }
        wait();
        inited_ = true;
        return avg_;
    }

    void run(int iters, bool mult, double lambda, double* stats) {
        SD_CHECK(inited_, SPIMDECON_ERR_STATE, "lrsim_init first");
        SD_CHECK(!dead_, SPIMDECON_ERR_STATE, "communicator aborted");
        SD_CHECK(iters >= 0, SPIMDECON_ERR_ARG, "iters must be >= 0");
        {
            DeviceGuard guard(grp_[0].dev);
            int64_t lb;
            std::memcpy(&lb, &lambda, 8);
            const int64_t mine[4] = {0x4c52534d32LL, iters, int64_t(mult), lb};
            agree(mine, 4, "lrsim_run");
        }
        const int64_t ncplx = pd_.complex_count();
        const unsigned gr = grid_of(g_.My * g_.Mz, kW);
        const unsigned gi = grid_of(g_.ny * g_.nz, kW);
        const unsigned gb = grid_of(n_, kB);
        LrGroup& G0 = grp_[0];
        for (int it = 0; it < iters; ++it) {
            for (auto& G : grp_) {   // every group's views, concurrently on their own streams
                DeviceGuard guard(G.dev);
                launch_pad_mirror(g_, G.psi.p, G.Ra.p, G.st);
                G.plan.forward(G.Ra.p);
                hipLaunchKernelGGL(k_lr_fill, dim3(grid_of(n_, kB, 4096)), dim3(kB), 0, G.st, G.value.p, n_,
                                   mult ? 1.0 : 0.0);
                for (auto& v : views_) {
                    if (v.grp != int(&G - grp_.data())) continue;
                    hipLaunchKernelGGL(k_lr_cmul, dim3(grid_of(ncplx / 2, kB, 256 * 32)), dim3(kB), 0, G.st,
                                       reinterpret_cast<const float4*>(G.Ra.p),
                                       reinterpret_cast<const float4*>(v.spec.p), reinterpret_cast<float4*>(G.Rb.p),
                                       ncplx / 2, reinterpret_cast<const float2*>(G.Ra.p) + (ncplx - 1),
                                       reinterpret_cast<const float2*>(v.spec.p) + (ncplx - 1),
                                       reinterpret_cast<float2*>(G.Rb.p) + (ncplx - 1), int(ncplx & 1));
                    G.plan.inverse(G.Rb.p);   // blurred = conv(psi, K) at the interior slots
                    hipLaunchKernelGGL(k_lr_quot_pad, dim3(gr), dim3(kB), 0, G.st, g_, v.img.p, G.Rb.p, G.Rc.p);
                    G.plan.forward(G.Rc.p);
                    launch_spec_mul(G.Rc.p, v.spec.p, ncplx, G.st);
                    G.plan.inverse(G.Rc.p);   // the view's contribution conv(img / blurred, K)
                    if (mult)
                        hipLaunchKernelGGL(k_lr_accum<true>, dim3(gi), dim3(kB), 0, G.st, g_, G.Rc.p, v.w.p,
                                           G.value.p);
                    else
                        hipLaunchKernelGGL(k_lr_accum<false>, dim3(gi), dim3(kB), 0, G.st, g_, G.Rc.p, v.w.p,
                                           G.value.p);
                    SD_HIP(hipGetLastError());
                }
            }
            DeviceGuard guard(G0.dev);
            // the compound correction of all views: merged over the groups, then one all-reduce
            // (product / sum) over the ranks
            merge_groups(&LrGroup::value, mult);
            allreduce(G0.value.p, n_, mult ? ncclProd : ncclSum);
            auto upd = [&](auto m, auto t) {
                hipLaunchKernelGGL((k_lr_update<decltype(m)::value, decltype(t)::value>), dim3(gb), dim3(kB), 0,
                                   G0.st, n_, G0.psi.p, G0.value.p, G0.num.p, lambda, part_.p);
            };
            using T = std::true_type;
            using F = std::false_type;
            if (mult && lambda > 0) upd(T{}, T{});
            else if (mult) upd(T{}, F{});
            else if (lambda > 0) upd(F{}, T{});
            else upd(F{}, F{});
            SD_HIP(hipGetLastError());
            launch_reduce_partials(part_.p, int64_t(gb), red_.p, 0, G0.st);
            // the new psi to the other groups (on group 0's stream; they wait for it)
            for (size_t g = 1; g < grp_.size(); ++g)
                SD_HIP(hipMemcpyAsync(grp_[g].psi.p, G0.psi.p, size_t(n_) * 4, hipMemcpyDefault, G0.st));
            if (grp_.size() > 1) {
                SD_HIP(hipEventRecord(G0.ev, G0.st));
                for (size_t g = 1; g < grp_.size(); ++g) {
                    DeviceGuard g2(grp_[g].dev);
                    SD_HIP(hipStreamWaitEvent(grp_[g].st, G0.ev, 0));
                }
            }
            double r[2];
            SD_HIP(hipMemcpyAsync(r, red_.p, sizeof(r), hipMemcpyDeviceToHost, G0.st));
            wait();
            if (stats) {
                stats[2 * it] = r[0];
                stats[2 * it + 1] = r[1];
            }
        }
    }

    void get_psi(float* out) {
        SD_CHECK(inited_, SPIMDECON_ERR_STATE, "lrsim_init first");
        SD_CHECK(out, SPIMDECON_ERR_ARG, "null argument");
        DeviceGuard guard(grp_[0].dev);
        SD_HIP(hipMemcpyAsync(out, grp_[0].psi.p, size_t(n_) * 4, hipMemcpyDefault, grp_[0].st));
        wait();
    }

    int owns(int v) const {
        SD_CHECK(v >= 0 && v < int(views_.size()), SPIMDECON_ERR_ARG, "bad view index");
        return views_[v].grp >= 0 ? 1 : 0;
    }

    int view_device(int v) const {
        SD_CHECK(v >= 0 && v < int(views_.size()), SPIMDECON_ERR_ARG, "bad view index");
        return views_[v].grp >= 0 ? grp_[views_[v].grp].dev : -1;
    }

    void fft_dims(int64_t* out3) const {
        SD_CHECK(inited_, SPIMDECON_ERR_STATE, "lrsim_init first");
        for (int d = 0; d < 3; ++d) out3[d] = pd_.M[d];
    }

private:
    static const float* const* imgs_of(const LrGroup& G) { return reinterpret_cast<const float* const*>(G.ptrs.p); }
    static const float* const* ws_of(const LrGroup& G) { return imgs_of(G) + G.nown; }

    // group 0's array (member `a`) merged with every other group's, in group order, on group
    // 0's stream after their streams' work so far: a sum, or a product (mult)
    void merge_groups(DBuf<double> LrGroup::*a, bool mult) {
        if (grp_.size() < 2) return;
        LrGroup& G0 = grp_[0];
        for (size_t g = 1; g < grp_.size(); ++g) {
            LrGroup& G = grp_[g];
            {
                DeviceGuard guard(G.dev);
                SD_HIP(hipEventRecord(G.ev, G.st));
            }
            DeviceGuard guard(G0.dev);
            SD_HIP(hipStreamWaitEvent(G0.st, G.ev, 0));
            SD_HIP(hipMemcpyAsync(G0.tmp.p, (G.*a).p, size_t(n_) * 8, hipMemcpyDefault, G0.st));
            hipLaunchKernelGGL(k_lr_merge, dim3(grid_of(n_, kB, 4096)), dim3(kB), 0, G0.st, (G0.*a).p, G0.tmp.p, n_,
                               int(mult));
            SD_HIP(hipGetLastError());
        }
    }

    void allreduce(double* p, int64_t n, ncclRedOp_t op) {
        if (!comm_) return;
        SD_NCCL_LR(ncclAllReduce(p, p, size_t(n), ncclDouble, op, comm_, grp_[0].st));
    }

    // waits for group 0's stream; with a communicator, bounded: an asynchronous RCCL error or
    // SPIMDECON_RCCL_TIMEOUT seconds without completion abort it (ranks that disagree on
    // the work fail instead of waiting for each other forever)
    void wait() {
        hipStream_t st = grp_[0].st;
        if (!comm_) {
            SD_HIP(hipStreamSynchronize(st));
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        int spins = 0;
        for (;;) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) SD_HIP(e);
            ncclResult_t ar = ncclSuccess;
            (void)ncclCommGetAsyncError(comm_, &ar);
            const double idle = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if ((ar != ncclSuccess && ar != ncclInProgress) || idle > timeout_s_) {
                (void)ncclCommAbort(comm_);
                comm_ = nullptr;
                dead_ = true;
                fail(SPIMDECON_ERR_COMM, "rank " + std::to_string(rank_) + ": " +
                                             (ar != ncclSuccess && ar != ncclInProgress
                                                  ? std::string("RCCL asynchronous error: ") + ncclGetErrorString(ar)
                                                  : std::string("no completion within SPIMDECON_RCCL_TIMEOUT")) +
                                             "; communicator aborted");
            }
            if (++spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }

    // every rank's K values all-gathered; refused on every rank unless all are equal
    // (a mismatch would post different collectives)
    void agree(const int64_t* mine, int K, const char* what) {
        if (!comm_) return;
        hipStream_t st = grp_[0].st;
        DeviceGuard guard(grp_[0].dev);
        DBuf<int64_t> d(size_t(K) * nranks_);
        std::vector<int64_t> all(size_t(K) * nranks_);
        SD_HIP(hipMemcpyAsync(d.p + size_t(K) * rank_, mine, size_t(K) * 8, hipMemcpyHostToDevice, st));
        SD_NCCL_LR(ncclAllGather(d.p + size_t(K) * rank_, d.p, size_t(K), ncclInt64, comm_, st));
        SD_HIP(hipMemcpyAsync(all.data(), d.p, all.size() * 8, hipMemcpyDeviceToHost, st));
        wait();
        for (int r = 0; r < nranks_; ++r)
            for (int k = 0; k < K; ++k)
                if (all[size_t(K) * r + k] != mine[k])
                    fail(SPIMDECON_ERR_ARG, std::string(what) + ": rank " + std::to_string(r) +
                                                " disagrees with rank " + std::to_string(rank_) + " (field " +
                                                std::to_string(k) + ")");
    }

    int64_t dims_[3] = {0, 0, 0};
    int64_t n_ = 0;
    int nranks_ = 1, rank_ = 0;
    ncclComm_t comm_ = nullptr;
    double timeout_s_ = 300.0;
    bool dead_ = false, inited_ = false;
    double avg_ = 1.0;
    std::vector<LrView> views_;
    std::vector<LrGroup> grp_;
    SlabGeom g_{};
    PadDims pd_;
    DBuf<double> part_, red_;   // (group 0)
};
}  // namespace spimdecon

using spimdecon::guarded;
using spimdecon::LrSim;

struct lrsim_session {
    LrSim* s;
};

#define LRS(h)                                                                        \
    SD_CHECK((h) && (h)->s, SPIMDECON_ERR_ARG, "null lrsim session");                \
    LrSim& S = *(h)->s

extern "C" {

int lrsim_create(const int64_t* dims, int device, int nranks, int rank, const char* comm_id, lrsim_session** out) {
    return guarded([&] {
        SD_CHECK(out, SPIMDECON_ERR_ARG, "null argument");
        *out = nullptr;
        auto s = std::make_unique<LrSim>(dims, std::vector<int>{device}, nranks, rank, comm_id);
        *out = new lrsim_session{s.release()};
    });
}

int lrsim_create_devices(const int64_t* dims, const int* devs, int ndev, lrsim_session** out) {
    return guarded([&] {
        SD_CHECK(out && devs && ndev >= 1, SPIMDECON_ERR_ARG, "null argument");
        *out = nullptr;
        auto s = std::make_unique<LrSim>(dims, std::vector<int>(devs, devs + ndev), 1, 0, nullptr);
        *out = new lrsim_session{s.release()};
    });
}

int lrsim_view_device(lrsim_session* h, int view, int* device) {
    return guarded([&] {
        LRS(h);
        SD_CHECK(device, SPIMDECON_ERR_ARG, "null argument");
        *device = S.view_device(view);
    });
}

void lrsim_destroy(lrsim_session* h) {
    if (!h) return;
    delete h->s;
    delete h;
}

int lrsim_add_view(lrsim_session* h, const float* img, const float* weight, const float* kernel, const int* kdims) {
    return guarded([&] { LRS(h); S.add_view(img, weight, kernel, kdims); });
}

int lrsim_owns_view(lrsim_session* h, int view, int* owned) {
    return guarded([&] {
        LRS(h);
        SD_CHECK(owned, SPIMDECON_ERR_ARG, "null argument");
        *owned = S.owns(view);
    });
}

int lrsim_init(lrsim_session* h, double* avg_out) {
    return guarded([&] {
        LRS(h);
        const double a = S.init();
        if (avg_out) *avg_out = a;
    });
}

int lrsim_run(lrsim_session* h, int iters, int multiplicative, double lambda, double* stats) {
    return guarded([&] { LRS(h); S.run(iters, multiplicative != 0, lambda, stats); });
}

int lrsim_get_psi(lrsim_session* h, float* out) {
    return guarded([&] { LRS(h); S.get_psi(out); });
}

int lrsim_fft_dims(lrsim_session* h, int64_t* out3) {
    return guarded([&] {
        LRS(h);
        SD_CHECK(out3, SPIMDECON_ERR_ARG, "null argument");
        S.fft_dims(out3);
    });
}

}  // extern "C"
