// legacy.cpp -- FourierConvolutionCUDALib + CUDAStandardFunctions ABI on MI355X.
//
// convolution3DfftCUDAInPlace (spim/process/cuda/CUDAFourierConvolution.java:10) is
// called concurrently from one Java thread per device (MVDeconFFT.java:424-446):
// every device owns a mutex, a stream, a plan cache keyed by block dims and a
// small kernel-spectrum cache (the reference recomputes the kernel FFT on every
// call; identical kernels are recognised by content and reused).
#include <array>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>

#include "common.hpp"
#include "fft.hpp"
#include "rl_kernels.hpp"

namespace spimdecon {

namespace {

struct CachedSpectrum {
    std::vector<float> kernel;
    int kd[3];
    DBuf<float> spec;
    uint64_t stamp;
};

struct PlanEntry {
    std::unique_ptr<FftPlan3D> fft;
    DBuf<float> buf;
    std::vector<CachedSpectrum> spectra;
    uint64_t stamp = 0;  // last use (LRU eviction beyond kMaxPlans)
};

struct DeviceCtx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    std::map<std::array<int64_t, 3>, PlanEntry> plans;
    uint64_t clock = 0;
};

std::mutex g_ctx_mu;
// never destroyed: a static destructor would free device buffers and rocFFT plans at
// process exit in an order relative to the HIP runtime's and rocFFT's own teardown that
// nothing guarantees (the OS reclaims the memory)
std::unordered_map<int, std::unique_ptr<DeviceCtx>>& g_ctx = *new std::unordered_map<int, std::unique_ptr<DeviceCtx>>();

DeviceCtx& device_ctx(int dev) {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto& p = g_ctx[dev];
    if (!p) p.reset(new DeviceCtx());
    return *p;
}

constexpr size_t kMaxSpectra = 16;
// block shapes cached per device: a long-lived JVM that walks datasets with different
// block sizes would otherwise keep a plan, a padded work block and up to kMaxSpectra
// kernel spectra per shape forever; the least recently used is dropped
constexpr size_t kMaxPlans = 4;

const float* spectrum_for(PlanEntry& pe, DeviceCtx& ctx, const SlabGeom& g, const PadDims& pd,
                          const float* kernel, const int kd[3]) {
    const size_t kn = size_t(kd[0]) * kd[1] * kd[2];
    for (auto& c : pe.spectra) {
        if (c.kd[0] == kd[0] && c.kd[1] == kd[1] && c.kd[2] == kd[2] &&
            std::memcmp(c.kernel.data(), kernel, kn * sizeof(float)) == 0) {
            c.stamp = ++ctx.clock;
            return c.spec.p;
        }
    }
    CachedSpectrum* slot;
    if (pe.spectra.size() < kMaxSpectra) {
        pe.spectra.emplace_back();
        slot = &pe.spectra.back();
    } else {
        slot = &pe.spectra[0];
        for (auto& c : pe.spectra)
            if (c.stamp < slot->stamp) slot = &c;
    }
    slot->kernel.assign(kernel, kernel + kn);
    std::memcpy(slot->kd, kd, sizeof(slot->kd));
    slot->stamp = ++ctx.clock;
    if (slot->spec.n != size_t(pd.real_floats())) slot->spec.alloc(pd.real_floats());
    DBuf<float> dk(kn);
    SD_HIP(hipMemcpyAsync(dk.p, kernel, kn * 4, hipMemcpyHostToDevice, ctx.stream));
    launch_place_kernel(g, dk.p, kd[0], kd[1], kd[2], float(1.0 / double(pd.logical())), slot->spec.p,
                        ctx.stream);
    pe.fft->forward(slot->spec.p);
    SD_HIP(hipStreamSynchronize(ctx.stream));
    return slot->spec.p;
}

}  // namespace

void check_device(int dev) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        fail(SPIMDECON_ERR_DEVICE, "no HIP device available (no CPU fallback)");
    if (dev < 0 || dev >= n)
        fail(SPIMDECON_ERR_DEVICE, "invalid device id " + std::to_string(dev) + " (" +
                                       std::to_string(n) + " devices; negative = CPU is not supported)");
}

// In-place circular convolution of one block (see spimdecon.h).
void fft_convolve_block(float* im, const int* imDim, const float* kernel, const int* kernelDim,
                        int dev, float* out) {
    SD_CHECK(im && imDim && kernel && kernelDim, SPIMDECON_ERR_ARG, "null argument");
    check_device(dev);
    const int64_t nz = imDim[0], ny = imDim[1], nx = imDim[2];
    const int kd[3] = {kernelDim[2], kernelDim[1], kernelDim[0]};
    SD_CHECK(nx >= 1 && ny >= 1 && nz >= 1, SPIMDECON_ERR_ARG, "bad block dims");
    SD_CHECK(kd[0] >= 1 && kd[1] >= 1 && kd[2] >= 1, SPIMDECON_ERR_ARG, "bad kernel dims");
    DeviceCtx& ctx = device_ctx(dev);
    std::lock_guard<std::mutex> lk(ctx.mu);
    DeviceGuard guard(dev);
    if (!ctx.stream) SD_HIP(hipStreamCreateWithFlags(&ctx.stream, hipStreamNonBlocking));
    PadDims pd;
    pd.M[0] = nx;
    pd.M[1] = ny;
    pd.M[2] = nz;
    const std::array<int64_t, 3> key{nx, ny, nz};
    if (!ctx.plans.count(key) && ctx.plans.size() >= kMaxPlans) {
        auto lru = ctx.plans.begin();
        for (auto it = ctx.plans.begin(); it != ctx.plans.end(); ++it)
            if (it->second.stamp < lru->second.stamp) lru = it;
        SD_HIP(hipStreamSynchronize(ctx.stream));
        ctx.plans.erase(lru);
    }
    PlanEntry& pe = ctx.plans[key];
    pe.stamp = ++ctx.clock;
    if (!pe.fft) {
        pe.fft.reset(new FftPlan3D());
        pe.fft->create(pd, ctx.stream);
        pe.buf.alloc(pd.real_floats());
    }
    SlabGeom g{};
    g.nx = nx; g.ny = ny; g.nz = nz; g.z0 = 0; g.nzg = nz;
    g.Mx = nx; g.My = ny; g.Mz = nz; g.Sx = pd.Sx();
    const float* spec = spectrum_for(pe, ctx, g, pd, kernel, kd);
    const size_t row = size_t(nx) * 4, pitch = size_t(pd.Sx()) * 4;
    SD_HIP(hipMemcpy2DAsync(pe.buf.p, pitch, im, row, row, size_t(ny * nz), hipMemcpyHostToDevice,
                            ctx.stream));
    pe.fft->forward(pe.buf.p);
    launch_spec_mul(pe.buf.p, spec, pd.complex_count(), ctx.stream);
    pe.fft->inverse(pe.buf.p);
    SD_HIP(hipMemcpy2DAsync(out, row, pe.buf.p, pitch, row, size_t(ny * nz), hipMemcpyDeviceToHost,
                            ctx.stream));
    SD_HIP(hipStreamSynchronize(ctx.stream));
}

}  // namespace spimdecon
