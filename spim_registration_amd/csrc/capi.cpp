// capi.cpp -- extern "C" entry points of libspimdecon.so (declared in include/spimdecon.h).
#include <rccl/rccl.h>
#include <rocfft/rocfft-version.h>

#include <cstdlib>
#include <cstring>
#include <string>

#include "common.hpp"
#include "kernel_prep.hpp"
#include "session.hpp"

namespace spimdecon {

thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
void clear_last_error() { g_last_error.clear(); }

void fft_convolve_block(float* im, const int* imDim, const float* kernel, const int* kernelDim,
                        int dev, float* out);
void slab_range(int64_t nz, int nparts, int idx, int64_t* z0, int64_t* z1);

}  // namespace spimdecon

using namespace spimdecon;

struct mvd_session {
    Session* s;
};

extern "C" {

const char* spimdecon_last_error(void) { return g_last_error.c_str(); }

const char* spimdecon_version(void) {
    static std::string v = std::string("spimdecon 0.1.0 gfx950 rocfft ") +
                           std::to_string(rocfft_version_major) + "." +
                           std::to_string(rocfft_version_minor) + "." +
                           std::to_string(rocfft_version_patch);
    return v.c_str();
}

// ---------------------------------------------------------------- legacy FFT ABI
int convolution3DfftCUDAInPlace(float* im, const int* imDim, const float* kernel,
                                const int* kernelDim, int devCUDA) {
    return guarded([&] { fft_convolve_block(im, imDim, kernel, kernelDim, devCUDA, im); });
}

float* convolution3DfftCUDA(const float* im, const int* imDim, const float* kernel,
                            const int* kernelDim, int devCUDA) {
    float* out = nullptr;
    int st = guarded([&] {
        SD_CHECK(imDim, SPIMDECON_ERR_ARG, "null imDim");
        const size_t n = size_t(imDim[0]) * imDim[1] * imDim[2];
        out = static_cast<float*>(std::malloc(n * sizeof(float)));
        SD_CHECK(out, SPIMDECON_ERR_OOM, "host out of memory");
        fft_convolve_block(const_cast<float*>(im), imDim, kernel, kernelDim, devCUDA, out);
    });
    if (st != SPIMDECON_OK) {
        std::free(out);
        return nullptr;
    }
    return out;
}

void spimdecon_free(void* p) { std::free(p); }

// ---------------------------------------------------------------- device query ABI
int getNumDevicesCUDA(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        // no driver / no device: the reference distinguishes "crash" (-1) from "none" (0)
        return 0;
    }
    return n;
}

void getNameDeviceCUDA(int devCUDA, char* name) {
    if (!name) return;
    name[0] = 0;
    guarded([&] {
        check_device(devCUDA);
        hipDeviceProp_t prop;
        SD_HIP(hipGetDeviceProperties(&prop, devCUDA));
        std::string s = std::string(prop.name) + " (" + prop.gcnArchName + ")";
        std::strncpy(name, s.c_str(), 255);
        name[255] = 0;
    });
}

int64_t getMemDeviceCUDA(int devCUDA) {
    int64_t r = -1;
    guarded([&] {
        check_device(devCUDA);
        hipDeviceProp_t prop;
        SD_HIP(hipGetDeviceProperties(&prop, devCUDA));
        r = int64_t(prop.totalGlobalMem);
    });
    return r;
}

int64_t getFreeMemDeviceCUDA(int devCUDA) {
    int64_t r = -1;
    guarded([&] {
        check_device(devCUDA);
        DeviceGuard g(devCUDA);
        size_t fr = 0, tot = 0;
        SD_HIP(hipMemGetInfo(&fr, &tot));
        r = int64_t(fr);
    });
    return r;
}

int getCUDAcomputeCapabilityMajorVersion(int devCUDA) {
    int r = -1;
    guarded([&] {
        check_device(devCUDA);
        hipDeviceProp_t prop;
        SD_HIP(hipGetDeviceProperties(&prop, devCUDA));
        r = prop.major;
    });
    return r;
}

int getCUDAcomputeCapabilityMinorVersion(int devCUDA) {
    int r = -1;
    guarded([&] {
        check_device(devCUDA);
        hipDeviceProp_t prop;
        SD_HIP(hipGetDeviceProperties(&prop, devCUDA));
        r = prop.minor;
    });
    return r;
}

int spimdecon_next_value(const float* last, const float* integral, const float* weight, int64_t n, double lambda,
                         float* out) {
    return guarded([&] {
        SD_CHECK(n >= 0, SPIMDECON_ERR_ARG, "n must be >= 0");
        SD_CHECK(n == 0 || (last && integral && weight && out), SPIMDECON_ERR_ARG, "null pointer");
        launch_next_value(last, integral, weight, n, lambda, out, nullptr);
        SD_HIP(hipStreamSynchronize(nullptr));
    });
}

// ---------------------------------------------------------------- kernel preparation
int mvd_prepare_kernels(int nviews, const float* const* k1_in, const int* kdims, int psftype,
                        int ij_threads, float* const* k1_out, float* const* k2_out, int devCUDA) {
    return guarded([&] {
        SD_CHECK(nviews >= 1 && k1_in && kdims && k1_out && k2_out, SPIMDECON_ERR_ARG, "bad arguments");
        std::vector<HostKernel> k1(nviews), k2;
        for (int v = 0; v < nviews; ++v) {
            for (int d = 0; d < 3; ++d) k1[v].dims[d] = kdims[3 * v + d];
            const int64_t n = int64_t(k1[v].dims[0]) * k1[v].dims[1] * k1[v].dims[2];
            SD_CHECK(n > 0 && k1_in[v], SPIMDECON_ERR_ARG, "bad kernel");
            k1[v].data.assign(k1_in[v], k1_in[v] + n);
        }
        prepare_kernels_gpu(k1, k2, psftype, ij_threads, devCUDA);
        for (int v = 0; v < nviews; ++v) {
            std::copy(k1[v].data.begin(), k1[v].data.end(), k1_out[v]);
            std::copy(k2[v].data.begin(), k2[v].data.end(), k2_out[v]);
        }
    });
}

// ---------------------------------------------------------------- session
void mvd_params_default(mvd_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->local_slabs = 1;
    p->nranks = 1;
    p->ij_threads = 8;
}

int mvd_comm_unique_id(char* out128) {
    return guarded([&] {
        SD_CHECK(out128, SPIMDECON_ERR_ARG, "null output");
        static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
        ncclUniqueId id;
        ncclResult_t r = ncclGetUniqueId(&id);
        SD_CHECK(r == ncclSuccess, SPIMDECON_ERR_COMM,
                 std::string("ncclGetUniqueId failed: ") + ncclGetErrorString(r));
        std::memcpy(out128, &id, 128);
    });
}

int mvd_slab_range(int64_t nz, int nparts, int idx, int64_t* z0, int64_t* z1) {
    return guarded([&] {
        SD_CHECK(nz >= 1 && nparts >= 1 && idx >= 0 && idx < nparts && z0 && z1, SPIMDECON_ERR_ARG,
                 "bad slab_range arguments");
        slab_range(nz, nparts, idx, z0, z1);
    });
}

int mvd_halo_plan(int64_t nz, int64_t Mz, int cz, int64_t plane_elems, int64_t* out5) {
    return guarded([&] {
        SD_CHECK(out5, SPIMDECON_ERR_ARG, "null argument");
        const HaloPlan h = halo_plan(nz, Mz, cz, plane_elems);
        out5[0] = h.send_lo;
        out5[1] = h.recv_lo;
        out5[2] = h.send_hi;
        out5[3] = h.recv_hi;
        out5[4] = h.count;
    });
}

int mvd_create(const mvd_params* params, mvd_session** out) {
    return guarded([&] {
        SD_CHECK(params && out, SPIMDECON_ERR_ARG, "null argument");
        *out = nullptr;
        auto* h = new mvd_session{nullptr};
        try {
            h->s = new Session(*params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int mvd_create_devices(const int* devs, int ndev, const mvd_params* params, mvd_session** out) {
    return guarded([&] {
        SD_CHECK(devs && ndev >= 1 && params && out, SPIMDECON_ERR_ARG, "null argument");
        *out = nullptr;
        std::vector<int> dl(devs, devs + ndev);
        auto* h = new mvd_session{nullptr};
        try {
            h->s = new Session(*params, dl);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

void mvd_destroy(mvd_session* h) {
    if (!h) return;
    guarded([&] { delete h->s; });
    delete h;
}

#define SESSION(h) \
    SD_CHECK((h) && (h)->s, SPIMDECON_ERR_ARG, "null session"); \
    Session& S = *(h)->s

int mvd_add_view(mvd_session* h, const float* img, const float* weight, const float* kernel1,
                 const int* kdims) {
    return guarded([&] { SESSION(h); S.add_view(img, weight, kernel1, kdims, false); });
}

int mvd_add_view_device(mvd_session* h, const float* d_img, const float* d_weight,
                        const float* kernel1, const int* kdims) {
    return guarded([&] { SESSION(h); S.add_view(d_img, d_weight, kernel1, kdims, true); });
}

int mvd_init(mvd_session* h, int psftype) {
    return guarded([&] { SESSION(h); S.init(psftype); });
}

int mvd_set_kernels(mvd_session* h, int view, const float* k1, const float* k2) {
    return guarded([&] { SESSION(h); S.set_kernels(view, k1, k2); });
}

int mvd_get_kernels(mvd_session* h, int view, float* k1, float* k2) {
    return guarded([&] { SESSION(h); S.get_kernels(view, k1, k2); });
}

int mvd_init_psi(mvd_session* h, const float* psi_or_null, double* avg_out) {
    return guarded([&] {
        SESSION(h);
        const double a = S.init_psi(psi_or_null);
        if (avg_out) *avg_out = a;
    });
}

int mvd_run(mvd_session* h, int iters, double lambda, double* stats) {
    return guarded([&] { SESSION(h); S.run(iters, lambda, stats); });
}

int mvd_apply_mask(mvd_session* h) {
    return guarded([&] { SESSION(h); S.apply_mask(); });
}

int mvd_get_psi(mvd_session* h, float* out) {
    return guarded([&] { SESSION(h); S.get_psi(out); });
}

float* mvd_psi_device(mvd_session* h, int slab) {
    float* r = nullptr;
    guarded([&] { SESSION(h); r = S.psi_device(slab); });
    return r;
}

int mvd_fft_dims(mvd_session* h, int slab, int64_t* out3) {
    return guarded([&] { SESSION(h); SD_CHECK(out3, SPIMDECON_ERR_ARG, "null"); S.fft_dims(slab, out3); });
}

int mvd_kernel_planes(mvd_session* h, int slab, int* planes) {
    return guarded([&] { SESSION(h); SD_CHECK(planes, SPIMDECON_ERR_ARG, "null"); *planes = S.kernel_planes(slab); });
}

int mvd_zpass_mode(mvd_session* h, int slab, int* mode) {
    return guarded([&] { SESSION(h); SD_CHECK(mode, SPIMDECON_ERR_ARG, "null"); *mode = S.zpass_mode(slab); });
}

int mvd_xpass_mode(mvd_session* h, int slab, int* mode) {
    return guarded([&] { SESSION(h); SD_CHECK(mode, SPIMDECON_ERR_ARG, "null"); *mode = S.xpass_mode(slab); });
}

void* mvd_stream(mvd_session* h) {
    void* r = nullptr;
    guarded([&] { SESSION(h); r = S.stream(); });
    return r;
}

int mvd_num_devices(mvd_session* h, int* ndev) {
    return guarded([&] { SESSION(h); SD_CHECK(ndev, SPIMDECON_ERR_ARG, "null"); *ndev = S.ndevices(); });
}

int mvd_slab_device(mvd_session* h, int slab, int* dev) {
    return guarded([&] { SESSION(h); SD_CHECK(dev, SPIMDECON_ERR_ARG, "null"); *dev = S.slab_device(slab); });
}

int mvd_num_slabs(mvd_session* h, int* nslabs) {
    return guarded([&] { SESSION(h); SD_CHECK(nslabs, SPIMDECON_ERR_ARG, "null"); *nslabs = S.nslabs(); });
}

int mvd_exchange_stats(mvd_session* h, int64_t* bytes, int64_t* copies) {
    return guarded([&] { SESSION(h); S.exchange_stats(bytes, copies); });
}

int mvd_slab_extent(mvd_session* h, int slab, int64_t* out3) {
    return guarded([&] { SESSION(h); SD_CHECK(out3, SPIMDECON_ERR_ARG, "null"); S.slab_extent(slab, out3); });
}

int mvd_enable_timing(mvd_session* h, int on) {
    return guarded([&] { SESSION(h); S.enable_timing(on != 0); });
}

int mvd_timing(mvd_session* h, double* out16) {
    return guarded([&] { SESSION(h); SD_CHECK(out16, SPIMDECON_ERR_ARG, "null"); S.timing(out16); });
}

}  // extern "C"
