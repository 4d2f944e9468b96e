// session.hpp -- GPU-resident multiview RL deconvolution session (mvd_* C-ABI).
//
// Replaces MVDeconvolution (spim/process/fusion/deconvolution/MVDeconvolution.java:73-444):
// psi, the views (img, weight), the kernel spectra and two padded FFT work
// volumes stay resident in HBM; one iteration is, per view v (sequential,
// MVDeconvolution.java:353-441):
//   Ra = pad_mirror(psi)             (fused into the previous view's update)
//   Ra = C2R(R2C(Ra) * FFT(K1_v))    convolve1
//   Rb = pad_one(img_v > 0 ? img_v / Ra : 1)                    computeQuotient
//   Rb = C2R(R2C(Rb) * FFT(K2_v))    convolve2
//   psi' = update(psi, Rb, w_v);  Ra = pad_mirror(psi')         computeFinalValues
// The volume is split into z-slabs (local virtual slabs and/or one slab per
// RCCL rank); halos of c_z padded planes are exchanged after each pad.
#pragma once

#include <rccl/rccl.h>

#include <memory>
#include <vector>

#include "common.hpp"
#include "fft.hpp"
#include "fftconv.hpp"
#include "kernel_prep.hpp"
#include "rl_kernels.hpp"

namespace spimdecon {

struct SlabState {
    SlabGeom g{};
    PadDims pd;
    int64_t local_z0 = 0;  // first plane within this rank's z-range
    int64_t n = 0;         // voxels
    DBuf<float> psi_a, psi_b;
    float* psi = nullptr;
    float* psi_next = nullptr;
    std::vector<DBuf<char>> img, w;
    std::vector<DBuf<float>> k1spec, k2spec;
    DBuf<float> Ra, Rb;                       // rocFFT backend work volumes
    SpectralPlan sp;                           // engine backend
    DBuf<float2> C1, C2;
    std::vector<DBuf<float2>> e1spec, e2spec;  // full kernel spectra, or compact ones (kcompact)
    bool kcompact = false;
    bool zexact = false;  // Mz = nz + 2 cz (direct z pass, no z FFT plan)
    DBuf<double> partials;
    DBuf<const void*> img_ptrs;
    std::unique_ptr<FftPlan3D> fft;
};

struct TimingRec {
    int cls;
    hipEvent_t a, b;
};

class Session {
public:
    explicit Session(const mvd_params& p);
    ~Session();

    void add_view(const float* img, const float* weight, const float* k1, const int* kdims,
                  bool device_ptrs);
    void init(int psftype);
    void set_kernels(int view, const float* k1, const float* k2);
    void get_kernels(int view, float* k1, float* k2) const;
    double init_psi(const float* psi_or_null);
    void run(int iters, double lambda, double* stats);
    void apply_mask();
    void get_psi(float* out);
    float* psi_device(int slab);
    void fft_dims(int slab, int64_t* out3) const;
    int kernel_planes(int slab) const;
    int zpass_mode(int slab) const;
    hipStream_t stream() const { return stream_; }
    void enable_timing(bool on) { timing_on_ = on; }
    void timing(double* out16);

private:
    void build_spectra();
    void exchange(bool buffer_a, hipStream_t st);
    void exchange_planes(float* (*get)(SlabState&, bool), bool which, size_t plane_floats, hipStream_t st);
    // x-pass pair ranges of a slab: the planes its neighbours need (bnd) and the rest
    bool split_pairs(const SlabState& sl, PairRanges& bnd, PairRanges& rest) const;
    void run_rocfft(int iters, double lambda);
    void run_engine(int iters, double lambda);
    void allreduce_sum(double* host, int n);
    void allreduce_max(double* host, int n);
    void tstart(int cls, hipStream_t st = nullptr);
    void tstop(hipStream_t st = nullptr);

    mvd_params p_{};
    int backend_ = 0;  // 0 = fused spectral engine, 1 = rocFFT (mvd_params.fft_backend)
    Store store_ = Store::F32;
    hipStream_t stream_ = nullptr;
    hipStream_t xstream_ = nullptr;  // halo exchanges overlapped with the interior x pass
    hipEvent_t ev_bnd_ = nullptr, ev_x_ = nullptr;
    ncclComm_t comm_ = nullptr;
    std::vector<SlabState> slabs_;
    std::vector<HostKernel> k1_, k2_;
    int nviews_ = 0;
    int halo_[3] = {0, 0, 0};
    bool kernels_ready_ = false;
    bool spectra_ready_ = false;
    bool psi_ready_ = false;
    DBuf<double> stats_dev_;
    bool timing_on_ = false;
    std::vector<TimingRec> trecs_;
    int tcur_ = -1;
    double tacc_[16] = {0};
    std::vector<hipEvent_t> event_pool_;
    hipEvent_t get_event();
};

}  // namespace spimdecon
