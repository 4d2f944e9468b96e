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
// The volume is split into z-slabs (local virtual slabs, slabs on several
// devices of this process, and/or one slab range per RCCL rank); halos of c_z
// padded planes are exchanged after each pad.
//
// Several devices in one process (mvd_create_devices, the reference's
// MVDeconFFT(..., int[] deviceList, ...) driven from one JVM, MVDeconFFT.java:58-64,
// 424-446): each device group owns consecutive slabs, a stream and an exchange
// stream; mvd_run drives every group from its own host thread, and the halo planes
// are pulled from the neighbouring groups' HBM (peer copies over xGMI) between two
// host barriers per exchange (events recorded before any stream waits on them).
#pragma once

#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "fft.hpp"
#include "fftconv.hpp"
#include "kernel_prep.hpp"
#include "rl_kernels.hpp"

namespace spimdecon {

struct SlabState {
    int grp = 0;           // device group (index into Session::groups_)
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
    int weight = 1;   // whole-slab passes the interval covers (counted into the class)
};

// one device of a multi-device session (or the only one)
struct DevGroup {
    int dev = 0;
    int s0 = 0, s1 = 0;                    // slabs [s0, s1)
    hipStream_t stream = nullptr;
    hipStream_t xstream = nullptr;          // halo exchanges overlapped with the interior x pass
    hipEvent_t ev_bnd = nullptr, ev_x = nullptr;
    hipEvent_t ev_pre = nullptr, ev_bu = nullptr;  // (boundary x launches on xstream: cbnd_)
    DBuf<double> stats;                     // iters * V * {sum, max} of this group's slabs
};

// The halo transfers of one slab, as element offsets into its spectrum buffer (plane =
// elements per padded z-plane).  The slab's interior planes are [0, nz); its upper halo
// is [nz, nz + cz), its lower halo the wrapped planes [Mz - cz, Mz).
//   to / from the LOWER neighbour: send [0, cz) (send_lo), receive into recv_lo
//   to / from the UPPER neighbour: send [nz - cz, nz) (send_hi), receive into recv_hi
// One helper for every deployment: the local copies between slabs of a device, the
// device-group peer pulls and the RCCL send / recv all address the buffers through it,
// so the one-GPU device-group tests exercise the offsets RCCL uses.
struct HaloPlan {
    int64_t send_lo, recv_lo, send_hi, recv_hi, count;
};
HaloPlan halo_plan(int64_t nz, int64_t Mz, int64_t cz, int64_t plane);

// reusable host barrier for the group threads; abort() releases every waiter with an
// error so that one failing thread cannot deadlock the others
class HostBarrier {
public:
    explicit HostBarrier(int n) : n_(n) {}
    void wait();
    void abort();

private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0;
    uint64_t gen_ = 0;
    bool aborted_ = false;
};

class Session {
public:
    // devs: the device of each group (repeats allowed: groups sharing one GPU run the
    // multi-device code path on it); empty = {p.device}
    explicit Session(const mvd_params& p, const std::vector<int>& devs = {});
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
    int xpass_mode(int slab) const;
    hipStream_t stream() const { return groups_[0].stream; }
    int ndevices() const { return int(groups_.size()); }
    int nslabs() const { return int(slabs_.size()); }
    void slab_extent(int slab, int64_t* out3) const;
    // halo bytes / copies moved between slabs (local, peer or RCCL sends) since creation
    void exchange_stats(int64_t* bytes, int64_t* copies) const;
    int slab_device(int slab) const;
    void enable_timing(bool on) { timing_on_ = on; }
    void timing(double* out16);

private:
    void build_spectra();
    // original-layout volume (this rank's part, odims_) <-> slab sl in the internal
    // layout (f32, sl.n floats on the slab's device); y-split sessions transpose rows
    void load_slab(const float* src, hipMemcpyKind kind, const SlabState& sl, float* dst, DBuf<float>& tmp,
                   hipStream_t st) const;
    void store_slab(const SlabState& sl, const float* src, float* out, DBuf<float>& tmp, hipStream_t st) const;
    // kernel k in the internal axis order (y and z swapped for y-split sessions)
    HostKernel internal_kernel(const HostKernel& k) const;
    static float* buf_ptr(SlabState& sl, bool a, int backend);
    size_t plane_floats() const;
    // halo exchange of one buffer (C1/Ra when buffer_a) among the slabs of group gi and,
    // with one group, over RCCL; issued on st (single group)
    void exchange(bool buffer_a, hipStream_t st);
    // multi-group exchange protocol (called by every group thread in step)
    void group_exchange_begin(int gi, bool buffer_a, HostBarrier& bar);
    void group_exchange_end(int gi);
    // x-pass pair ranges of a slab: the planes its neighbours need (bnd) and the rest
    bool split_pairs(const SlabState& sl, PairRanges& bnd, PairRanges& rest) const;
    void run_rocfft(int iters, double lambda);
    // the engine schedule of group gi; bar == nullptr: the only group (RCCL halos)
    void run_engine(int gi, int iters, double lambda, HostBarrier* bar);
    void run_groups(int iters, double lambda);
    void sync_all();
    void allreduce_sum(double* host, int n);
    void allreduce_max(double* host, int n);
    void tstart(int cls, hipStream_t st = nullptr);
    void tstop(hipStream_t st = nullptr);
    // class 7: the overlap window of a halo exchange -- the compute stream's work queued
    // between the exchange's start and the wait for it (group 0's stream)
    void wstart(hipStream_t st);
    void wstop(hipStream_t st);
    // an interval of class cls covering `weight` whole-slab passes, independent of tcur_
    // (the concurrent boundary / rest x launches: one interval across both streams)
    int rstart(int cls, hipStream_t st, int weight);
    void rstop(int rec, hipStream_t st);
    int wcur_ = -1;

    mvd_params p_{};        // internal geometry (dims / halo with y and z swapped when axis_ == 1)
    int64_t odims_[3] = {0, 0, 0};  // this rank's volume in the caller's layout {nx, ny, nz}
    int axis_ = 0;          // slab axis: 0 = z, 1 = y (mvd_params.slab_axis)
    int backend_ = 0;  // 0 = fused spectral engine, 1 = rocFFT (mvd_params.fft_backend)
    Store store_ = Store::F32;
    std::vector<DevGroup> groups_;
    hipStream_t stream_ = nullptr;   // groups_[0].stream
    ncclComm_t comm_ = nullptr;
    std::vector<SlabState> slabs_;
    std::vector<HostKernel> k1_, k2_;
    int nviews_ = 0;
    int halo_[3] = {0, 0, 0};
    bool kernels_ready_ = false;
    bool spectra_ready_ = false;
    bool psi_ready_ = false;
    // a multi-device run aborted mid-iteration: the slabs hold psi of different
    // iterations, so nothing but destruction is allowed afterwards
    bool poisoned_ = false;
    bool warned_fallback_ = false;  // the Stockham-fallback warning is printed once
    // one device group with neighbours (RCCL ranks, local slabs): the boundary x launches
    // run on the exchange stream, concurrently with the rest of the x pass on the compute
    // stream, and the exchange follows them there (SPIMDECON_CBND=0: both on the compute
    // stream, the exchange after the boundary launches)
    bool cbnd_ = true;
    // halo copies between slabs of this process (local slabs, device-group peer pulls) by
    // a copy kernel instead of hipMemcpyAsync (SPIMDECON_PULL=kernel); RCCL is unaffected
    bool pull_kernel_ = false;
    void copy_halo(float* dst, const float* src, size_t bytes, hipStream_t st, bool peer);
    std::atomic<int64_t> xbytes_{0}, xcopies_{0};  // (group threads add concurrently)
    bool timing_on_ = false;
    std::vector<TimingRec> trecs_;
    int tcur_ = -1;
    double tacc_[16] = {0};
    std::vector<hipEvent_t> event_pool_;
    hipEvent_t get_event();

    // RCCL watchdog (nranks > 1).  Every host wait on a stream that RCCL work feeds is
    // bounded: when the stream's progress events (one per RL iteration) stop completing
    // for rccl_timeout_s_ seconds, or RCCL reports an asynchronous error, the communicator
    // is aborted (ncclCommAbort) and the call fails with SPIMDECON_ERR_COMM -- ranks whose
    // sends and receives do not match fail instead of waiting forever.
    double rccl_timeout_s_ = 300.0;  // SPIMDECON_RCCL_TIMEOUT (seconds)
    bool rccl_dead_ = false;          // aborted: the session's streams may hold dead work
    std::vector<hipEvent_t> progress_;  // recorded on the compute stream after each iteration
    size_t nprogress_ = 0;              // progress_ entries recorded in the current run
    void wait_stream(hipStream_t st);
    void record_progress(hipStream_t st);
    // all-gathers every rank's exchange geometry (RCCL) once the spectra are built and
    // fails on every rank when they disagree (counts, halo planes, z ranges, views)
    void verify_ranks();
};

}  // namespace spimdecon
