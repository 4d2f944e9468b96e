// session.cpp -- see session.hpp.
#include "session.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <exception>
#include <thread>

namespace spimdecon {

#define SD_NCCL(expr)                                                                          \
    do {                                                                                       \
        ncclResult_t _r = (expr);                                                              \
        if (_r != ncclSuccess)                                                                 \
            ::spimdecon::fail(SPIMDECON_ERR_COMM,                                              \
                              std::string(#expr " failed: ") + ncclGetErrorString(_r));        \
    } while (0)

void slab_range(int64_t nz, int nparts, int idx, int64_t* z0, int64_t* z1) {
    const int64_t base = nz / nparts, rem = nz % nparts;
    *z0 = int64_t(idx) * base + std::min<int64_t>(idx, rem);
    *z1 = *z0 + base + (idx < rem ? 1 : 0);
}

HaloPlan halo_plan(int64_t nz, int64_t Mz, int64_t cz, int64_t plane) {
    SD_CHECK(cz >= 0 && nz >= cz && Mz >= nz + 2 * cz && plane > 0, SPIMDECON_ERR_ARG, "bad halo geometry");
    HaloPlan h;
    h.send_lo = 0;
    h.recv_lo = (Mz - cz) * plane;
    h.send_hi = (nz - cz) * plane;
    h.recv_hi = nz * plane;
    h.count = cz * plane;
    return h;
}

void HostBarrier::wait() {
    std::unique_lock<std::mutex> lk(mu_);
    if (aborted_) fail(SPIMDECON_ERR_STATE, "device group aborted");
    const uint64_t gen = gen_;
    if (++count_ == n_) {
        count_ = 0;
        ++gen_;
        cv_.notify_all();
        return;
    }
    cv_.wait(lk, [&] { return gen_ != gen || aborted_; });
    if (gen_ == gen) fail(SPIMDECON_ERR_STATE, "device group aborted");
}

void HostBarrier::abort() {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
    cv_.notify_all();
}

// caller's geometry -> internal geometry: a y-split session swaps the roles of y
// and z (dims and halo), so the engine always slabs its outermost axis
static mvd_params internal_params(const mvd_params& p, int nslabs, int* axis) {
    SD_CHECK(p.slab_axis >= -1 && p.slab_axis <= 1, SPIMDECON_ERR_ARG, "slab_axis must be -1, 0 or 1");
    int a = p.slab_axis;
    // auto: split the longer of y and z (fewer halo rows per slab); an unsplit volume
    // keeps its own layout (no transposition)
    if (a == -1) a = (p.nranks == 1 && nslabs > 1 && p.dims[1] > p.dims[2]) ? 1 : 0;
    *axis = a;
    mvd_params q = p;
    if (a == 1) {
        std::swap(q.dims[1], q.dims[2]);
        std::swap(q.halo[1], q.halo[2]);
    }
    return q;
}

Session::Session(const mvd_params& p0, const std::vector<int>& devs) {
    for (int d = 0; d < 3; ++d) odims_[d] = p0.dims[d];
    p_ = internal_params(p0, int(std::max<size_t>(devs.size(), 1)) * std::max(p0.local_slabs, 1), &axis_);
    const mvd_params& p = p_;
    SD_CHECK(p.dims[0] >= 1 && p.dims[1] >= 1 && p.dims[2] >= 1, SPIMDECON_ERR_ARG, "bad dims");
    SD_CHECK(p.local_slabs >= 1, SPIMDECON_ERR_ARG, "local_slabs must be >= 1");
    SD_CHECK(p.nranks >= 1 && p.rank >= 0 && p.rank < p.nranks, SPIMDECON_ERR_ARG, "bad rank");
    SD_CHECK(p.ij_threads >= 1, SPIMDECON_ERR_ARG, "ij_threads must be >= 1");
    std::vector<int> dl = devs.empty() ? std::vector<int>{p.device} : devs;
    const int G = int(dl.size());
    SD_CHECK(G == 1 || p.nranks == 1, SPIMDECON_ERR_ARG,
             "several devices per process and several RCCL ranks cannot be combined");
    SD_CHECK(G == 1 || p.fft_backend == 0, SPIMDECON_ERR_ARG, "several devices need the engine backend");
    // Engine slabs whose buffers outgrow the 32-bit offsets of the fast passes (a 1024^3
    // psi is 2^32 B) are split further on their device: exact slabs with halos, the
    // same arithmetic as any other split.  Kernel half sizes are not known yet: up to
    // 16 (33-plane kernels) is assumed unless mvd_params.halo says more.  An automatic
    // split axis is re-decided for the new slab count (the longer of y and z).
    static const bool auto_slabs = [] {
        const char* e = std::getenv("SPIMDECON_AUTO_SLABS");
        return !(e && e[0] == '0');
    }();
    if (p0.fft_backend == 0 && auto_slabs && p0.local_slabs >= 1) {
        auto needed = [&](const mvd_params& q, int ls) {
            const int hal[3] = {std::max(q.halo[0], 16), std::max(q.halo[1], 16), std::max(q.halo[2], 16)};
            auto fits = [&](int64_t nzs) {
                return engine_slab_fits(q.dims[0], q.dims[1], nzs, hal, q.fft_pad_policy);
            };
            // when even one-plane slabs are past the fast passes' offsets no split helps:
            // keep the caller's slab count (the Stockham passes run it, as before)
            if (!fits(1)) return ls;
            while (int64_t(G) * ls < q.dims[2] && !fits(ceil_div(q.dims[2], int64_t(G) * ls))) ++ls;
            return ls;
        };
        int ls = needed(p_, p0.local_slabs);
        if (ls != p0.local_slabs && p0.slab_axis == -1) {
            p_ = internal_params(p0, G * ls, &axis_);
            ls = needed(p_, ls);
        }
        p_.local_slabs = ls;
    }
    const int nslabs = G * p.local_slabs;
    SD_CHECK(nslabs <= p.dims[2], SPIMDECON_ERR_ARG, "more slabs than z planes");
    if (p_.nz_global <= 0) p_.nz_global = p.dims[2];
    SD_CHECK(p_.z_offset >= 0 && p_.z_offset + p.dims[2] <= p_.nz_global, SPIMDECON_ERR_ARG,
             "z range outside nz_global");
    SD_CHECK(p_.nranks == 1 || p_.comm_id != nullptr, SPIMDECON_ERR_ARG,
             "nranks > 1 needs comm_id");
    for (int d : dl) check_device(d);
    p_.device = dl[0];
    store_ = p.storage_fp16 ? Store::F16 : Store::F32;
    backend_ = p.fft_backend;
    SD_CHECK(backend_ == 0 || backend_ == 1, SPIMDECON_ERR_ARG, "unknown fft_backend");
    groups_.resize(G);
    for (int gi = 0; gi < G; ++gi) {
        DevGroup& gr = groups_[gi];
        gr.dev = dl[gi];
        gr.s0 = gi * p.local_slabs;
        gr.s1 = gr.s0 + p.local_slabs;
        DeviceGuard guard(gr.dev);
        SD_HIP(hipStreamCreateWithFlags(&gr.stream, hipStreamNonBlocking));
        SD_HIP(hipStreamCreateWithFlags(&gr.xstream, hipStreamNonBlocking));
        SD_HIP(hipEventCreateWithFlags(&gr.ev_bnd, hipEventDisableTiming));
        SD_HIP(hipEventCreateWithFlags(&gr.ev_x, hipEventDisableTiming));
        SD_HIP(hipEventCreateWithFlags(&gr.ev_pre, hipEventDisableTiming));
        SD_HIP(hipEventCreateWithFlags(&gr.ev_bu, hipEventDisableTiming));
        // halo planes are pulled straight from the neighbours' HBM (xGMI peer access)
        for (int o : {gi - 1, gi + 1}) {
            if (o < 0 || o >= G || dl[o] == gr.dev) continue;
            int can = 0;
            SD_HIP(hipDeviceCanAccessPeer(&can, gr.dev, dl[o]));
            if (can) {
                const hipError_t e = hipDeviceEnablePeerAccess(dl[o], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) SD_HIP(e);
                (void)hipGetLastError();
            }
        }
    }
    stream_ = groups_[0].stream;
    if (const char* e = std::getenv("SPIMDECON_CBND")) cbnd_ = e[0] != '0';
    if (const char* e = std::getenv("SPIMDECON_PULL")) pull_kernel_ = e[0] == 'k';
    // a communicator for several ranks -- or for one when the caller passes an id (the
    // single-GPU tests run the collectives and the watchdog through RCCL that way)
    if (p_.nranks > 1 || p_.comm_id != nullptr) {
        if (const char* e = std::getenv("SPIMDECON_RCCL_TIMEOUT")) rccl_timeout_s_ = std::max(1.0, std::atof(e));
        DeviceGuard guard(p_.device);
        ncclUniqueId id;
        std::memcpy(&id, p_.comm_id, sizeof(id));
        SD_NCCL(ncclCommInitRank(&comm_, p_.nranks, id, p_.rank));
        p_.comm_id = nullptr;  // caller-owned; not retained
    }
    slabs_.resize(nslabs);
    for (int s = 0; s < nslabs; ++s) {
        int64_t a, b;
        slab_range(p.dims[2], nslabs, s, &a, &b);
        SlabState& sl = slabs_[s];
        sl.grp = s / p.local_slabs;
        sl.local_z0 = a;
        sl.g.nx = p.dims[0];
        sl.g.ny = p.dims[1];
        sl.g.nz = b - a;
        sl.g.z0 = p_.z_offset + a;
        sl.g.nzg = p_.nz_global;
        sl.n = sl.g.nx * sl.g.ny * sl.g.nz;
    }
}

Session::~Session() {
    if (rccl_dead_) {
        // an aborted communicator: its kernels should drain; if a stream still holds work
        // after 30 s, leak the buffers rather than block in hipFree (the process is failing)
        bool busy = false;
        for (auto& gr : groups_) {
            DeviceGuard guard(gr.dev);
            for (hipStream_t st : {gr.stream, gr.xstream}) {
                const auto t0 = std::chrono::steady_clock::now();
                while (st && hipStreamQuery(st) == hipErrorNotReady) {
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
                        busy = true;
                        break;
                    }
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                }
            }
        }
        if (busy) {
            new std::vector<SlabState>(std::move(slabs_));   // intentionally leaked
            new std::vector<DevGroup>(std::move(groups_));
            return;
        }
    }
    for (auto& gr : groups_) {
        DeviceGuard guard(gr.dev);
        if (gr.stream) (void)hipStreamSynchronize(gr.stream);
        if (gr.xstream) (void)hipStreamSynchronize(gr.xstream);
    }
    {
        DeviceGuard guard(p_.device);
        for (auto& r : trecs_) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto e : event_pool_) (void)hipEventDestroy(e);
        for (auto e : progress_) (void)hipEventDestroy(e);
        if (comm_) ncclCommDestroy(comm_);
    }
    for (auto& sl : slabs_) {  // buffers and plans released on their own device
        DeviceGuard guard(groups_[sl.grp].dev);
        sl = SlabState{};
    }
    for (auto& gr : groups_) {
        DeviceGuard guard(gr.dev);
        gr.stats.release();
        if (gr.ev_bnd) (void)hipEventDestroy(gr.ev_bnd);
        if (gr.ev_x) (void)hipEventDestroy(gr.ev_x);
        if (gr.ev_pre) (void)hipEventDestroy(gr.ev_pre);
        if (gr.ev_bu) (void)hipEventDestroy(gr.ev_bu);
        if (gr.xstream) (void)hipStreamDestroy(gr.xstream);
        if (gr.stream) (void)hipStreamDestroy(gr.stream);
    }
}

int Session::slab_device(int slab) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    return groups_[slabs_[slab].grp].dev;
}

void Session::exchange_stats(int64_t* bytes, int64_t* copies) const {
    if (bytes) *bytes = xbytes_.load();
    if (copies) *copies = xcopies_.load();
}

void Session::slab_extent(int slab, int64_t* out3) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    const SlabGeom& g = slabs_[slab].g;
    out3[0] = g.nx;
    out3[1] = g.ny;
    out3[2] = g.nz;
}

void Session::sync_all() {
    for (auto& gr : groups_) {
        DeviceGuard guard(gr.dev);
        wait_stream(gr.stream);
        wait_stream(gr.xstream);
    }
}

void Session::load_slab(const float* src, hipMemcpyKind kind, const SlabState& sl, float* dst, DBuf<float>& tmp,
                        hipStream_t st) const {
    const int64_t nx = odims_[0], ny = odims_[1], nz = odims_[2];
    if (axis_ == 0) {
        SD_HIP(hipMemcpyAsync(dst, src + sl.local_z0 * nx * ny, size_t(sl.n) * 4, kind, st));
        return;
    }
    // y rows [y0, y0 + ys) of every z plane -> tmp [nz][ys][nx] -> dst [ys][nz][nx]
    const int64_t y0 = sl.local_z0, ys = sl.g.nz;
    if (tmp.n < size_t(sl.n)) tmp.alloc(sl.n);
    SD_HIP(hipMemcpy2DAsync(tmp.p, size_t(ys * nx) * 4, src + y0 * nx, size_t(ny * nx) * 4, size_t(ys * nx) * 4,
                            size_t(nz), kind, st));
    launch_swap_outer(tmp.p, dst, nx, ys, nz, st);
}

void Session::store_slab(const SlabState& sl, const float* src, float* out, DBuf<float>& tmp, hipStream_t st) const {
    const int64_t nx = odims_[0], ny = odims_[1], nz = odims_[2];
    if (axis_ == 0) {
        SD_HIP(hipMemcpyAsync(out + sl.local_z0 * nx * ny, src, size_t(sl.n) * 4, hipMemcpyDefault, st));
        return;
    }
    const int64_t y0 = sl.local_z0, ys = sl.g.nz;
    if (tmp.n < size_t(sl.n)) tmp.alloc(sl.n);
    launch_swap_outer(src, tmp.p, nx, nz, ys, st);  // [ys][nz][nx] -> [nz][ys][nx]
    SD_HIP(hipMemcpy2DAsync(out + y0 * nx, size_t(ny * nx) * 4, tmp.p, size_t(ys * nx) * 4, size_t(ys * nx) * 4,
                            size_t(nz), hipMemcpyDefault, st));
}

HostKernel Session::internal_kernel(const HostKernel& k) const {
    if (axis_ == 0) return k;
    HostKernel o;
    const int kx = k.dims[0], ky = k.dims[1], kz = k.dims[2];
    o.dims[0] = kx;
    o.dims[1] = kz;
    o.dims[2] = ky;
    o.data.resize(k.data.size());
    for (int z = 0; z < kz; ++z)
        for (int y = 0; y < ky; ++y)
            std::copy(k.data.begin() + (int64_t(z) * ky + y) * kx, k.data.begin() + (int64_t(z) * ky + y + 1) * kx,
                      o.data.begin() + (int64_t(y) * kz + z) * kx);
    return o;
}

void Session::add_view(const float* img, const float* weight, const float* k1, const int* kdims,
                       bool device_ptrs) {
    SD_CHECK(img && weight && k1 && kdims, SPIMDECON_ERR_ARG, "null argument");
    SD_CHECK(!spectra_ready_, SPIMDECON_ERR_STATE, "views must be added before mvd_init");
    HostKernel hk;
    for (int d = 0; d < 3; ++d) {
        SD_CHECK(kdims[d] >= 1 && (kdims[d] & 1), SPIMDECON_ERR_ARG, "kernel dims must be odd");
        hk.dims[d] = kdims[d];
    }
    hk.data.assign(k1, k1 + int64_t(kdims[0]) * kdims[1] * kdims[2]);
    // device pointers live on the first device; other groups copy them peer to peer
    const hipMemcpyKind kind = device_ptrs ? hipMemcpyDefault : hipMemcpyHostToDevice;
    if (device_ptrs) {
        // the caller may still be writing them on another stream (torch's default stream
        // does not order against the session's non-blocking streams): wait for the device
        DeviceGuard guard(p_.device);
        SD_HIP(hipDeviceSynchronize());
    }
    std::vector<std::vector<DBuf<char>>> bufs(slabs_.size());
    for (auto& gr : groups_) {
        DeviceGuard guard(gr.dev);
        DBuf<float> tmp, f32;
        for (int s = gr.s0; s < gr.s1; ++s) {
            SlabState& sl = slabs_[s];
            const size_t esz = store_ == Store::F32 ? 4 : 2;
            for (int which = 0; which < 2; ++which) {
                const float* src = which == 0 ? img : weight;
                DBuf<char> buf(size_t(sl.n) * esz);
                if (store_ == Store::F32) {
                    load_slab(src, kind, sl, reinterpret_cast<float*>(buf.p), tmp, gr.stream);
                } else {
                    if (f32.n < size_t(sl.n)) f32.alloc(sl.n);
                    load_slab(src, kind, sl, f32.p, tmp, gr.stream);
                    launch_to_half(f32.p, buf.p, sl.n, gr.stream);
                }
                bufs[s].push_back(std::move(buf));
            }
        }
        wait_stream(gr.stream);
    }
    for (size_t s = 0; s < slabs_.size(); ++s) {
        slabs_[s].img.push_back(std::move(bufs[s][0]));
        slabs_[s].w.push_back(std::move(bufs[s][1]));
    }
    k1_.push_back(std::move(hk));
    ++nviews_;
    kernels_ready_ = false;
}

void Session::init(int psftype) {
    SD_CHECK(nviews_ >= 1, SPIMDECON_ERR_STATE, "no views added");
    std::vector<HostKernel> k1 = k1_;
    prepare_kernels_gpu(k1, k2_, psftype, p_.ij_threads, p_.device);
    k1_ = std::move(k1);
    kernels_ready_ = true;
    build_spectra();
}

void Session::set_kernels(int view, const float* k1, const float* k2) {
    SD_CHECK(view >= 0 && view < nviews_, SPIMDECON_ERR_ARG, "bad view index");
    SD_CHECK(k1 && k2, SPIMDECON_ERR_ARG, "null kernel");
    if (k2_.size() != size_t(nviews_)) k2_.resize(nviews_);
    const int64_t n = int64_t(k1_[view].dims[0]) * k1_[view].dims[1] * k1_[view].dims[2];
    k1_[view].data.assign(k1, k1 + n);
    std::memcpy(k2_[view].dims, k1_[view].dims, sizeof(k1_[view].dims));
    k2_[view].data.assign(k2, k2 + n);
    spectra_ready_ = false;
    bool all = true;
    for (auto& k : k2_) all &= !k.data.empty();
    if (all) {
        kernels_ready_ = true;
        build_spectra();
    }
}

void Session::get_kernels(int view, float* k1, float* k2) const {
    SD_CHECK(kernels_ready_, SPIMDECON_ERR_STATE, "kernels not prepared");
    SD_CHECK(view >= 0 && view < nviews_, SPIMDECON_ERR_ARG, "bad view index");
    if (k1) std::copy(k1_[view].data.begin(), k1_[view].data.end(), k1);
    if (k2) std::copy(k2_[view].data.begin(), k2_[view].data.end(), k2);
}

void Session::build_spectra() {
    // kernels in the internal axis order (prepared in the caller's order: the normImg
    // portions of AdjustInput.java:93-97 follow the original flat order)
    std::vector<HostKernel> ik1(nviews_), ik2(nviews_);
    for (int v = 0; v < nviews_; ++v) {
        ik1[v] = internal_kernel(k1_[v]);
        ik2[v] = internal_kernel(k2_[v]);
    }
    int h[3] = {0, 0, 0};
    for (int v = 0; v < nviews_; ++v)
        for (int d = 0; d < 3; ++d) h[d] = std::max(h[d], ik1[v].dims[d] / 2);
    for (int d = 0; d < 3; ++d) halo_[d] = std::max(h[d], p_.halo[d]);
    const int total_slabs = int(slabs_.size()) * p_.nranks;
    const EngineKnobs knobs = EngineKnobs::from_env();   // read once: sizing and plans agree
    for (auto& sl : slabs_) {
        DeviceGuard guard(groups_[sl.grp].dev);
        hipStream_t stream_ = groups_[sl.grp].stream;  // this slab's device stream
        SlabGeom& g = sl.g;
        g.cx = halo_[0];
        g.cy = halo_[1];
        g.cz = halo_[2];
        if (total_slabs > 1)
            SD_CHECK(g.nz >= g.cz + 1, SPIMDECON_ERR_ARG,
                     "slab thinner than kernel half size + 1 (" + std::to_string(g.nz) + " < " +
                         std::to_string(g.cz + 1) + ")");
        const int pol = backend_ == 1 ? 2 : p_.fft_pad_policy;
        sl.pd.M[0] = engine_fast_size(g.nx + 2 * g.cx, true, pol);
        sl.pd.M[1] = engine_fast_size(g.ny + 2 * g.cy, false, pol);
        sl.pd.M[2] = engine_fast_size(g.nz + 2 * g.cz, false, pol);
        // the direct z convolution needs no z FFT: Mz = nz + 2 cz exactly (unless the
        // full kernel spectra are asked for, SPIMDECON_ZK=full/reg)
        const char* zk = std::getenv("SPIMDECON_ZK");
        const bool zk_full = zk && (zk[0] == 'f' || zk[0] == 'r');
        sl.zexact = backend_ == 0 && !zk_full &&
                    engine_zdirect_dims_ok(sl.pd.M[0], sl.pd.M[1], g.nz + 2 * g.cz, g.cz, knobs.zdirect);
        if (sl.zexact) sl.pd.M[2] = g.nz + 2 * g.cz;
        g.Mx = sl.pd.M[0];
        g.My = sl.pd.M[1];
        g.Mz = sl.pd.M[2];
        g.Sx = sl.pd.Sx();
        // stats partials: one {sum, max} per x-pass block; the x tiles may run one
        // tile (>= 1 row pair) per block, split over two launches (boundary + rest)
        sl.partials.alloc(size_t(2) * std::max<int64_t>(256 * 16, (g.My * g.Mz + 1) / 2 + 64));
        std::vector<const void*> ptrs(nviews_);
        for (int v = 0; v < nviews_; ++v) ptrs[v] = sl.img[v].p;
        sl.img_ptrs.alloc(nviews_);
        SD_HIP(hipMemcpyAsync(sl.img_ptrs.p, ptrs.data(), nviews_ * sizeof(void*),
                              hipMemcpyHostToDevice, stream_));
        const float scale = float(1.0 / double(sl.pd.logical()));
        DBuf<float> kd;  // this slab's device
        if (backend_ == 1) {
            const size_t rf = size_t(sl.pd.real_floats());
            sl.Ra.alloc(rf);
            sl.Rb.alloc(rf);
            sl.fft.reset(new FftPlan3D());
            sl.fft->create(sl.pd, stream_);
            sl.k1spec.clear();
            sl.k2spec.clear();
            for (int v = 0; v < nviews_; ++v) {
                for (int which = 0; which < 2; ++which) {
                    const HostKernel& hk = which == 0 ? ik1[v] : ik2[v];
                    kd.alloc(hk.data.size());
                    SD_HIP(hipMemcpyAsync(kd.p, hk.data.data(), kd.bytes(), hipMemcpyHostToDevice, stream_));
                    DBuf<float> spec(rf);
                    launch_place_kernel(g, kd.p, hk.dims[0], hk.dims[1], hk.dims[2], scale, spec.p, stream_);
                    sl.fft->forward(spec.p);
                    wait_stream(stream_);
                    (which == 0 ? sl.k1spec : sl.k2spec).push_back(std::move(spec));
                }
            }
        } else {
            sl.sp.create(g, p_.fft_pad_policy != 2, !sl.zexact, knobs);
            const size_t ne = size_t(sl.sp.spectrum_elems());
            sl.C1.alloc(ne);
            sl.C2.alloc(ne);
            SD_HIP(hipMemsetAsync(sl.C1.p, 0, sl.C1.bytes(), stream_));
            SD_HIP(hipMemsetAsync(sl.C2.p, 0, sl.C2.bytes(), stream_));
            sl.e1spec.clear();
            sl.e2spec.clear();
            // compact kernels (2cz+1 z-planes, z transform in the z pass) unless
            // SPIMDECON_ZK=full / =reg asks for the full spectra (A/B runs)
            const char* zk = std::getenv("SPIMDECON_ZK");  // read per session (tests toggle it)
            const bool full_k = zk && (zk[0] == 'f' || zk[0] == 'r');
            sl.kcompact = !full_k && (engine_zdirect_ok(sl.sp) || engine_kernel_compact_ok(sl.sp));
            SD_CHECK(!sl.zexact || (sl.kcompact && engine_zdirect_ok(sl.sp)), SPIMDECON_ERR_STATE,
                     "exact-Mz slab without the direct z pass");
            DBuf<float2> work;
            if (sl.kcompact) work.alloc(ne);
            for (int v = 0; v < nviews_; ++v) {
                for (int which = 0; which < 2; ++which) {
                    const HostKernel& hk = which == 0 ? ik1[v] : ik2[v];
                    kd.alloc(hk.data.size());
                    SD_HIP(hipMemcpyAsync(kd.p, hk.data.data(), kd.bytes(), hipMemcpyHostToDevice, stream_));
                    DBuf<float2> spec;
                    if (sl.kcompact) {
                        spec.alloc(size_t(engine_kernel_compact_elems(sl.sp)));
                        engine_kernel_compact(sl.sp, kd.p, hk.dims[0], hk.dims[1], hk.dims[2], scale, work.p,
                                              spec.p, stream_);
                    } else {
                        spec.alloc(ne);
                        engine_kernel_spectrum(sl.sp, kd.p, hk.dims[0], hk.dims[1], hk.dims[2], scale, spec.p,
                                               stream_);
                    }
                    (which == 0 ? sl.e1spec : sl.e2spec).push_back(std::move(spec));
                }
            }
        }
        wait_stream(stream_);
    }
    spectra_ready_ = true;
    verify_ranks();
}

double Session::init_psi(const float* psi_or_null) {
    SD_CHECK(nviews_ >= 1, SPIMDECON_ERR_STATE, "no views added");
    double avg = std::nan("");
    for (auto& sl : slabs_) {
        DeviceGuard guard(groups_[sl.grp].dev);
        hipStream_t st = groups_[sl.grp].stream;
        if (!sl.psi_a.p) {
            sl.psi_a.alloc(sl.n);
            sl.psi_b.alloc(sl.n);
        }
        sl.psi = sl.psi_a.p;
        sl.psi_next = sl.psi_b.p;
        if (sl.img_ptrs.n != size_t(nviews_)) {
            std::vector<const void*> ptrs(nviews_);
            for (int v = 0; v < nviews_; ++v) ptrs[v] = sl.img[v].p;
            sl.img_ptrs.alloc(nviews_);
            SD_HIP(hipMemcpyAsync(sl.img_ptrs.p, ptrs.data(), nviews_ * sizeof(void*),
                                  hipMemcpyHostToDevice, st));
            wait_stream(st);
        }
    }
    if (psi_or_null) {
        for (auto& sl : slabs_) {
            DeviceGuard guard(groups_[sl.grp].dev);
            hipStream_t st = groups_[sl.grp].stream;
            DBuf<float> tmp;
            load_slab(psi_or_null, hipMemcpyHostToDevice, sl, sl.psi, tmp, st);
            launch_clamp_min(sl.psi, sl.n, st);
            wait_stream(st);
        }
    } else {
        // FirstIteration + fuseFirstIteration (MVDeconvolution.java:192-235)
        double acc[2] = {0.0, 0.0};
        std::vector<double> part;
        for (auto& sl : slabs_) {
            DeviceGuard guard(groups_[sl.grp].dev);
            hipStream_t st = groups_[sl.grp].stream;
            DBuf<double> dpart(2 * 2048);
            const int64_t nb = launch_first_iteration(sl.n, nviews_, store_, sl.img_ptrs.p, dpart.p, st);
            part.resize(2 * nb);
            SD_HIP(hipMemcpyAsync(part.data(), dpart.p, part.size() * 8, hipMemcpyDeviceToHost, st));
            wait_stream(st);
            for (int64_t i = 0; i < nb; ++i) {
                acc[0] += part[2 * i];
                acc[1] += part[2 * i + 1];
            }
        }
        allreduce_sum(acc, 2);
        avg = acc[0] / acc[1];  // NaN when no voxel has data
        const double a = std::isnan(avg) ? 0.5 : avg;  // :117-121
        for (auto& sl : slabs_) {
            DeviceGuard guard(groups_[sl.grp].dev);
            launch_fill(sl.psi, sl.n, float(a), groups_[sl.grp].stream);
        }
    }
    sync_all();
    psi_ready_ = true;
    poisoned_ = false;  // every slab holds the same (new) starting psi again
    return avg;
}

hipEvent_t Session::get_event() {
    if (!event_pool_.empty()) {
        hipEvent_t e = event_pool_.back();
        event_pool_.pop_back();
        return e;
    }
    hipEvent_t e;
    SD_HIP(hipEventCreate(&e));
    return e;
}

void Session::tstart(int cls, hipStream_t st) {
    if (!timing_on_) return;
    TimingRec r{cls, get_event(), nullptr};
    SD_HIP(hipEventRecord(r.a, st ? st : stream_));
    trecs_.push_back(r);
    tcur_ = int(trecs_.size()) - 1;
}

void Session::tstop(hipStream_t st) {
    if (!timing_on_ || tcur_ < 0) return;
    trecs_[tcur_].b = get_event();
    SD_HIP(hipEventRecord(trecs_[tcur_].b, st ? st : stream_));
    tcur_ = -1;
}

void Session::wstart(hipStream_t st) {
    if (!timing_on_) return;
    TimingRec r{7, get_event(), nullptr};
    SD_HIP(hipEventRecord(r.a, st));
    trecs_.push_back(r);
    wcur_ = int(trecs_.size()) - 1;
}

void Session::wstop(hipStream_t st) {
    if (!timing_on_ || wcur_ < 0) return;
    trecs_[wcur_].b = get_event();
    SD_HIP(hipEventRecord(trecs_[wcur_].b, st));
    wcur_ = -1;
}

int Session::rstart(int cls, hipStream_t st, int weight) {
    if (!timing_on_) return -1;
    TimingRec r{cls, get_event(), nullptr, weight};
    SD_HIP(hipEventRecord(r.a, st));
    trecs_.push_back(r);
    return int(trecs_.size()) - 1;
}

void Session::rstop(int rec, hipStream_t st) {
    if (!timing_on_ || rec < 0) return;
    trecs_[rec].b = get_event();
    SD_HIP(hipEventRecord(trecs_[rec].b, st));
}

void Session::timing(double* out16) {
    for (int i = 0; i < 16; ++i) out16[i] = tacc_[i];
}

float* Session::buf_ptr(SlabState& sl, bool a, int backend) {
    if (backend == 1) return a ? sl.Ra.p : sl.Rb.p;
    return reinterpret_cast<float*>(a ? sl.C1.p : sl.C2.p);
}

size_t Session::plane_floats() const {
    if (backend_ == 1) return size_t(slabs_[0].g.Sx * slabs_[0].g.My);
    return size_t(2 * slabs_[0].sp.Hp * slabs_[0].g.My);
}

bool Session::split_pairs(const SlabState& sl, PairRanges& bnd, PairRanges& rest) const {
    const int64_t My = sl.g.My, nz = sl.g.nz, cz = halo_[2];
    const int64_t npairs = (My * sl.g.Mz + 1) / 2;
    const int64_t e1 = ceil_div(cz * My, int64_t(2));   // pairs holding planes [0, cz)
    const int64_t s2 = ((nz - cz) * My) / 2;            // ... planes [nz - cz, nz)
    const int64_t e2 = ceil_div(nz * My, int64_t(2));
    if (cz <= 0 || s2 < e1) return false;
    bnd.b0 = 0;
    bnd.n0 = int(e1);
    bnd.b1 = int(s2);
    bnd.n1 = int(e2 - s2);
    rest.b0 = int(e1);
    rest.n0 = int(s2 - e1);
    rest.b1 = int(e2);
    rest.n1 = int(npairs - e2);
    // Halo planes the neighbours provide ([nz, nz + cz) from the upper one, [Mz - cz, Mz)
    // from the lower one) are skip rows: the x pass would transform zeros and store
    // nothing there, so their pairs are left out (an interior slab of C3's 8-rank split:
    // 24 of 152 planes).  Halo planes at the global boundary are mirror rows and stay.
    if (sl.g.Mz == nz + 2 * cz) {
        const bool hi_skip = sl.g.z0 + nz < sl.g.nzg;   // an upper neighbour exists
        const bool lo_skip = sl.g.z0 > 0;               // a lower neighbour exists
        const int64_t m0 = ((nz + cz) * My) / 2;             // first pair touching plane nz + cz
        const int64_t m1 = ceil_div((nz + cz) * My, int64_t(2));   // pairs past plane nz + cz - 1
        if (hi_skip && lo_skip) {
            rest.n1 = 0;
        } else if (hi_skip) {
            rest.b1 = int(m0);
            rest.n1 = int(npairs - m0);
        } else if (lo_skip) {
            rest.n1 = int(m1 - e2);
        }
    }
    return true;
}

// halo exchange of cz padded z-planes between neighbouring slabs of the only device
// group (local copies) and with the neighbouring RCCL ranks
void Session::exchange(bool which, hipStream_t st) {
    const int S = int(slabs_.size());
    if (S == 1 && p_.nranks == 1) return;
    const int cz = halo_[2];
    if (cz <= 0) return;
    const int64_t plane = int64_t(plane_floats());
    auto get = [&](SlabState& sl) { return buf_ptr(sl, which, backend_); };
    auto hp = [&](const SlabState& sl) { return halo_plan(sl.g.nz, sl.g.Mz, cz, plane); };
    tstart(5, st);
    const size_t bytes = size_t(cz) * size_t(plane) * sizeof(float);
    for (int s = 1; s < S; ++s) {
        SlabState& lo = slabs_[s - 1];
        SlabState& hi = slabs_[s];
        const HaloPlan hl = hp(lo), hh = hp(hi);
        // hi's first cz planes -> lo's upper halo
        copy_halo(get(lo) + hl.recv_hi, get(hi) + hh.send_lo, bytes, st, false);
        // lo's last cz planes -> hi's lower halo
        copy_halo(get(hi) + hh.recv_lo, get(lo) + hl.send_hi, bytes, st, false);
    }
    xbytes_ += int64_t(2) * (S - 1) * int64_t(bytes);
    xcopies_ += int64_t(2) * (S - 1);
    if (p_.nranks > 1) {
        const size_t count = size_t(cz) * size_t(plane);
        SD_NCCL(ncclGroupStart());
        if (p_.rank > 0) {
            SlabState& s0 = slabs_[0];
            const HaloPlan h = hp(s0);
            SD_NCCL(ncclSend(get(s0) + h.send_lo, count, ncclFloat, p_.rank - 1, comm_, st));
            SD_NCCL(ncclRecv(get(s0) + h.recv_lo, count, ncclFloat, p_.rank - 1, comm_, st));
        }
        if (p_.rank < p_.nranks - 1) {
            SlabState& sl = slabs_[S - 1];
            const HaloPlan h = hp(sl);
            SD_NCCL(ncclSend(get(sl) + h.send_hi, count, ncclFloat, p_.rank + 1, comm_, st));
            SD_NCCL(ncclRecv(get(sl) + h.recv_hi, count, ncclFloat, p_.rank + 1, comm_, st));
        }
        SD_NCCL(ncclGroupEnd());
        const int nsend = (p_.rank > 0 ? 1 : 0) + (p_.rank < p_.nranks - 1 ? 1 : 0);
        xbytes_ += int64_t(nsend) * int64_t(count * sizeof(float));
        xcopies_ += nsend;
    }
    tstop(st);
}

// One halo transfer between slabs of this process.  hipMemcpyAsync: between two GPUs a
// peer copy (ROCm runs it on an SDMA engine unless HSA_ENABLE_SDMA=0), on one GPU a blit
// kernel; SPIMDECON_PULL=kernel: k_pull_copy on the receiving device's stream, whose
// loads read the sender's HBM over xGMI (peer access is enabled between neighbours).
void Session::copy_halo(float* dst, const float* src, size_t bytes, hipStream_t st, bool peer) {
    if (pull_kernel_) launch_pull_copy(dst, src, bytes, st);
    else SD_HIP(hipMemcpyAsync(dst, src, bytes, peer ? hipMemcpyDefault : hipMemcpyDeviceToDevice, st));
}

// Multi-device exchange, run by every group thread at the same point of the schedule.
// (1) each group marks its boundary planes written (ev_bnd); barrier, so every event
// is recorded before anyone waits on it; (2) each group's exchange stream waits for
// its own and its neighbours' boundary events and PULLS the halo planes of its own
// slabs (peer reads over xGMI; local copies between slabs of one device); barrier.
// group_exchange_end: the compute stream waits for its own pulls and for the
// neighbours' pulls out of its buffer (which its next x pass overwrites).
void Session::group_exchange_begin(int gi, bool which, HostBarrier& bar) {
    DevGroup& gr = groups_[gi];
    const int G = int(groups_.size());
    const int S = int(slabs_.size());
    const int cz = halo_[2];
    SD_HIP(hipEventRecord(gr.ev_bnd, gr.stream));
    bar.wait();
    for (int o : {gi - 1, gi, gi + 1})
        if (o >= 0 && o < G) SD_HIP(hipStreamWaitEvent(gr.xstream, groups_[o].ev_bnd, 0));
    if (gi == 0) tstart(5, gr.xstream);
    if (cz > 0) {
        const int64_t plane = int64_t(plane_floats());
        const size_t bytes = size_t(cz) * size_t(plane) * sizeof(float);
        for (int s = gr.s0; s < gr.s1; ++s) {
            SlabState& me = slabs_[s];
            const HaloPlan hm = halo_plan(me.g.nz, me.g.Mz, cz, plane);
            if (s > 0) {  // lower neighbour's last cz planes -> my lower halo
                SlabState& lo = slabs_[s - 1];
                const HaloPlan hl = halo_plan(lo.g.nz, lo.g.Mz, cz, plane);
                copy_halo(buf_ptr(me, which, backend_) + hm.recv_lo, buf_ptr(lo, which, backend_) + hl.send_hi,
                          bytes, gr.xstream, true);
            }
            if (s < S - 1) {  // upper neighbour's first cz planes -> my upper halo
                SlabState& hi = slabs_[s + 1];
                const HaloPlan hh = halo_plan(hi.g.nz, hi.g.Mz, cz, plane);
                copy_halo(buf_ptr(me, which, backend_) + hm.recv_hi, buf_ptr(hi, which, backend_) + hh.send_lo,
                          bytes, gr.xstream, true);
            }
            const int npull = (s > 0 ? 1 : 0) + (s < S - 1 ? 1 : 0);
            xbytes_ += int64_t(npull) * int64_t(bytes);
            xcopies_ += npull;
        }
    }
    if (gi == 0) tstop(gr.xstream);
    SD_HIP(hipEventRecord(gr.ev_x, gr.xstream));
    bar.wait();
}

void Session::group_exchange_end(int gi) {
    DevGroup& gr = groups_[gi];
    const int G = int(groups_.size());
    for (int o : {gi - 1, gi, gi + 1})
        if (o >= 0 && o < G) SD_HIP(hipStreamWaitEvent(gr.stream, groups_[o].ev_x, 0));
}

void Session::allreduce_sum(double* host, int n) {
    if (!comm_) return;
    DeviceGuard guard(p_.device);
    DBuf<double> d(n);
    SD_HIP(hipMemcpyAsync(d.p, host, n * 8, hipMemcpyHostToDevice, stream_));
    SD_NCCL(ncclAllReduce(d.p, d.p, n, ncclDouble, ncclSum, comm_, stream_));
    SD_HIP(hipMemcpyAsync(host, d.p, n * 8, hipMemcpyDeviceToHost, stream_));
    wait_stream(stream_);
}

void Session::allreduce_max(double* host, int n) {
    if (!comm_) return;
    DeviceGuard guard(p_.device);
    DBuf<double> d(n);
    SD_HIP(hipMemcpyAsync(d.p, host, n * 8, hipMemcpyHostToDevice, stream_));
    SD_NCCL(ncclAllReduce(d.p, d.p, n, ncclDouble, ncclMax, comm_, stream_));
    SD_HIP(hipMemcpyAsync(host, d.p, n * 8, hipMemcpyDeviceToHost, stream_));
    wait_stream(stream_);
}

void Session::record_progress(hipStream_t st) {
    // (one device group: with several, run_engine runs on a thread per group and only the
    // RCCL-free device-group exchange is used)
    if (!comm_ || groups_.size() > 1) return;
    if (nprogress_ == progress_.size()) {
        hipEvent_t e;
        SD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        progress_.push_back(e);
    }
    SD_HIP(hipEventRecord(progress_[nprogress_++], st));
}

void Session::wait_stream(hipStream_t st) {
    if (!comm_) {
        SD_HIP(hipStreamSynchronize(st));
        return;
    }
    using clk = std::chrono::steady_clock;
    auto last = clk::now();
    size_t done = 0;   // progress events seen complete
    int spins = 0;
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) SD_HIP(e);
        while (done < nprogress_ && hipEventQuery(progress_[done]) == hipSuccess) {
            ++done;
            last = clk::now();
        }
        ncclResult_t ar = ncclSuccess;
        (void)ncclCommGetAsyncError(comm_, &ar);
        const double idle = std::chrono::duration<double>(clk::now() - last).count();
        if ((ar != ncclSuccess && ar != ncclInProgress) || idle > rccl_timeout_s_) {
            const std::string why = ar != ncclSuccess && ar != ncclInProgress
                                        ? std::string("RCCL asynchronous error: ") + ncclGetErrorString(ar)
                                        : "no progress for " + std::to_string(int(idle)) +
                                              " s (SPIMDECON_RCCL_TIMEOUT): mismatched halo exchanges across ranks?";
            (void)ncclCommAbort(comm_);
            comm_ = nullptr;
            rccl_dead_ = true;
            poisoned_ = true;
            fail(SPIMDECON_ERR_COMM, "rank " + std::to_string(p_.rank) + ": " + why + "; communicator aborted");
        }
        // spin briefly (a run's last iteration usually ends within microseconds), then sleep
        if (++spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (st == stream_) nprogress_ = 0;
}

// the exchange geometry of this rank, all-gathered; refused on every rank when any two
// ranks' sends and receives could not match (they would wait for each other forever)
void Session::verify_ranks() {
    if (!comm_) return;
    constexpr int K = 12;
    int64_t ext = 0;
    for (auto& sl : slabs_) ext += sl.g.nz;
    const int64_t mine[K] = {0x5350494d44454301LL, p_.nranks, p_.rank, p_.nz_global, p_.z_offset, ext,
                             int64_t(axis_), int64_t(store_ == Store::F16), int64_t(backend_), int64_t(nviews_),
                             int64_t(halo_[2]), int64_t(plane_floats())};
    DeviceGuard guard(p_.device);
    const int R = p_.nranks;
    DBuf<int64_t> d(size_t(K) * R);
    std::vector<int64_t> all(size_t(K) * R, 0);
    SD_HIP(hipMemcpyAsync(d.p + size_t(K) * p_.rank, mine, sizeof(mine), hipMemcpyHostToDevice, stream_));
    SD_NCCL(ncclAllGather(d.p + size_t(K) * p_.rank, d.p, K, ncclInt64, comm_, stream_));
    SD_HIP(hipMemcpyAsync(all.data(), d.p, all.size() * 8, hipMemcpyDeviceToHost, stream_));
    wait_stream(stream_);
    static const char* names[K] = {"build", "nranks", "rank", "nz_global", "z_offset", "extent", "slab_axis",
                                   "storage_fp16", "fft_backend", "views", "halo planes", "plane floats"};
    std::string bad;
    for (int r = 0; r < R && bad.empty(); ++r) {
        const int64_t* q = all.data() + size_t(K) * r;
        for (int k = 0; k < K; ++k) {
            const bool must_equal = k != 2 && k != 4 && k != 5;
            if ((must_equal && q[k] != mine[k]) || (k == 2 && q[k] != r)) {
                bad = std::string(names[k]) + ": rank " + std::to_string(r) + " has " + std::to_string(q[k]) +
                      ", rank " + std::to_string(p_.rank) + " has " + std::to_string(mine[k]);
                break;
            }
        }
        if (bad.empty() && r + 1 < R) {   // adjacent ranks own adjacent ranges
            const int64_t* n = q + K;
            if (q[4] + q[5] != n[4])
                bad = "rank " + std::to_string(r) + " owns [" + std::to_string(q[4]) + ", " +
                      std::to_string(q[4] + q[5]) + ") but rank " + std::to_string(r + 1) + " starts at " +
                      std::to_string(n[4]);
        }
    }
    if (bad.empty()) {
        const int64_t* l = all.data() + size_t(K) * (R - 1);
        if (all[4] != 0 || l[4] + l[5] != p_.nz_global)
            bad = "the ranks' ranges do not cover [0, nz_global)";
    }
    SD_CHECK(bad.empty(), SPIMDECON_ERR_ARG, "ranks disagree on the exchange geometry (" + bad + ")");
}

void Session::run(int iters, double lambda, double* stats) {
    SD_CHECK(!poisoned_, SPIMDECON_ERR_STATE, "an earlier multi-device run failed mid-iteration; destroy the session");
    SD_CHECK(iters >= 0, SPIMDECON_ERR_ARG, "iters must be >= 0");
    SD_CHECK(spectra_ready_, SPIMDECON_ERR_STATE, "call mvd_init (or mvd_set_kernels) first");
    SD_CHECK(psi_ready_, SPIMDECON_ERR_STATE, "call mvd_init_psi first");
    if (iters == 0) return;
    const int V = nviews_;
    nprogress_ = 0;
    for (auto& gr : groups_) {
        DeviceGuard guard(gr.dev);
        gr.stats.alloc(size_t(iters) * V * 2);
    }
    try {
        if (backend_ == 1) {
            DeviceGuard guard(p_.device);
            run_rocfft(iters, lambda);
        } else if (groups_.size() == 1) {
            DeviceGuard guard(p_.device);
            run_engine(0, iters, lambda, nullptr);
        } else {
            run_groups(iters, lambda);
        }
    } catch (...) {
        if (slabs_.size() > 1 || p_.nranks > 1) poisoned_ = true;
        throw;
    }
    static const bool quiet = [] {
        const char* e = std::getenv("SPIMDECON_WARN_FALLBACK");
        return e && e[0] == '0';
    }();
    if (backend_ == 0 && !quiet && !warned_fallback_) {
        // the fast paths are a layout choice, not a semantic one: a slab outside them runs
        // the Stockham passes with the same results, several times slower -- say so once
        // (SPIMDECON_WARN_FALLBACK=0 silences it; callers can query mvd_xpass_mode / mvd_zpass_mode)
        for (int s = 0; s < int(slabs_.size()); ++s) {
            const int xm = slabs_[s].sp.xmode_update, zm = zpass_mode(s);
            if (xm != 2 || zm != 3) {
                std::fprintf(stderr,
                             "[spimdecon] warning: slab %d (%lld x %lld x %lld, padded %lld x %lld x %lld) runs "
                             "outside the fast engine passes (x pass %d, z pass %d; fast = 2 and 3): same "
                             "results, lower throughput\n",
                             s, (long long)slabs_[s].g.nx, (long long)slabs_[s].g.ny, (long long)slabs_[s].g.nz,
                             (long long)slabs_[s].g.Mx, (long long)slabs_[s].g.My, (long long)slabs_[s].g.Mz, xm,
                             zm);
                warned_fallback_ = true;
                break;
            }
        }
    }
    // per-group {sum, max} -> totals (sum over groups in double, max)
    std::vector<double> st(size_t(iters) * V * 2, 0.0), part(st.size());
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
        DevGroup& gr = groups_[gi];
        DeviceGuard guard(gr.dev);
        SD_HIP(hipMemcpyAsync(part.data(), gr.stats.p, part.size() * 8, hipMemcpyDeviceToHost, gr.stream));
        wait_stream(gr.stream);
        for (size_t i = 0; i < st.size(); i += 2) {
            st[i] = gi == 0 ? part[i] : st[i] + part[i];
            st[i + 1] = gi == 0 ? part[i + 1] : std::max(st[i + 1], part[i + 1]);
        }
    }
    if (comm_) {
        DeviceGuard guard(p_.device);
        std::vector<double> sums(size_t(iters) * V), maxs(size_t(iters) * V);
        for (size_t i = 0; i < sums.size(); ++i) {
            sums[i] = st[2 * i];
            maxs[i] = st[2 * i + 1];
        }
        allreduce_sum(sums.data(), int(sums.size()));
        allreduce_max(maxs.data(), int(maxs.size()));
        for (size_t i = 0; i < sums.size(); ++i) {
            st[2 * i] = sums[i];
            st[2 * i + 1] = maxs[i];
        }
    }
    if (stats) std::copy(st.begin(), st.end(), stats);
    if (timing_on_) {
        DeviceGuard guard(p_.device);
        for (auto& r : trecs_) {
            float ms = 0.f;
            SD_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            tacc_[r.cls] += ms;
            tacc_[8 + r.cls] += double(r.weight);
            event_pool_.push_back(r.a);
            event_pool_.push_back(r.b);
        }
        trecs_.clear();
    }
}

// one host thread per device group; the exchanges keep them in step (HostBarrier)
void Session::run_groups(int iters, double lambda) {
    const int G = int(groups_.size());
    HostBarrier bar(G);
    std::vector<std::exception_ptr> errs(G);
    std::vector<std::thread> th;
    th.reserve(G);
    for (int gi = 0; gi < G; ++gi) {
        th.emplace_back([&, gi] {
            try {
                SD_HIP(hipSetDevice(groups_[gi].dev));
                run_engine(gi, iters, lambda, &bar);
            } catch (...) {
                errs[gi] = std::current_exception();
                bar.abort();
            }
        });
    }
    for (auto& t : th) t.join();
    for (auto& e : errs)
        if (e) poisoned_ = true;  // the groups stopped at different views / iterations
    for (auto& e : errs)  // the first failure that is not another group's abort
        if (e) {
            try {
                std::rethrow_exception(e);
            } catch (const Error& x) {
                if (std::string(x.what()) != "device group aborted") throw;
            }
        }
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    sync_all();
}

void Session::run_rocfft(int iters, double lambda) {
    const int V = nviews_;
    for (auto& sl : slabs_) {
        tstart(0);
        launch_pad_mirror(sl.g, sl.psi, sl.Ra.p, stream_);
        tstop();
    }
    exchange(true, stream_);
    for (int it = 0; it < iters; ++it) {
        for (int v = 0; v < V; ++v) {
            const bool last = (it == iters - 1) && (v == V - 1);
            for (auto& sl : slabs_) {                    // convolve1 + quotient
                tstart(2); sl.fft->forward(sl.Ra.p); tstop();
                tstart(3); launch_spec_mul(sl.Ra.p, sl.k1spec[v].p, sl.pd.complex_count(), stream_); tstop();
                tstart(4); sl.fft->inverse(sl.Ra.p); tstop();
                tstart(1); launch_quotient_pad(sl.g, store_, sl.img[v].p, sl.Ra.p, sl.Rb.p, stream_); tstop();
            }
            exchange(false, stream_);
            for (size_t s = 0; s < slabs_.size(); ++s) {  // convolve2 + update
                SlabState& sl = slabs_[s];
                tstart(2); sl.fft->forward(sl.Rb.p); tstop();
                tstart(3); launch_spec_mul(sl.Rb.p, sl.k2spec[v].p, sl.pd.complex_count(), stream_); tstop();
                tstart(4); sl.fft->inverse(sl.Rb.p); tstop();
                tstart(0);
                const int64_t nb = launch_update_pad(sl.g, store_, sl.psi, sl.Rb.p, sl.w[v].p, lambda,
                                                     sl.psi_next, sl.Ra.p, sl.partials.p, !last, stream_);
                tstop();
                tstart(6);
                launch_reduce_partials(sl.partials.p, nb, groups_[0].stats.p + (size_t(it) * V + v) * 2,
                                       s > 0 ? 1 : 0, stream_);
                tstop();
                std::swap(sl.psi, sl.psi_next);
            }
            if (!last) exchange(true, stream_);
        }
        record_progress(stream_);
    }
}

// timing classes: 0 update x-pass, 1 quotient x-pass, 2 y passes, 3 z pass,
// 4 initial psi x-pass, 5 halo exchange, 6 stats reduce, 7 overlap window of an
// overlapped exchange (recorded by group 0 only)
void Session::run_engine(int gi, int iters, double lambda, HostBarrier* bar) {
    const int V = nviews_;
    DevGroup& gr = groups_[gi];
    hipStream_t st = gr.stream;
    const int s0 = gr.s0, s1 = gr.s1;
    const bool tm = gi == 0;
    auto T0 = [&](int cls) { if (tm) tstart(cls, st); };
    auto T1 = [&]() { if (tm) tstop(st); };
    const bool halo = slabs_.size() > 1 || p_.nranks > 1;
    // overlap: the x pass writes the planes the neighbours need first; their exchange
    // (xstream) runs while the x pass covers the rest of the slab
    std::vector<PairRanges> bnd(slabs_.size()), rest(slabs_.size());
    bool overlap = halo;
    for (int s = s0; s < s1; ++s) overlap = overlap && split_pairs(slabs_[s], bnd[s], rest[s]);
    // exchange of one buffer: begin after the boundary launches, end before the y pass
    auto xbegin = [&](bool buffer_a, bool window = true) {
        if (bar) {
            group_exchange_begin(gi, buffer_a, *bar);
        } else {
            SD_HIP(hipEventRecord(gr.ev_bnd, st));
            SD_HIP(hipStreamWaitEvent(gr.xstream, gr.ev_bnd, 0));
            exchange(buffer_a, gr.xstream);
            SD_HIP(hipEventRecord(gr.ev_x, gr.xstream));
        }
        if (tm && window) wstart(st);
    };
    // (cbnd_) one group, exchange over RCCL or between its own slabs: the boundary launches
    // were issued on xstream (after ev_pre), the exchange follows them there
    const bool cb = cbnd_ && !bar;
    auto xbegin_cb = [&](bool buffer_a) {
        exchange(buffer_a, gr.xstream);
        SD_HIP(hipEventRecord(gr.ev_x, gr.xstream));
        if (tm) wstart(st);
    };
    auto xend = [&]() {
        if (tm) wstop(st);   // (no-op after an unwindowed begin)
        if (bar) group_exchange_end(gi);
        else SD_HIP(hipStreamWaitEvent(st, gr.ev_x, 0));
    };
    auto xfull = [&](bool buffer_a) {  // not overlapped
        if (!halo) return;
        if (bar) {
            xbegin(buffer_a, false);
            xend();
        } else {
            exchange(buffer_a, st);
        }
    };
    auto convolve = [&](SlabState& sl, float2* Cb, const float2* K, bool fwd_done) {
        if (!fwd_done) { T0(2); engine_ypass(sl.sp, Cb, false, st); T1(); }
        T0(3);
        if (sl.kcompact) engine_zpass_compact(sl.sp, Cb, K, st);
        else engine_zpass(sl.sp, Cb, K, st);
        T1();
        T0(2); engine_ypass(sl.sp, Cb, true, st); T1();
    };
    // Both convolutions of every slab, for buffer C1 (buffer_a) or C2 of view v.  With an
    // exchange in flight (pending) the forward y pass of the planes nobody exchanges,
    // [cz, nz - cz), runs before waiting for it: the neighbours still read my boundary
    // planes [0, cz) and [nz - cz, nz) (the y pass works in place), and my halo planes
    // [nz, Mz) are still arriving.
    const int czx = halo_[2];
    auto convolve_all = [&](bool buffer_a, int v, bool pending) {
        auto buf = [&](SlabState& sl) { return buffer_a ? sl.C1.p : sl.C2.p; };
        auto ker = [&](SlabState& sl) { return buffer_a ? sl.e1spec[v].p : sl.e2spec[v].p; };
        bool split = pending;
        for (int s = s0; s < s1 && split; ++s)
            split = slabs_[s].sp.fy.n1 != 0 && int(slabs_[s].g.nz) > 2 * czx;
        if (split) {
            for (int s = s0; s < s1; ++s) {
                SlabState& sl = slabs_[s];
                T0(2);
                SD_CHECK(engine_ypass_planes(sl.sp, buf(sl), czx, int(sl.g.nz) - czx, st), SPIMDECON_ERR_STATE,
                         "y pass of a plane range not available");
                T1();
            }
            xend();
            for (int s = s0; s < s1; ++s) {
                SlabState& sl = slabs_[s];
                T0(2);
                // the planes that waited, [0, cz) and [nz - cz, Mz), in one launch (two small
                // launches ran two partial rounds: C3 as 8 slabs +0.5 %, bit-identical;
                // profiles/r06_ymerge_ab.txt)
                SD_CHECK(engine_ypass_planes2(sl.sp, buf(sl), 0, czx, int(sl.g.nz) - czx, int(sl.g.Mz), st),
                         SPIMDECON_ERR_STATE, "y pass of a plane range not available");
                T1();
            }
            for (int s = s0; s < s1; ++s) convolve(slabs_[s], buf(slabs_[s]), ker(slabs_[s]), true);
            return;
        }
        if (pending) xend();
        for (int s = s0; s < s1; ++s) convolve(slabs_[s], buf(slabs_[s]), ker(slabs_[s]), false);
    };

    for (int s = s0; s < s1; ++s) {
        T0(4);
        engine_forward_psi(slabs_[s].sp, slabs_[s].psi, slabs_[s].C1.p, st);
        T1();
    }
    xfull(true);
    bool pending = false;  // the update's exchange of C1 is still in flight
    for (int it = 0; it < iters; ++it) {
        for (int v = 0; v < V; ++v) {
            const bool last = (it == iters - 1) && (v == V - 1);
            convolve_all(true, v, pending);
            pending = false;
            // quotient (+ forward x of the quotient: C1 -> C2) and its halo exchange
            auto qin = [&](SlabState& sl) { return sl.C1.p; };
            auto qout = [&](SlabState& sl) { return sl.C2.p; };
            if (overlap && cb) {
                // boundary pairs on the exchange stream, the exchange right behind them there,
                // the rest of the pass concurrently on the compute stream; timed as one
                // interval (compute stream, through the boundary launches' end) per pass
                const int rq = tm ? rstart(1, st, s1 - s0) : -1;
                SD_HIP(hipEventRecord(gr.ev_pre, st));
                SD_HIP(hipStreamWaitEvent(gr.xstream, gr.ev_pre, 0));
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    engine_quotient(sl.sp, store_, qin(sl), sl.img[v].p, qout(sl), bnd[s], gr.xstream);
                }
                SD_HIP(hipEventRecord(gr.ev_bu, gr.xstream));
                xbegin_cb(false);
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    engine_quotient(sl.sp, store_, qin(sl), sl.img[v].p, qout(sl), rest[s], st);
                }
                if (rq >= 0) {
                    SD_HIP(hipStreamWaitEvent(st, gr.ev_bu, 0));   // (timing only)
                    rstop(rq, st);
                }
            } else if (overlap) {
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    T0(1); engine_quotient(sl.sp, store_, qin(sl), sl.img[v].p, qout(sl), bnd[s], st); T1();
                }
                xbegin(false);
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    T0(1); engine_quotient(sl.sp, store_, qin(sl), sl.img[v].p, qout(sl), rest[s], st); T1();
                }
            } else {
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    T0(1);
                    engine_quotient(sl.sp, store_, qin(sl), sl.img[v].p, qout(sl), all_pairs(sl.sp), st);
                    T1();
                }
                xfull(false);
            }
            convolve_all(false, v, overlap);   // (second convolution: kernel 2)
            // update (+ forward x of the next psi) and its halo exchange
            const bool ov = overlap && !last;
            std::vector<int64_t> nb(slabs_.size(), 0);
            const bool ovc = ov && cb;
            int ru = -1;
            if (ovc) {   // (as the quotient: boundary pairs and the exchange on xstream)
                ru = tm ? rstart(0, st, s1 - s0) : -1;
                SD_HIP(hipEventRecord(gr.ev_pre, st));
                SD_HIP(hipStreamWaitEvent(gr.xstream, gr.ev_pre, 0));
            }
            for (int s = s0; s < s1; ++s) {
                SlabState& sl = slabs_[s];
                if (!ovc) T0(0);
                nb[s] = engine_update(sl.sp, store_, sl.C2.p, sl.psi, sl.w[v].p, lambda, sl.psi_next,
                                      last ? nullptr : sl.C1.p, sl.partials.p, ov ? bnd[s] : all_pairs(sl.sp),
                                      ovc ? gr.xstream : st);
                if (!ovc) T1();
            }
            if (ovc) SD_HIP(hipEventRecord(gr.ev_bu, gr.xstream));   // the boundary partials
            if (ov) {
                if (ovc) xbegin_cb(true);
                else xbegin(true);
                for (int s = s0; s < s1; ++s) {
                    SlabState& sl = slabs_[s];
                    if (!ovc) T0(0);
                    nb[s] += engine_update(sl.sp, store_, sl.C2.p, sl.psi, sl.w[v].p, lambda, sl.psi_next,
                                           sl.C1.p, sl.partials.p + 2 * nb[s], rest[s], st);
                    if (!ovc) T1();
                }
            }
            if (ovc) {
                SD_HIP(hipStreamWaitEvent(st, gr.ev_bu, 0));
                rstop(ru, st);
            }
            for (int s = s0; s < s1; ++s) {
                SlabState& sl = slabs_[s];
                T0(6);
                launch_reduce_partials(sl.partials.p, nb[s], gr.stats.p + (size_t(it) * V + v) * 2,
                                       s > s0 ? 1 : 0, st);
                T1();
                std::swap(sl.psi, sl.psi_next);
            }
            if (ov) pending = true;  // ended inside the next view's convolve_all
            else if (!last) xfull(true);
        }
        record_progress(st);   // (RCCL watchdog: one event per iteration)
    }
}

void Session::apply_mask() {
    SD_CHECK(!poisoned_, SPIMDECON_ERR_STATE, "an earlier multi-device run failed mid-iteration; psi is inconsistent");
    SD_CHECK(psi_ready_, SPIMDECON_ERR_STATE, "psi not initialised");
    for (auto& sl : slabs_) {
        DeviceGuard guard(groups_[sl.grp].dev);
        launch_mask(sl.psi, sl.n, nviews_, store_, sl.img_ptrs.p, groups_[sl.grp].stream);
    }
    sync_all();
}

void Session::get_psi(float* out) {
    SD_CHECK(!poisoned_, SPIMDECON_ERR_STATE, "an earlier multi-device run failed mid-iteration; psi is inconsistent");
    SD_CHECK(psi_ready_, SPIMDECON_ERR_STATE, "psi not initialised");
    SD_CHECK(out, SPIMDECON_ERR_ARG, "null output");
    for (auto& sl : slabs_) {
        DeviceGuard guard(groups_[sl.grp].dev);
        DBuf<float> tmp;
        store_slab(sl, sl.psi, out, tmp, groups_[sl.grp].stream);
        wait_stream(groups_[sl.grp].stream);
    }
}

float* Session::psi_device(int slab) {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    return slabs_[slab].psi;
}

void Session::fft_dims(int slab, int64_t* out3) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    SD_CHECK(spectra_ready_, SPIMDECON_ERR_STATE, "not initialised");
    for (int d = 0; d < 3; ++d) out3[d] = slabs_[slab].pd.M[d];
}

int Session::zpass_mode(int slab) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    SD_CHECK(spectra_ready_, SPIMDECON_ERR_STATE, "not initialised");
    if (backend_ != 0) return -1;
    return engine_zpass_mode(slabs_[slab].sp, slabs_[slab].kcompact);
}

int Session::xpass_mode(int slab) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    SD_CHECK(spectra_ready_, SPIMDECON_ERR_STATE, "not initialised");
    if (backend_ != 0) return -2;
    return slabs_[slab].sp.xmode_update;
}

int Session::kernel_planes(int slab) const {
    SD_CHECK(slab >= 0 && slab < int(slabs_.size()), SPIMDECON_ERR_ARG, "bad slab");
    SD_CHECK(spectra_ready_, SPIMDECON_ERR_STATE, "not initialised");
    const SlabState& sl = slabs_[slab];
    if (backend_ != 0) return int(sl.pd.M[2]);
    return sl.kcompact ? int(2 * sl.sp.g.cz + 1) : int(sl.sp.g.Mz);
}

}  // namespace spimdecon
