// fft.cpp -- rocFFT plan wrapper (see fft.hpp).
#include "fft.hpp"

#include <cstdlib>
#include <mutex>

namespace spimdecon {

#define SD_FFT(expr)                                                                       \
    do {                                                                                   \
        rocfft_status _s = (expr);                                                         \
        if (_s != rocfft_status_success)                                                   \
            ::spimdecon::fail(SPIMDECON_ERR_FFT, std::string(#expr " failed, status ") +   \
                                                     std::to_string(int(_s)));             \
    } while (0)

static bool smooth2357(int64_t m) {
    for (int64_t p : {2, 3, 5, 7})
        while (m % p == 0) m /= p;
    return m == 1;
}

int64_t fft_fast_size(int64_t need, bool even) {
    int64_t m = need < 1 ? 1 : need;
    for (;; ++m) {
        if (even && (m & 1)) continue;
        if (smooth2357(m)) return m;
    }
}

void rocfft_init_once() {
    static std::once_flag once;
    std::call_once(once, [] {
        // compile runtime kernels in-process: no helper-process spawn from a
        // GPU-initialised process (unless the user chose otherwise)
        setenv("ROCFFT_RTC_PROCESS", "0", 0);
        if (rocfft_setup() != rocfft_status_success)
            fail(SPIMDECON_ERR_FFT, "rocfft_setup failed");
    });
}

FftPlan3D::~FftPlan3D() { destroy(); }

void FftPlan3D::destroy() {
    if (fwd_) rocfft_plan_destroy(fwd_);
    if (inv_) rocfft_plan_destroy(inv_);
    if (info_) rocfft_execution_info_destroy(info_);
    if (work_) (void)hipFree(work_);
    fwd_ = inv_ = nullptr;
    info_ = nullptr;
    work_ = nullptr;
    work_bytes_ = 0;
}

void FftPlan3D::create(const PadDims& pd, hipStream_t stream) {
    rocfft_init_once();
    destroy();
    pd_ = pd;
    const size_t lengths[3] = {size_t(pd.M[0]), size_t(pd.M[1]), size_t(pd.M[2])};
    const size_t Sx = size_t(pd.Sx()), Hx = size_t(pd.Hx());
    const size_t rstr[3] = {1, Sx, Sx * size_t(pd.M[1])};
    const size_t cstr[3] = {1, Hx, Hx * size_t(pd.M[1])};
    const size_t rdist = rstr[2] * size_t(pd.M[2]);
    const size_t cdist = cstr[2] * size_t(pd.M[2]);

    for (int dir = 0; dir < 2; ++dir) {
        rocfft_plan_description desc = nullptr;
        SD_FFT(rocfft_plan_description_create(&desc));
        rocfft_status st;
        if (dir == 0)
            st = rocfft_plan_description_set_data_layout(desc, rocfft_array_type_real,
                                                         rocfft_array_type_hermitian_interleaved,
                                                         nullptr, nullptr, 3, rstr, rdist, 3, cstr,
                                                         cdist);
        else
            st = rocfft_plan_description_set_data_layout(desc, rocfft_array_type_hermitian_interleaved,
                                                         rocfft_array_type_real, nullptr, nullptr,
                                                         3, cstr, cdist, 3, rstr, rdist);
        if (st != rocfft_status_success) {
            rocfft_plan_description_destroy(desc);
            fail(SPIMDECON_ERR_FFT, "rocfft_plan_description_set_data_layout failed");
        }
        rocfft_plan* plan = dir == 0 ? &fwd_ : &inv_;
        st = rocfft_plan_create(plan, rocfft_placement_inplace,
                                dir == 0 ? rocfft_transform_type_real_forward
                                         : rocfft_transform_type_real_inverse,
                                rocfft_precision_single, 3, lengths, 1, desc);
        rocfft_plan_description_destroy(desc);
        if (st != rocfft_status_success)
            fail(SPIMDECON_ERR_FFT, "rocfft_plan_create failed for " + std::to_string(pd.M[0]) +
                                        "x" + std::to_string(pd.M[1]) + "x" +
                                        std::to_string(pd.M[2]));
        size_t wb = 0;
        SD_FFT(rocfft_plan_get_work_buffer_size(*plan, &wb));
        if (wb > work_bytes_) work_bytes_ = wb;
    }
    SD_FFT(rocfft_execution_info_create(&info_));
    if (work_bytes_) {
        SD_HIP(hipMalloc(&work_, work_bytes_));
        SD_FFT(rocfft_execution_info_set_work_buffer(info_, work_, work_bytes_));
    }
    SD_FFT(rocfft_execution_info_set_stream(info_, stream));
}

void FftPlan3D::forward(float* buf) {
    void* in[1] = {buf};
    SD_FFT(rocfft_execute(fwd_, in, nullptr, info_));
}

void FftPlan3D::inverse(float* buf) {
    void* in[1] = {buf};
    SD_FFT(rocfft_execute(inv_, in, nullptr, info_));
}

}  // namespace spimdecon
