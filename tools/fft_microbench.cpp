// fft_microbench: rocFFT in-place 3D R2C / C2R timing for candidate padded sizes.
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { auto e = (x); if (e != 0) { printf("err %d at %s:%d\n", int(e), __FILE__, __LINE__); exit(1);} } while (0)
int main(int argc, char** argv) {
    rocfft_setup();
    std::vector<int> sizes;
    for (int i = 1; i < argc; ++i) sizes.push_back(atoi(argv[i]));
    for (int M : sizes) {
        size_t Hx = M / 2 + 1, Sx = 2 * Hx;
        size_t lens[3] = {size_t(M), size_t(M), size_t(M)};
        size_t rstr[3] = {1, Sx, Sx * M}, cstr[3] = {1, Hx, Hx * M};
        size_t rdist = Sx * M * M, cdist = Hx * M * M;
        rocfft_plan p[2];
        size_t wmax = 0;
        for (int d = 0; d < 2; ++d) {
            rocfft_plan_description desc;
            CK(rocfft_plan_description_create(&desc));
            if (d == 0) CK(rocfft_plan_description_set_data_layout(desc, rocfft_array_type_real, rocfft_array_type_hermitian_interleaved, nullptr, nullptr, 3, rstr, rdist, 3, cstr, cdist));
            else CK(rocfft_plan_description_set_data_layout(desc, rocfft_array_type_hermitian_interleaved, rocfft_array_type_real, nullptr, nullptr, 3, cstr, cdist, 3, rstr, rdist));
            CK(rocfft_plan_create(&p[d], rocfft_placement_inplace, d == 0 ? rocfft_transform_type_real_forward : rocfft_transform_type_real_inverse, rocfft_precision_single, 3, lens, 1, desc));
            size_t w; CK(rocfft_plan_get_work_buffer_size(p[d], &w)); if (w > wmax) wmax = w;
            rocfft_plan_description_destroy(desc);
        }
        float* buf; CK(hipMalloc(&buf, rdist * 4));
        CK(hipMemset(buf, 0, rdist * 4));
        void* work = nullptr; if (wmax) CK(hipMalloc(&work, wmax));
        rocfft_execution_info info; CK(rocfft_execution_info_create(&info));
        if (wmax) CK(rocfft_execution_info_set_work_buffer(info, work, wmax));
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        void* in[1] = {buf};
        for (int w = 0; w < 3; ++w) { rocfft_execute(p[0], in, nullptr, info); rocfft_execute(p[1], in, nullptr, info); }
        float ms[2];
        for (int d = 0; d < 2; ++d) {
            hipEventRecord(a);
            for (int it = 0; it < 10; ++it) rocfft_execute(p[d], in, nullptr, info);
            hipEventRecord(b); hipEventSynchronize(b);
            hipEventElapsedTime(&ms[d], a, b); ms[d] /= 10;
        }
        double bytes = double(cdist) * 8 * 2;  // one read + one write of the complex volume
        printf("M=%d work=%zuMB r2c %.3f ms c2r %.3f ms  ns/pt %.3f %.3f  (1-pass GB/s r2c %.0f)\n", M, wmax >> 20, ms[0], ms[1],
               ms[0] * 1e6 / (double(M) * M * M), ms[1] * 1e6 / (double(M) * M * M), bytes / (ms[0] * 1e-3) / 1e9);
        rocfft_plan_destroy(p[0]); rocfft_plan_destroy(p[1]); hipFree(buf); if (work) hipFree(work);
        rocfft_execution_info_destroy(info);
    }
    return 0;
}
