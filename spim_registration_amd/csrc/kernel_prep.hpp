// kernel_prep.hpp -- GPU implementation of MVDeconFFT.init kernel preparation.
#pragma once

#include <vector>

#include "common.hpp"

namespace spimdecon {

struct HostKernel {
    int dims[3] = {0, 0, 0};  // {kx, ky, kz}
    std::vector<float> data;  // x-fastest
};

// k1: raw kernels in (normalised out); k2: compound/inverted kernels out.
// Views processed in list order exactly as MVDeconInput.init (MVDeconInput.java:41-47).
void prepare_kernels_gpu(std::vector<HostKernel>& k1, std::vector<HostKernel>& k2, int psftype,
                         int ij_threads, int dev);

}  // namespace spimdecon
