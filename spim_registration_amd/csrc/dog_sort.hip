// dog_sort.hip -- device radix sort of DoG peak candidates into the reference order.
//
// The fused DoG kernels emit candidates in tile order; the reference's order is
// per-thread lists by x % T, each in flat (x-fastest) order
// (mpicbg/spim/segmentation/InteractiveIntegral.java:394,437-438), i.e. ascending
// key (x % T) << 40 | flat.  Kept in its own translation unit: hipcub is heavy to
// compile and nothing else needs it.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace spimdecon {

size_t peak_sort_temp_bytes(int64_t n, int end_bit) {
    size_t bytes = 0;
    SD_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const uint64_t*>(nullptr),
                                              static_cast<uint64_t*>(nullptr),
                                              static_cast<const uint32_t*>(nullptr),
                                              static_cast<uint32_t*>(nullptr), int(n), 0, end_bit));
    return bytes;
}

void peak_sort(void* tmp, size_t tmp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
               uint32_t* vout, int64_t n, int end_bit, hipStream_t s) {
    SD_CHECK(n < (int64_t(1) << 31), SPIMDECON_ERR_ARG, "too many DoG peak candidates to sort");
    SD_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, int(n), 0, end_bit, s));
}

// Order-preserving selection of the localised interest points that pass the threshold
// (the host loop of Localization.computeQuadraticLocalization's caller, on the device):
// only the survivors travel to the host.
size_t point_select_temp_bytes(int64_t n) {
    size_t bytes = 0;
    SD_HIP(hipcub::DeviceSelect::Flagged(nullptr, bytes, static_cast<const spim_interest_point*>(nullptr),
                                         static_cast<const unsigned char*>(nullptr),
                                         static_cast<spim_interest_point*>(nullptr), static_cast<int*>(nullptr),
                                         int(n)));
    return bytes;
}

void point_select(void* tmp, size_t tmp_bytes, const spim_interest_point* in, const unsigned char* flags,
                  spim_interest_point* out, int* nsel, int64_t n, hipStream_t s) {
    SD_CHECK(n < (int64_t(1) << 31), SPIMDECON_ERR_ARG, "too many DoG candidates to select");
    SD_HIP(hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, in, flags, out, nsel, int(n), s));
}

}  // namespace spimdecon
