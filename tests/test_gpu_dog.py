"""GPU parity of the DoG bead-detection pass against the oracle."""
import ctypes as C

import numpy as np
import pytest
import torch  # before the library loads: one shared HIP runtime (spim_registration_amd._lib.load)

from oracle import dog_ref
from spim_registration_amd import dog, synthetic

pytestmark = pytest.mark.gpu


def bead_stack(shape=(40, 44, 48), cid=11):
    rng = synthetic.rng_for(cid)
    t = synthetic.truth_volume(shape, rng, bead_density=1.0 / 10 ** 3)
    k = synthetic.psf(0, 1, (9, 9, 13), sigma=(1.0, 1.0, 1.6))
    from oracle import mvdecon_ref as ref
    img = ref.convolve(t.astype(np.float32), k, "mirror")
    img = (rng.poisson(np.maximum(img * 2000 + 50, 0)) + rng.normal(0, 2, shape)).astype(np.float32)
    return img


@pytest.mark.parametrize("find_min,find_max", [(False, True), (True, True)])
def test_dog_matches_oracle(gpu, find_min, find_max):
    img = bead_stack()
    pts, d = dog.compute(img, sigma=1.8, threshold=0.008, find_min=find_min, find_max=find_max,
                         return_dog=True, keep_intensity=True)
    exp, dref = dog_ref.process_dog(img, 1.8, 0.008, find_min=find_min, find_max=find_max)
    # same float32 op order: bit-identical DoG image
    np.testing.assert_array_equal(d, dref)
    assert len(pts) == len(exp) and len(exp) > 10
    got = [(int(p.location[0]), int(p.location[1]), int(p.location[2])) for p in pts]
    assert got == [(e[0], e[1], e[2]) for e in exp]          # same order (x % T lists)
    np.testing.assert_array_equal([p.intensity for p in pts], np.float32([e[3] for e in exp]))


def test_dog_given_intensity_range(gpu):
    img = bead_stack(shape=(24, 26, 30), cid=12)
    pts, d = dog.compute(img, sigma=2.0, threshold=0.004, min_intensity=0.0, max_intensity=4000.0,
                         return_dog=True)
    exp, dref = dog_ref.process_dog(img, 2.0, 0.004, min_intensity=0.0, max_intensity=4000.0)
    np.testing.assert_array_equal(d, dref)
    assert [tuple(int(c) for c in p.location) for p in pts] == [e[:3] for e in exp]


def test_dog_flat_image_has_no_peaks_and_no_nan(gpu):
    img = np.full((12, 12, 12), 3.0, np.float32)   # min == max: normalisation skipped
    pts, d = dog.compute(img, return_dog=True)
    exp, dref = dog_ref.process_dog(img)
    np.testing.assert_array_equal(d, dref)
    assert len(pts) == len(exp)


@pytest.mark.parametrize("find_min,find_max", [(False, True), (True, True)])
def test_dog_quadratic_localization(gpu, find_min, find_max):
    """Localization 1 (the reference's default, DifferenceOf.java:46): candidates at
    threshold/10, quadratic sub-pixel fit, |fitted value| > threshold."""
    img = bead_stack(cid=13)
    pts, d = dog.compute(img, sigma=1.8, threshold=0.008, localization=1, find_min=find_min,
                         find_max=find_max, return_dog=True, keep_intensity=True)
    exp, dref = dog_ref.process_dog(img, 1.8, 0.008, localization=1, find_min=find_min,
                                    find_max=find_max)
    np.testing.assert_array_equal(d, dref)
    assert len(pts) == len(exp) and len(exp) > 10
    got = np.array([p.location for p in pts])
    want = np.array([e[:3] for e in exp])
    # identical double arithmetic; float32-rounded positions
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)
    np.testing.assert_allclose([p.intensity for p in pts], [e[3] for e in exp], rtol=1e-6, atol=1e-9)
    assert np.any(np.abs(got - np.round(got)) > 1e-3)      # genuinely sub-pixel


def test_dog_simple_peaks_threshold_tenth(gpu):
    """getSimplePeaks at localization 1 uses threshold / 10 (ProcessDOG.java:63-67)."""
    img = bead_stack(shape=(24, 26, 30), cid=14)
    p0 = dog.simple_peaks(img, threshold=0.008, localization=0)
    p1 = dog.simple_peaks(img, threshold=0.008, localization=1)
    _, dref = dog_ref.process_dog(img, 1.8, 0.008)
    e1 = dog_ref.find_peaks(dref, float(np.float32(0.008) / np.float32(10.0)))
    assert len(p1) >= len(p0)
    assert [q[:3] for q in p1] == [e[:3] for e in e1 if e[5]]


def test_dog_device_resident_input(gpu):
    """The same C-ABI entry point with device pointers (a view already in HBM): the
    DoG image and the interest points equal the host-pointer call's, bit for bit."""
    from spim_registration_amd import _lib
    img = bead_stack(shape=(24, 26, 30), cid=13)
    pts, d = dog.compute(img, localization=1, return_dog=True, keep_intensity=True)
    lib = _lib.load()
    dimg = torch.from_numpy(img).to("cuda:0")
    ddog = torch.empty_like(dimg)
    p = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(p))
    p.localization = 1
    dims = (C.c_int64 * 3)(img.shape[2], img.shape[1], img.shape[0])
    cap = max(16, 2 * len(pts))
    out = (_lib.InterestPointC * cap)()
    n = C.c_int64(0)
    fp = C.POINTER(C.c_float)
    _lib.check(lib.spim_dog_interest_points(C.cast(C.c_void_p(dimg.data_ptr()), fp), dims, C.byref(p),
                                            C.cast(C.c_void_p(ddog.data_ptr()), fp), out, cap, C.byref(n)))
    torch.cuda.synchronize()
    assert int(n.value) == len(pts) > 0
    np.testing.assert_array_equal(ddog.cpu().numpy(), d)
    for i, q in enumerate(pts):
        assert tuple(out[i].pos) == tuple(q.location)
