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


def test_dog_localized_threshold_is_a_float(gpu):
    """ProcessDOG takes a float threshold and Localization keeps |fitted value| >
    threshold in float (Localization.java:47,74): a double threshold just below a
    fitted value, which rounds to that value as a float, drops the point."""
    img = bead_stack(cid=13)
    pts = dog.compute(img, sigma=1.8, threshold=0.008, localization=1, keep_intensity=True)
    v = np.float32(abs(pts[len(pts) // 2].intensity))
    thr = float(v) - float(np.spacing(v)) / 4          # < v as a double, == v as a float
    assert np.float32(thr) == v and thr < float(v)
    got = dog.compute(img, sigma=1.8, threshold=thr, localization=1, keep_intensity=True)
    exp, _ = dog_ref.process_dog(img, 1.8, thr, localization=1)
    assert len(got) == len(exp)
    assert not any(np.float32(abs(p.intensity)) == v for p in got)
    np.testing.assert_allclose([p.location for p in got], [e[:3] for e in exp], rtol=0, atol=1e-5)


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


# ---------------------------------------------------------------- fused DoG path (k_dog_xy / k_dog_z)

@pytest.mark.parametrize("sigma,taps", [(1.0, 7), (1.8, 15), (4.0, 31), (8.0, 63)])
def test_dog_tap_sizes_tiles_and_chunks(gpu, sigma, taps):
    """Every Gaussian size class: 7 / 15 / 31 taps on the fused kernels, 63 on the
    separate passes + candidate pass.  150 planes = 3 z chunks of 64 (the last one
    ragged); 70 rows = several 16-row boxes and 32-row xy tiles; 131 columns = three
    64-column boxes with their 1-voxel halo rings.  Bit-identical DoG and peak list."""
    s1, s2, _, _ = dog_ref.dog_sigmas(sigma, (0.5, 0.5, 0.5))
    assert len(dog_ref.cuda_kernels(s1)[0]) == taps or len(dog_ref.cuda_kernels(s2)[0]) == taps
    img = bead_stack(shape=(150, 70, 131), cid=21)
    pts, d = dog.compute(img, sigma=sigma, threshold=0.002, find_min=True, find_max=True, return_dog=True,
                         keep_intensity=True)
    exp, dref = dog_ref.process_dog(img, sigma, 0.002, find_min=True, find_max=True)
    np.testing.assert_array_equal(d, dref)
    assert len(exp) > 5
    assert [tuple(int(c) for c in p.location) for p in pts] == [e[:3] for e in exp]
    np.testing.assert_array_equal([p.intensity for p in pts], np.float32([e[3] for e in exp]))


@pytest.mark.parametrize("shape", [(1, 1, 1), (1, 5, 7), (3, 3, 3), (2, 9, 4), (5, 1, 70), (70, 3, 65),
                                   (4, 17, 3), (66, 18, 66)])
def test_dog_small_and_thin_volumes(gpu, shape):
    """Volumes thinner than the kernel, the boxes or the peak border (mirror indices
    folding several times); threshold 0 on noise: every extremum is a candidate."""
    rng = np.random.default_rng(sum(shape))
    img = rng.random(shape, dtype=np.float32)
    pts, d = dog.compute(img, threshold=0.0, find_min=True, find_max=True, return_dog=True,
                         keep_intensity=True, ij_threads=3)
    exp, dref = dog_ref.process_dog(img, 1.8, 0.0, find_min=True, find_max=True, ij_threads=3)
    np.testing.assert_array_equal(d, dref)
    assert [tuple(int(c) for c in p.location) for p in pts] == [e[:3] for e in exp]


def test_dog_plateau_overflows_candidate_capacity(gpu):
    """A constant volume at threshold 0: every interior voxel is a (plateau) extremum
    (238,328 > the 65,536 initial candidate capacity): the library reruns the peak
    kernel with room for all and keeps the reference order."""
    img = np.full((64, 64, 64), 3.0, np.float32)
    pk = dog.simple_peaks(img, threshold=0.0, find_min=True, find_max=True)
    _, dref = dog_ref.process_dog(img, 1.8, 0.0)
    exp = dog_ref.find_peaks(dref, 0.0)
    assert len(pk) == len(exp) == 62 ** 3
    assert [q[:3] for q in pk] == [e[:3] for e in exp]
    assert [(q[4], q[5]) for q in pk] == [(e[4], e[5]) for e in exp]


def test_dog_nan_planes_take_the_comparison_loop(gpu):
    """NaN in the image spreads into the DoG; a NaN neighbour fails every comparison
    in the reference (isSpecialPoint), which the min/max box test would not see --
    the planes holding NaN are tested by the comparison loop.  Checked against the
    oracle's peak finder on the library's own DoG image (the oracle's convolution
    skips zero taps, so its NaN footprint differs for padded kernels)."""
    img = bead_stack(shape=(40, 44, 48), cid=22)
    img[20, 22, 24] = np.nan
    img[5, 40, 3] = np.nan
    pk = dog.simple_peaks(img, threshold=0.001, find_min=True, find_max=True, min_intensity=0.0,
                          max_intensity=4000.0)
    _, d = dog.compute(img, threshold=0.001, min_intensity=0.0, max_intensity=4000.0, return_dog=True)
    assert np.isnan(d).sum() > 1000
    exp = dog_ref.find_peaks(d, 0.001)
    assert [q[:3] for q in pk] == [e[:3] for e in exp] and len(exp) > 10
    assert [(q[4], q[5]) for q in pk] == [(e[4], e[5]) for e in exp]


@pytest.mark.parametrize("sigma", [1.0, 1.8, 4.0])
def test_dog_split_and_fused_z_stages_agree(gpu, sigma, monkeypatch):
    """The split z stage (k_dog_zconv + k_dog_peaks, the default) and the fused
    k_dog_z (SPIMDECON_DOG_SPLIT=0) give the same DoG image and the same ordered
    candidate list, NaN planes (the comparison loop) and several row / plane
    chunks included; 7 / 15 / 31 taps."""
    img = bead_stack(shape=(150, 70, 131), cid=24)
    img[70, 30, 64] = np.nan
    img[3, 68, 2] = np.nan
    out = {}
    for split in ("1", "0"):
        monkeypatch.setenv("SPIMDECON_DOG_SPLIT", split)
        pk = dog.simple_peaks(img, sigma=sigma, threshold=0.001, find_min=True, find_max=True,
                              min_intensity=0.0, max_intensity=4000.0, ij_threads=5)
        _, d = dog.compute(img, sigma=sigma, threshold=0.001, min_intensity=0.0, max_intensity=4000.0,
                           return_dog=True)
        out[split] = (pk, d)
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
    assert len(out["1"][0]) > 10
    assert out["1"][0] == out["0"][0]


def test_dog_workspace_release_and_reuse(gpu):
    """The per-device workspace grows to the largest view and is reused; releasing it
    and calling again gives the same result."""
    from spim_registration_amd import _lib
    img = bead_stack(shape=(24, 26, 30), cid=23)
    a = dog.compute(img, localization=1, keep_intensity=True)
    _lib.check(_lib.load().spim_dog_release_workspace(0))
    b = dog.compute(img, localization=1, keep_intensity=True)
    assert [(p.location, p.intensity) for p in a] == [(p.location, p.intensity) for p in b]


@pytest.mark.parametrize("zchunk", [None, "128"])
def test_dog_partial_last_z_chunk_after_full_ones(gpu, zchunk, monkeypatch):
    """The split z stage's last chunk partial and not the first: 300 planes at the
    default 256-plane chunks (256 + 44) and at 128 (128 + 128 + 44) -- the boundary a
    round-3 experiment build read past.  Bit-identical DoG image and peak list."""
    if zchunk:
        monkeypatch.setenv("SPIMDECON_DOG_ZC_CHUNK", zchunk)
    img = bead_stack(shape=(300, 40, 72), cid=25)
    pts, d = dog.compute(img, sigma=1.8, threshold=0.002, find_min=True, find_max=True, return_dog=True,
                         keep_intensity=True)
    exp, dref = dog_ref.process_dog(img, 1.8, 0.002, find_min=True, find_max=True)
    np.testing.assert_array_equal(d, dref)
    assert len(exp) > 5
    assert [tuple(int(c) for c in p.location) for p in pts] == [e[:3] for e in exp]
    np.testing.assert_array_equal([p.intensity for p in pts], np.float32([e[3] for e in exp]))


def test_dog_own_range_division_edges(gpu, monkeypatch):
    """k_dog_xy skips the per-value range check of its reciprocal division when min / max
    are the image's own (SPIMDECON_DOG_MM_EXACT=1, the default).  At the edges of that
    argument -- min = -2^-20, values one ulp above min, a range near 2^48 -- the DoG
    image and the ordered peaks must equal those of the checked division (=0), bit for
    bit, and the oracle's."""
    rng = np.random.default_rng(77)
    img = bead_stack(shape=(40, 44, 48), cid=26)
    mn = np.float32(-2.0 ** -20)
    img[5, 5, 5] = mn
    up = np.nextafter(mn, np.float32(1))
    idx = rng.integers(0, img.size, 400)
    img.reshape(-1)[idx] = up
    img[30, 30, 30] = np.float32(2.0 ** 48)
    img[31, 10, 7] = np.float32(2.0 ** 48) - np.float32(2.0 ** 24)
    out = {}
    for mm in ("1", "0"):
        monkeypatch.setenv("SPIMDECON_DOG_MM_EXACT", mm)
        pk, d = dog.compute(img, sigma=1.8, threshold=1e-9, find_min=True, find_max=True, return_dog=True,
                            keep_intensity=True)
        out[mm] = ([(p.location, p.intensity) for p in pk], d)
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
    assert out["1"][0] == out["0"][0]
    exp, dref = dog_ref.process_dog(img, 1.8, 1e-9, find_min=True, find_max=True)
    np.testing.assert_array_equal(out["1"][1], dref)
    assert [tuple(int(c) for c in q[0]) for q in out["1"][0]] == [e[:3] for e in exp]


@pytest.mark.parametrize("sigma", [1.0, 1.8, 4.0])
def test_dog_zero_tap_trim_bit_identical(gpu, sigma, monkeypatch):
    """k_dog_xy skips the padded taps that are zero for both sigmas when k_minmax found
    every value finite and normalised the image by its own range (SPIMDECON_DOG_TRIM=1,
    the default): the DoG image and the ordered peaks equal those of every padded tap (=0)
    bit for bit.  With a NaN or an infinity in the image the trim is off, so the NaN
    footprint stays that of all padded taps."""
    img = bead_stack(shape=(40, 44, 48), cid=27)
    nan_img = img.copy()
    nan_img[20, 22, 24] = np.nan
    inf_img = img.copy()
    inf_img[7, 30, 11] = np.inf
    for im in (img, nan_img, inf_img):
        out = {}
        for t in ("1", "0"):
            monkeypatch.setenv("SPIMDECON_DOG_TRIM", t)
            pk, d = dog.compute(im, sigma=sigma, threshold=1e-4, find_min=True, find_max=True, return_dog=True,
                                keep_intensity=True)
            out[t] = ([(tuple(p.location), p.intensity) for p in pk], d)
        np.testing.assert_array_equal(out["1"][1], out["0"][1])
        assert out["1"][0] == out["0"][0]
