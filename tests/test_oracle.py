"""CPU: the oracle against the committed golden vectors and the reference's
known-answer harnesses (MVDeconvolution.main, Block.main, ...).

PARITY UNPINNED (see oracle/__init__.py): no reference output is available, so
the KATs are the analytic values the reference's own ``main()`` harnesses
print, plus algebraic identities.
"""
import glob
import math
import os

import numpy as np
import pytest

from conftest import rel_l2
from oracle import dog_ref, mvdecon_ref as ref
from spim_registration_amd import legacy, synthetic

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "rl_*.npz"))))
def test_oracle_reproduces_golden_rl(path):
    g = np.load(path)
    pt = ref.PSFTYPE(int(g["psftype"]))
    T = int(g["ij_threads"])
    psfs = list(g["psfs"])
    k1, k2 = ref.prepare_kernels(psfs, pt, T)
    np.testing.assert_array_equal(np.stack(k1), g["k1"])
    np.testing.assert_allclose(np.stack(k2), g["k2"], rtol=1e-6, atol=1e-12)
    res = ref.mv_deconvolution(list(g["imgs"]), list(g["weights"]), psfs, pt, int(g["iters"]),
                               float(g["lam"]), ij_threads=T)
    assert rel_l2(res.psi, g["psi"]) < 1e-6
    np.testing.assert_allclose(np.array(res.stats), g["stats"], rtol=1e-6)
    assert res.avg == float(g["avg"])


def test_oracle_reproduces_golden_conv():
    g = np.load(os.path.join(GOLD, "conv.npz"))
    assert rel_l2(ref.convolve(g["a"], g["k"], "mirror"), g["mirror"]) < 1e-7
    assert rel_l2(ref.convolve(g["a"], g["k"], "one"), g["one"]) < 1e-7
    assert rel_l2(ref.circular_convolve_block(g["block"], g["k"]), g["circular"]) < 1e-7


def test_oracle_reproduces_golden_dog():
    g = np.load(os.path.join(GOLD, "dog.npz"))
    peaks, dog = dog_ref.process_dog(g["img"], 1.8, 0.008)
    np.testing.assert_array_equal(dog, g["dog"])
    np.testing.assert_array_equal(np.array([p[:3] for p in peaks]).reshape(-1, 3), g["peaks"])


def test_tikhonov_kat():
    """MVDeconvolution.main (:707-714) prints tikhonov(d, 0.0006) for d in [0,10)
    and d*1e4: (sqrt(1 + 2 l d) - 1) / l."""
    lam = 0.0006
    for d in np.arange(0, 10, 0.1):
        for v in (d, d * 10000):
            exp = (math.sqrt(1.0 + 2.0 * lam * v) - 1.0) / lam
            assert float(ref.tikhonov(v, lam)) == exp
    assert float(ref.tikhonov(10000.0, lam)) < 10000.0      # damping of bright voxels
    assert abs(float(ref.tikhonov(1e-6, lam)) - 1e-6) < 1e-12


@pytest.mark.parametrize("lam", [0.006, 0.0006, 0.05, 0.3, 1e-7])
def test_tikhonov_division_correctly_rounded(lam):
    """The engine divides d = sqrt(1 + 2 l v) - 1 by l as q0 = d * RN(1/l) plus two fma
    corrections (rl_math.hpp div_rn_by).  Restated here with exact rational fma: it
    must equal Java's correctly rounded double d / l (MVDeconvolution.java:681-690)
    for float32 values over 2^-40 .. 2^20, and keep an infinite d infinite."""
    from fractions import Fraction as Fr

    def fma(a, b, c):
        return float(Fr(a) * Fr(b) + Fr(c))

    def div_rn_by(d, lam, inv):
        q0 = d * inv
        if not math.isfinite(q0):
            return q0
        q1 = fma(fma(-lam, q0, d), inv, q0)
        return fma(fma(-lam, q1, d), inv, q1)

    inv = 1.0 / lam
    rng = np.random.default_rng(11)
    vals = np.float32(2.0) ** rng.uniform(-40, 20, 6000).astype(np.float32)
    vals = np.concatenate([vals, rng.random(2000, dtype=np.float32) * 4])
    for v in vals:
        d = math.sqrt(1.0 + 2.0 * lam * float(v)) - 1.0
        assert div_rn_by(d, lam, inv) == d / lam, (float(v), lam)
    assert div_rn_by(math.inf, lam, inv) == math.inf


def test_compute_next_value_rules():
    """computeNextValue (:671-703): value <= 0 or NaN -> minValue; weight blend."""
    psi = np.float32([1.0, 1.0, 1.0, 2.0, 0.5])
    integ = np.float32([0.0, -1.0, np.nan, 1.5, 3.0])
    w = np.float32([1.0, 1.0, 1.0, 0.5, 0.0])
    out = ref.compute_next_value(psi, integ, w, 0.0)
    one = np.float32(1.0)
    blended = np.float32(one + np.float32(np.float32(ref.MIN_VALUE - one) * one))   # last + (next-last)*w
    assert out[0] == blended and out[1] == blended and out[2] == blended
    assert out[3] == np.float32(2.0 + (3.0 - 2.0) * 0.5)
    assert out[4] == np.float32(0.5)


def test_quotient_rules():
    q = ref.compute_quotient(np.float32([2.0, 2.0, 0.5]), np.float32([1.0, 0.0, -1.0]))
    np.testing.assert_array_equal(q, np.float32([0.5, 1.0, 1.0]))


def test_block_main_layout():
    """Block.main (CUDA/Block.java:367-402): 1024x1024 image, 384x384 blocks,
    kernel 16x32 -> effective 369x353, 3x3 blocks, last ones clipped."""
    gen = legacy.BlockGeneratorFixedSizePrecise((384, 384))
    blocks = gen.divide_into_blocks((1024, 1024), (16, 32))
    assert len(blocks) == 9
    assert blocks[0].offset == (-8, -16) and blocks[0].effective_size == (369, 353)
    assert blocks[1].effective_offset == (369, 0)           # x varies fastest
    assert blocks[-1].effective_offset == (738, 706)
    assert blocks[-1].effective_size == (1024 - 738, 1024 - 706)
    assert blocks[0].effective_local_offset == (8, 16)
    # identical to the oracle's restatement
    ob = ref.divide_into_blocks((1024, 1024, 1), (16, 32, 1), (384, 384, 1))
    assert [b.offset[:2] for b in ob] == [b.offset for b in blocks]


def test_block_layout_config3_256():
    """C3 (1024x1024x512) with 256^3 blocks, K=25: eff 232 -> 5x5x3."""
    blocks = legacy.BlockGeneratorFixedSizePrecise((256, 256, 256)).divide_into_blocks(
        (1024, 1024, 512), (25, 25, 25))
    assert len(blocks) == 75
    assert blocks[0].effective_size == (232, 232, 232)
    assert legacy.BlockGeneratorFixedSizePrecise((20, 20, 20)).divide_into_blocks((30,) * 3, (25,) * 3) is None


def test_precise_blocks_equal_whole_convolution():
    rng = np.random.default_rng(0)
    a = rng.random((23, 25, 27)).astype(np.float32)
    k = synthetic.psf(1, 3, (7, 5, 9))
    for ext in ("mirror", "one"):
        assert rel_l2(ref.blocked_convolve(a, k, (15, 14, 16), ext), ref.convolve(a, k, ext)) < 1e-6


def test_norm_quirk():
    """AdjustInput.sumImg adds portion 0 twice (:93-97): sum = S + P0."""
    k = synthetic.psf(0, 1, (19, 19, 25))
    flat = k.ravel().astype(np.float64)
    for T in (1, 4, 8):
        chunk = flat.size // (2 * T)
        p0 = flat[:chunk].sum()
        assert abs(ref.sum_img(k, T) - (flat.sum() + p0)) < 1e-12
        n = ref.norm_img(k, T)
        assert abs(n.astype(np.float64).sum() - flat.sum() / (flat.sum() + p0)) < 1e-6
    assert ref.norm_img(k, 1).sum() < 0.7          # T=1: portion 0 is half the kernel


def test_mirror_even_quirk():
    a = np.arange(6, dtype=np.float32).reshape(1, 1, 6)
    np.testing.assert_array_equal(ref.mirror_axis(a, 2).ravel(), [5, 4, 2, 3, 1, 0])
    b = np.arange(5, dtype=np.float32).reshape(1, 1, 5)
    np.testing.assert_array_equal(ref.mirror_axis(b, 2).ravel(), [4, 3, 2, 1, 0])


def test_delta_psf_identity_oracle():
    imgs, _, _, _ = synthetic.make_views((10, 12, 14), 1, config_id=3, ksize=(3, 3, 3), weights="ones")
    k = np.zeros((3, 3, 3), np.float32)
    k[1, 1, 1] = 1
    r = ref.mv_deconvolution(imgs, [np.ones_like(imgs[0])], [k], ref.PSFTYPE.INDEPENDENT, 1, 0.0)
    np.testing.assert_allclose(r.psi, imgs[0], rtol=1e-5)


def test_first_iteration_average():
    a = np.zeros((2, 2, 2), np.float32)
    b = np.zeros((2, 2, 2), np.float32)
    a[0, 0, 0], b[0, 0, 0] = 2.0, 4.0          # mean 3 over 2 views
    a[1, 1, 1] = 5.0                           # mean 5 over 1 view
    cnt, avg = ref.first_iteration([a, b])
    assert cnt[0, 0, 0] == 2 and cnt[1, 1, 1] == 1 and cnt.sum() == 3
    assert avg == 4.0
    _, avg0 = ref.first_iteration([np.zeros((2, 2, 2), np.float32)])
    assert math.isnan(avg0)


def test_dog_sigma_math():
    """ProcessDOG.java:88-105 for the defaults sigma=1.8, imageSigma=0.5."""
    s1, s2, k, kinv = dog_ref.dog_sigmas(1.8)
    assert k == np.float32(2 ** 0.25)
    assert abs(s1[0] - math.sqrt(1.8 ** 2 - 0.25)) < 1e-6
    assert abs(s2[0] - math.sqrt((1.8 * 2 ** 0.25) ** 2 - 0.25)) < 1e-5
    assert [len(dog_ref.gaussian_kernel_1d(s)) for s in (s1[0], s2[0])] == [11, 13]
    assert all(len(x) == 15 for x in dog_ref.cuda_kernels(s1))


def test_find_peaks_order_and_labels():
    d = np.zeros((5, 5, 9), np.float32)
    d[2, 2, 2] = -1.0       # all neighbours >= centre -> MAX (bright bead)
    d[2, 2, 6] = 1.0        # all neighbours <= centre -> MIN
    p = dog_ref.find_peaks(d, 0.5, ij_threads=4)
    # x % 4 == 2 for both -> one thread list, flat order
    assert [(q[0], q[4], q[5]) for q in p] == [(2, False, True), (6, True, False)]
    p2 = dog_ref.find_peaks(d, 0.5, ij_threads=3)   # x%3: 6->0 first, 2->2
    assert [q[0] for q in p2] == [6, 2]


def test_quadratic_localization_recovers_paraboloid_vertex():
    """A sampled paraboloid has its exact vertex as the quadratic fit; starting one
    voxel off, the fit moves (LaPlaceFunctions.java:94-119) and converges."""
    z, y, x = np.mgrid[0:12, 0:13, 0:14].astype(np.float64)
    x0, y0, z0 = 6.3, 5.8, 7.4
    f = (-(1 - ((x - x0) ** 2 + 2 * (y - y0) ** 2 + 3 * (z - z0) ** 2) / 50)).astype(np.float32)
    for start in [(6, 6, 7, 0.9), (8, 5, 7, 0.5), (5, 7, 8, 0.5)]:
        (px, py, pz, v), = dog_ref.quadratic_localization(f, [start])
        assert abs(px - x0) < 1e-4 and abs(py - y0) < 1e-4 and abs(pz - z0) < 1e-4
        assert abs(v + 1.0) < 1e-5
    # flat neighbourhood: singular Hessian -> the peak stays as detected
    flat = np.zeros((5, 5, 5), np.float32)
    assert dog_ref.quadratic_localization(flat, [(2, 2, 2, 0.25)]) == [(2.0, 2.0, 2.0, np.float32(0.25))]


def test_input_prep_oracle_rules():
    """SURVEY 8f #1 restatement: blending table, identity resampling, weight
    normalisation rules (BlendingRealRandomAccess.java:25-104,
    WeightNormalizer.java:117-205, NormalizingRandomAccess.java:36-45)."""
    from oracle import input_ref as ir
    assert ir.LUT[0] == 0.0 and abs(ir.LUT[1000] - 1.0) < 1e-12 and abs(ir.LUT[500] - 0.5) < 1e-9
    w = ir.blending_weight(np.array([[0, 5, 5], [10, 5, 5], [5, 5, 5]], np.float32), (11, 11, 11),
                           (0, 0, 0), (4, 4, 4))
    assert w[0] == 0 and w[1] == 0 and w[2] == 1
    rng = np.random.default_rng(3)
    src = (rng.random((6, 7, 8)) + 0.5).astype(np.float32)
    ident = np.hstack([np.eye(3), np.zeros((3, 1))])
    img, _ = ir.transform_view(src, ident, (0, 0, 0), (8, 7, 6), (0, 0, 0), (3, 3, 3), ir.NO_WEIGHTS)
    np.testing.assert_array_equal(img, src)
    shifted = ident.copy()
    shifted[0, 3] = 3.0                                    # view 2 moved 3 voxels in x
    imgs, ws, _ = ir.prepare_inputs([src, src], [ident, shifted], (0, 0, 0), (11, 7, 6), (0, 0, 0),
                                    (2, 2, 2), ir.PRECOMPUTED_WEIGHTS)
    tot = ws[0] + ws[1]
    covered = np.isfinite(tot)
    np.testing.assert_allclose(tot[covered], 1.0, rtol=1e-6)
    imgs, ws, _ = ir.prepare_inputs([src, src], [ident, shifted], (0, 0, 0), (11, 7, 6), (0, 0, 0),
                                    (2, 2, 2), ir.VIRTUAL_WEIGHTS, osem_index=0, osem=3.0)
    assert max(float(w.max()) for w in ws) <= 1.0


def test_psf_oracle_known_answers():
    """ExtractPSF restatement: one bead at an integer location gives the
    normalised crop; the identity model keeps the PSF; a pure z scaling keeps
    the centre voxel and produces odd sizes (ExtractPSF.java:309-346)."""
    from oracle import psf_ref as pr
    rng = np.random.default_rng(3)
    img = rng.random((12, 14, 16)).astype(np.float32)
    p = pr.extract_psf_local(img, [(8.0, 7.0, 6.0)], (5, 5, 3))
    np.testing.assert_array_equal(p, img[5:8, 5:10, 6:11])
    q = pr.extract_psf_local(img, [(0.0, 0.0, 0.0)], (3, 3, 3))     # periodic wrap
    assert q[0, 0, 0] == img[-1, -1, -1]
    n = pr.normalize(p)
    assert n.min() == 0 and n.max() == 1
    np.testing.assert_array_equal(pr.transform_psf(n, np.eye(3, 4)), n)
    size, off = pr.transformed_size((5, 5, 3), [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 2.0, 0])
    assert size == [5, 5, 5] and off == [0.0, 0.0, 0.0]
    t = pr.transform_psf(n, [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 2.0, 0])
    np.testing.assert_array_equal(t[2], n[1])                        # centre plane kept
    np.testing.assert_allclose(t[1], 0.5 * (n[0] + n[1]), rtol=1e-6)


def test_psf_oracle_batched_extraction_is_bit_identical():
    """The chunked extraction used for the many-bead C4 PSFs sums in location order,
    exactly like the per-bead restatement of ExtractPSF.extractPSFLocal (:383-422)."""
    from oracle import psf_ref as pr
    rng = np.random.default_rng(7)
    img = rng.random((30, 26, 22), dtype=np.float32) * 3
    locs = rng.uniform([0, 0, 0], [21, 25, 29], size=(37, 3))
    a = pr.extract_psf_local(img, locs, (7, 5, 9))
    b = pr.extract_psf_local_batched(img, locs, (7, 5, 9), chunk=8)
    np.testing.assert_array_equal(a, b)
