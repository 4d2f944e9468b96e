"""GPU parity of PSF extraction / transformation against
oracle/psf_ref.py (parity unpinned: see DESIGN.md)."""
import numpy as np
import pytest
import torch   # before libspimdecon loads: one HIP runtime in the process (torch's), as in bench.py

from oracle import psf_ref as pr
from spim_registration_amd import psf, synthetic

pytestmark = pytest.mark.gpu

ROT = np.array([[0.92, 0.31, 0.05, 140.0], [-0.29, 0.95, 0.12, -33.0], [0.02, -0.15, 2.4, 7.5]])


def bead_view(shape=(40, 56, 64), cid=21):
    rng = synthetic.rng_for(cid)
    img = rng.normal(100, 3, shape).astype(np.float32)
    locs = []
    z, y, x = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
    for _ in range(12):
        c = rng.uniform([0, 0, 0], [shape[2], shape[1], shape[0]])      # (x, y, z), some near borders
        locs.append(c + rng.normal(0, 0.3, 3))
        img += (500 * np.exp(-((x - c[0]) ** 2 + (y - c[1]) ** 2) / 3.0 - (z - c[2]) ** 2 / 8.0)).astype(np.float32)
    return img.astype(np.float32), np.array(locs)


@pytest.mark.parametrize("size", [(9, 9, 11), (13, 11, 21), (8, 10, 12)])
def test_extract_psf_matches_oracle(gpu, size):
    img, locs = bead_view()
    orig, trans = psf.extract_psf(img, locs, size, ROT)
    eo, et = pr.extract_next_img(img, ROT, locs, size)
    assert orig.shape == eo.shape and trans.shape == et.shape
    np.testing.assert_allclose(orig, eo, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(trans, et, rtol=1e-5, atol=1e-6)
    assert np.mean(orig == eo) > 0.99 and orig.max() == 1.0 and orig.min() == 0.0


def test_extract_psf_identity_model_and_device_input(gpu):
    img, locs = bead_view(cid=22)
    orig, trans = psf.extract_psf(torch.from_numpy(img).cuda(), locs, (11, 11, 15), np.eye(3, 4))
    np.testing.assert_array_equal(orig, trans)                    # identity keeps the centre voxel
    np.testing.assert_allclose(orig, pr.extract_next_img(img, np.eye(3, 4), locs, (11, 11, 15))[0],
                               rtol=1e-6, atol=1e-7)


def test_extract_psf_no_beads_is_nan(gpu):
    img, _ = bead_view(cid=23)
    orig, trans = psf.extract_psf(img, np.zeros((0, 3)), (5, 5, 5))
    assert trans is None and np.isnan(orig).all()                 # 0 / 0 as in normalize


@pytest.mark.parametrize("model", [ROT, np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 3.2, 0.0]]),
                                   np.array([[0, -1.0, 0, 5], [1.0, 0, 0, 2], [0, 0, 1.7, 1]])])
def test_transform_psf_matches_oracle(gpu, model):
    rng = np.random.default_rng(5)
    p = rng.random((21, 17, 15)).astype(np.float32)
    assert psf.transformed_size((15, 17, 21), model) == tuple(map(list, pr.transformed_size((15, 17, 21), model)))
    got = psf.transform_psf(p, model)
    want = pr.transform_psf(p, model)
    assert got.shape == want.shape and all(n % 2 == 1 for n in got.shape)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)


def test_average_transformed_psf_and_max_projection(gpu):
    rng = np.random.default_rng(6)
    ps = [rng.random(s).astype(np.float32) for s in [(21, 13, 11), (17, 15, 12), (9, 9, 9)]]
    np.testing.assert_array_equal(psf.average_transformed_psf(ps), pr.average_transformed_psf(ps))
    a = pr.average_transformed_psf(ps)
    for d in (-1, 0, 1, 2):
        got, used = psf.max_projection(a, d)
        want, wused = pr.max_projection(a, d)
        assert used == wused
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("nbeads", [65, 300])
def test_extract_psf_many_beads_two_phase(gpu, nbeads):
    """More than 64 beads: all (bead, voxel) samples in parallel, then each voxel's
    float sum in bead order -- the same bits as the per-voxel loop and the oracle."""
    img, _ = bead_view(cid=23)
    rng = np.random.default_rng(nbeads)
    locs = rng.uniform([0, 0, 0], [64, 56, 40], size=(nbeads, 3))
    few = psf.extract_psf(img, locs[:64], (9, 9, 11), ROT)[0]          # per-voxel loop path
    orig, trans = psf.extract_psf(img, locs, (9, 9, 11), ROT)
    eo, et = pr.extract_next_img(img, ROT, locs, (9, 9, 11))
    np.testing.assert_allclose(orig, eo, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(trans, et, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(few, pr.extract_next_img(img, ROT, locs[:64], (9, 9, 11))[0], rtol=1e-6, atol=1e-7)


def test_extract_psfs_batch_equals_per_view(gpu):
    """spim_extract_psfs: several views (device tensors, few and many beads, one view
    without beads) at once give the bits of per-view spim_extract_psf calls."""
    views, beads, models = [], [], []
    rng = np.random.default_rng(5)
    for v, nb in enumerate([12, 0, 300, 70]):
        img, locs = bead_view(cid=30 + v)
        if nb != 12:
            locs = rng.uniform([0, 0, 0], [64, 56, 40], size=(nb, 3))
        views.append(torch.from_numpy(img).cuda())
        beads.append(locs)
        models.append(ROT if v % 2 == 0 else np.hstack([np.eye(3), np.zeros((3, 1))]))
    got = psf.extract_psfs(views, beads, (9, 9, 11), models)
    for v in range(4):
        o, t = psf.extract_psf(views[v], beads[v], (9, 9, 11), models[v])
        np.testing.assert_array_equal(got[v][0], o)
        np.testing.assert_array_equal(got[v][1], t)
    host = psf.extract_psfs([x.cpu().numpy() for x in views], beads, (9, 9, 11), None)
    for v in range(4):
        np.testing.assert_array_equal(host[v][0], got[v][0])
        assert host[v][1] is None


def test_release_workspace_then_extract_again(gpu):
    """spim_psf_release_workspace frees the per-view buffers the extraction keeps
    between calls (on one device and on all); later calls reallocate and give the
    same bits."""
    img, locs = bead_view(cid=41)
    first = psf.extract_psfs([img, img], [locs, locs[:5]], (9, 9, 11), [ROT, ROT])
    psf.release_workspace(0)
    again = psf.extract_psfs([img, img], [locs, locs[:5]], (9, 9, 11), [ROT, ROT])
    psf.release_workspace()
    single = psf.extract_psf(img, locs, (9, 9, 11), ROT)
    for a, b in zip(first, again):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(single[1], first[0][1])
    psf.release_workspace(0)
