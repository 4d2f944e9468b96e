"""GPU: the HIP path against the committed golden vectors (tests/golden)."""
import glob
import os

import numpy as np
import pytest

from conftest import rel_l2
from spim_registration_amd import dog, legacy
from spim_registration_amd.decon import PSFTYPE, Session

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "rl_*.npz"))))
def test_rl_against_golden(gpu, path):
    g = np.load(path)
    imgs, ws, psfs = g["imgs"], g["weights"], g["psfs"]
    nz, ny, nx = imgs.shape[1:]
    with Session((nx, ny, nz), ij_threads=int(g["ij_threads"])) as s:
        for i, w, k in zip(imgs, ws, psfs):
            s.add_view(i, w, k)
        s.init(PSFTYPE(int(g["psftype"])))
        for v in range(len(psfs)):
            k1, k2 = s.get_kernels(v, psfs[v].shape)
            assert rel_l2(k1, g["k1"][v]) < 1e-6
            assert rel_l2(k2, g["k2"][v]) < 1e-5
        avg = s.init_psi()
        assert abs(avg - float(g["avg"])) <= 1e-12 * abs(float(g["avg"]))
        st = s.run(int(g["iters"]), float(g["lam"]))
        s.apply_mask()
        psi = s.get_psi()
    assert rel_l2(psi, g["psi"]) < 1e-4
    np.testing.assert_allclose(st[:, :, 0], g["stats"][:, :, 0], rtol=1e-3)


def test_conv_against_golden(gpu):
    g = np.load(os.path.join(GOLD, "conv.npz"))
    cuda = legacy.CUDAFourierConvolution()
    blk = g["block"].copy()
    cuda.convolution3DfftCUDAInPlace(blk.reshape(-1), list(blk.shape), g["k"], list(g["k"].shape), 0)
    assert rel_l2(blk, g["circular"]) < 1e-6
    for ext in ("mirror", "one"):
        out = legacy.convolve_blocks_cuda(g["a"], g["k"], (16, 14, 12), ext, cuda, 0)
        assert rel_l2(out, g[ext]) < 1e-6


def test_dog_against_golden(gpu):
    g = np.load(os.path.join(GOLD, "dog.npz"))
    pts, d = dog.compute(g["img"], 1.8, 0.008, return_dog=True, keep_intensity=True)
    np.testing.assert_array_equal(d, g["dog"])
    np.testing.assert_array_equal(dog.peaks_array(pts), g["peaks"])
