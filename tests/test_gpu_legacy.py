"""GPU parity of the legacy JNA-facing exports (FourierConvolutionCUDALib,
CUDAStandardFunctions, SeparableConvolutionCUDALib) against the oracle."""
import numpy as np
import pytest

from conftest import rel_l2
from oracle import dog_ref, mvdecon_ref as ref
from spim_registration_amd import legacy, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bdims,kdims", [((32, 30, 28), (7, 9, 11)), ((17, 23, 29), (5, 5, 5)),
                                         ((16, 16, 16), (15, 15, 15))])
def test_convolution3dfft_inplace_circular(gpu, bdims, kdims):
    rng = np.random.default_rng(1)
    blk = rng.random(bdims).astype(np.float32)
    k = rng.random(kdims).astype(np.float32)
    cuda = legacy.CUDAFourierConvolution()
    im = blk.copy()
    cuda.convolution3DfftCUDAInPlace(im.reshape(-1), list(bdims), k, list(kdims), 0)
    exp = ref.circular_convolve_block(blk, k)
    assert rel_l2(im, exp) < 1e-6
    out = cuda.convolution3DfftCUDA(blk.reshape(-1), list(bdims), k, list(kdims), 0)
    assert rel_l2(out.reshape(bdims), exp) < 1e-6


@pytest.mark.parametrize("ext", ["mirror", "one"])
def test_blocked_convolution_matches_whole(gpu, ext):
    """MVDeconFFTThreads.convolve{1,2}BlockCUDA: precise blocks == whole-volume conv."""
    rng = np.random.default_rng(2)
    img = rng.random((37, 41, 45)).astype(np.float32)
    k = synthetic.psf(1, 3, (9, 7, 11))
    cuda = legacy.CUDAFourierConvolution()
    out = legacy.convolve_blocks_cuda(img, k, (24, 20, 28), ext, cuda, 0)
    exp = ref.convolve(img, k, ext)
    assert rel_l2(out, exp) < 1e-6
    exp2 = ref.blocked_convolve(img, k, (24, 20, 28), ext)
    assert rel_l2(out, exp2) < 1e-6


def test_device_query(gpu):
    f = legacy.CUDAStandardFunctions()
    n = f.getNumDevicesCUDA()
    assert n >= 1
    name = f.getNameDeviceCUDA(0)
    assert "gfx950" in name
    assert f.getMemDeviceCUDA(0) > 200 * 2 ** 30
    assert 0 < f.getFreeMemDeviceCUDA(0) <= f.getMemDeviceCUDA(0)
    assert f.getCUDAcomputeCapabilityMajorVersion(0) == 9
    assert f.getCUDAcomputeCapabilityMinorVersion(0) == 5
    assert f.getMemDeviceCUDA(-1) == -1          # invalid device -> error, no CPU emulation


@pytest.mark.parametrize("sigmas", [[1.7, 2.0, 1.2],     # 15-tap kernels
                                    [6.0, 3.0, 9.5]])    # 63-tap kernels: halos wider than the image
@pytest.mark.parametrize("oob", [legacy.OutOfBounds.ZERO, legacy.OutOfBounds.VALUE,
                                 legacy.OutOfBounds.EXTEND_BORDER_PIXELS, legacy.OutOfBounds.MIRROR_SINGLE])
def test_separable_convolve_n(gpu, oob, sigmas):
    rng = np.random.default_rng(3)
    img = rng.random((13, 17, 19)).astype(np.float32)
    cuda = legacy.CUDASeparableConvolution()
    im = img.copy().reshape(-1)
    ok = legacy.gauss(im, [19, 17, 13], sigmas, oob, 0.25, cuda, 0)
    assert ok
    ks = legacy.get_cuda_kernels(sigmas)
    mode = {0: "zero", 1: "value", 2: "border", 3: "mirror"}[int(oob)]
    exp = dog_ref.gauss3d(img, ks, mode, 0.25)
    np.testing.assert_array_equal(im.reshape(img.shape), exp)


def test_separable_convolve_bad_device(gpu):
    cuda = legacy.CUDASeparableConvolution()
    im = np.ones(27, np.float32)
    k = np.zeros(7, np.float32)
    k[3] = 1
    assert cuda.convolve_7(im, k, k, k, 3, 3, 3, True, True, True, 0, 0.0, -1) is False


def test_convolution3dfft_concurrent_threads(gpu):
    """MVDeconFFT.java:424-446 calls convolution3DfftCUDAInPlace from one Java thread
    per device at once: the export serialises per device (mutex, stream, caches) and
    every concurrent call returns its own block's convolution.  ctypes releases the
    GIL around the foreign call, so the calls really overlap."""
    import threading
    rng = np.random.default_rng(3)
    shapes = [(32, 30, 28), (24, 26, 20), (32, 30, 28), (17, 23, 29)] * 3
    blks = [rng.random(s).astype(np.float32) for s in shapes]
    ks = [rng.random((5, 7, 9)).astype(np.float32) for _ in shapes]
    cuda = legacy.CUDAFourierConvolution()
    outs = [b.copy() for b in blks]
    errs = []

    def work(i):
        try:
            cuda.convolution3DfftCUDAInPlace(outs[i].reshape(-1), list(shapes[i]), ks[i], [5, 7, 9], 0)
        except Exception as e:      # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(blks))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for b, k, o in zip(blks, ks, outs):
        assert rel_l2(o, ref.circular_convolve_block(b, k)) < 1e-6


def test_convolution3dfft_plan_cache_bounded(gpu):
    """the per-device plan cache keeps at most 4 block shapes, so walking
    many block sizes does not grow device memory without bound."""
    f = legacy.CUDAStandardFunctions()
    cuda = legacy.CUDAFourierConvolution()
    rng = np.random.default_rng(4)
    k = rng.random((3, 3, 3)).astype(np.float32)
    free = []
    for i in range(12):
        s = (96 + 2 * i, 96, 96)
        blk = rng.random(s).astype(np.float32)
        cuda.convolution3DfftCUDAInPlace(blk.reshape(-1), list(s), k, [3, 3, 3], 0)
        free.append(f.getFreeMemDeviceCUDA(0))
    # after the cache is full (4 shapes), free memory stops falling by a block's worth per call
    assert min(free[6:]) > free[5] - 64 * 2 ** 20, [x >> 20 for x in free]
