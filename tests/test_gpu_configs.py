"""GPU: every BASELINE.json config exercised at its full size.

The oracle is a numpy restatement, so full-size comparisons against it use its
float32 scipy.fft variant (``precision="f32"``, 16 worker threads -- the box's CPU
share) for a bounded number of iterations; the rest of each config is checked
through size-independent properties and against the rocFFT backend (an
independent FFT implementation of the same RL) at full size:

  C1  2-view 256x256x128 weighted-average fusion       vs oracle, every voxel
  C2  4-view 512^3 RL, INDEPENDENT, lambda 0            vs oracle (2 iterations, rel-L2 1e-4);
                                                        10 iterations: finite, change shrinking, no voxel masked
  C3  6-view 1024x1024x512, EFFICIENT_BAYESIAN, 0.006   20 iterations on the 8-device code path (8 device
                                                        groups on this GPU) and on one slab, both vs the
                                                        rocFFT backend (rel-L2 1e-5); the same path vs the
                                                        oracle on a 256x256x128 instance
  C4  768^3 view DoG                                    bit-exact DoG and identical peaks vs oracle on crops
                                                        (the DoG at a voxel depends on a 15^3 neighbourhood)
  C5  6-view 2048x2048x128 fp16 slab, OPTIMIZATION_I    engine (fast path asserted) vs rocFFT backend
"""
import numpy as np
import pytest
import torch  # before the library loads (one shared HIP runtime, spim_registration_amd._lib.load)

from conftest import rel_l2
from oracle import dog_ref
from oracle import fusion_ref as fr
from oracle import mvdecon_ref as ref
from spim_registration_amd import dog, synthetic
from spim_registration_amd.decon import PSFTYPE, Session
from spim_registration_amd.input_prep import fuse_weighted_average

pytestmark = pytest.mark.gpu

TOL = 1e-4            # north star: within 1e-4 rel-L2 of the CPU reference
ENGINE_VS_ROCFFT = 1e-5
CPU_WORKERS = 16      # the GPU box's CPU share per GPU


def release():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def session_from_device(imgs, ws, psfs, psftype, **kw):
    shape = tuple(imgs[0].shape)
    s = Session(shape[::-1], **kw)
    for i, w, k in zip(imgs, ws, psfs):
        s.add_view_device(i.data_ptr(), w.data_ptr(), k)
    s.init(psftype)
    s.init_psi()
    return s


def run_to_host(imgs, ws, psfs, psftype, iters, lam, **kw):
    with session_from_device(imgs, ws, psfs, psftype, **kw) as s:
        st = s.run(iters, lam)
        s.apply_mask()
        info = {"fft_dims": s.fft_dims(0), "zpass": s.zpass_mode(0), "xpass": s.xpass_mode(0),
                "slabs": s.num_slabs(), "extent0": s.slab_extent(0)}
        return s.get_psi(), st, info


# ------------------------------------------------------------------ C1

@pytest.mark.timeout(300)
def test_c1_fusion_2view_256x256x128(gpu):
    """BASELINE configs[0]: 2-view weighted-average fusion (n-linear, blending: the
    reference defaults) into a 256x256x128 box, every voxel against the oracle."""
    rng = np.random.default_rng(20140612)
    shape = (120, 200, 210)                       # source stacks [z, y, x]
    srcs, models = [], []
    for v in range(2):
        srcs.append((rng.random(shape, dtype=np.float32) * 100 + 1).astype(np.float32))
        c, s = np.cos(np.radians(90.0 * v + 3)), np.sin(np.radians(90.0 * v + 3))
        a = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]]) @ np.diag([1.0, 1.0, 1.4])
        m = np.zeros((3, 4))
        m[:, :3] = a
        m[:, 3] = [60.0 + 37.5 * v, 20.25, 40.0 - 11.0 * v]
        models.append(m)
    bb_min, bb_dims = (-40, 0, -60), (256, 256, 128)
    borders, ranges = [(0, 0, 0), (0, 0, 0)], [(12, 12, 12), (12, 12, 12)]
    got = fuse_weighted_average(srcs, models, bb_min, bb_dims, 1.0, 1, True, borders, ranges)
    want = fr.fuse_weighted_average(srcs, models, bb_min, bb_dims, 1.0, 1, True, borders, ranges)
    assert got.shape == (128, 256, 256)
    assert (want > 0).mean() > 0.3 and (want == 0).any()
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=1e-4)


# ------------------------------------------------------------------ C2

@pytest.fixture(scope="module")
def c2_data(gpu):
    imgs, ws, psfs = synthetic.make_views_torch((512, 512, 512), 4, config_id=2, ksize=(25, 25, 25),
                                                device="cuda:0")
    release()
    yield imgs, ws, psfs
    del imgs, ws
    release()


@pytest.mark.timeout(600)
def test_c2_4view_512_matches_oracle(gpu, c2_data):
    imgs, ws, psfs = c2_data
    psi, st, info = run_to_host(imgs, ws, psfs, PSFTYPE.INDEPENDENT, 2, 0.0)
    assert info["zpass"] in (2, 3, 4) and info["xpass"] == 2, info  # the fast engine passes ran
    himgs = [i.cpu().numpy() for i in imgs]
    hws = [w.cpu().numpy() for w in ws]
    res = ref.mv_deconvolution(himgs, hws, psfs, PSFTYPE.INDEPENDENT, 2, 0.0, precision="f32",
                               workers=CPU_WORKERS)
    err = rel_l2(psi, res.psi)
    assert err < TOL, err
    np.testing.assert_allclose(st[:, :, 0], np.array(res.stats)[:, :, 0], rtol=1e-3)


@pytest.mark.timeout(300)
def test_c2_4view_512_ten_iterations(gpu, c2_data):
    imgs, ws, psfs = c2_data
    psi, st, _ = run_to_host(imgs, ws, psfs, PSFTYPE.INDEPENDENT, 10, 0.0)
    assert np.isfinite(psi).all() and np.isfinite(st).all()
    assert (psi > 0).all()                 # every voxel covered: the final mask keeps all
    tot = st[:, :, 0].sum(axis=1)          # sumChange over the views, per iteration
    assert tot[-1] < 0.5 * tot[0], tot
    assert all(tot[i + 1] <= tot[i] * 1.0001 for i in range(1, len(tot) - 1)), tot


# ------------------------------------------------------------------ C3

@pytest.mark.timeout(600)
def test_c3_6view_1024x1024x512_tikhonov_20_iterations(gpu):
    imgs, ws, psfs = synthetic.make_views_torch((512, 1024, 1024), 6, config_id=3, ksize=(25, 25, 25),
                                                device="cuda:0")
    release()
    args = (imgs, ws, psfs, PSFTYPE.EFFICIENT_BAYESIAN, 20, 0.006)
    # the 8-GPU decomposition (the longer axis: 8 y-slabs of 128 rows, kept as (x, z, y)
    # rows; halo pulls between device groups), all groups on this GPU
    psi8, st8, info8 = run_to_host(*args, devices=[0] * 8)
    release()
    assert info8["slabs"] == 8 and info8["extent0"] == (1024, 512, 128), info8
    # one slab of 1024x1024x512: spectra of 2.38 GB on the fast engine passes
    psi1, st1, info1 = run_to_host(*args)
    release()
    assert info1["fft_dims"] == (1050, 1050, 536) and info1["zpass"] in (2, 3, 4) and info1["xpass"] == 2, info1
    psir, str_, _ = run_to_host(*args, fft_backend="rocfft")
    del imgs, ws
    release()
    assert np.isfinite(psi8).all()
    assert rel_l2(psi8, psir) < ENGINE_VS_ROCFFT
    assert rel_l2(psi1, psir) < ENGINE_VS_ROCFFT
    np.testing.assert_allclose(st8, str_, rtol=1e-4)
    np.testing.assert_allclose(st1, str_, rtol=1e-4)


@pytest.mark.timeout(300)
def test_c3_decomposition_matches_oracle_256x256x128(gpu):
    imgs, ws, psfs = synthetic.make_views_torch((128, 256, 256), 6, config_id=30, ksize=(25, 25, 25),
                                                device="cuda:0")
    psi, st, _ = run_to_host(imgs, ws, psfs, PSFTYPE.EFFICIENT_BAYESIAN, 3, 0.006, devices=[0] * 8)
    himgs = [i.cpu().numpy() for i in imgs]
    hws = [w.cpu().numpy() for w in ws]
    del imgs, ws
    release()
    res = ref.mv_deconvolution(himgs, hws, psfs, PSFTYPE.EFFICIENT_BAYESIAN, 3, 0.006, precision="f32",
                               workers=CPU_WORKERS)
    assert rel_l2(psi, res.psi) < TOL
    np.testing.assert_allclose(st[:, :, 0], np.array(res.stats)[:, :, 0], rtol=1e-3)


# ------------------------------------------------------------------ C4

def bead_stack_torch(shape, seed, spacing=20):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    n = int(np.prod(shape))
    img = torch.full(shape, 0.05, device="cuda:0")
    nb = n // spacing ** 3
    nz, ny, nx = shape
    zyx = [torch.randint(1, m - 1, (nb,), generator=g, device="cuda:0") for m in shape]
    idx = (zyx[0] * ny + zyx[1]) * nx + zyx[2]
    amp = 0.5 + torch.rand(nb, generator=g, device="cuda:0")
    for dz in (-1, 0, 1):                  # a 3x3x3 bead footprint
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                f = 0.6 ** (abs(dz) + abs(dy) + abs(dx))
                img.view(-1).index_add_(0, idx + (dz * ny + dy) * nx + dx, amp * f)
    img.clamp_(max=2.0)                    # (coinciding beads must not set the intensity range)
    img += 0.01 * torch.randn(shape, generator=g, device="cuda:0")
    return img.cpu().numpy()


@pytest.mark.timeout(600)
def test_c4_dog_768_matches_oracle_on_crops(gpu):
    shape = (768, 768, 768)
    img = bead_stack_torch(shape, 20140614)
    release()
    pts, d = dog.compute(img, sigma=1.8, threshold=0.008, return_dog=True, keep_intensity=True)
    mn, mx = float(img.min()), float(img.max())
    T = 8
    got = np.array([[int(c) for c in p.location] for p in pts], np.int64)   # x, y, z
    assert len(got) > 10000
    # global order: per-thread lists by x % T, each in flat order (InteractiveIntegral.java:394)
    flat = (got[:, 2] * shape[1] + got[:, 1]) * shape[2] + got[:, 0]
    key = (got[:, 0] % T) * (np.int64(1) << 40) + flat
    assert (np.diff(key) > 0).all()
    # DoG at a voxel depends on its 15^3 neighbourhood (7-voxel kernel radius per pass):
    # an oracle run on a crop with a 7-voxel rim reproduces the full-volume DoG bit for
    # bit inside the rim (and up to a face that is the volume's own face)
    R = 7
    n = 96
    starts = [(0, 0, 0), (768 - n, 768 - n, 768 - n), (0, 768 - n, 384), (352, 200, 768 - n),
              (400, 400, 400), (123, 611, 40)]
    for z0, y0, x0 in starts:
        c0 = [max(0, z0 - R), max(0, y0 - R), max(0, x0 - R)]
        c0[2] -= c0[2] % T                           # crop-local x % T == global x % T
        c1 = [min(768, z0 + n + R), min(768, y0 + n + R), min(768, x0 + n + R)]
        crop = img[c0[0]:c1[0], c0[1]:c1[1], c0[2]:c1[2]]
        peaks, dref = dog_ref.process_dog(crop, 1.8, 0.008, min_intensity=mn, max_intensity=mx)
        # verified region: R voxels inside every crop face that is not a volume face
        lo = [0 if c0[a] == 0 else R for a in range(3)]
        hi = [dref.shape[a] - (0 if c1[a] == 768 else R) for a in range(3)]
        np.testing.assert_array_equal(
            d[c0[0] + lo[0]:c0[0] + hi[0], c0[1] + lo[1]:c0[1] + hi[1], c0[2] + lo[2]:c0[2] + hi[2]],
            dref[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]])
        # peaks need their 26 neighbours inside the verified region
        plo = [lo[a] + (1 if lo[a] else 0) for a in range(3)]
        phi = [hi[a] - (1 if hi[a] < dref.shape[a] else 0) for a in range(3)]
        exp = [(p[0] + c0[2], p[1] + c0[1], p[2] + c0[0]) for p in peaks
               if plo[2] <= p[0] < phi[2] and plo[1] <= p[1] < phi[1] and plo[0] <= p[2] < phi[0]]
        sel = ((got[:, 0] >= c0[2] + plo[2]) & (got[:, 0] < c0[2] + phi[2]) & (got[:, 1] >= c0[1] + plo[1])
               & (got[:, 1] < c0[1] + phi[1]) & (got[:, 2] >= c0[0] + plo[0]) & (got[:, 2] < c0[0] + phi[0]))
        assert [tuple(int(v) for v in r) for r in got[sel]] == exp, (z0, y0, x0)


# ------------------------------------------------------------------ C5

@pytest.mark.timeout(600)
def test_c5_fp16_2048x2048x128_slab(gpu):
    imgs, ws, psfs = synthetic.make_views_torch((128, 2048, 2048), 6, config_id=5, ksize=(25, 25, 25),
                                                device="cuda:0")
    release()
    args = (imgs, ws, psfs, PSFTYPE.OPTIMIZATION_I, 2, 0.006)
    psi, st, info = run_to_host(*args, storage_fp16=True)
    release()
    assert info["fft_dims"] == (2100, 2100, 152), info
    assert info["zpass"] in (2, 3, 4) and info["xpass"] == 2, info  # the fast engine, not Stockham
    psir, str_, _ = run_to_host(*args, storage_fp16=True, fft_backend="rocfft")
    del imgs, ws
    release()
    assert np.isfinite(psi).all()
    assert rel_l2(psi, psir) < ENGINE_VS_ROCFFT
    np.testing.assert_allclose(st, str_, rtol=1e-4)
