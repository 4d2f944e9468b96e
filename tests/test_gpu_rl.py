"""GPU parity of the RL deconvolution path against the oracle (through the C-ABI).

Tolerance: the north star's 1e-4 relative L2 on psi (float32 FFT on the GPU vs
float64-FFT oracle); observed values are ~1e-6.  Pointwise kernels are
bit-exact given identical convolution outputs (tested separately with a delta
PSF, where the convolution is exact).
"""
import numpy as np
import pytest

from conftest import rel_l2
from oracle import mvdecon_ref as ref
from spim_registration_amd import synthetic
from spim_registration_amd.decon import (MVDeconFFT, MVDeconInput, MVDeconvolution, PSFTYPE,
                                         Session, prepare_kernels)

pytestmark = pytest.mark.gpu

TOL = 1e-4


def small_case(shape=(20, 24, 28), V=3, ksize=(7, 9, 11), weights="blend", partial=False, cid=7):
    return synthetic.make_views(shape, V, config_id=cid, ksize=ksize, weights=weights,
                                partial=partial, bead_density=1.0 / 6 ** 3)


@pytest.mark.parametrize("psftype", list(PSFTYPE))
def test_prepare_kernels_matches_oracle(gpu, psftype):
    # different kernel sizes per view exercise the 'same'-size compound convolutions
    ks = [synthetic.psf(0, 3, (7, 9, 11)), synthetic.psf(1, 3, (9, 7, 11)), synthetic.psf(2, 3, (5, 9, 7))]
    ks = [(k * 3.7).astype(np.float32) for k in ks]   # un-normalised input
    views = [MVDeconFFT(np.ones((4, 4, 4)), np.ones((4, 4, 4)), k) for k in ks]
    k1, k2 = prepare_kernels(views, psftype, ij_threads=8)
    r1, r2 = ref.prepare_kernels(ks, psftype, 8)
    for a, b in zip(k1, r1):
        assert rel_l2(a, b) < 1e-6
    for a, b in zip(k2, r2):
        assert rel_l2(a, b) < 1e-5


@pytest.mark.parametrize("psftype", [PSFTYPE.OPTIMIZATION_I, PSFTYPE.OPTIMIZATION_II])
def test_prepare_kernels_large_compound(gpu, psftype):
    """Kernels of 45-degree-transformed PSFs (31 x 19 x 31): the compound convolutions
    split each output's taps over a block (k_conv_same_zero_blk)."""
    ks = [synthetic.psf(v, 4, (31, 19, 31)) for v in range(3)] + [synthetic.psf(3, 4, (25, 19, 21))]
    views = [MVDeconFFT(np.ones((4, 4, 4)), np.ones((4, 4, 4)), k) for k in ks]
    k1, k2 = prepare_kernels(views, psftype, ij_threads=8)
    r1, r2 = ref.prepare_kernels(ks, psftype, 8)
    for a, b in zip(k1, r1):
        assert rel_l2(a, b) < 1e-6
    for a, b in zip(k2, r2):
        assert rel_l2(a, b) < 1e-5


@pytest.mark.parametrize("T", [1, 3, 8])
def test_norm_quirk_thread_count(gpu, T):
    k = synthetic.psf(0, 1, (9, 9, 13))
    views = [MVDeconFFT(np.ones((2, 2, 2)), np.ones((2, 2, 2)), k)]
    k1, _ = prepare_kernels(views, PSFTYPE.INDEPENDENT, ij_threads=T)
    r1 = ref.norm_img(k, T)
    np.testing.assert_allclose(k1[0], r1, rtol=2e-7, atol=0)
    # the double count makes the kernel sum S / (S + P0) < 1 (AdjustInput.java:93-97)
    assert float(k1[0].astype(np.float64).sum()) < 1.0 - 1e-6


@pytest.mark.parametrize("psftype,lam,weights,partial", [
    (PSFTYPE.INDEPENDENT, 0.0, "ones", False),
    (PSFTYPE.INDEPENDENT, 0.006, "blend", False),
    (PSFTYPE.OPTIMIZATION_I, 0.006, "blend", True),
    (PSFTYPE.OPTIMIZATION_II, 0.0, "blend", False),
    (PSFTYPE.EFFICIENT_BAYESIAN, 0.006, "blend", True),
])
def test_mvdeconvolution_matches_oracle(gpu, psftype, lam, weights, partial):
    imgs, ws, ks, _ = small_case(weights=weights, partial=partial)
    iters = 5
    inp = MVDeconInput()
    for i, w, k in zip(imgs, ws, ks):
        inp.add(MVDeconFFT(i, w, k, device_list=[0]))
    dec = MVDeconvolution(inp, psftype, iters, lam, ij_threads=8)
    psi = dec.get_psi()
    res = ref.mv_deconvolution(imgs, ws, ks, psftype, iters, lam, ij_threads=8)
    assert np.isfinite(psi).all()
    err = rel_l2(psi, res.psi)
    assert err < TOL, err
    # per-view statistics (sumChange, maxChange) follow the reference's log
    st = np.array(res.stats)
    np.testing.assert_allclose(dec.stats[:, :, 0], st[:, :, 0], rtol=1e-3)
    np.testing.assert_allclose(dec.stats[:, :, 1], st[:, :, 1], rtol=1e-2, atol=1e-6)
    assert abs(dec.avg - res.avg) <= 1e-12 * abs(res.avg)
    if partial:
        # voxels covered by no view stay masked exactly like the reference
        assert ((psi == 0) == (res.psi == 0)).all()


def test_delta_psf_identity(gpu):
    """Delta PSF: both convolutions are the identity up to the float32 FFT round
    trip, so psi follows the oracle to ~1 ulp-level relative error."""
    imgs, ws, _, _ = small_case(V=2)
    k = np.zeros((3, 3, 3), np.float32)
    k[1, 1, 1] = 1.0
    with Session((28, 24, 20)) as s:
        for i, w in zip(imgs, ws):
            s.add_view(i, w, k)
        s.init(PSFTYPE.INDEPENDENT)
        s.init_psi()
        s.run(3, 0.006)
        psi = s.get_psi()                      # (no mask step here)
    res = ref.mv_deconvolution(imgs, ws, [k, k], PSFTYPE.INDEPENDENT, 3, 0.006)
    cnt, _ = ref.first_iteration(imgs)
    a, b = psi[cnt > 0], res.psi[cnt > 0]
    assert rel_l2(a, b) < 1e-6
    assert np.max(np.abs(a - b) / np.abs(b)) < 1e-4


@pytest.mark.parametrize("slabs", [2, 3, 4, 6])   # 6: slabs too thin for the overlapped exchange
def test_virtual_slabs_match_single(gpu, slabs):
    """z-slab decomposition with halo exchange (the multi-GPU path on one GPU)."""
    imgs, ws, ks, _ = small_case(shape=(40, 20, 22), V=2, ksize=(5, 7, 9))
    out = []
    for S in (1, slabs):
        with Session((22, 20, 40), local_slabs=S) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            s.init_psi()
            st = s.run(4, 0.006)
            s.apply_mask()
            out.append((s.get_psi(), st))
    assert rel_l2(out[1][0], out[0][0]) < 1e-5
    np.testing.assert_allclose(out[1][1], out[0][1], rtol=1e-4)
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 4, 0.006)
    assert rel_l2(out[1][0], res.psi) < TOL


@pytest.mark.parametrize("shape,ksize", [((20, 24, 28), (7, 9, 11)), ((33, 17, 46), (5, 7, 3)),
                                         ((9, 40, 12), (11, 5, 9))])
def test_engine_matches_rocfft_backend(gpu, shape, ksize):
    """The fused spectral engine and the rocFFT backend compute the same RL."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for be in ("engine", "rocfft"):
        with Session(shape[::-1], fft_backend=be) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.EFFICIENT_BAYESIAN)
            s.init_psi()
            st = s.run(3, 0.006)
            s.apply_mask()
            out.append((s.get_psi(), st))
    assert rel_l2(out[0][0], out[1][0]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.EFFICIENT_BAYESIAN, 3, 0.006)
    assert rel_l2(out[0][0], res.psi) < TOL


@pytest.mark.parametrize("policy", ["fast", "smooth"])
@pytest.mark.parametrize("shape,ksize", [((20, 24, 28), (7, 9, 11)), ((33, 17, 46), (5, 7, 3)),
                                         ((30, 61, 40), (9, 5, 7)), ((12, 14, 500), (3, 3, 25)),
                                         ((10, 500, 12), (3, 25, 3)), ((500, 10, 12), (25, 3, 3)),
                                         # M = 1050 = 30*35: the TR = 64 two-factor passes (x tile,
                                         # y column pass; the z pass falls back to Stockham)
                                         ((12, 14, 1024), (3, 3, 27)), ((10, 1024, 12), (3, 27, 3)),
                                         ((1024, 10, 12), (27, 3, 3))])
def test_engine_pad_policies(gpu, shape, ksize, policy):
    """Two-factor register passes ("fast") and Stockham passes ("smooth") agree
    with the rocFFT backend and the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for be, pol in (("engine", policy), ("rocfft", "auto")):
        with Session(shape[::-1], fft_backend=be, fft_pad_policy=pol) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_II)
            s.init_psi()
            st = s.run(3, 0.0)
            s.apply_mask()
            out.append((s.get_psi(), st, s.fft_dims()))
    assert rel_l2(out[0][0], out[1][0]) < 1e-5, out[0][2]
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_II, 3, 0.0)
    assert rel_l2(out[0][0], res.psi) < TOL


@pytest.mark.parametrize("fp16", [False, True])
@pytest.mark.parametrize("psftype,lam", [(PSFTYPE.OPTIMIZATION_II, 0.0), (PSFTYPE.EFFICIENT_BAYESIAN, 0.006)])
def test_x_tiles_2100_wave_tiles(gpu, fp16, psftype, lam):
    """x = 2048 pads to Mx = 2100 = 42 * 50: the wave x tiles (one wave per block, one row
    pair, no block barrier; xt_wave) in every mode -- psi spectra, quotient, plain and
    Tikhonov update -- for f32 and fp16 storage, against the rocFFT backend and the oracle
    (on the fp16-rounded inputs when fp16)."""
    shape, ksize = (10, 12, 2048), (21, 3, 3)
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for be in ("engine", "rocfft"):
        with Session(shape[::-1], fft_backend=be, storage_fp16=fp16) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(psftype)
            s.init_psi()
            st = s.run(3, lam)
            s.apply_mask()
            out.append((s.get_psi(), st, s.fft_dims(), s.xpass_mode()))
    assert out[0][2][0] == 2100 and out[0][3] == 2, out[0][2:]
    assert rel_l2(out[0][0], out[1][0]) < 1e-5
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-3)
    if fp16:
        imgs = [i.astype(np.float16).astype(np.float32) for i in imgs]
        ws = [w.astype(np.float16).astype(np.float32) for w in ws]
    res = ref.mv_deconvolution(imgs, ws, ks, psftype, 3, lam)
    assert rel_l2(out[0][0], res.psi) < TOL


def test_initial_image_and_incremental_iterations(gpu):
    imgs, ws, ks, _ = small_case(V=2)
    init = imgs[0].copy()
    init[0, 0, :4] = -1.0      # checkNumbers clamp: <= 0 -> minValue
    with Session((28, 24, 20)) as s:
        for i, w, k in zip(imgs, ws, ks):
            s.add_view(i, w, k)
        s.init(PSFTYPE.INDEPENDENT)
        s.init_psi(init)
        s.run(2, 0.0)
        s.run(1, 0.0)           # iterations continue from the resident psi
        psi = s.get_psi()
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.INDEPENDENT, 3, 0.0, initial_psi=init)
    cnt, _ = ref.first_iteration(imgs)
    res_psi = res.psi.copy()
    assert rel_l2(psi[cnt > 0], res_psi[cnt > 0]) < TOL


def test_fp16_storage(gpu):
    """img/weights stored as fp16 (config-5 mode): compared with the oracle run
    on the fp16-rounded inputs; psi and all arithmetic stay fp32."""
    imgs, ws, ks, _ = small_case(V=2)
    with Session((28, 24, 20), storage_fp16=True) as s:
        for i, w, k in zip(imgs, ws, ks):
            s.add_view(i, w, k)
        s.init(PSFTYPE.OPTIMIZATION_I)
        s.init_psi()
        s.run(4, 0.006)
        s.apply_mask()
        psi = s.get_psi()
    hi = [i.astype(np.float16).astype(np.float32) for i in imgs]
    hw = [w.astype(np.float16).astype(np.float32) for w in ws]
    res = ref.mv_deconvolution(hi, hw, ks, PSFTYPE.OPTIMIZATION_I, 4, 0.006)
    assert rel_l2(psi, res.psi) < TOL


def test_no_cpu_device(gpu):
    with pytest.raises(ValueError):
        MVDeconFFT(np.ones((3, 3, 3)), np.ones((3, 3, 3)), np.ones((3, 3, 3)), device_list=[-1])
    from spim_registration_amd._lib import SpimDeconError
    with pytest.raises(SpimDeconError):
        Session((8, 8, 8), device=-1)


@pytest.mark.parametrize("shape,ksize", [((40, 18, 22), (9, 5, 7)),       # Mz 48 = 6*8
                                         ((520, 10, 12), (3, 3, 17)),     # Mz 540 = 20*27, kc 8
                                         ((516, 10, 12), (3, 3, 25)),     # Mz 540, kc 12 (4 outputs)
                                         ((100, 16, 14), (5, 7, 15))])    # Mz 128 = 8*16
def test_compact_kernel_z_pass(gpu, shape, ksize, monkeypatch):
    """The two compact-kernel z passes -- the direct circular convolution with the
    kernel's 2cz+1 non-zero planes (default) and the fused FFT z pass that builds the
    kernel's z transform from them (SPIMDECON_ZDIRECT=0; needs 2cz+1 <= N2 of the
    two-factor z length) -- agree with the full precomputed kernel spectra
    (SPIMDECON_ZK=full) and the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for zk, zd, mode in (("compact", "1", (3,)), ("compact", "0", (1,)), ("full", "1", (0,))):
        monkeypatch.setenv("SPIMDECON_ZK", zk)
        monkeypatch.setenv("SPIMDECON_ZDIRECT", zd)
        with Session(shape[::-1], fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            assert s.zpass_mode() in mode
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            out.append(s.get_psi())
    assert not np.array_equal(out[0], out[2]), "direct path not taken (identical bits)"
    assert not np.array_equal(out[1], out[2]), "compact FFT path not taken (identical bits)"
    assert rel_l2(out[0], out[2]) < 1e-5
    assert rel_l2(out[1], out[2]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL



@pytest.mark.parametrize("shape,ksize", [((100, 10, 12), (3, 3, 31)),     # kc 15: 33-tap bound, OPT 1 / 5
                                         ((300, 10, 12), (3, 5, 33)),     # kc 16, 9 outputs per round
                                         ((60, 12, 14), (3, 3, 25)),      # kc 12 on the LDS-DMA kernel
                                         ((530, 8, 12), (3, 3, 9)),       # kc 4, 17 outputs per round
                                         ((512, 13, 12), (3, 3, 25)),     # 2 chunks of 256, My odd: half tile
                                         ((770, 9, 12), (3, 3, 31))])     # 33 taps, 4 chunks of 193
def test_direct_z_pass_lds_dma(gpu, shape, ksize, monkeypatch):
    """The LDS-DMA direct z pass (k_zdmc, mode 3): z chunks of 32-column tiles carried
    inside one block, against the full kernel spectra and the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for zk, mode in (("compact", 3), ("full", 0)):
        monkeypatch.setenv("SPIMDECON_ZK", zk)
        with Session(shape[::-1], fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            assert s.zpass_mode() == mode
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            out.append(s.get_psi())
    assert not np.array_equal(out[0], out[1]), "direct path not taken (identical bits)"
    assert rel_l2(out[0], out[1]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL


@pytest.mark.parametrize("shape,ksize", [((200, 10, 12), (3, 3, 23)),    # kc 11 in the KC-12 layout
                                         ((300, 10, 12), (3, 5, 31))])   # kc 15 in the KC-16 layout
def test_z_tap_trim_bit_identical(gpu, shape, ksize, monkeypatch):
    """Kernels of 2 KC - 1 planes skip the two zero outer taps of the KC layout at compile
    time (k_zdmc KD = 1); the skipped products are exact zeros, so psi is bit-identical to
    the runtime-masked kernel (SPIMDECON_ZKD=0) and on the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True, cid=44)
    out = []
    for zkd in ("1", "0"):
        monkeypatch.setenv("SPIMDECON_ZKD", zkd)
        with Session(shape[::-1], fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            assert s.zpass_mode() == 3
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            out.append(s.get_psi())
    assert np.array_equal(out[0], out[1])
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL


@pytest.mark.parametrize("shape,ksize,env,zmode", [
    ((20, 776, 12), (3, 25, 3), {}, 3),                               # My 800 = 25*32: 8-column y tiles
    ((616, 8, 12), (3, 3, 25), {"SPIMDECON_ZDIRECT": "0"}, 1),        # Mz 640: compact FFT z, 8-column tiles
    ((770, 8, 12), (3, 3, 31), {}, 3)])                               # Mz 800: 33-tap chunked direct z
def test_long_columns_on_8_column_tiles(gpu, shape, ksize, env, zmode, monkeypatch):
    """Two-factor lengths whose 16-column tile exceeds the 80-KB budget of 32 threads
    per column (640, 800, 1024) run 8-column tiles instead of the Stockham passes;
    33-tap kernels on long columns run the chunked LDS-DMA z pass."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize, partial=True)
    out = []
    for backend in ("engine", "rocfft"):
        with Session(shape[::-1], fft_backend=backend, fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            if backend == "engine":
                assert s.zpass_mode() == zmode
                assert max(s.fft_dims()) in (640, 800)
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            out.append(s.get_psi())
    assert rel_l2(out[0], out[1]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL


@pytest.mark.parametrize("shape,my", [((8, 616, 12), 640), ((6, 776, 10), 800), ((5, 1000, 8), 1024)])
def test_y_pass_prefetch_bit_identical(gpu, shape, my, monkeypatch):
    """The y pass at one block per CU (16-column tiles of 640-, 800- and 1024-point
    columns) prefetches the next tile's inputs into registers (k_col2f PF); the
    arithmetic is the plain kernel's, so psi is bit-identical with SPIMDECON_YPF=0, and
    both agree with the rocFFT backend (1e-5) and the oracle (1e-4)."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=(3, 25, 3), partial=True, cid=43)
    out = []
    for backend, ypf in (("engine", "1"), ("engine", "0"), ("rocfft", "1")):
        monkeypatch.setenv("SPIMDECON_YPF", ypf)
        with Session(shape[::-1], fft_backend=backend, fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            if backend == "engine":
                assert s.fft_dims()[1] == my
            out.append(s.get_psi())
    assert np.array_equal(out[0], out[1])
    assert rel_l2(out[0], out[2]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL


@pytest.mark.parametrize("shape,lx", [((6, 10, 360), 384), ((6, 10, 552), 576), ((5, 9, 776), 800)])
def test_x_tiles_with_global_twiddles(gpu, shape, lx):
    """Row lengths whose x tiles fit one more block per CU without the LDS twiddle
    table (384, 576, 800: xt_twg) read the phase-A twiddles from global memory;
    the tile path must still agree with the rocFFT backend and the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=(25, 5, 3), partial=True)
    out = []
    for backend in ("engine", "rocfft"):
        with Session(shape[::-1], fft_backend=backend, fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            if backend == "engine":
                assert s.fft_dims()[0] == lx
            s.init_psi()
            s.run(3, 0.006)
            if backend == "engine":
                assert s.xpass_mode() == 2, "x tile path not taken"
            s.apply_mask()
            out.append(s.get_psi())
    assert rel_l2(out[0], out[1]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL


@pytest.mark.parametrize("shape,ksize", [((1, 16, 20), (5, 5, 3)), ((2, 12, 16), (3, 5, 3)),
                                         ((3, 10, 12), (3, 3, 5))])
def test_thin_volumes(gpu, shape, ksize):
    """nz = 1..3 with 3- or 5-plane kernels: Mz = nz + 2cz is below the direct z pass's
    tap bound (unwritten window slots); such slabs take another z pass
    and stay finite and on the oracle."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=ksize)
    with Session(shape[::-1]) as s:
        for i, w, k in zip(imgs, ws, ks):
            s.add_view(i, w, k)
        s.init(PSFTYPE.OPTIMIZATION_I)
        s.init_psi()
        s.run(3, 0.006)
        s.apply_mask()
        psi = s.get_psi()
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert np.isfinite(psi).all()
    assert rel_l2(psi, res.psi) < TOL


@pytest.mark.parametrize("lam", [0.0, 0.006, 0.0006, 0.3, 1e-7])
def test_next_value_rule_bit_exact(gpu, lam):
    """spimdecon_next_value (the per-voxel update rule of both update paths:
    Tikhonov sqrt and division by lambda included) against the oracle's
    computeNextValue (MVDeconvolution.java:671-703), bit for bit, over random
    voxels and the special cases: value <= 0, NaN, +-inf, denormal, huge."""
    import torch
    from spim_registration_amd import _lib
    rng = np.random.default_rng(3)
    n = 1 << 20
    last = (rng.random(n, dtype=np.float32) * 10).astype(np.float32)
    integ = (np.float32(2.0) ** rng.uniform(-40, 40, n)).astype(np.float32)
    integ[: n // 8] = rng.standard_normal(n // 8).astype(np.float32)
    special = np.float32([0.0, -0.0, -1.0, np.nan, np.inf, -np.inf, 1e-45, 1e-38, 3e38, 1.0])
    integ[n // 8: n // 8 + special.size] = special
    w = rng.random(n, dtype=np.float32)
    w[:16] = [0.0, 1.0] * 8
    d = [torch.from_numpy(a).cuda() for a in (last, integ, w)]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    _lib.check(_lib.load().spimdecon_next_value(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, lam,
                                                  out.data_ptr()))
    got = out.cpu().numpy()
    want = ref.compute_next_value(last, integ, w, lam)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), want[~nan].view(np.uint32))


@pytest.mark.parametrize("shape,lx", [((12, 24, 516), 540), ((10, 16, 1024), 1050)])
@pytest.mark.parametrize("psftype", [PSFTYPE.EFFICIENT_BAYESIAN, PSFTYPE.OPTIMIZATION_I])
def test_tikhonov_update_tiles_match_oracle(gpu, shape, lx, psftype):
    """The Tikhonov update x tiles in their voxel batches of 2 float4 per row (the
    540-class rows of up to 5 float4 per lane, and the 1050 rows at 64 threads per
    pair, where larger batches spilled registers) against the oracle (1e-4) and the
    rocFFT backend (1e-5); lambda 0.006 (MVDeconvolution.java:671-705)."""
    imgs, ws, ks, _ = small_case(shape=shape, V=2, ksize=(9, 9, 9), partial=True, cid=41)
    out = []
    for backend in ("engine", "rocfft"):
        with Session(shape[::-1], fft_backend=backend, fft_pad_policy="fast") as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(psftype)
            s.init_psi()
            s.run(3, 0.006)
            s.apply_mask()
            if backend == "engine":
                assert s.fft_dims()[0] == lx and s.xpass_mode() == 2
            out.append(s.get_psi())
    assert rel_l2(out[0], out[1]) < 1e-5
    res = ref.mv_deconvolution(imgs, ws, ks, psftype, 3, 0.006)
    assert rel_l2(out[0], res.psi) < TOL
