"""GPU: one session over several devices of this process (``mvd_create_devices``)
and the virtual-slab paths of the fast x tiles.

The reference drives several GPUs from one JVM through
``MVDeconFFT(..., int[] deviceList, ...)`` (MVDeconFFT.java:58-64,91-100,424-446).
Here one ``mvd_run`` drives every device of the list from its own host thread;
the halo planes move between neighbouring devices as peer copies.  Device ids
may repeat, so the one-GPU box runs exactly the multi-device code (threads,
barriers, cross-stream events, pull copies) with every group on device 0.

Tolerances: psi within 1e-5 relative L2 of the single-slab session (only the
FFT rounding of the slab-sized transforms differs) and 1e-4 of the oracle (the
north-star bound); per-view stats within rtol 1e-4 of the single-slab session.
"""
import numpy as np
import pytest

from conftest import rel_l2
from oracle import mvdecon_ref as ref
from spim_registration_amd import synthetic
from spim_registration_amd._lib import SpimDeconError
from spim_registration_amd.decon import MVDeconFFT, MVDeconInput, MVDeconvolution, PSFTYPE, Session

pytestmark = pytest.mark.gpu

TOL = 1e-4

# nx % 4 == 0 and Mx = 256 = 16 * 16 (two-factor x table): the update / quotient
# passes run the row-pair tiles (k_xtile), with slab row maps and the split
# boundary / rest launches of the overlapped exchange
TILE_SHAPE = (60, 20, 248)      # [z, y, x]
TILE_K = (9, 7, 9)              # kx, ky, kz -> cz = 4


def tile_case(V=2, cid=11, partial=True):
    return synthetic.make_views(TILE_SHAPE, V, config_id=cid, ksize=TILE_K, weights="blend",
                                partial=partial, bead_density=1.0 / 6 ** 3)


def run_session(imgs, ws, ks, iters=3, lam=0.006, psftype=PSFTYPE.OPTIMIZATION_I, **kw):
    shape = imgs[0].shape
    with Session(shape[::-1], **kw) as s:
        for i, w, k in zip(imgs, ws, ks):
            s.add_view(i, w, k)
        s.init(psftype)
        s.init_psi()
        st = s.run(iters, lam)
        s.apply_mask()
        nslab = kw.get("local_slabs", 1) * max(1, len(kw.get("devices") or [0]))
        modes = [s.xpass_mode(i) for i in range(nslab)]
        ndev = s.num_devices()
        devs = [s.slab_device(i) for i in range(nslab)]
        return s.get_psi(), st, modes, ndev, devs


@pytest.fixture(scope="module")
def tile_ref():
    imgs, ws, ks, _ = tile_case()
    psi, st, modes, _, _ = run_session(imgs, ws, ks)
    assert modes == [2], modes          # the two-factor x tiles ran
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.OPTIMIZATION_I, 3, 0.006)
    assert rel_l2(psi, res.psi) < TOL
    return imgs, ws, ks, psi, st, res


@pytest.mark.parametrize("slabs", [2, 3, 6])
def test_virtual_slabs_on_tile_path(gpu, tile_ref, slabs):
    """local slabs with the k_xtile passes (overlapped boundary / rest
    split, psi x tiles on slab row maps, two-launch stats partials)."""
    imgs, ws, ks, psi1, st1, res = tile_ref
    psi, st, modes, ndev, _ = run_session(imgs, ws, ks, local_slabs=slabs)
    assert ndev == 1 and modes == [2] * slabs, modes
    assert rel_l2(psi, psi1) < 1e-5
    np.testing.assert_allclose(st, st1, rtol=1e-4)
    assert rel_l2(psi, res.psi) < TOL


@pytest.mark.parametrize("devices,slabs", [([0, 0], 1), ([0, 0, 0], 1), ([0, 0], 2), ([0, 0, 0, 0], 3)])
def test_device_groups_match_single(gpu, tile_ref, devices, slabs):
    """Several device groups in one session: one host thread per group, halo pulls
    between groups, stats combined over the groups."""
    imgs, ws, ks, psi1, st1, res = tile_ref
    psi, st, modes, ndev, devs = run_session(imgs, ws, ks, devices=devices, local_slabs=slabs)
    assert ndev == len(devices)
    assert devs == [d for d in devices for _ in range(slabs)]
    assert modes == [2] * (len(devices) * slabs), modes
    assert rel_l2(psi, psi1) < 1e-5
    np.testing.assert_allclose(st, st1, rtol=1e-4)
    assert rel_l2(psi, res.psi) < TOL


def test_mvdeconvolution_device_list(gpu):
    """decon.MVDeconvolution routes the views' device_list into one multi-device
    session (the reference's deviceList), not just its first entry."""
    imgs, ws, ks, _ = synthetic.make_views((40, 20, 22), 3, config_id=5, ksize=(5, 7, 9),
                                           weights="blend", partial=True, bead_density=1.0 / 6 ** 3)
    inp = MVDeconInput()
    for i, w, k in zip(imgs, ws, ks):
        inp.add(MVDeconFFT(i, w, k, device_list=[0, 0, 0]))
    dec = MVDeconvolution(inp, PSFTYPE.EFFICIENT_BAYESIAN, 4, 0.006)
    assert dec.session.num_devices() == 3
    psi = dec.get_psi()
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.EFFICIENT_BAYESIAN, 4, 0.006)
    assert rel_l2(psi, res.psi) < TOL
    np.testing.assert_allclose(dec.stats[:, :, 0], np.array(res.stats)[:, :, 0], rtol=1e-3)
    assert ((psi == 0) == (res.psi == 0)).all()


def test_device_groups_fp16_and_initial_image(gpu):
    imgs, ws, ks, _ = tile_case(V=3, cid=12, partial=False)
    init = imgs[1].copy()
    out = []
    for kw in ({}, {"devices": [0, 0]}):
        with Session(TILE_SHAPE[::-1], storage_fp16=True, **kw) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.INDEPENDENT)
            s.init_psi(init)
            s.run(2, 0.0)
            s.run(1, 0.0)       # continues from the resident psi on every device
            out.append(s.get_psi())
    assert rel_l2(out[1], out[0]) < 1e-5


def test_device_groups_reject_bad_arguments(gpu):
    with pytest.raises(SpimDeconError):
        Session((16, 16, 16), devices=[0, 0], fft_backend="rocfft")
    with pytest.raises(SpimDeconError):
        Session((16, 16, 3), devices=[0, 0], local_slabs=2, slab_axis="z")     # 4 slabs > 3 planes
    with pytest.raises(SpimDeconError):
        Session((16, 16, 16), devices=[0, -1])


# y-split sessions (mvd_params.slab_axis = 1): the engine slabs its outermost axis, so
# the session keeps (x, z, y) rows internally; ny > nz here, so "auto" picks y
Y_SHAPE = (20, 60, 248)        # [z, y, x]


@pytest.mark.parametrize("devices,slabs", [(None, 2), ([0, 0], 1), ([0, 0, 0], 2)])
def test_y_split_matches_z_split_and_oracle(gpu, devices, slabs):
    imgs, ws, ks, _ = synthetic.make_views(Y_SHAPE, 3, config_id=13, ksize=(9, 7, 5), weights="blend",
                                           partial=True, bead_density=1.0 / 6 ** 3)
    out = {}
    for axis in ("z", "y", "auto"):
        kw = dict(local_slabs=slabs if axis != "z" else 1, slab_axis=axis)
        if devices and axis != "z":
            kw["devices"] = devices
        out[axis] = run_session(imgs, ws, ks, psftype=PSFTYPE.EFFICIENT_BAYESIAN, **kw)
    assert out["y"][2] == [2] * (slabs * len(devices or [0]))   # x tiles ran on the y slabs
    assert rel_l2(out["y"][0], out["z"][0]) < 1e-5
    assert np.array_equal(out["auto"][0], out["y"][0])
    np.testing.assert_allclose(out["y"][1], out["z"][1], rtol=1e-4)
    res = ref.mv_deconvolution(imgs, ws, ks, PSFTYPE.EFFICIENT_BAYESIAN, 3, 0.006)
    assert rel_l2(out["y"][0], res.psi) < TOL
    assert ((out["y"][0] == 0) == (res.psi == 0)).all()


def test_y_split_fp16_initial_image_and_kernels(gpu):
    imgs, ws, ks, _ = synthetic.make_views(Y_SHAPE, 2, config_id=14, ksize=(5, 9, 3), weights="blend",
                                           bead_density=1.0 / 6 ** 3)
    init = imgs[0].copy()
    out = []
    for axis in ("z", "y"):
        with Session(Y_SHAPE[::-1], storage_fp16=True, local_slabs=2 if axis == "y" else 1, slab_axis=axis) as s:
            for i, w, k in zip(imgs, ws, ks):
                s.add_view(i, w, k)
            s.init(PSFTYPE.OPTIMIZATION_I)
            k1, k2 = s.get_kernels(1, ks[1].shape)          # the caller's axis order
            s.init_psi(init)
            s.run(3, 0.006)
            out.append((s.get_psi(), k1, k2))
    assert rel_l2(out[1][0], out[0][0]) < 1e-5
    np.testing.assert_array_equal(out[1][1], out[0][1])
    np.testing.assert_array_equal(out[1][2], out[0][2])


@pytest.mark.timeout(600)
def test_c3_strong_decomposition_exchange_accounting(gpu):
    """BASELINE configs[2] as the 8-GPU strong decomposition (8 device groups, all on
    this GPU): 8 y-slabs of 128 rows, one halo exchange of every boundary in both
    directions per pad (the initial psi pad, then the quotient and the next psi per
    view; the last update pads nothing): 2 * iters * V exchanges of 2 * 7 copies of
    cz planes each.  Prints the exchange time the timing class measured."""
    import torch
    imgs, ws, psfs = synthetic.make_views_torch((512, 1024, 1024), 6, config_id=3, ksize=(25, 25, 25),
                                                device="cuda:0")
    iters, V, G = 2, 6, 8
    with Session((1024, 1024, 512), devices=[0] * G) as s:
        for i, w, k in zip(imgs, ws, psfs):
            s.add_view_device(i.data_ptr(), w.data_ptr(), k)
        del imgs, ws
        torch.cuda.empty_cache()
        s.init(PSFTYPE.EFFICIENT_BAYESIAN)
        s.init_psi()
        assert s.num_slabs() == G and s.slab_extent(0) == (1024, 512, 128)
        Mx, My, Mz = s.fft_dims(0)
        Hp = -(-(Mx // 2 + 1) // 16) * 16
        plane = 2 * Hp * My * 4                      # bytes of one padded x-spectrum plane
        cz = 12                                      # 25-plane kernels
        b0, c0 = s.exchange_stats()
        s.enable_timing(True)
        s.run(iters, 0.006)
        tm = s.timing()
        b1, c1 = s.exchange_stats()
        copies = 2 * iters * V * 2 * (G - 1)
        assert c1 - c0 == copies, (c1 - c0, copies)
        assert b1 - b0 == copies * cz * plane, (b1 - b0, copies * cz * plane)
        assert tm[8 + 5] == 2 * iters * V               # group 0's exchange intervals
        print(f"\nC3 8-group exchange: {plane * cz / 1e6:.1f} MB per copy, {(b1 - b0) / iters / 1e9:.2f} GB "
              f"per iteration (all boundaries), {tm[5] / tm[13]:.3f} ms per exchange on group 0's stream")


@pytest.mark.skipif(__import__("torch").cuda.device_count() < 2, reason="needs 2 distinct GPUs (the pool's boxes have 1)")
def test_distinct_devices_match_single(gpu):
    """Peer pulls over xGMI between distinct GPUs: the same psi and stats as one
    device (runs wherever >= 2 GPUs are visible, e.g. the 8-GPU node; on one GPU the
    same code path is covered by the repeated-id tests above)."""
    import torch
    n = min(torch.cuda.device_count(), 4)
    imgs, ws, ks, _ = tile_case(V=3, cid=15)
    psi1, st1, _, _, _ = run_session(imgs, ws, ks)
    psi, st, modes, ndev, devs = run_session(imgs, ws, ks, devices=list(range(n)))
    assert ndev == n and devs == list(range(n))
    assert rel_l2(psi, psi1) < 1e-5
    np.testing.assert_allclose(st, st1, rtol=1e-4)


def test_auto_slabs_keep_the_count_when_no_split_fits(gpu):
    """One z-plane's spectrum alone past the fast passes' 32-bit offsets (33000 x 33000):
    no z split can help, so the session keeps the caller's slab count (the Stockham
    passes run it, as before the automatic split) instead of one-plane slabs, or 'more
    slabs than z planes' with two devices.  Geometry only: nothing is allocated."""
    with Session((33000, 33000, 3), slab_axis="z") as s:
        assert s.num_slabs() == 1
    with Session((33000, 33000, 3), devices=[0, 0], slab_axis="z") as s:
        assert s.num_slabs() == 2


def test_single_rank_rccl_communicator(gpu, tile_ref, monkeypatch):
    """A one-rank RCCL communicator (comm_id given with nranks = 1; the only RCCL
    configuration one GPU admits -- two ranks cannot share a device): ncclCommInitRank,
    the rank-geometry all-gather of Session::verify_ranks, the first-iteration and
    per-view statistics all-reduces, and the watchdog's bounded waits on the progress
    events all run through RCCL; psi and the statistics equal the session without a
    communicator bit for bit (a one-rank sum / max is the identity), twice in a row."""
    from spim_registration_amd.distributed import unique_id_bytes
    monkeypatch.setenv("SPIMDECON_RCCL_TIMEOUT", "120")
    imgs, ws, ks, _ = tile_case()
    psi0, st0, _, _, _ = run_session(imgs, ws, ks)
    for _ in range(2):
        psi, st, modes, _, _ = run_session(imgs, ws, ks, comm_id=unique_id_bytes())
        assert modes == [2]
        np.testing.assert_array_equal(psi, psi0)
        np.testing.assert_array_equal(st, st0)
    assert rel_l2(psi, tile_ref[3]) < 1e-6


@pytest.mark.parametrize("slabs", [2, 4])
def test_concurrent_boundary_launches_bit_identical(gpu, tile_ref, slabs, monkeypatch):
    """One device group with neighbouring slabs: the boundary x launches on the exchange
    stream, concurrently with the rest of the pass (default), compute the same bits as
    both on the compute stream (SPIMDECON_CBND=0) -- the launches write disjoint rows and
    stats partials, and the reduction order is fixed."""
    imgs, ws, ks, _ = tile_case()
    out = []
    for cb in ("0", "1"):
        monkeypatch.setenv("SPIMDECON_CBND", cb)
        psi, st, modes, _, _ = run_session(imgs, ws, ks, local_slabs=slabs)
        assert modes == [2] * slabs
        out.append((psi, st))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert rel_l2(out[1][0], tile_ref[3]) < 1e-5


@pytest.mark.parametrize("kw", [dict(devices=[0, 0], local_slabs=2), dict(local_slabs=3)])
def test_kernel_pull_bit_identical(gpu, kw, monkeypatch):
    """Halo planes moved by the pull kernel (SPIMDECON_PULL=kernel: k_pull_copy reads the
    sender's buffer) instead of hipMemcpyAsync -- device-group pulls and local slab copies
    -- give the same bits."""
    imgs, ws, ks, _ = tile_case()
    out = []
    for pull in ("copy", "kernel"):
        monkeypatch.setenv("SPIMDECON_PULL", pull)
        psi, st, _, _, _ = run_session(imgs, ws, ks, **kw)
        out.append((psi, st))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
