"""GPU: the largest BASELINE geometries at their real size on one MI355X.

  1024^3       6-view 1024^3 (the north star's scaling workload) on ONE device: psi is
               2^32 B, past the fast passes' 32-bit buffer offsets, so the session splits
               it into exact slabs on the device and stays on the fast engine passes
               (asserted) -- vs the rocFFT backend, rel-L2 1e-5
  C5 full      6-view 2048x2048x1024 fp16 OPTIMIZATION_I 0.006 as 8 y-slabs of
               2048x256x1024 on one GPU (the 8-GPU decomposition, ~190 GB resident):
               2 iterations, finite, exact final mask, sumChange falling
  C5 rank slab the geometry one of 8 ranks holds (2048x256x1024 + halos, padded
               2100x1050x280) through the y-split path vs the rocFFT backend, 1e-5
  C5 aspect    the same decomposition on a 232x256x104 instance vs the oracle, 1e-4, on
               C5's fp16 two-factor x tiles (asserted)
  C4           one timepoint of 8-view 768^3 through pipeline.process_timepoint:
               input preparation vs the oracle on sub-boxes, PSFs vs the oracle per view,
               10 RL iterations (800-point lengths, 31-plane kernels) vs the rocFFT
               backend on the same prepared inputs and PSFs; two timepoints back to back
               through one Pipeline == a fresh process's timepoint, bit for bit

References (paths under /root/reference/src/main/java/spim/process/):
fusion/deconvolution/MVDeconvolution.java:333-444 (the iteration),
cuda/BlockGeneratorFixedSizePrecise.java:25-101 (exact blocks of any size),
fusion/deconvolution/ProcessForDeconvolution.java:105-349 (the C4 inputs).
"""
import numpy as np
import pytest
import torch  # before the library loads (one shared HIP runtime, spim_registration_amd._lib.load)

from conftest import rel_l2
from oracle import input_ref, mvdecon_ref as ref, psf_ref
from spim_registration_amd import input_prep, pipeline, synthetic
from spim_registration_amd.decon import PSFTYPE, Session

pytestmark = pytest.mark.gpu

TOL = 1e-4
ENGINE_VS_ROCFFT = 1e-5
CPU_WORKERS = 16


def release():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def engine_modes(s):
    n = s.num_slabs()
    return [s.xpass_mode(i) for i in range(n)], [s.zpass_mode(i) for i in range(n)]


def assert_fast(s):
    xm, zm = engine_modes(s)
    assert set(xm) == {2} and set(zm) <= {2, 3, 4}, (xm, zm)


def run_views(shape_zyx, views, psftype, iters, lam, keep=None, **kw):
    """views: iterable of (img, w, psf) torch/numpy triples (added one by one, so a
    generator can hand out one full-size view at a time).  Returns (psi on the host
    unless keep == 'device', stats, session info)."""
    with Session(shape_zyx[::-1], **kw) as s:
        for img, w, k in views:
            s.add_view_device(img.data_ptr(), w.data_ptr(), k)
            del img, w
        s.init(psftype)
        s.init_psi()
        st = s.run(iters, lam)
        s.apply_mask()
        info = {"slabs": s.num_slabs(), "extent0": s.slab_extent(0), "fft_dims": s.fft_dims(0)}
        if kw.get("fft_backend", "engine") == "engine":
            info["xpass"], info["zpass"] = engine_modes(s)
        if keep == "device":
            psi = torch.empty(shape_zyx, dtype=torch.float32, device="cuda:0")
            import ctypes as C
            from spim_registration_amd import _lib
            _lib.check(s.lib.mvd_get_psi(s.h, C.cast(C.c_void_p(psi.data_ptr()), _lib._pf)))
            torch.cuda.synchronize()
        else:
            psi = s.get_psi()
        return psi, st, info


# ------------------------------------------------------------------ 1024^3, one device

@pytest.mark.timeout(900)
def test_1024_cube_one_device_fast_engine_vs_rocfft(gpu):
    imgs, ws, psfs = synthetic.make_views_torch((1024, 1024, 1024), 6, config_id=6, ksize=(25, 25, 25),
                                                device="cuda:0")
    release()
    views = lambda: zip(imgs, ws, psfs)          # noqa: E731
    psi, st, info = run_views((1024, 1024, 1024), views(), PSFTYPE.OPTIMIZATION_I, 2, 0.006)
    release()
    # psi alone is 2^32 B: two exact z-slabs of 512 planes on the device, both fast
    assert info["slabs"] == 2 and info["extent0"] == (1024, 1024, 512), info
    assert set(info["xpass"]) == {2} and set(info["zpass"]) <= {2, 3, 4}, info
    assert info["fft_dims"] == (1050, 1050, 536), info
    psir, str_, _ = run_views((1024, 1024, 1024), views(), PSFTYPE.OPTIMIZATION_I, 2, 0.006,
                              fft_backend="rocfft")
    del imgs, ws
    release()
    assert np.isfinite(psi).all()
    assert rel_l2(psi, psir) < ENGINE_VS_ROCFFT
    np.testing.assert_allclose(st, str_, rtol=1e-4)


# ------------------------------------------------------------------ C5

def tiled_views(shape_zyx, V, cid, base=(256, 512, 512), hole=None):
    """One full-size (img, w, psf) view at a time (fp32, on the GPU): the base-size
    synthetic views (make_views_torch, same PSFs) tiled periodically, with the
    VIRTUAL-normalised cosine blending recomputed at full size.  ``hole`` = (z, y, x)
    corner box where no view has data (img = w = 0): the final mask must zero it."""
    nz, ny, nx = shape_zyx
    bimgs, _, psfs = synthetic.make_views_torch(base, V, config_id=cid, ksize=(25, 25, 25), device="cuda:0")
    prof = [torch.from_numpy(synthetic.blend_weight((nz, 1, nx), v, V).astype(np.float32)).to("cuda:0")
            for v in range(V)]
    norm = torch.clamp(sum(prof), min=1.0)
    reps = [-(-nz // base[0]), -(-ny // base[1]), -(-nx // base[2])]
    for v in range(V):
        print(f"  [tiled views] view {v} of {V} ({nx}x{ny}x{nz})", flush=True)   # (progress: long test)
        img = bimgs[v].repeat(*reps)[:nz, :ny, :nx].contiguous()
        w = (prof[v] / norm).expand(nz, ny, nx).contiguous()
        if hole is not None:
            img[:hole[0], :hole[1], :hole[2]] = 0.0
            w[:hole[0], :hole[1], :hole[2]] = 0.0
        torch.cuda.synchronize()
        yield img, w, psfs[v]
        del img, w
        release()


@pytest.mark.timeout(1200)
def test_c5_full_2048x2048x1024_fp16_eight_y_slabs(gpu):
    shape = (1024, 2048, 2048)                    # [z, y, x]
    hole = (64, 96, 128)
    psi, st, info = run_views(shape, tiled_views(shape, 6, 50, hole=hole), PSFTYPE.OPTIMIZATION_I, 2, 0.006,
                              keep="device", storage_fp16=True, local_slabs=8)
    # the 8-rank decomposition: y-slabs of 2048 x 256 rows x 1024, kept as (x, z, y) rows
    assert info["slabs"] == 8 and info["extent0"] == (2048, 1024, 256), info
    assert info["fft_dims"] == (2100, 1050, 280), info
    assert set(info["xpass"]) == {2} and set(info["zpass"]) <= {2, 3, 4}, info
    assert bool(torch.isfinite(psi).all())
    assert bool((psi[:hole[0], :hole[1], :hole[2]] == 0).all())          # MVDeconvolution.java:180-187
    psi[:hole[0], :hole[1], :hole[2]] = 1.0
    assert bool((psi > 0).all())
    del psi
    release()
    assert np.isfinite(st).all()
    tot = st[:, :, 0].sum(axis=1)
    assert tot[1] < tot[0], tot


@pytest.mark.timeout(900)
def test_c5_rank_slab_geometry_vs_rocfft(gpu):
    """The slab one of 8 ranks holds (2048 x 256 y-rows x 1024, padded 2100 x 1050 x 280
    internally) through the y-split path: 2 y-slabs of a 2048 x 512 x 1024 volume."""
    shape = (1024, 512, 2048)
    views = list(tiled_views(shape, 6, 51))
    psi, st, info = run_views(shape, views, PSFTYPE.OPTIMIZATION_I, 2, 0.006, storage_fp16=True, local_slabs=2,
                              slab_axis="y")
    release()
    assert info["slabs"] == 2 and info["extent0"] == (2048, 1024, 256), info
    assert info["fft_dims"] == (2100, 1050, 280), info
    assert set(info["xpass"]) == {2} and set(info["zpass"]) <= {2, 3, 4}, info
    psir, str_, _ = run_views(shape, views, PSFTYPE.OPTIMIZATION_I, 2, 0.006, storage_fp16=True,
                              fft_backend="rocfft")
    del views
    release()
    assert np.isfinite(psi).all()
    assert rel_l2(psi, psir) < ENGINE_VS_ROCFFT
    np.testing.assert_allclose(st, str_, rtol=1e-4)


@pytest.mark.timeout(300)
def test_c5_decomposition_matches_oracle_232x256x104(gpu):
    """C5's decomposition (8 y-slabs, fp16 img / weight storage, OPTIMIZATION_I 0.006)
    on an instance the oracle runs in seconds, on C5's own arithmetic path: x = 232 + 24
    pads to 256, a two-factor tile length, so every slab runs the fp16 x tiles
    (k_xtile<..., S = 1, ...>) -- asserted -- and the direct z pass.  The oracle sees the
    fp16-rounded inputs (MVDeconvolution.java:582-703 on the stored values)."""
    imgs, ws, ks, _ = synthetic.make_views((104, 256, 232), 6, config_id=52, ksize=(25, 25, 25),
                                           weights="blend", partial=True)
    with Session((232, 256, 104), storage_fp16=True, local_slabs=8) as s:
        for i, w, k in zip(imgs, ws, ks):
            s.add_view(i, w, k)
        s.init(PSFTYPE.OPTIMIZATION_I)
        s.init_psi()
        st = s.run(2, 0.006)
        s.apply_mask()
        # y-slabs of 32 rows, kept as (x, z, y) rows: padded 256 x 128 x 56
        assert s.num_slabs() == 8 and s.slab_extent(0) == (232, 104, 32)
        assert s.fft_dims(0)[0] == 256, s.fft_dims(0)
        xm, zm = engine_modes(s)
        assert set(xm) == {2} and set(zm) <= {2, 3, 4}, (xm, zm)
        psi = s.get_psi()
    hi = [i.astype(np.float16).astype(np.float32) for i in imgs]
    hw = [w.astype(np.float16).astype(np.float32) for w in ws]
    res = ref.mv_deconvolution(hi, hw, ks, PSFTYPE.OPTIMIZATION_I, 2, 0.006, precision="f32", workers=CPU_WORKERS)
    assert rel_l2(psi, res.psi) < TOL
    assert ((psi == 0) == (res.psi == 0)).all()
    np.testing.assert_allclose(st[:, :, 0], np.array(res.stats)[:, :, 0], rtol=1e-3)


# ------------------------------------------------------------------ C4

@pytest.mark.timeout(1200)
def test_c4_timepoint_8view_768(gpu):
    from test_gpu_input_prep import assert_mismatches_on_ties
    from spim_registration_amd import psf as psf_mod
    n = 768
    log = lambda m: print(f"  [c4] {m}", flush=True)   # noqa: E731  (progress: long stages)
    views, models = synthetic.make_timepoint_torch((n, n, n), (n, n, n), 8, timepoint=1, device="cuda:0")
    release()
    res = pipeline.process_timepoint(views, models, (0, 0, 0), (n, n, n), psf_size=(19, 19, 25), iterations=10)
    log(f"pipeline done: {res.ms}")
    assert res.engine["zpass_mode"] in (2, 3, 4) and res.engine["xpass_mode"] == 2, res.engine
    assert res.engine["fft_dims_xyz"] == [800, 800, 798] and res.engine["kernel_planes"] == 31, res.engine
    assert all(len(c) > 1000 for c in res.corresponding)
    psi = res.psi.cpu().numpy()
    assert np.isfinite(psi).all() and (psi > 0).mean() > 0.3
    assert all(np.isfinite(p).all() and p.max() <= 1.0 + 1e-6 for p in res.psfs)

    # input preparation: the GPU's full bounding box vs the oracle on sub-boxes
    imgs, ws, _ = input_prep.prepare_inputs(views, models, (0, 0, 0), (n, n, n), (-8, -8, -8), (12, 12, 12))
    hv = [v.cpu().numpy() for v in views]
    for b0 in [(0, 0, 0), (352, 360, 368), (n - 40, 200, n - 40), (100, n - 40, 500)]:
        bd = (40, 40, 40)
        ei, ew, _ = input_ref.prepare_inputs(hv, models, b0, bd, (-8, -8, -8), (12, 12, 12))
        for v in range(len(views)):
            gi = imgs[v][b0[2]:b0[2] + bd[2], b0[1]:b0[1] + bd[1], b0[0]:b0[0] + bd[0]].cpu().numpy()
            gw = ws[v][b0[2]:b0[2] + bd[2], b0[1]:b0[1] + bd[1], b0[0]:b0[0] + bd[0]].cpu().numpy()
            assert_mismatches_on_ties(gi, ei[v], [models[v]], b0, bd)
            np.testing.assert_allclose(gw, ew[v], rtol=1e-5, atol=1e-6)
    log("input preparation matches the oracle on 4 sub-boxes x 8 views")

    # PSFs: the pipeline's batch extraction (spim_extract_psfs, views in flight together)
    # vs the oracle on the first 1500 corresponding beads of a 0- and a 45-degree view
    # (the oracle's per-bead float sum over ~70k beads would take minutes per view)
    sel = [0, 1]
    locs = [res.points[v][res.corresponding[v]][:1500] for v in sel]
    got = psf_mod.extract_psfs([views[v] for v in sel], locs, (19, 19, 25), [models[v] for v in sel])
    for (orig_g, tr_g), v, lc in zip(got, sel, locs):
        orig = psf_ref.normalize(psf_ref.extract_psf_local_batched(hv[v], lc, (19, 19, 25)))
        want = psf_ref.transform_psf(orig, models[v])
        np.testing.assert_allclose(orig_g, orig, rtol=1e-5, atol=1e-6)
        assert tr_g.shape == want.shape == res.psfs[v].shape
        np.testing.assert_allclose(tr_g, want, rtol=1e-5, atol=1e-6)
    log("PSF extraction matches the oracle")
    del hv, views
    release()

    # RL: 10 iterations on the rocFFT backend from the same prepared inputs and PSFs
    psir, _, _ = run_views((n, n, n), zip(imgs, ws, res.psfs), PSFTYPE.OPTIMIZATION_I, 10, 0.006,
                           fft_backend="rocfft")
    del imgs, ws
    release()
    err = rel_l2(psi, psir)
    log(f"RL engine vs rocFFT backend: rel-L2 {err:.2e}")
    assert err < ENGINE_VS_ROCFFT


@pytest.mark.timeout(1200)
def test_c4_two_timepoints_back_to_back_equal_fresh_process(gpu):
    """Two C4 timepoints (8-view 768^3) back to back through one Pipeline (the DoG
    workspace, PSF / resampling scratch and plan caches carried over): timepoint 1's psi,
    RL statistics and detections equal, bit for bit, those of a fresh process that runs
    timepoint 1 alone (tools/c4_pipeline.py --only 1 --digest)."""
    import json
    import os
    import subprocess
    import sys
    n = 768
    pipe = pipeline.Pipeline(psf_size=(19, 19, 25), iterations=10)
    digests = []
    for t in (0, 1):
        views, models = synthetic.make_timepoint_torch((n, n, n), (n, n, n), 8, timepoint=t, device="cuda:0")
        res = pipe.process(views, models, (0, 0, 0), (n, n, n), digest=True)
        digests.append(pipeline.result_digest(res))
        print(f"  [c4x2] timepoint {t}: {res.ms}", flush=True)
        del views, res
        release()
    assert digests[0]["psi_sha256"] != digests[1]["psi_sha256"]     # the beads drift: a different result
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "c4_pipeline.py"), "--only", "1", "--digest",
                        "--timepoints", "2"], capture_output=True, text=True, timeout=900, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    fresh = json.loads(r.stdout.strip().splitlines()[-1])["timepoints"][0]
    keys = ("points_sha256", "corresponding_sha256", "inputs_sha256", "psfs_sha256", "stats_sha256", "psi_sha256")
    differ = [k for k in keys if fresh[k] != digests[1][k]]   # the stages in pipeline order
    assert not differ, differ
