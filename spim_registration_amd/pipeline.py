"""One timepoint of the multiview pipeline, device resident (BASELINE configs[3]).

The Fiji workflow the reference runs per timepoint, restated over this library:

  1. Detect Interest Points   ProcessDOG.compute per view (spim/process/interestpointdetection/
                              ProcessDOG.java:40-178) -> bead positions in view pixels
  2. Register                 the view models are given (descriptor matching stays out of
                              scope); the correspondences the registration would
                              record are recovered from them (a detection corresponds when
                              another view detected a bead within ``radius`` world pixels of
                              it).  With ``refine`` = "translation" / "rigid" / "affine" the
                              given models are first refined on the host: mutual nearest
                              detections -> GlobalOpt.compute (globalopt.py, GlobalOpt.java:
                              44-135), view 0 fixed
  3. Input preparation        ProcessForDeconvolution.fuseStacksAndGetPSFs (:159-384): views
                              resampled into the bounding box, blending weights normalised,
                              and per view the PSF extracted from its corresponding beads
                              (getLocationsOfCorrespondingBeads :444-462, ExtractPSF.
                              extractNextImg :260-279) and transformed with the view model
  4. Deconvolution            MVDeconvolution (EfficientBayesianBased.java:166-286 defaults:
                              OPTIMIZATION_I, lambda 0.006)

Every volume stays in HBM (torch tensors are only device-memory plumbing); the
stages are the library's C-ABI calls.  ``process_timepoint`` returns psi as a
torch tensor and per-stage wall times.
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib, dog, input_prep, psf as psf_mod
from .decon import PSFTYPE, Session


@dataclass
class TimepointResult:
    psi: object                              # torch tensor [z, y, x] on the GPU
    points: list                             # per view: (n, 3) detections, view pixels (x, y, z)
    corresponding: list                      # per view: indices of detections with a correspondence
    psfs: list                               # per view: transformed PSF [z, y, x] (numpy)
    stats: np.ndarray                        # RL (iterations, views, 2)
    ms: dict = field(default_factory=dict)   # stage wall times
    engine: dict = field(default_factory=dict)   # RL FFT dims and z / x pass modes
    stage_digests: dict = field(default_factory=dict)   # SHA-256 per stage output (digest=True)
    models: list = field(default_factory=list)   # the view models used (refined when refine is set)
    globalopt: object = None                     # globalopt.GlobalOptResult (refine is set)


def apply_model(model, pts):
    """AffineTransform3D.apply for (n, 3) points (x, y, z)."""
    m = np.asarray(model, np.float64).reshape(3, 4)
    return np.asarray(pts, np.float64) @ m[:, :3].T + m[:, 3]


def corresponding_detections(points, models, radius: float = 2.0, device=None):
    """The detections of each view that lie within ``radius`` world pixels of a
    detection of another view: the set ``getLocationsOfCorrespondingBeads`` reads
    from the registration's correspondence lists (ProcessForDeconvolution.java:444-462).

    All pairs within the radius are found exactly through a hash of radius-sized
    cells (sorted cell keys, the 27 neighbouring cells of each point looked up by
    binary search), in torch on ``device`` (the GPU in the pipeline, the CPU in
    the host tests)."""
    import torch
    dev = torch.device(device if device is not None else "cpu")
    world = [apply_model(m, p) if len(p) else np.zeros((0, 3)) for p, m in zip(points, models)]
    sizes = [len(w) for w in world]
    n = sum(sizes)
    if n == 0:
        return [np.zeros(0, np.int64) for _ in world]
    P = torch.from_numpy(np.concatenate(world)).to(dev, torch.float64)
    lab = torch.cat([torch.full((k,), v, dtype=torch.int64) for v, k in enumerate(sizes)]).to(dev)
    cell = torch.floor(P / radius).to(torch.int64)
    cell = cell - cell.min(dim=0).values + 1
    dims = cell.max(dim=0).values + 2
    key = (cell[:, 0] * dims[1] + cell[:, 1]) * dims[2] + cell[:, 2]
    skey, order = torch.sort(key)
    Ps, Ls = P[order], lab[order]
    r2 = float(radius) ** 2
    offs = torch.tensor([(dx * dims[1] + dy) * dims[2] + dz for dx in (-1, 0, 1) for dy in (-1, 0, 1)
                         for dz in (-1, 0, 1)], dtype=torch.int64, device=dev)
    nk = key[None, :] + offs[:, None]                          # [27, n] neighbouring cell keys
    lo = torch.searchsorted(skey, nk, side="left")
    cnt = torch.searchsorted(skey, nk, side="right") - lo
    hit = torch.zeros(n, dtype=torch.bool, device=dev)
    for j in range(int(cnt.max())):                            # (a cell rarely holds more than 2)
        idx = (lo + j).clamp(max=n - 1)
        d2 = ((Ps[idx] - P[None]) ** 2).sum(dim=2)
        hit |= ((j < cnt) & (Ls[idx] != lab[None]) & (d2 <= r2)).any(dim=0)
    hit = hit.cpu().numpy()
    out, o = [], 0
    for k in sizes:
        out.append(np.nonzero(hit[o:o + k])[0])
        o += k
    return out


def process_timepoint(views, models, bb_min, bb_dims, *, psf_size=(19, 19, 25), iterations: int = 10,
                      psftype: PSFTYPE = PSFTYPE.OPTIMIZATION_I, lam: float = 0.006, sigma: float = 1.8,
                      threshold: float = 0.008, localization: int = 1, radius: float = 2.0,
                      blending_border=(-8, -8, -8), blending_range=(12, 12, 12),
                      weight_type=input_prep.WeightType.VIRTUAL_WEIGHTS, device: int = 0,
                      log=None, digest: bool = False, refine: str | None = None) -> TimepointResult:
    """views: per view a [z, y, x] float32 torch tensor on the GPU (the acquired
    stack); models: 3x4 view -> world affines; bb_min / bb_dims (x, y, z)."""
    import torch
    ms = {}

    def lap(name, t0):
        torch.cuda.synchronize(device)
        ms[name] = round((time.perf_counter() - t0) * 1e3, 2)
        if log:
            log(f"{name}: {ms[name]} ms")
        return time.perf_counter()

    torch.cuda.synchronize(device)
    t = time.perf_counter()
    points = []
    for v in views:          # 1. ProcessDOG per view, read in place
        pos, _ = dog.interest_points_array(v, sigma=sigma, threshold=threshold, localization=localization,
                                           device=device)
        points.append(pos)
    t = lap("detect", t)
    gres = None
    models = [np.asarray(m, np.float64).reshape(3, 4) for m in models]
    if refine is not None:   # 2'. GlobalOpt over mutual-nearest detections (host)
        from . import globalopt
        gres = globalopt.compute(len(models), globalopt.correspondences(points, models, radius),
                                 model=refine, fixed=(0,))
        if gres is not None:   # (a caught fit failure keeps the tiles' models as they stand, as the reference)
            if gres.failure and log:
                log(gres.failure)
            models = [globalopt.concatenate(c, m) for c, m in zip(gres.models, models)]
        t = lap("register", t)
    corr = corresponding_detections(points, models, radius, device=f"cuda:{device}")   # 2. (registration given)
    t = lap("correspondences", t)
    imgs, ws, info = input_prep.prepare_inputs(views, models, bb_min, bb_dims, blending_border, blending_range,
                                               weight_type, device=device)   # 3a.
    t = lap("prepare_inputs", t)
    # 3b. ExtractPSF from the corresponding beads, all views at once (a view with no
    # corresponding bead -- registration would have failed for it -- takes all of its
    # detections rather than an all-zero PSF)
    beads = [p[c] if len(c) else p for p, c in zip(points, corr)]
    psfs = [tr for _, tr in psf_mod.extract_psfs(list(views), beads, psf_size, list(models), device=device)]
    psf_mod.release_workspace(device)   # (the bead samples and per-view buffers: HBM the RL session can use)
    t = lap("extract_psf", t)
    sd = {}
    if digest:   # (outside the timed stages' accounting: after the lap)
        # one volume on the host at a time (a C4 timepoint is 16 volumes of 768^3 float32)
        sd["inputs"] = _sha(x.cpu().numpy() for x in list(imgs) + list(ws))
        sd["psfs"] = _sha(np.ascontiguousarray(p, np.float32) for p in psfs)
        sd["corresponding"] = _sha(np.ascontiguousarray(c, np.int64) for c in corr)
        t = time.perf_counter()
    shape = tuple(imgs[0].shape)
    t_setup = t
    sess = Session((shape[2], shape[1], shape[0]), device=device)            # 4. MVDeconvolution
    try:
        t = lap("rl_setup_create", t)
        for i, w, k in zip(imgs, ws, psfs):
            sess.add_view_device(i.data_ptr(), w.data_ptr(), k)
        t = lap("rl_setup_add_views", t)
        sess.init(psftype)
        sess.init_psi()
        engine = {"fft_dims_xyz": list(sess.fft_dims(0)), "zpass_mode": sess.zpass_mode(0),
                  "kernel_planes": sess.kernel_planes(0)}
        t = lap("rl_setup_init", t)
        ms["rl_setup"] = round((t - t_setup) * 1e3, 2)
        stats = sess.run(iterations, lam)
        engine["xpass_mode"] = sess.xpass_mode(0)
        sess.apply_mask()
        t = lap("rl_iterations", t)
        psi = torch.empty(shape, dtype=torch.float32, device=imgs[0].device)
        _lib.check(sess.lib.mvd_get_psi(sess.h, C.cast(C.c_void_p(psi.data_ptr()), _lib._pf)))
    finally:
        sess.close()
    del imgs, ws
    lap("rl_result", t)
    return TimepointResult(psi, points, corr, psfs, stats, ms, engine, sd, models, gres)


def _sha(parts) -> str:
    """SHA-256 of the concatenated bytes of `parts` (arrays), fed one part at a time."""
    import hashlib
    h = hashlib.sha256()
    for a in parts:
        h.update(memoryview(np.ascontiguousarray(a)).cast("B"))
    return h.hexdigest()


class Pipeline:
    """The per-timepoint driver held across a time series (BASELINE configs[3]): the
    parameters of every stage, and the device whose library-side state (the DoG
    workspace, the PSF / resampling scratch, plan caches) carries over from one
    timepoint to the next -- as the reference's plugin processes timepoint after
    timepoint (EfficientBayesianBased.java:166-286).  Carried state must not change a
    result: timepoint t processed after others equals timepoint t processed alone
    (``result_digest``; tests/test_gpu_scale.py)."""

    def __init__(self, **params):
        self.params = params

    def process(self, views, models, bb_min, bb_dims, log=None, digest=False) -> TimepointResult:
        return process_timepoint(views, models, bb_min, bb_dims, log=log, digest=digest, **self.params)


def result_digest(res: TimepointResult) -> dict:
    """SHA-256 of psi's bytes and of the RL statistics, plus the detection counts."""
    import hashlib
    psi = res.psi.cpu().numpy()
    return {**{f"{k}_sha256": v for k, v in res.stage_digests.items()},
            "psi_sha256": hashlib.sha256(psi.tobytes()).hexdigest(),
            "stats_sha256": hashlib.sha256(np.ascontiguousarray(res.stats, np.float64).tobytes()).hexdigest(),
            "points_sha256": hashlib.sha256(b"".join(np.ascontiguousarray(p, np.float64).tobytes()
                                                     for p in res.points)).hexdigest()}
