"""Host-side mirror of the legacy simultaneous-update multiview RL (opt-in mode).

Mirrors ``mpicbg.spim.postprocessing.deconvolution`` (paths under
/root/reference/src/main/java/mpicbg/spim/postprocessing/deconvolution/):

  LucyRichardsonFFT                     LucyRichardsonFFT.java:7-38 (image, weight, kernel)
  LucyRichardsonMultiViewDeconvolution  LucyRichardsonMultiViewDeconvolution.java:19-491
    .lucyRichardsonMultiView(data, minIterations, maxIterations, multiplicative,
                             lambda, numThreads)                            :24-358

The arithmetic runs in libspimdecon.so (``lrsim_*``, include/spimdecon.h section 10).
With ``comm_id`` / ``nranks`` / ``rank`` the views are sharded over RCCL ranks (view v on
rank v % nranks, as the reference hands view v to thread v % numThreads, :127-128) and
the per-voxel combination of the views' corrections is one all-reduce per iteration.
Volumes are numpy float32 [z, y, x] arrays (x fastest).

This is NOT the maintained ``MVDeconvolution`` rule (``decon.py``): the reference's
plugin comments the call out (``fiji/plugin/Multi_View_Deconvolution.java:226-231``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check

MIN_VALUE = 0.0001   # LucyRichardsonMultiViewDeconvolution.java:30 (double)


def _vol(a, name):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 3:
        raise ValueError(f"{name} must be a 3D [z, y, x] array, got shape {a.shape}")
    return a


class LucyRichardsonFFT:
    """One view (LucyRichardsonFFT.java:14-22).  ``cpus_per_view`` is accepted for API
    parity (the FFTs run on the GPU).  ``image`` / ``weight`` may be None for a view
    another rank owns; ``kernel`` may then be a shape-only placeholder (its dims are
    needed on every rank)."""

    def __init__(self, image, weight, kernel, cpus_per_view: int = 1):
        self.image = None if image is None else _vol(image, "image")
        self.weight = None if weight is None else _vol(weight, "weight")
        self.kernel = _vol(kernel, "kernel")
        if any(s % 2 == 0 for s in self.kernel.shape):
            raise ValueError(f"kernel dims must be odd, got {self.kernel.shape}")
        self.cpus_per_view = cpus_per_view
        self.view_contribution = None

    def getImage(self):
        return self.image

    def getWeight(self):
        return self.weight

    def getKernel(self):
        return self.kernel


class LucyRichardsonMultiViewDeconvolution:
    """LucyRichardsonMultiViewDeconvolution.java:19-358."""

    debug = False
    debugInterval = 10

    @staticmethod
    def lucyRichardsonMultiView(data, minIterations, maxIterations, multiplicative, lambda_, numThreads,
                                device: int = 0, nranks: int = 1, rank: int = 0, comm_id: bytes | None = None,
                                stats_out: list | None = None, avg_out: list | None = None):
        return lucy_richardson_multi_view(data, maxIterations, multiplicative, lambda_, device=device,
                                          nranks=nranks, rank=rank, comm_id=comm_id, stats_out=stats_out,
                                          avg_out=avg_out)


def lucy_richardson_multi_view(data, max_iterations: int, multiplicative: bool, lambda_: float, device: int = 0,
                               nranks: int = 1, rank: int = 0, comm_id: bytes | None = None,
                               stats_out: list | None = None, avg_out: list | None = None,
                               devices=None) -> np.ndarray:
    """Runs LucyRichardsonMultiViewDeconvolution.lucyRichardsonMultiView (:24-358) and
    returns psi.  ``minIterations`` of the reference is unused there too; the do-while
    (:98-351) runs max(1, maxIterations) iterations.  ``stats_out`` receives
    (sumChange, maxChange) per iteration, ``avg_out`` the initial average (:63).
    ``devices``: several GPUs of this process (view v on devices[v % len]; ids may
    repeat), as the reference's threads; not combined with RCCL ranks."""
    if not data:
        raise ValueError("no views")
    lib = _lib.load()
    dims = None
    for v in data:
        if v.image is not None:
            dims = v.image.shape
            break
    if dims is None:
        raise ValueError("at least one view must carry its image on every rank that owns one")
    nz, ny, nx = dims
    d = (C.c_int64 * 3)(nx, ny, nz)
    h = C.c_void_p()
    cid = None if comm_id is None else C.create_string_buffer(bytes(comm_id), 128)
    if devices is not None:
        if nranks != 1 or comm_id is not None:
            raise ValueError("devices and RCCL ranks cannot be combined")
        dv = (C.c_int * len(devices))(*[int(x) for x in devices])
        check(lib.lrsim_create_devices(d, dv, len(devices), C.byref(h)))
    else:
        check(lib.lrsim_create(d, int(device), int(nranks), int(rank), cid, C.byref(h)))
    try:
        for i, v in enumerate(data):
            kz, ky, kx = v.kernel.shape
            kd = np.array([kx, ky, kz], np.int32)
            mine = i % nranks == rank
            if mine:
                for a, nm in ((v.image, "image"), (v.weight, "weight")):
                    if a is None:
                        raise ValueError(f"view {i} is owned by rank {rank} and needs its {nm} "
                                         "(normAllImages reads every weight, :401)")
                    if a.shape != tuple(dims):
                        raise ValueError(f"view {i}: {nm} shape {a.shape} != {tuple(dims)}")
                check(lib.lrsim_add_view(h, v.image.ctypes.data, v.weight.ctypes.data, v.kernel.ctypes.data,
                                         kd.ctypes.data_as(_lib._pi)))
            else:
                check(lib.lrsim_add_view(h, None, None, None, kd.ctypes.data_as(_lib._pi)))
        avg = C.c_double()
        check(lib.lrsim_init(h, C.byref(avg)))
        if avg_out is not None:
            avg_out.append(avg.value)
        iters = max(1, int(max_iterations))
        st = np.zeros(2 * iters, np.float64)
        check(lib.lrsim_run(h, iters, 1 if multiplicative else 0, float(lambda_),
                            st.ctypes.data_as(_lib._pd)))
        if stats_out is not None:
            stats_out.extend((float(st[2 * i]), float(st[2 * i + 1])) for i in range(iters))
        out = np.empty(dims, np.float32)
        check(lib.lrsim_get_psi(h, out.ctypes.data))
        return out
    finally:
        lib.lrsim_destroy(h)


def views_of_rank(nviews: int, nranks: int, rank: int) -> list:
    """The views rank ``rank`` owns: v % nranks == rank (LRMV:127-128 over threads)."""
    return [v for v in range(nviews) if v % nranks == rank]
