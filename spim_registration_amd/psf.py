"""Host-side mirror of ``ExtractPSF``.

spim/process/fusion/deconvolution/ExtractPSF.java: PSFs are extracted from the
bead detections of each view (``extractNextImg``: ``extractPSFLocal`` +
``normalize``), transformed with the view model (``transformPSF``), and
averaged / max-projected for display -- each a GPU kernel in ``csrc/psf.hip``
behind ``spim_extract_psf`` & co.  Images are [z, y, x] float32 arrays, sizes
and locations (x, y, z) as in the reference.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, fptr


def _dims(a: np.ndarray):
    return (C.c_int64 * 3)(a.shape[2], a.shape[1], a.shape[0])


def _model(model):
    return (C.c_double * 12)(*[float(v) for v in np.asarray(model, np.float64).reshape(12)])


def transformed_size(psf_size, model):
    """transformPSF (:309-346): (odd size (x, y, z), offset)."""
    lib = _lib.load()
    out = (C.c_int64 * 3)()
    off = (C.c_double * 3)()
    check(lib.spim_psf_transformed_size((C.c_int64 * 3)(*[int(v) for v in psf_size]), _model(model), out, off))
    return [int(v) for v in out], [float(v) for v in off]


def transform_psf(psf: np.ndarray, model, device: int = 0) -> np.ndarray:
    """ExtractPSF.transformPSF (:309-346, :424-460)."""
    lib = _lib.load()
    psf = np.ascontiguousarray(psf, np.float32)
    (nx, ny, nz), _ = transformed_size((psf.shape[2], psf.shape[1], psf.shape[0]), model)
    out = np.empty((nz, ny, nx), np.float32)
    check(lib.spim_transform_psf(fptr(psf), _dims(psf), _model(model), fptr(out), device))
    return out


def extract_psf(img, locations, psf_size, model=None, device: int = 0):
    """ExtractPSF.extractNextImg (:260-279): (normalised PSF in the view's
    calibration, transformed PSF or None without a model).  img: [z, y, x]
    float32 numpy array or a torch tensor already on the GPU."""
    lib = _lib.load()
    on_dev = 0
    if hasattr(img, "is_cuda") and img.is_cuda:
        img = img.contiguous().float()
        ptr, shape, on_dev = C.c_void_p(img.data_ptr()), tuple(img.shape), 1
    else:
        img = np.ascontiguousarray(img, np.float32)
        ptr, shape = C.c_void_p(img.ctypes.data), img.shape
    dims = (C.c_int64 * 3)(shape[2], shape[1], shape[0])
    locs = np.ascontiguousarray(np.asarray(locations, np.float64).reshape(-1, 3))
    size = [int(v) for v in psf_size]
    orig = np.empty((size[2], size[1], size[0]), np.float32)
    trans = None
    if model is not None:
        (tx, ty, tz), _ = transformed_size(size, model)
        trans = np.empty((tz, ty, tx), np.float32)
    check(lib.spim_extract_psf(ptr, dims, on_dev, locs.ctypes.data_as(_lib._pd) if len(locs) else None,
                               len(locs), (C.c_int64 * 3)(*size), _model(model) if model is not None else None,
                               fptr(orig), fptr(trans) if trans is not None else None, device))
    return orig, trans


def extract_psfs(imgs, locations, psf_size, models=None, device: int = 0):
    """extract_psf for the views of a timepoint in one call (ExtractPSF.extract over
    the views): the views run concurrently on the GPU; results are identical to
    per-view extract_psf calls.  imgs: torch tensors on the GPU (all of them) or
    numpy arrays; models: per view, or None."""
    lib = _lib.load()
    n = len(imgs)
    on_dev = 1 if n and hasattr(imgs[0], "is_cuda") and imgs[0].is_cuda else 0
    keep, ptrs, dims = [], [], []
    for im in imgs:
        if on_dev:
            if not (hasattr(im, "is_cuda") and im.is_cuda):
                raise ValueError("imgs must be all GPU tensors or all host arrays")
            im = im.contiguous().float()
            ptrs.append(im.data_ptr())
        else:
            im = np.ascontiguousarray(im, np.float32)
            ptrs.append(im.ctypes.data)
        keep.append(im)
        dims += [im.shape[2], im.shape[1], im.shape[0]]
    locs = [np.ascontiguousarray(np.asarray(l, np.float64).reshape(-1, 3)) for l in locations]
    size = [int(v) for v in psf_size]
    origs = [np.empty((size[2], size[1], size[0]), np.float32) for _ in range(n)]
    trans = None
    if models is not None:
        trans = []
        for m in models:
            (tx, ty, tz), _ = transformed_size(size, m)
            trans.append(np.empty((tz, ty, tx), np.float32))
    vp = C.c_void_p * max(n, 1)
    check(lib.spim_extract_psfs(n, vp(*ptrs), (C.c_int64 * max(3 * n, 1))(*dims), on_dev,
                                vp(*[l.ctypes.data if len(l) else None for l in locs]),
                                (C.c_int64 * max(n, 1))(*[len(l) for l in locs]), (C.c_int64 * 3)(*size),
                                (C.c_double * (12 * n))(*[float(v) for m in models
                                                          for v in np.asarray(m, np.float64).reshape(12)])
                                if models is not None else None,
                                vp(*[o.ctypes.data for o in origs]),
                                vp(*[t.ctypes.data for t in trans]) if trans is not None else None, device))
    return [(origs[v], trans[v] if trans is not None else None) for v in range(n)]


def release_workspace(device: int = -1) -> None:
    """Frees the buffers and streams the PSF extraction keeps per view between calls
    (spim_psf_release_workspace; -1: every device)."""
    check(_lib.load().spim_psf_release_workspace(int(device)))


def average_transformed_psf(psfs, device: int = 0) -> np.ndarray:
    """ExtractPSF.computeAverageTransformedPSF (:164-208)."""
    lib = _lib.load()
    psfs = [np.ascontiguousarray(p, np.float32) for p in psfs]
    n = len(psfs)
    ptrs = (_lib._pf * n)(*[fptr(p) for p in psfs])
    dims = (C.c_int64 * (3 * n))(*[v for p in psfs for v in (p.shape[2], p.shape[1], p.shape[0])])
    ad = (C.c_int64 * 3)()
    check(lib.spim_average_transformed_psf(n, ptrs, dims, None, ad, device))
    out = np.empty((ad[2], ad[1], ad[0]), np.float32)
    check(lib.spim_average_transformed_psf(n, ptrs, dims, fptr(out), ad, device))
    return out


def max_projection(img: np.ndarray, min_dim: int = -1, device: int = 0):
    """ExtractPSF.computeMaxProjection (:110-162): (2-D [b, a] projection with
    a, b the remaining dims in order, the projected dim)."""
    lib = _lib.load()
    img = np.ascontiguousarray(img, np.float32)
    od = (C.c_int64 * 2)()
    used = C.c_int()
    check(lib.spim_max_projection(fptr(img), _dims(img), min_dim, None, od, C.byref(used), device))
    out = np.empty((od[1], od[0]), np.float32)
    check(lib.spim_max_projection(fptr(img), _dims(img), min_dim, fptr(out), od, C.byref(used), device))
    return out, used.value
