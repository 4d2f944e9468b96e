"""Host-side mirror of the deconvolution input preparation.

``ProcessForDeconvolution.fuseStacksAndGetPSFs``
(spim/process/fusion/deconvolution/ProcessForDeconvolution.java:159-384): each
view is resampled into the fused bounding box through the inverse of its
affine model, cosine blending weights are computed at the same source
positions, normalised across views (``WeightNormalizer``) and adjusted for the
OSEM speed-up -- all on the GPU in ``spim_prepare_inputs``.
"""
from __future__ import annotations

import ctypes as C
from enum import IntEnum

import numpy as np

from . import _lib
from ._lib import check, fptr


class WeightType(IntEnum):
    """ProcessForDeconvolution.WeightType members on the deconvolution path."""
    NO_WEIGHTS = 0
    PRECOMPUTED_WEIGHTS = 1
    VIRTUAL_WEIGHTS = 2


def prepare_inputs(srcs, models, bb_min, bb_dims, blending_border=(-8, -8, -8), blending_range=(12, 12, 12),
                   weight_type: WeightType = WeightType.VIRTUAL_WEIGHTS, osem_index: int = 0,
                   osem_speedup: float = 1.0, ij_threads: int = 8, device: int = 0):
    """srcs: [z, y, x] float32 stacks; models: 3x4 (source -> world) affine per
    view; bb_min / bb_dims: (x, y, z).  Returns (imgs, weights, info) with
    imgs/weights [z, y, x] float32 per view and info = {osem, min_overlap,
    avg_overlap}."""
    lib = _lib.load()
    V = len(srcs)
    if V < 1 or len(models) != V:
        raise ValueError("need one model per view")
    if all(hasattr(s, "is_cuda") and s.is_cuda for s in srcs):
        return _prepare_inputs_device(lib, srcs, models, bb_min, bb_dims, blending_border, blending_range,
                                      weight_type, osem_index, osem_speedup, ij_threads, device)
    srcs = [np.ascontiguousarray(s, np.float32) for s in srcs]
    views = (_lib.ViewSource * V)()
    for v, (s, m) in enumerate(zip(srcs, models)):
        if s.ndim != 3:
            raise ValueError("sources must be 3D [z, y, x]")
        views[v].img = fptr(s)
        views[v].dims[:] = [s.shape[2], s.shape[1], s.shape[0]]
        views[v].model[:] = [float(x) for x in np.asarray(m, np.float64).reshape(12)]
    p = _lib.InputParams()
    lib.spim_input_params_default(C.byref(p))
    p.bb_min[:] = [int(x) for x in bb_min]
    p.bb_dims[:] = [int(x) for x in bb_dims]
    p.blending_border[:] = [float(x) for x in blending_border]
    p.blending_range[:] = [float(x) for x in blending_range]
    p.weight_type = int(weight_type)
    p.osem_index = int(osem_index)
    p.osem_speedup = float(osem_speedup)
    p.ij_threads = int(ij_threads)
    p.device = int(device)
    shape = (int(bb_dims[2]), int(bb_dims[1]), int(bb_dims[0]))
    imgs = [np.empty(shape, np.float32) for _ in range(V)]
    ws = [np.empty(shape, np.float32) for _ in range(V)]
    ip = (_lib._pf * V)(*[fptr(a) for a in imgs])
    wp = (_lib._pf * V)(*[fptr(a) for a in ws])
    osem, mn, av = C.c_double(), C.c_int(), C.c_double()
    check(lib.spim_prepare_inputs(V, views, C.byref(p), ip, wp, C.byref(osem), C.byref(mn), C.byref(av)))
    return imgs, ws, {"osem": osem.value, "min_overlap": mn.value, "avg_overlap": av.value}


def _prepare_inputs_device(lib, srcs, models, bb_min, bb_dims, blending_border, blending_range, weight_type,
                           osem_index, osem_speedup, ij_threads, device):
    """prepare_inputs for torch tensors on the GPU: read in place, results as torch
    tensors on the same device (no host round trip)."""
    import torch
    V = len(srcs)
    srcs = [s.contiguous().float() for s in srcs]
    torch.cuda.synchronize(srcs[0].device)   # the library runs on its own stream
    views = (_lib.ViewSource * V)()
    for v, (s, m) in enumerate(zip(srcs, models)):
        if s.dim() != 3:
            raise ValueError("sources must be 3D [z, y, x]")
        views[v].img = C.cast(C.c_void_p(s.data_ptr()), _lib._pf)
        views[v].dims[:] = [s.shape[2], s.shape[1], s.shape[0]]
        views[v].model[:] = [float(x) for x in np.asarray(m, np.float64).reshape(12)]
    p = _lib.InputParams()
    lib.spim_input_params_default(C.byref(p))
    p.bb_min[:] = [int(x) for x in bb_min]
    p.bb_dims[:] = [int(x) for x in bb_dims]
    p.blending_border[:] = [float(x) for x in blending_border]
    p.blending_range[:] = [float(x) for x in blending_range]
    p.weight_type = int(weight_type)
    p.osem_index = int(osem_index)
    p.osem_speedup = float(osem_speedup)
    p.ij_threads = int(ij_threads)
    p.device = int(device)
    p.src_on_device = 1
    p.out_on_device = 1
    shape = (int(bb_dims[2]), int(bb_dims[1]), int(bb_dims[0]))
    imgs = [torch.empty(shape, dtype=torch.float32, device=srcs[0].device) for _ in range(V)]
    ws = [torch.empty(shape, dtype=torch.float32, device=srcs[0].device) for _ in range(V)]
    ip = (_lib._pf * V)(*[C.cast(C.c_void_p(a.data_ptr()), _lib._pf) for a in imgs])
    wp = (_lib._pf * V)(*[C.cast(C.c_void_p(a.data_ptr()), _lib._pf) for a in ws])
    osem, mn, av = C.c_double(), C.c_int(), C.c_double()
    check(lib.spim_prepare_inputs(V, views, C.byref(p), ip, wp, C.byref(osem), C.byref(mn), C.byref(av)))
    return imgs, ws, {"osem": osem.value, "min_overlap": mn.value, "avg_overlap": av.value}


def fuse_weighted_average(srcs, models, bb_min, bb_dims, downsampling: float = 1.0, interpolation: int = 1,
                          use_blending: bool = True, blending_borders=None, blending_ranges=None,
                          device: int = 0) -> np.ndarray:
    """Weighted-average fusion (spim/process/fusion/weightedavg/ProcessParalell*.java):
    [z, y, x] float32 fused volume.  blending_borders / ranges: (x, y, z) per view."""
    lib = _lib.load()
    V = len(srcs)
    srcs = [np.ascontiguousarray(s, np.float32) for s in srcs]
    views = (_lib.ViewSource * V)()
    for v, (s, m) in enumerate(zip(srcs, models)):
        views[v].img = fptr(s)
        views[v].dims[:] = [s.shape[2], s.shape[1], s.shape[0]]
        views[v].model[:] = [float(x) for x in np.asarray(m, np.float64).reshape(12)]
    p = _lib.FusionParams()
    lib.spim_fusion_params_default(C.byref(p))
    p.bb_min[:] = [int(x) for x in bb_min]
    p.bb_dims[:] = [int(x) for x in bb_dims]
    p.downsampling = float(downsampling)
    p.interpolation = int(interpolation)
    p.use_blending = int(bool(use_blending))
    p.device = int(device)
    b = r = None
    if use_blending:
        b = np.ascontiguousarray(np.asarray(blending_borders, np.float32).reshape(V, 3))
        r = np.ascontiguousarray(np.asarray(blending_ranges, np.float32).reshape(V, 3))
    out = np.empty((int(bb_dims[2]), int(bb_dims[1]), int(bb_dims[0])), np.float32)
    check(lib.spim_fuse_weighted_average(V, views, C.byref(p), fptr(b) if b is not None else None,
                                         fptr(r) if r is not None else None, fptr(out)))
    return out
